# device-side input validation: new tests, commit parity, the sharded case, pcie_inclusive
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_prover.py -m gpu > gpurun_out/r03_devcheck_parity.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_dist.py -m gpu -k "matches_single" > gpurun_out/r03_devcheck_dist.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py > gpurun_out/r03_devcheck_bench.json 2> gpurun_out/r03_devcheck_bench.err || exit 3
