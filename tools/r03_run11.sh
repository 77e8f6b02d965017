# reproduce the stall in the 2^20 non-canonical case with stack dumps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "noncanonical" > gpurun_out/r03_devcheck_repro.log 2>&1
echo "rc=$?" >> gpurun_out/r03_devcheck_repro.log
