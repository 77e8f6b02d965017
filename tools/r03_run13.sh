# six-level quad leaf kernel (DEEP): parity, commit A/B against no-deep and deep-from-2^22, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_prover.py -m gpu > gpurun_out/r03_deep_parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_dist.py -m gpu -k "matches_single or loopback" > gpurun_out/r03_deep_dist.log 2>&1 || exit 2
bash tools/abn.sh 4 20 libfri_amd.so libfri_amd_nodeep.so libfri_amd_deep22.so > gpurun_out/r03_ab_deep.txt || exit 3
bash tools/kt_ab.sh 1 libfri_amd.so libfri_amd_nodeep.so || exit 4
