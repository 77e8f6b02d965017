set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_dist.py -m gpu -k "matches_single or configs4 or loopback" > gpurun_out/r03_coef_dist.log 2>&1 || exit 1
bash tools/r03_proj_ab.sh 3 libfri_amd.so libfri_amd_coefold.so || exit 2
