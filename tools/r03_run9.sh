# k_tree_mid<1024>: per-lane nodes on wide levels vs lane pairs everywhere (midold)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "commit or merkle or fold" > gpurun_out/r03_mid_parity.log 2>&1 || exit 1
bash tools/abn.sh 4 20 libfri_amd.so libfri_amd_midold.so > gpurun_out/r03_ab_mid.txt || exit 2
bash tools/kt_ab.sh 1 libfri_amd.so libfri_amd_midold.so || exit 3
