# parity of the default build, then interleaved commit A/B and a kernel-trace
# A/B against a variant:  bash tools/r03_ab_run.sh TAG VARIANT.so
set -o pipefail
TAG=$1; V=$2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/r03_${TAG}_parity.log 2>&1 || exit 1
bash tools/abn.sh 4 20 libfri_amd.so $V > gpurun_out/r03_ab_${TAG}.txt || exit 2
bash tools/kt_ab.sh 1 libfri_amd.so $V || exit 3
