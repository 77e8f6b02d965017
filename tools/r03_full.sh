# the driver's round-end checks, as it runs them: the whole -m gpu suite, then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 900 --timeout-method thread > gpurun_out/r03_full_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit 2
