# round-3 GPU session: new tests, then wide-first-pass A/B (bench --log-n L, two builds interleaved)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "releases_scratch" > gpurun_out/r03_scratch.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_dist.py -m gpu > gpurun_out/r03_dist2.log 2>&1 || exit 2
timeout -k 10 200 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cpp_host.py -m gpu > gpurun_out/r03_cpp.log 2>&1 || exit 3
for L in 28 25 20; do for lib in libfri_amd_nowide.so libfri_amd.so libfri_amd_nowide.so libfri_amd.so; do
  FRI_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --log-n $L --steps 5 --warmup 1 --no-cpu-baseline --no-extras >> gpurun_out/r03_ab_wide_$L.jsonl 2>/dev/null || exit 4
  echo "$lib $L" >> gpurun_out/r03_ab_wide_order.txt
done; done
