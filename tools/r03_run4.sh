# wide-first-pass A/B (bench --log-n L, two builds interleaved), then the bench rehearsals
set -o pipefail
mkdir -p gpurun_out
for L in 28 25 20; do for lib in libfri_amd_nowide.so libfri_amd.so libfri_amd_nowide.so libfri_amd.so; do
  echo "$lib $L" >> gpurun_out/r03_ab_wide_order.txt
  FRI_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --log-n $L --steps 5 --warmup 1 --no-cpu-baseline --no-extras >> gpurun_out/r03_ab_wide_$L.jsonl 2>> gpurun_out/r03_ab_wide.err || exit 4
done; done
bash tools/r03_run3.sh
