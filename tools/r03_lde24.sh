#!/bin/bash
# 2^24 coset LDE (NTT_LDE24): parity of the LDE / commit cases at 2^24, then
# an interleaved A/B against the three-pass build (lib/libfri_amd_ab3p.so,
# -DNTT_LDE24=0) and a kernel trace of the new build.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "lde or interpolate or commit_2p24 or golden or matches_fast_oracle or noncanonical or tiny" \
  > gpurun_out/r03_lde24_parity.log 2>&1 || { echo parity failed; exit 1; }
tail -1 gpurun_out/r03_lde24_parity.log
timeout -k 10 600 tools/ab.sh libfri_amd.so libfri_amd_ab3p.so 4 20 > gpurun_out/r03_lde24_ab.txt 2>&1 || exit 1
cat gpurun_out/r03_lde24_ab.txt
for lib in libfri_amd.so libfri_amd_ab3p.so; do
  FRI_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
    > gpurun_out/r03_lde24_bench_$lib.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03_lde24_bench_$lib.json')); print('$lib', d['ms_per_step'], d['roofline']['lde_ntt'])"
done
