#!/bin/bash
# 2^24 coset LDE build: parity of the 2^24 LDE/commit cases, kernel trace
# (per-kernel averages), then A/B against the three-pass build.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "lde or commit_2p24 or golden" > gpurun_out/r03_lde24_parity2.log 2>&1 || { echo parity failed; tail -20 gpurun_out/r03_lde24_parity2.log; exit 1; }
tail -1 gpurun_out/r03_lde24_parity2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_lde24_kt -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-profile > gpurun_out/r03_lde24_kt.json 2>/dev/null || exit 1
f=$(find gpurun_out/r03_lde24_kt -name '*kernel_stats.csv' | head -1)
grep -E "lde24|ntt_pass|Name" "$f" | cut -c1-160
timeout -k 10 600 tools/ab.sh libfri_amd.so libfri_amd_ab3p.so 3 20 > gpurun_out/r03_lde24_ab2.txt 2>&1 || exit 1
cat gpurun_out/r03_lde24_ab2.txt
