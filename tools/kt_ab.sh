#!/bin/bash
# Kernel-trace A/B of library builds (interleaved, ROUNDS rounds; run through
# gpurun from the repo root):  bash tools/kt_ab.sh ROUNDS A.so B.so ...
# -> gpurun_out/kt_<lib>_<round>/ (rocprofv3 --kernel-trace --stats)
set -e
R=$PWD
N=$1; shift
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 $N); do for L in "$@"; do
FRI_AMD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_${L%.so}_$i -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-profile > $R/gpurun_out/kt_${L%.so}_$i.json 2>/dev/null
done; done
