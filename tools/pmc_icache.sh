#!/bin/bash
# Instruction-cache counters of the layer kernels (one --pmc pass; run
# through gpurun from the repo root):  bash tools/pmc_icache.sh [lib.so ...]
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
for L in "${@:-libfri_amd.so}"; do
  FRI_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU \
    --output-format csv -d $R/gpurun_out/pmc_ic_${L%.so} -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras > /dev/null
done
