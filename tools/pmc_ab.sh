#!/bin/bash
# VALU issue counters of each build named on the command line (one
# rocprofv3 --pmc pass per library; run through gpurun from the repo root):
#   bash tools/pmc_ab.sh libfri_amd.so libfri_amd_base.so
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  FRI_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/pmc_${L%.so} -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras > /dev/null
done
