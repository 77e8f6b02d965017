#!/bin/bash
# Issue / wait / LDS counters of the NTT passes (two --pmc passes, <= 8 SQ
# counters each; run through gpurun from the repo root).
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/pmc_ntt1 -o run -- $B > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_ANY \
    --output-format csv -d $R/gpurun_out/pmc_ntt2 -o run -- $B > /dev/null
