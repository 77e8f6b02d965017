#!/bin/bash
# HBM traffic per NTT pass of the coset LDE at 2^L (FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 passes, MI355X_MICROARCH.md HBM recipe); run through
# gpurun from the repo root:  bash tools/pmc_lde.sh L OUT_JSON
set -e
L=${1:-28}; OUT=${2:-profiles/pmc_lde.json}
R=$PWD
O=$R/gpurun_out/pmc_lde_$L
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --log-n $L --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-extras"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > /dev/null
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > /dev/null
cd $R
python3 tools/pmc_traffic.py $O/fetch $O/write $L $R/$OUT
