#!/bin/bash
# Round evidence on one MI355X (run through gpurun from the repo root):
#   bash tools/collect_profiles.sh TAG
# writes gpurun_out/prof_TAG/: bench line (defaults), rocprofv3 kernel stats +
# trace of the same bench command, FETCH_SIZE / WRITE_SIZE passes (separate
# runs, MI355X_MICROARCH.md HBM recipe) -> pmc_traffic.json, and the 2^20 /
# 2^28 bench lines.  Every GPU step has its own time limit; the first failure
# ends the script.
set -e
TAG=${1:-rNN}
R=$PWD
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python3 bench.py --log-n 20 --steps 50 --no-cpu-baseline --no-extras > $O/bench_2p20.json 2>> $O/bench.err
timeout -k 10 300 python3 bench.py --log-n 28 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/bench_2p28.json 2>> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench_under_rocprof.json 2> $O/rocprof.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-extras > /dev/null 2>> $O/rocprof.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-extras > /dev/null 2>> $O/rocprof.err
cd $R
python3 tools/pmc_traffic.py $O/fetch $O/write 24 $O/pmc_traffic.json
echo "collected into $O"
