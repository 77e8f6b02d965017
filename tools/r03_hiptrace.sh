# host API timing around the commit graph: hip + kernel trace of a short bench
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/hiptrace -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-profile > $R/gpurun_out/hiptrace.json 2> $R/gpurun_out/hiptrace.err
