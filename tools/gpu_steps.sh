#!/bin/bash
# GPU evidence steps, run through gpurun from the repo root:
#
#   bash tools/gpu_steps.sh STEP TAG [args]
#
# Every GPU step runs under its own time limit; the first failure ends the
# script (set -e), so a fault or timeout never starts another GPU step.
# Output goes to gpurun_out/TAG_*; the files worth keeping are copied into
# profiles/ by hand (profiles/README.md lists them).
#
#   suite   TAG            the driver's round-end checks: the whole -m gpu suite, then smoke()
#   parity  TAG            the parity tests only (1-GPU parity, fuzz, prover, sharded vs single)
#   collect TAG            bench lines, rocprofv3 kernel stats, PMC traffic (collect_profiles.sh)
#                          and the LDE passes at 2^24 / 2^28 (pmc_lde.sh)
#   proj    TAG [L...]     1-GPU bench lines at 2^28 and 2^24, then one rank's share of the
#                          sharded commit at each codeword L (default 28 24) over 2, 4, 8 ranks
#                          (loopback transport, recorded degree schedule, inputs resident)
#   projkt  TAG [L]        kernel trace of one rank's share (rank 0 of 8) at 2^L (default 28),
#                          summarised per kernel (tools/shard_projection.py)
#   hiptrace TAG           HIP API + kernel trace around the commit graph (host turnaround)
#   final   TAG            end-of-round evidence in one call: suite (+ smoke), collect, proj,
#                          and the 5000-shape commit fuzz
#   lanesab TAG A.so B.so  commit lanes (1 and 3 lanes) and synchronous commits, the two library
#                          builds interleaved over 3 rounds (tools/lanes_probe.py, tools/abn.sh)
set -e
STEP=${1:?step}
TAG=${2:?tag}
shift 2
R=$PWD
O=$R/gpurun_out
mkdir -p $O
case $STEP in
suite)
    timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 900 --timeout-method thread \
        > $O/${TAG}_full_gpu.log 2>&1
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
    ;;
parity)
    timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
        tests/test_gpu_fuzz.py tests/test_gpu_prover.py tests/test_gpu_pipelined.py -m gpu > $O/${TAG}_parity.log 2>&1
    timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_dist.py -m gpu \
        -k "matches_single or loopback" > $O/${TAG}_dist.log 2>&1
    ;;
collect)
    bash tools/collect_profiles.sh $TAG
    bash tools/pmc_lde.sh 28 gpurun_out/prof_$TAG/pmc_lde_2p28.json
    bash tools/pmc_lde.sh 24 gpurun_out/prof_$TAG/pmc_lde_2p24.json
    ;;
proj)
    LS=${*:-28 24}
    timeout -k 10 300 python3 bench.py --log-n 28 --steps 5 --warmup 2 --no-cpu-baseline --no-extras \
        > $O/${TAG}_proj_bench28.json
    timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-extras > $O/${TAG}_proj_bench24.json
    for W in 8 4 2; do for L in $LS; do
        timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world $W --rank 0 --steps 5 \
            > $O/${TAG}_proj_wall_${L}_w$W.txt 2>&1
    done; done
    ;;
projkt)
    L=${1:-28}
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${TAG}_projkt_$L -o run -- \
        python3 $R/tools/shard_projection.py --log-n $L --world 8 --rank 0 --steps 3 > $O/${TAG}_projkt_$L.txt 2>&1
    python3 $R/tools/shard_projection.py --summarise $O/${TAG}_projkt_$L >> $O/${TAG}_projkt_$L.txt
    ;;
hiptrace)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
        -d $O/${TAG}_hiptrace -o run -- \
        python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-profile \
        > $O/${TAG}_hiptrace.json 2> $O/${TAG}_hiptrace.err
    ;;
final)
    bash tools/gpu_steps.sh suite $TAG
    bash tools/gpu_steps.sh collect $TAG
    bash tools/gpu_steps.sh proj $TAG
    FRI_FUZZ_N=5000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -q -m gpu --timeout 500 \
        --timeout-method thread > $O/${TAG}_fuzz5000.log 2>&1
    ;;
lanesab)
    for i in 1 2 3; do for lib in "$@"; do
        echo "== $(basename $lib) round $i" >> $O/${TAG}_lanesab.txt
        FRI_AMD_LIB=$lib timeout -k 10 120 python3 tools/lanes_probe.py --pairs 1:1,3:3 --commits 30 \
            >> $O/${TAG}_lanesab.txt 2>&1
    done; done
    timeout -k 10 600 bash tools/abn.sh 3 20 "$@" > $O/${TAG}_syncab.txt 2>&1
    ;;
*)
    echo "unknown step $STEP" >&2
    exit 2
    ;;
esac
