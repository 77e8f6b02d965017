# on ONE box: the 1-GPU 2^28 and 2^24 commits (bench) and one rank's share of
# the same codewords sharded over 8 (loopback transport), for the projection
set -e
R=$PWD
timeout -k 10 300 python3 bench.py --log-n 28 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/proj_bench28.json
timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/proj_bench24.json
for L in 28 24; do
timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world 8 --rank 0 --steps 5 > gpurun_out/proj_wall_$L.txt 2>&1
done
for L in 28 24; do
timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world 4 --rank 0 --steps 5 > gpurun_out/proj_wall_${L}_w4.txt 2>&1
timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world 2 --rank 0 --steps 5 > gpurun_out/proj_wall_${L}_w2.txt 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/proj_24 -o run -- \
    python3 $R/tools/shard_projection.py --log-n 24 --world 8 --rank 0 --steps 3 > $R/gpurun_out/proj_24.txt 2>&1
python3 $R/tools/shard_projection.py --summarise $R/gpurun_out/proj_24 >> $R/gpurun_out/proj_24.txt
