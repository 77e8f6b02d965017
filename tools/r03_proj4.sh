# one rank's share of 2^28 / 2^24 sharded over 2, 4, 8 (loopback, inputs resident), same box as a 1-GPU 2^28 bench
set -e
timeout -k 10 300 python3 bench.py --log-n 28 --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/proj_bench28.json
timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/proj_bench24.json
for W in 8 4 2; do for L in 28 24; do
timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world $W --rank 0 --steps 5 > gpurun_out/proj_wall_${L}_w$W.txt 2>&1
done; done
