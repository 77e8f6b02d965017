# A/B of sharded-path builds on one rank's share (loopback), interleaved:
#   bash tools/r03_proj_ab.sh ROUNDS A.so B.so ...   -> gpurun_out/proj_ab.txt
set -e
N=$1; shift
for i in $(seq 1 $N); do for lib in "$@"; do for L in 28 24; do
  echo "$lib 2^$L $(FRI_AMD_LIB=$lib timeout -k 10 300 python3 tools/shard_projection.py --log-n $L --world 8 --rank 0 --steps 5 | grep wall)" >> gpurun_out/proj_ab.txt
done; done; done
