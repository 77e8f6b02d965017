# per-rank GPU work of the sharded commit on one device (loopback transport):
# 2^28 x 8 with the coefficient folds beside / before the block trees, 2^24 x 8
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
run() {   # tag log_n extra-args
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/proj_$1 -o run -- \
    python3 $R/tools/shard_projection.py --log-n $2 --world 8 --rank 0 --steps 3 $3 > $R/gpurun_out/proj_$1.txt 2>&1
python3 $R/tools/shard_projection.py --summarise $R/gpurun_out/proj_$1 >> $R/gpurun_out/proj_$1.txt
}
run 28 28 ""
run 28s 28 --serial-coef
run 24 24 ""
