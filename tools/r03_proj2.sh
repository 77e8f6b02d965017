# sharded per-rank work at 2^28 x 8 with the coefficient folds serialised (no side stream)
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/proj_28s -o run -- \
    python3 $R/tools/shard_projection.py --log-n 28 --world 8 --rank 0 --steps 3 --serial-coef > $R/gpurun_out/proj_28s.txt 2>&1
python3 $R/tools/shard_projection.py --summarise $R/gpurun_out/proj_28s >> $R/gpurun_out/proj_28s.txt
