# round-3 GPU session: bench.py end to end. N=1 default line; N=8 rehearsals on
# one GPU: RCCL (two ranks on one device cannot form a communicator -> the
# replicas fallback line) and the host-staged transport (the sharded line).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r03_bench_n1.json 2> gpurun_out/r03_bench_n1.err || exit 1
export FRI_RCCL_TIMEOUT_S=30
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r03_bench_n8_rccl1gpu.json 2> gpurun_out/r03_bench_n8_rccl1gpu.err || exit 2
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 \
    bench.py --gpus 8 --steps 3 --warmup 1 --transport host > gpurun_out/r03_bench_n8_host.json 2> gpurun_out/r03_bench_n8_host.err || exit 3
