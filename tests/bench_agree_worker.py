"""gloo worker for tests/test_bench_host.py: bench.agree_step with rank 1
failing a setup step (as an RCCL attach failing on one rank would)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import bench

    def attach():
        if rank == 1:
            raise RuntimeError("ncclCommInitRank: invalid usage")

    ok1, note1 = bench.agree_step(dist, world, rank, lambda: None, "attach (rccl)")
    ok2, note2 = bench.agree_step(dist, world, rank, attach, "attach (rccl)")
    ok3, note3 = bench.agree_step(dist, world, rank, lambda: False, "first sharded commit 2^28 (strong_primary)")
    with open(os.path.join(sys.argv[1], f"rank{rank}.json"), "w") as f:
        json.dump({"ok": [ok1, ok2, ok3], "notes": [note1, note2, note3]}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
