"""Leaf kernel of a commit (k_layer_leaf<false, true>) against the same kernel
without the coefficient task (k_layer_leaf<false, false>: fri_merkle_root,
and the block trees of a sharded commit) on 2^24 values; run under
rocprofv3 --kernel-trace and compare the two kernels' durations."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fri_amd  # noqa: E402
import fri_oracle as fo  # noqa: E402

ctx = fri_amd.Context(0, 24)
c = fo.splitmix64_np(42, 1 << 21).astype("uint32")
vals = fo.splitmix64_np(7, 1 << 24).astype("uint32")
for _ in range(5):
    ctx.commit(c, 24)
    ctx.merkle_root(vals)
print("done", flush=True)
ctx.close()
