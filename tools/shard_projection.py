"""Per-rank GPU work of the coset-sharded commit, measured on ONE GPU.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- \
        python3 tools/shard_projection.py --log-n 28 --world 8 --rank 0
    python3 tools/shard_projection.py --summarise DIR

One rank's share of a fri_commit_sharded (BASELINE configs[4]: 2^28 over 8
ranks) runs on a context sized for its shard.  The collectives are the
library's loopback transport (fri_debug_attach_loopback): every exchange
returns this rank's own bytes as a device-to-device copy on the stream RCCL
would use, so the GPU never idles on a host round trip.  The transcript is
NOT the real one (the run is not checked), but every kernel the rank would
launch runs, on data of the right shape.
The coefficient fold is sharded (each rank folds its chunk of poly_k and
the degree comes from the maxima of all ranks' chunks), and the loopback
all-gather returns this rank's own maxima only, so the degree schedule of a
1-GPU commit of the same polynomial is handed to the rehearsal
(fri_debug_loopback_degrees): the same rounds are gated on as in the real run.

The kernel trace then gives the rank's GPU time per commit, and the host
clock the per-commit wall time with collectives that cost only a local copy.
DESIGN.md §7 adds a transfer model for xGMI to that time.
"""
import argparse
import csv
import ctypes
import glob
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def run(log_n, world, rank, steps, serial_coef=False):
    import fri_amd
    import fri_oracle as fo
    logw = world.bit_length() - 1
    d = (1 << log_n) >> 3
    coeffs = fo.splitmix64_np(42, d).astype("uint32")
    one = fri_amd.Context(0, log_n)          # the degree schedule of the real commit
    try:
        one.commit(coeffs, log_n)
        degrees = one.commit_degrees()
    finally:
        one.close()
    ctx = fri_amd.Context(0, log_n - logw)
    ctx.attach_loopback(rank, world)
    ctx.loopback_degrees(degrees)
    if serial_coef:
        ctx.set_profiling(True)              # profiled commits run the coefficient folds on the main stream
    t0 = time.perf_counter()
    for _ in range(steps + 1):
        r = ctx.commit_sharded(coeffs, log_n)
    assert r.n_layers == len(degrees), (r.n_layers, len(degrees))
    print(f"rank {rank}/{world}, 2^{log_n}: {r.n_layers} layers, {r.n_rounds} rounds; "
          f"{steps + 1} loopback commits in {time.perf_counter() - t0:.4f} s", flush=True)
    # timed as bench.py times the sharded step: coefficients resident in HBM
    dptr = ctypes.c_void_p(ctx.input_upload(coeffs))     # the context's input buffer, filled once
    res = fri_amd.CommitResult()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx._check(ctx.lib.fri_commit_sharded_device(ctx.h, dptr, d, log_n, fri_amd.GENERATOR, None, 0, None,
                                                     ctypes.byref(res)))
    print(f"wall time per commit, inputs resident (after the first): "
          f"{1000 * (time.perf_counter() - t0) / steps:.3f} ms", flush=True)
    cur, peak = ctx.device_bytes()
    print(f"HBM per rank: {peak / 2**30:.2f} GiB", flush=True)
    ctx.detach()
    ctx.close()


def summarise(d):
    """Kernel time per commit from the trace: commits are delimited by the
    first NTT pass of the rank's LDE slice; the first commit (plan build,
    cold caches) is dropped."""
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    first = [i for i, r in enumerate(rows)
             if re.search(r"k_ntt_first_wide|k_ntt_pass<\d+, \d+, true", r["Kernel_Name"])]
    segs = [rows[a:b] for a, b in zip(first, first[1:] + [len(rows)])][1:]
    per = {}
    for seg in segs:
        seg = [r for r in seg if "rocclr" not in r["Kernel_Name"]]   # the loopback copies
        for r in seg:
            key = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[key] = per.get(key, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / len(segs)
    side = per.get("fri::k_coef", 0.0)       # on its own stream, beside the block trees
    main = sum(v for k, v in per.items() if k != "fri::k_coef")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {k[:64]:64s} {v:9.1f} us per commit")
    print(f"{len(segs)} commits; kernel time per commit on the rank's main stream: {main / 1e3:.3f} ms "
          f"(+ {side / 1e3:.3f} ms of coefficient folds on the side stream)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=28)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--summarise", default=None)
    ap.add_argument("--serial-coef", action="store_true",
                    help="coefficient folds on the main stream (profiling mode) instead of beside the block trees")
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.log_n, a.world, a.rank, a.steps, a.serial_coef)
