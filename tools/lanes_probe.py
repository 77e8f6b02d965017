"""Commit lanes on one context: wall time per 2^24 commit for (lanes, depth)
pairs, and (with --summarise DIR, on a rocprofv3 --kernel-trace of this
script) which hardware queue each lane's kernels ran on and how long the
lanes overlapped.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- \
        python3 tools/lanes_probe.py --pairs 3:3,4:4 --commits 12
    python3 tools/lanes_probe.py --summarise DIR
"""
import argparse
import csv
import ctypes
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, ROOT)


def run(pairs, commits, log_n=24):
    import fri_amd
    import bench
    d = (1 << log_n) >> 3
    ctx = fri_amd.Context(0, log_n)
    ctx.commit(bench._coeffs(42, d, fri_amd.P), log_n)
    hip = bench._hip_runtime()
    st = ctypes.c_void_p()
    hip.hipStreamCreate(ctypes.byref(st))
    ptrs = []
    for sd in (42, 43, 44):
        host = bench._coeffs(sd, d, fri_amd.P)
        p = ctypes.c_void_p()
        hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(4 * d))
        hip.hipMemcpyAsync(p, host.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(4 * d), 1, st)
        hip.hipStreamSynchronize(st)
        ptrs.append(p)
    hip.hipStreamDestroy(st)
    for lanes, depth in pairs:
        ctx.set_lanes(lanes)

        def go(k):
            pend = []
            for i in range(k):
                pend.append(ctx.commit_device_async(ptrs[i % 3], d, log_n))
                if len(pend) == depth:
                    ctx.commit_wait(pend.pop(0))
            for t in pend:
                ctx.commit_wait(t)

        go(2 * depth)
        t0 = time.perf_counter()
        go(commits)
        print(f"lanes {lanes} depth {depth}: {1000 * (time.perf_counter() - t0) / commits:.3f} ms per commit",
              flush=True)
        time.sleep(0.05)             # a gap in the trace between the configurations
    ctx.close()


def summarise(dr):
    f = glob.glob(os.path.join(dr, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # configurations are separated by the 50 ms sleeps
    groups, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 20_000_000:
            groups.append(cur)
            cur = []
        cur.append(b)
    groups.append(cur)
    for g in groups:
        qs = {}
        for r in g:
            qs.setdefault((r["Queue_Id"], r.get("Stream_Id", "?")), []).append(r)
        t0 = int(g[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in g)
        # time with >= 2 kernels running at once
        ev = sorted([(int(r["Start_Timestamp"]), 1) for r in g] + [(int(r["End_Timestamp"]), -1) for r in g])
        live, last, multi = 0, t0, 0
        for t, dl in ev:
            if live >= 2:
                multi += t - last
            live += dl
            last = t
        print(f"{len(g)} kernels over {(t1 - t0) / 1e6:.2f} ms; overlapped {multi / 1e6:.2f} ms; "
              f"(queue, stream) -> kernels: " + ", ".join(f"{k}: {len(v)}" for k, v in sorted(qs.items())))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="1:2,2:2,3:3,3:4,4:4")
    ap.add_argument("--commits", type=int, default=24)
    ap.add_argument("--summarise", default=None)
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run([tuple(int(x) for x in p.split(":")) for p in a.pairs.split(",")], a.commits)
