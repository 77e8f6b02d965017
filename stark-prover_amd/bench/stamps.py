"""Diagnostic: per-layer top-kernel phase durations (us) from the FRI_STAMPS
build.  Usage: FRI_AMD_LIB=libfri_amd_stamps.so python stark-prover_amd/bench/stamps.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "python"))
import fri_amd  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
d = 1 << (log_n - 3)
ctx = fri_amd.Context(0, log_n)
c = (np.arange(d, dtype=np.uint64) * 2654435761 % fri_amd.P).astype(np.uint32)
for _ in range(3):
    res = ctx.commit(c, log_n)
buf = (ctypes.c_uint64 * (33 * 64))()
ctx._check(ctx.lib.fri_debug_stamps(ctx.h, buf, 33 * 64))
a = np.frombuffer(buf, dtype=np.uint64).reshape(33, 64).astype(np.int64)
prev_end = 0
for k in range(res.n_layers):
    row = a[k]
    t0 = row[0]
    marks = [(i, (row[i] - t0) / 100.0) for i in list(range(1, 17)) + [20, 21, 22] if row[i] > 0 and not (i in (13, 14) and row[i] < t0)]
    if row[17] and row[18] and row[19] > row[1]:
        marks.append(("MHz", (row[18] - row[17]) / ((row[19] - row[1]) / 100.0)))
    last = max(row[i] for i in list(range(17)) + [19])
    gap = (t0 - prev_end) / 100.0 if k else 0.0
    prev_end = last
    wide = ""
    if row[60] and row[62]:                        # wide leaf kernel (workgroup 0), relative to the top's start
        wide = f" wide[start {(row[60] - t0) / 100.0:.1f} leaves {(row[61] - t0) / 100.0:.1f} end {(row[62] - t0) / 100.0:.1f}]"
    print(f"layer {k:2d} L={log_n - k:2d} since-prev-top={gap:6.1f}: " + " ".join(f"{i}:{us:.1f}" for i, us in marks) + wide)
    nodes = [(row[25 + 2 * j] - row[24 + 2 * j]) / 1000.0 for j in range(18) if row[25 + 2 * j] > row[24 + 2 * j] > 0]
    print("      node kcycles per level: " + " ".join(f"{c:.1f}" for c in nodes))
