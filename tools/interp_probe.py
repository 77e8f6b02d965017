"""fri_interpolate_points timing (Polynomial::interpolate on arbitrary
points, O(n^2)) at n = 2^12..2^17, and the C oracle's Lagrange sum (the
reference algorithm, one thread) at 2^12 for scale.  Run through gpurun."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fri_amd  # noqa: E402
import fri_oracle as fo  # noqa: E402

P = fri_amd.P
ctx = fri_amd.Context(0, 17)
for log_n in range(12, 18):
    n = 1 << log_n
    r = np.random.default_rng(log_n)
    xs = np.unique(r.integers(0, P, n + 1024, dtype=np.uint64))[:n].astype(np.uint32)
    ys = r.integers(0, P, n, dtype=np.uint64).astype(np.uint32)
    ctx.interpolate_points(xs, ys)
    t0 = time.perf_counter()
    c = ctx.interpolate_points(xs, ys)
    t = time.perf_counter() - t0
    ok = np.array_equal(ctx.evaluate(c, xs), ys)
    print(f"n=2^{log_n}: {1e3 * t:9.2f} ms  (evaluates back: {ok})", flush=True)
    if log_n == 12:
        corc = fo.load_c_oracle()
        corc.orc_set_num_threads(1)
        x64, y64 = xs.astype(np.uint64), ys.astype(np.uint64)
        out = np.empty(n, dtype=np.uint64)
        t0 = time.perf_counter()
        corc.orc_interpolate_lagrange(x64.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                      y64.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), P)
        print(f"   C oracle Lagrange (reference algorithm, 1 thread) at 2^12: {time.perf_counter() - t0:.2f} s, "
              f"equal: {np.array_equal(out[:c.size], c.astype(np.uint64))}", flush=True)
ctx.close()
