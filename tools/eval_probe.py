"""fri_evaluate timing (Polynomial::evaluate, Horner semantics) for few points
and many coefficients, against Horner in the C oracle (one thread).  Run
through gpurun."""
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
ctx = fri_amd.Context(0, 22)
corc = fo.load_c_oracle()
for log_d, count in ((10, 1), (13, 1), (16, 1), (21, 1), (21, 16), (21, 1024)):
    d = 1 << log_d
    r = np.random.default_rng(log_d)
    c = r.integers(0, P, d, dtype=np.uint64).astype(np.uint32)
    xs = r.integers(0, P, count, dtype=np.uint64).astype(np.uint32)
    ctx.evaluate(c, xs)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        got = ctx.evaluate(c, xs)
    t = (time.perf_counter() - t0) / reps
    c64 = c.astype(np.uint64)
    pc = c64.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    t0 = time.perf_counter()
    want = corc.orc_poly_evaluate(pc, d, int(xs[0]), P)
    tc = time.perf_counter() - t0
    print(f"d=2^{log_d} points={count:5d}: GPU {1e3 * t:8.3f} ms per call (host copies included); "
          f"C Horner one point {1e3 * tc:8.3f} ms; equal {int(got[0]) == want}", flush=True)
ctx.close()
