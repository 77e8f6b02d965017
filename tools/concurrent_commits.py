"""Aggregate throughput of C concurrent FRI commits on one GPU (one context
and stream per commit, host threads; ctypes releases the GIL).  The tree
tops of one commit (a single workgroup on the serial Fiat-Shamir chain)
overlap the leaf hashing of the others.

    python tools/concurrent_commits.py [log_n=24] [C=2] [steps=10]
"""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stark-prover_amd", "python"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fri_amd  # noqa: E402
from bench import _coeffs  # noqa: E402

log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
C = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
d = 1 << (log_n - 3)
ctxs, ptrs, res, want = [], [], [], []
for c in range(C):
    ctx = fri_amd.Context(0, log_n)
    co = _coeffs(42 + c, d, fri_amd.P)
    want.append(ctx.commit(co, log_n))
    p = ctypes.c_void_p(ctx.input_upload(co))
    ctxs.append(ctx); ptrs.append(p); res.append(fri_amd.CommitResult())


def run(c, k):
    for _ in range(k):
        ctxs[c]._check(ctxs[c].lib.fri_commit_device(ctxs[c].h, ptrs[c], d, log_n, 5, None, 0, None,
                                                     ctypes.byref(res[c])))


for c in range(C):
    run(c, 2)
t0 = time.perf_counter()
run(0, steps)
single = (time.perf_counter() - t0) / steps
th = [threading.Thread(target=run, args=(c, steps)) for c in range(C)]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
wall = time.perf_counter() - t0
ok = all(bytes(res[c].roots[0]) == bytes(want[c].roots[0]) and res[c].final_value == want[c].final_value
         for c in range(C))
print(f"log_n={log_n} C={C}: single {1000 * single:.3f} ms/commit; concurrent {1000 * wall / (C * steps):.3f} "
      f"ms/commit ({C * steps} commits in {wall:.3f} s) = {C * steps * (1 << log_n) / wall / 1e9:.3f} G elems/s; "
      f"transcripts ok={ok}")
