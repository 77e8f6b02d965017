"""One host thread, K contexts (one stream each), commits enqueued round-robin
with fri_commit_async (host coefficients) or fri_commit_device_async (each
context's resident input buffer) and collected with fri_commit_wait:
concurrent commits without host threads.  2^24; transcripts checked."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import fri_amd
from bench import _coeffs, _same

log_n = 24; d = 1 << 21
c = _coeffs(42, d, fri_amd.P)
ctxs = [fri_amd.Context(0, log_n) for _ in range(4)]
ref = ctxs[0].commit(c, log_n)
dptr = {}
for x in ctxs:
    x.commit(c, log_n)
    p = ctypes.c_void_p(x.input_upload(c))
    dptr[id(x)] = p
for K, dev in ((1, False), (2, False), (3, False), (4, False), (1, True), (2, True), (3, True), (4, True)):
    cx = ctxs[:K]
    enq = (lambda x: x.commit_device_async(dptr[id(x)], d, log_n)) if dev else (lambda x: x.commit_async(c, log_n))
    for x in cx:                                   # warm-up: plans, slot graphs, buffers
        for t in [enq(x) for _ in range(2)]:
            x.commit_wait(t)
    n = 24
    pend = []
    ok = True
    t0 = time.perf_counter()
    for i in range(n):
        x = cx[i % K]
        if len(pend) == 2 * K:
            xi, ti = pend.pop(0)
            ok &= _same(xi.commit_wait(ti), ref)
        pend.append((x, enq(x)))
    for xi, ti in pend:
        ok &= _same(xi.commit_wait(ti), ref)
    dt = time.perf_counter() - t0
    print(f"K={K} contexts, {'device-resident' if dev else 'host'} input, one host thread: "
          f"{1000 * dt / n:.3f} ms per 2^24 commit, transcripts ok: {ok}")
