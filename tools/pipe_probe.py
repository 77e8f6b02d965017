"""Host-side timing of pipelined commits (fri_commit_async / fri_commit_device_async):
per-call durations of the enqueue and the wait, 2 in flight, 2^24."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import fri_amd
from bench import _coeffs

log_n = 24; d = 1 << 21
ctx = fri_amd.Context(0, log_n)
c = _coeffs(42, d, fri_amd.P)
ctx.commit(c, log_n)
dptr = ctypes.c_void_p(ctx.input_upload(c))
for kind in ("device", "host", "host", "device"):
    enq, wt = [], []
    pend = []
    t0 = time.perf_counter()
    for i in range(20):
        a = time.perf_counter()
        pend.append(ctx.commit_device_async(dptr, d, log_n) if kind == "device" else ctx.commit_async(c, log_n))
        enq.append(time.perf_counter() - a)
        if len(pend) == 2:
            a = time.perf_counter(); ctx.commit_wait(pend.pop(0)); wt.append(time.perf_counter() - a)
    ctx.commit_wait(pend.pop(0))
    tot = time.perf_counter() - t0
    print(f"{kind:6s} {1000*tot/20:.3f} ms/commit  enqueue median {1000*np.median(enq):.3f} ms  wait median {1000*np.median(wt):.3f} ms")
t0 = time.perf_counter()
for i in range(20):
    ctx.commit(c, log_n)
print(f"sync host {1000*(time.perf_counter()-t0)/20:.3f} ms/commit")
