"""Per-stage wall time of fri_amd.prove_fibsq (BASELINE configs[3]) on GPU 0."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stark-prover_amd", "python"))
import fri_amd  # noqa: E402

log_t, lb, q = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (16, 3, 3)))
L = log_t + lb
ctx = fri_amd.Context(0, L)
fri_amd.prove_fibsq(3141592, log_t, lb, q, fri_amd.Channel(), ctx=ctx)
for rep in range(3):
    T = {}
    t = time.perf_counter()
    trace = fri_amd.fibsq_trace(3141592, 1 << log_t)
    T["trace_gen"] = time.perf_counter() - t; t = time.perf_counter()
    root, _, _ = ctx.trace_commit(trace, lb, readback=False)
    T["trace_commit"] = time.perf_counter() - t; t = time.perf_counter()
    ch = fri_amd.Channel()
    ch.send(root.hex().encode())
    al = [ch.receive_random_field_element() for _ in range(3)]
    T["channel"] = time.perf_counter() - t; t = time.perf_counter()
    res = ctx.fibsq_composition_commit(log_t, lb, int(trace[-1]), al, channel_state=bytes.fromhex(ch.state))
    T["composition+fri"] = time.perf_counter() - t; t = time.perf_counter()
    fri = fri_amd._mirror_commit(res, ctx, L, ch)
    for _ in range(q):
        idx = ch.receive_random_int(0, (1 << L) - 2 * (1 << lb) - 1, True)
        for v, path in ctx.trace_decommit(idx, 1 << lb, 3, L):
            ch.send(v.to_bytes(8, "big")); ch.send(path)
        fri_amd.decommit_fri_layers(idx, fri, ch)
    T["queries"] = time.perf_counter() - t
    print(" ".join(f"{k}={1000 * v:.3f}ms" for k, v in T.items()), f"total={1000 * sum(T.values()):.3f}ms", flush=True)
ctx.set_profiling(True)
fri_amd.prove_fibsq(3141592, log_t, lb, q, fri_amd.Channel(), ctx=ctx)
ctx.set_profiling(False)
for cls in ("composition", "lde", "layer0", "layers"):
    print(cls, ctx.profile(cls))
