import faulthandler, sys, os
faulthandler.enable()
sys.path.insert(0, "stark-prover_amd/python"); sys.path.insert(0, "oracle")
import numpy as np, fri_amd, fri_oracle as fo
print("load", flush=True)
ctx = fri_amd.Context(0, 20)
print("ctx ok", flush=True)
for log_n in (10, 12, 16, 20):
    c = fo.splitmix64_field(3, (1 << log_n) // 8)
    r = ctx.commit(c, log_n, graph=False)
    print("commit", log_n, bytes(r.roots[0]).hex()[:16], flush=True)
    ch = fo.Channel(); o = fo.fri_commit(c, log_n, ch, keep=False) if log_n <= 16 else None
    if o is not None: print("  match", [x.hex() for x in o.roots] == [bytes(r.roots[k]).hex() for k in range(r.n_layers)], flush=True)
ctx.close()
print("done", flush=True)
