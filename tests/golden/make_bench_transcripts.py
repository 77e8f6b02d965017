"""Expected FRI transcripts of bench.py's synthetic workloads, from the OpenMP
C oracle (oracle/fri_oracle.c, orc_fri_commit_fast; test infrastructure).

bench.py commits splitmix64(42) % p coefficients (d = 2^log_n / 8) and, on
N > 1 GPUs, checks the sharded transcript against these before it times
anything, so the multi-GPU line is bit-exact against the CPU restatement
without a 1-GPU re-commit of 2^28 on every rank.  The oracle's commit itself
is checked against the reference's KATs and the golden vectors
(tests/test_oracle_*.py).

    python tests/golden/make_bench_transcripts.py [min_log max_log]
"""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import fri_oracle as fo  # noqa: E402

OUT = os.path.join(HERE, "bench_transcripts.json")


def transcript(lib, log_n, seed=42, blowup_log=3):
    d = (1 << log_n) >> blowup_log
    c = np.ascontiguousarray(fo.splitmix64_np(seed, d))
    och = fo.OrcChannel()
    lib.orc_channel_init(ctypes.byref(och))
    r = fo.OrcFriResult()
    assert lib.orc_fri_commit_fast(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, log_n, 5, 5, fo.P,
                                   ctypes.byref(och), None, ctypes.byref(r), None, None) == 0
    return {"log_n": log_n, "seed": seed, "blowup_log": blowup_log,
            "roots": [bytes(r.roots[k]).hex() for k in range(r.n_layers)],
            "betas": [int(r.betas[i]) for i in range(r.n_rounds)],
            "final_value": int(r.final_value), "final_degree": int(r.final_degree),
            "state": och.state.decode()}


def main():
    lo, hi = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (20, 28)
    lib = fo.load_c_oracle()
    data = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            data = json.load(f)
    for log_n in range(lo, hi + 1):
        t0 = time.time()
        data[f"{log_n}/42/3"] = transcript(lib, log_n)
        print(f"2^{log_n}: {time.time() - t0:.1f} s", flush=True)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
    # the distinct inputs of bench.py's pipelined stage (seeds 43, 44 at 2^20 and 2^24)
    for log_n in (20, 24):
        for seed in (43, 44):
            if lo <= log_n <= hi:
                data[f"{log_n}/{seed}/3"] = transcript(lib, log_n, seed)
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
