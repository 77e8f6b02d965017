"""Soak test of one context under a random mix of commit entry points (GPU).

Thousands of commits on ONE fri_ctx, drawn at random from: synchronous
commits from host coefficients or from a device buffer, pipelined commits of
device buffers, of host coefficients (fri_commit_async) and of the context's
own input buffer (fri_ctx_input_buffer), with the number of commit lanes and
the codeword shape changing now and then.  Every result is compared with the
C oracle's transcript of the same polynomial (oracle/fri_oracle.c, the
restatement of src/fri/fri_commit.rs:72-122), so an ordering race between
lanes, stagings or slots shows up as a wrong transcript.  The input buffer's
expected contents follow call order: a commit handed that buffer commits what
the last synchronous commit or lane-0 staging put there.

    python3 tools/soak.py [--commits N] [--seed S]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def oracle_transcript(corc, fo, c, log_n):
    cs = np.ascontiguousarray(c, dtype=np.uint64)
    och = fo.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    res = fo.OrcFriResult()
    assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, log_n, 5, 5, fo.P,
                                    ctypes.byref(och), None, ctypes.byref(res), None, None) == 0
    return ([bytes(res.roots[k]) for k in range(res.n_layers)], [res.betas[r] for r in range(res.n_rounds)],
            res.final_value, och.state.decode())


def transcript(r):
    return ([bytes(r.roots[k]) for k in range(r.n_layers)], [r.betas[i] for i in range(r.n_rounds)], r.final_value,
            bytes(r.channel_out.digest).hex())


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--commits", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args(argv)
    import torch
    import fri_amd
    import fri_oracle as fo
    corc = fo.load_c_oracle()
    rng = np.random.default_rng(a.seed)
    shapes = [16, 18, 20]                          # log_n; d = n / 8
    polys = {}                                     # (log_n, j) -> (host u32, device tensor, transcript)
    for L in shapes:
        d = (1 << L) >> 3
        for j in range(4):
            c = fo.splitmix64_np(7000 + 10 * L + j, d).astype(np.uint32)
            dev = torch.from_numpy(c.view(np.int32).copy()).cuda()
            polys[(L, j)] = (c, dev, oracle_transcript(corc, fo, c, L))
    ctx = fri_amd.Context(0, max(shapes))
    lanes = 3
    ctx.set_lanes(lanes)
    slots = {}                                     # ticket -> result slot (lowest free slot, fri_api.hip async_enqueue)
    L = shapes[0]
    in_buf = None                                  # (log_n, poly index) the input buffer holds, in call order
    pend = []                                      # (ticket, expected transcript key)
    n_ok = 0
    kinds = {}
    t0 = time.time()

    def next_lane():
        return min(set(range(fri_amd.MAX_INFLIGHT)) - set(slots.values())) % lanes

    def enqueue(t, key):
        slots[t] = min(set(range(fri_amd.MAX_INFLIGHT)) - set(slots.values()))
        pend.append((t, key))

    def expect(t, key):
        nonlocal n_ok
        slots.pop(t)
        r = ctx.commit_wait(t)
        assert transcript(r) == polys[key][2], f"pipelined commit of {key} gave a wrong transcript"
        n_ok += 1

    def drain():
        while pend:
            expect(*pend.pop(0))

    for i in range(a.commits):
        u = rng.random()
        if u < 0.02:                               # another shape: the plans of every lane are rebuilt
            drain()
            L = int(rng.choice(shapes))
            in_buf = None
        elif u < 0.04:                             # another number of lanes (no commit may be pending)
            drain()
            lanes = int(rng.integers(1, fri_amd.MAX_INFLIGHT + 1))
            ctx.set_lanes(lanes)
        d = (1 << L) >> 3
        j = int(rng.integers(0, 4))
        kind = int(rng.integers(0, 5))
        if kind == 4 and in_buf is None:
            kind = 0
        if len(pend) == fri_amd.MAX_INFLIGHT:
            expect(*pend.pop(0))
        c, dev, want = polys[(L, j)]
        if kind == 0:                              # synchronous, host coefficients: stages them (lane 0)
            assert transcript(ctx.commit(c, L)) == want
            n_ok += 1
            in_buf = (L, j)
        elif kind == 1:                            # synchronous, device buffer: staged into the input buffer
            r = fri_amd.CommitResult()
            ctx._check(ctx.lib.fri_commit_device(ctx.h, ctypes.c_void_p(dev.data_ptr()), d, L, fri_amd.GENERATOR,
                                                 None, 0, None, ctypes.byref(r)))
            assert transcript(r) == want
            n_ok += 1
            in_buf = (L, j)
        elif kind == 2:                            # pipelined, device buffer
            slot_lane0 = next_lane() == 0
            enqueue(ctx.commit_device_async(dev.data_ptr(), d, L), (L, j))
            if slot_lane0:
                in_buf = (L, j)                    # a lane-0 commit stages it into the input buffer
        elif kind == 3:                            # pipelined, host coefficients (per-slot pinned copy)
            slot_lane0 = next_lane() == 0
            enqueue(ctx.commit_async(c, L), (L, j))
            if slot_lane0:
                in_buf = (L, j)
        else:                                      # pipelined, the context's own input buffer
            p0 = ctypes.c_void_p()
            ctx._check(ctx.lib.fri_ctx_input_buffer(ctx.h, d, ctypes.byref(p0)))
            enqueue(ctx.commit_device_async(p0.value, d, L), in_buf)
        kinds[kind] = kinds.get(kind, 0) + 1
        if i % 500 == 0:
            print(f"[soak] {i} commits, {n_ok} checked, {time.time() - t0:.1f} s", flush=True)
    drain()
    ctx.close()
    print(f"soak ok: {n_ok} commits checked against the C oracle in {time.time() - t0:.1f} s "
          f"(kinds: sync-host {kinds.get(0, 0)}, sync-device {kinds.get(1, 0)}, async-device {kinds.get(2, 0)}, "
          f"async-host {kinds.get(3, 0)}, async-input-buffer {kinds.get(4, 0)})", flush=True)
    return n_ok, kinds


if __name__ == "__main__":
    main()
