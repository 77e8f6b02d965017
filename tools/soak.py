"""Soak test of commit contexts under a random mix of entry points (GPU).

Thousands of commits on one or more fri_ctx driven from ONE host thread,
each drawn at random from: synchronous commits from host coefficients or from
a device buffer, pipelined commits of device buffers, of host coefficients
(fri_commit_async; every context's uploads share the device's upload stream)
and of the context's own input buffer (fri_ctx_input_buffer, refilled now and
then with fri_ctx_input_upload), with the number of commit lanes and the
codeword shape of a context changing now and then.  Every result is compared
with the C oracle's transcript of the same polynomial (oracle/fri_oracle.c,
the restatement of src/fri/fri_commit.rs:72-122), so an ordering race between
lanes, stagings, result slots or contexts shows up as a wrong transcript.  The
model of a context's input buffer needs nothing from the library: the buffer
is the caller's, so it holds what the last upload put there, whatever the
commits in between and however they were dealt to lanes.

    python3 tools/soak.py [--commits N] [--seed S] [--contexts K]
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

SHAPES = [16, 18, 20]                              # log_n; d = n / 8


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


class Driven:
    """One context and the model of its state: the result slot of every
    pending ticket (lowest free slot, fri_lanes.hip async_enqueue), its lanes,
    its shape and what its input buffer holds (the last upload's
    polynomial)."""

    def __init__(self, fri_amd, polys, rng):
        self.fa, self.polys, self.rng = fri_amd, polys, rng
        self.ctx = fri_amd.Context(0, max(SHAPES))
        self.lanes = 3
        self.ctx.set_lanes(self.lanes)
        self.slots, self.pend = {}, []
        self.L = SHAPES[0]
        self.in_buf = None
        self.n_ok = 0

    def enqueue(self, t, key):
        self.slots[t] = min(set(range(self.fa.MAX_INFLIGHT)) - set(self.slots.values()))
        self.pend.append((t, key))

    def expect_oldest(self):
        t, key = self.pend.pop(0)
        self.slots.pop(t)
        r = self.ctx.commit_wait(t)
        assert transcript(r) == self.polys[key][2], f"pipelined commit of {key} gave a wrong transcript"
        self.n_ok += 1

    def drain(self):
        while self.pend:
            self.expect_oldest()

    def step(self, kinds):
        fa, rng, ctx = self.fa, self.rng, self.ctx
        u = rng.random()
        if u < 0.02:                               # another shape: every lane's plan is rebuilt
            self.drain()
            self.L = int(rng.choice(SHAPES))
        elif u < 0.04:                             # another number of lanes (no commit may be pending)
            self.drain()
            self.lanes = int(rng.integers(1, fa.MAX_INFLIGHT + 1))
            ctx.set_lanes(self.lanes)
        L = self.L
        d = (1 << L) >> 3
        j = int(rng.integers(0, 4))
        kind = int(rng.integers(0, 6))
        if kind == 4 and (self.in_buf is None or self.in_buf[0] != L):
            kind = 5                               # the buffer holds no polynomial of this shape yet
        if len(self.pend) == fa.MAX_INFLIGHT:
            self.expect_oldest()
        c, dev, want = self.polys[(L, j)]
        if kind == 0:                              # synchronous, host coefficients (staged privately)
            assert transcript(ctx.commit(c, L)) == want
            self.n_ok += 1
        elif kind == 1:                            # synchronous, another device buffer (staged privately)
            r = fa.CommitResult()
            ctx._check(ctx.lib.fri_commit_device(ctx.h, ctypes.c_void_p(dev.data_ptr()), d, L, fa.GENERATOR,
                                                 None, 0, None, ctypes.byref(r)))
            assert transcript(r) == want
            self.n_ok += 1
        elif kind in (2, 3):                       # pipelined, device buffer / host coefficients
            t = ctx.commit_device_async(dev.data_ptr(), d, L) if kind == 2 else ctx.commit_async(c, L)
            self.enqueue(t, (L, j))
        elif kind == 4:                            # pipelined, the context's own input buffer, read in place
            self.enqueue(ctx.commit_device_async(ctx.input_buffer(d), d, L), self.in_buf)
        else:                                      # refill the input buffer (waits for its pending readers)
            ctx.input_upload(c)
            self.in_buf = (L, j)
            # ... and, half the time, commit it at once (synchronously)
            if rng.random() < 0.5:
                r = fa.CommitResult()
                ctx._check(ctx.lib.fri_commit_device(ctx.h, ctypes.c_void_p(ctx.input_buffer(d)), d, L,
                                                     fa.GENERATOR, None, 0, None, ctypes.byref(r)))
                assert transcript(r) == want
                self.n_ok += 1
        kinds[kind] = kinds.get(kind, 0) + 1


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--commits", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--contexts", type=int, default=1)
    a = ap.parse_args(argv)
    import fri_amd
    import fri_oracle as fo
    corc = fo.load_c_oracle()
    rng = np.random.default_rng(a.seed)
    polys = {}                                     # (log_n, j) -> (host u32, device tensor, transcript)
    for L in SHAPES:
        d = (1 << L) >> 3
        for j in range(4):
            c = fo.splitmix64_np(7000 + 10 * L + j, d).astype(np.uint32)
            dev = fri_amd.DeviceBuffer(c)        # the library's own HIP runtime (no torch)
            polys[(L, j)] = (c, dev, oracle_transcript(corc, fo, c, L))
    cx = [Driven(fri_amd, polys, rng) for _ in range(a.contexts)]
    kinds = {}
    t0 = time.time()
    for i in range(a.commits):
        cx[int(rng.integers(0, len(cx)))].step(kinds)
        if i % 500 == 0:
            print(f"[soak] {i} commits, {sum(c.n_ok for c in cx)} checked, {time.time() - t0:.1f} s", flush=True)
    for c in cx:
        c.drain()
        c.ctx.close()
    n_ok = sum(c.n_ok for c in cx)
    print(f"soak ok: {n_ok} commits on {len(cx)} context(s) checked against the C oracle in {time.time() - t0:.1f} s "
          f"(kinds: sync-host {kinds.get(0, 0)}, sync-device {kinds.get(1, 0)}, async-device {kinds.get(2, 0)}, "
          f"async-host {kinds.get(3, 0)}, async-input-buffer {kinds.get(4, 0)}, upload {kinds.get(5, 0)})", flush=True)
    return n_ok, kinds


if __name__ == "__main__":
    main()
