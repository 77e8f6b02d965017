"""Randomised commit parity: many small commits with random shapes against the
OpenMP C oracle (oracle/fri_oracle.c orc_fri_commit_fast, which follows
src/fri/fri_commit.rs:72-122 with the SURVEY.md §8 frozen spec).

Each case draws a codeword size 2^1..2^17, a coefficient count anywhere in
[0, n] (blowups 1..2^log_n, non-powers of two, trailing zeros, all-zero and
constant polynomials), a random nonzero coset offset and, half of the time, a
pre-filled channel state.  Every root, beta, the final value and degree and
the channel state after the commit must match bit for bit.  FRI_FUZZ_N sets
the number of small cases (default 200; 400 ran green on an MI355X), plus a
few cases at 2^18..2^22.  The seed sequence is fixed, so a failure names a
reproducible case."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 3221225473


def _case(i, lo=1, hi=18):
    r = np.random.default_rng(1000 + i)
    log_n = int(r.integers(lo, hi))
    n = 1 << log_n
    kind = int(r.integers(0, 6))
    if kind == 0:
        d = n >> int(r.integers(0, min(log_n, 4) + 1))          # blowup 2^0..2^4
    elif kind == 1:
        d = int(r.integers(0, n + 1))                             # any count, 0 included
    elif kind == 2:
        d = int(r.integers(1, max(2, n // 8) + 1))                # small polynomial
    else:
        d = n >> 3 if log_n >= 3 else n                           # the bench shape
    c = r.integers(0, P, size=d, dtype=np.uint64)
    if d and kind == 3:
        c[int(r.integers(0, d)):] = 0                             # trailing zeros
    if d and kind == 4:
        c[:] = 0                                                  # zero polynomial
    if d and kind == 5:
        c[1:] = 0                                                 # constant
    offset = int(r.integers(1, P))
    state = r.bytes(32) if r.integers(0, 2) else None
    return log_n, c, offset, state


CASES = [(i, 1, 18) for i in range(int(os.environ.get("FRI_FUZZ_N", "200")))] + \
        [(100000 + i, 18, 23) for i in range(6)]


@pytest.mark.parametrize("i,lo,hi", CASES)
def test_commit_fuzz_vs_c_oracle(ctx, corc, oracle, i, lo, hi):
    log_n, c, offset, state = _case(i, lo, hi)
    d = c.size
    res = ctx.commit(c, log_n, offset=offset, channel_state=state)
    cs = np.ascontiguousarray(c, dtype=np.uint64)
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    if state is not None:
        och.state = state.hex().encode()
        och.state_len = 64
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, log_n, offset, 5, P,
                                    ctypes.byref(och), None, ctypes.byref(ores), None, None) == 0
    what = f"case {i}: log_n={log_n} d={d} offset={offset} prefilled={state is not None}"
    assert res.n_layers == ores.n_layers, what
    assert res.n_rounds == ores.n_rounds, what
    assert [bytes(res.roots[k]) for k in range(res.n_layers)] == [bytes(ores.roots[k]) for k in range(ores.n_layers)], what
    assert [res.betas[r] for r in range(res.n_rounds)] == [ores.betas[r] for r in range(ores.n_rounds)], what
    assert res.final_value == ores.final_value, what
    assert res.final_degree == ores.final_degree, what
    assert bytes(res.channel_out.digest).hex() == och.state.decode(), what


def _lane_cases(n_groups=8, per_group=4):
    """Groups of commits that share a plan (log_n, d, offset) but not their
    coefficients or channel state, each group a new shape."""
    out = []
    for g in range(n_groups):
        r = np.random.default_rng(70000 + g)
        log_n = int(r.integers(10, 19))
        n = 1 << log_n
        d = int(r.integers(0, n + 1)) if g % 2 else n >> int(r.integers(0, 5))
        offset = int(r.integers(1, P))
        for j in range(per_group):
            c = r.integers(0, P, size=d, dtype=np.uint64)
            if d and j == 1:
                c[int(r.integers(0, d)):] = 0
            out.append((log_n, c, offset, r.bytes(32) if j % 2 else None))
    return out


def test_lanes_fuzz_vs_c_oracle(corc, oracle):
    """Pipelined commits on ONE context over three commit lanes, three pending
    at a time, through plan changes (every fourth commit a new shape, which
    frees every lane's plan behind the commits still pending): each result
    equals the OpenMP C oracle's commit of the same input."""
    import fri_amd
    cases = _lane_cases()
    cx = fri_amd.Context(0, 18)
    try:
        cx.set_lanes(3)
        pend, results = [], {}
        for i, (log_n, c, offset, state) in enumerate(cases):
            pend.append((i, cx.commit_async(c.astype(np.uint32), log_n, offset, channel_state=state)))
            if len(pend) == 3:
                j, t = pend.pop(0)
                results[j] = cx.commit_wait(t)
        for j, t in pend:
            results[j] = cx.commit_wait(t)
    finally:
        cx.close()
    for i, (log_n, c, offset, state) in enumerate(cases):
        res = results[i]
        cs = np.ascontiguousarray(c, dtype=np.uint64)
        och = oracle.OrcChannel()
        corc.orc_channel_init(ctypes.byref(och))
        if state is not None:
            och.state = state.hex().encode()
            och.state_len = 64
        ores = oracle.OrcFriResult()
        assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, log_n, offset, 5,
                                        P, ctypes.byref(och), None, ctypes.byref(ores), None, None) == 0
        what = f"commit {i}: log_n={log_n} d={c.size} offset={offset} prefilled={state is not None}"
        assert [bytes(res.roots[k]) for k in range(res.n_layers)] == \
               [bytes(ores.roots[k]) for k in range(ores.n_layers)], what
        assert [res.betas[r] for r in range(res.n_rounds)] == [ores.betas[r] for r in range(ores.n_rounds)], what
        assert res.final_value == ores.final_value and res.final_degree == ores.final_degree, what
        assert bytes(res.channel_out.digest).hex() == och.state.decode(), what
