"""CPU: the prover slice's oracle (STARK-101 FibonacciSq, BASELINE configs[3])
and the host-side verifier.

The reference's src/prover, src/trace and src/composition are empty files, so
the composition polynomial is PARITY UNPINNED against the reference; what is
pinned here is internal consistency between independent restatements:
  * fibsq_cp_faithful — the reference's own polynomial arithmetic
    (ops.rs div_rem / mul / compose, interpolation.rs Lagrange), every
    division exact;
  * fibsq_cp_evals_np — evaluation form with numpy;
  * orc_fibsq_cp_evals / orc_fibsq_prove_commit — the C oracle (batch
    inverse, NTT interpolation, fast FRI);
  * the committed golden transcripts (tests/golden, make_golden.py).
"""
import ctypes
import hashlib

import numpy as np
import pytest

P = 3221225473


def _proof_sha(msgs):
    return hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m for m in msgs)).hexdigest()


def test_fibsq_trace_recurrence(oracle, corc):
    t = oracle.fibsq_trace(3141592, 64)
    assert t[0] == 1 and t[1] == 3141592
    assert all(t[i + 2] == (t[i + 1] ** 2 + t[i] ** 2) % P for i in range(62))
    out = (ctypes.c_uint64 * 64)()
    corc.orc_fibsq_trace(3141592, 64, P, out)
    assert list(out) == t


def test_library_trace_generator_matches_oracle(oracle):
    """fri_fibsq_trace is host code in libfri_amd.so (no device needed)."""
    import fri_amd
    for a1, log_t in ((3141592, 10), (P - 1, 4), (0, 3), (7, 1)):
        assert fri_amd.fibsq_trace(a1, 1 << log_t).tolist() == oracle.fibsq_trace(a1, 1 << log_t)


def test_python_twin_reproduces_golden_prover_transcripts(oracle, golden):
    for c in golden["fibsq"]:
        ch = oracle.Channel(state=c["channel_in"])
        pr = oracle.fibsq_prove(c["a1"], c["log_t"], c["log_blowup"], c["queries"], ch)
        assert pr.trace_root.hex() == c["trace_root"], c["name"]
        assert pr.alphas == c["alphas"] and pr.fri.betas == c["betas"], c["name"]
        assert [r.hex() for r in pr.fri.roots] == c["roots"], c["name"]
        assert pr.queries == c["query_indices"], c["name"]
        assert ch.state == c["channel_out"] and _proof_sha(ch.proof) == c["proof_sha256"], c["name"]


@pytest.mark.parametrize("log_t,lb", [(3, 1), (4, 2), (5, 3), (6, 3), (5, 4)])
def test_composition_three_ways(oracle, corc, log_t, lb):
    """Coefficient form (reference polynomial ops) == numpy evaluation form
    == C evaluation form, on the whole LDE coset; deg CP == T exactly."""
    T, L = 1 << log_t, log_t + lb
    trace = oracle.fibsq_trace(2718281, T)
    f = oracle.interpolate_lagrange_polynomials(oracle.coset_domain(log_t, offset=1), trace, P)
    dom = oracle.coset_domain(L)
    fe = [oracle.poly_evaluate(f, x, P) for x in dom]
    alphas = [11, 22, 33 + log_t]
    cp = oracle.fibsq_cp_faithful(f, log_t, trace[-1], alphas)
    assert len(cp) - 1 == T
    want = [oracle.poly_evaluate(cp, x, P) for x in dom]
    assert [int(v) for v in oracle.fibsq_cp_evals_np(fe, log_t, lb, 5, trace[-1], alphas)] == want
    fa = np.ascontiguousarray(np.array(fe, dtype=np.uint64))
    out = np.zeros(1 << L, dtype=np.uint64)
    al = (ctypes.c_uint64 * 3)(*alphas)
    pu = ctypes.POINTER(ctypes.c_uint64)
    assert corc.orc_fibsq_cp_evals(fa.ctypes.data_as(pu), log_t, lb, 5, 5, P, trace[-1], al,
                                   out.ctypes.data_as(pu)) == 0
    assert out.tolist() == want


def test_composition_rejects_a_wrong_trace(oracle):
    """A trace that breaks the transition or a boundary constraint makes a
    division inexact (the reference's div_rem leaves a remainder)."""
    T, log_t = 16, 4
    trace = oracle.fibsq_trace(5, T)
    xs = oracle.coset_domain(log_t, offset=1)
    bad = list(trace)
    bad[7] = (bad[7] + 1) % P
    f = oracle.interpolate_lagrange_polynomials(xs, bad, P)
    with pytest.raises(ValueError):
        oracle.fibsq_cp_faithful(f, log_t, bad[-1], [1, 2, 3])
    f = oracle.interpolate_lagrange_polynomials(xs, trace, P)
    with pytest.raises(ValueError):                         # wrong claimed a_{T-1}
        oracle.fibsq_cp_faithful(f, log_t, (trace[-1] + 1) % P, [1, 2, 3])


@pytest.mark.parametrize("log_t,lb", [(5, 3), (6, 3), (4, 1), (10, 3)])
def test_c_prover_commit_matches_python_twin(oracle, corc, log_t, lb):
    """orc_fibsq_prove_commit (NTT, batch inverse, fast FRI) vs the faithful
    twin; at 2^10 (too slow for Lagrange) vs the twin's evaluation-form path."""
    a1 = 3141592
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    root = ctypes.create_string_buffer(32)
    al = (ctypes.c_uint64 * 3)()
    res = oracle.OrcFriResult()
    assert corc.orc_fibsq_prove_commit(a1, log_t, lb, 5, 5, P, ctypes.byref(och), root, al, ctypes.byref(res),
                                       None, None, None, None) == 0
    if log_t <= 6:
        ch = oracle.Channel()
        pr = oracle.fibsq_prove(a1, log_t, lb, 0, ch)
        assert root.raw == pr.trace_root and list(al) == pr.alphas
        assert [bytes(res.roots[k]) for k in range(res.n_layers)] == pr.fri.roots
        assert och.state.decode() == ch.state
    else:
        L = log_t + lb
        trace = oracle.fibsq_trace(a1, 1 << log_t)
        ys = np.ascontiguousarray(np.array(trace, dtype=np.uint64))
        pu = ctypes.POINTER(ctypes.c_uint64)
        fc = np.zeros(1 << log_t, dtype=np.uint64)
        ln = corc.orc_interpolate_coset(ys.ctypes.data_as(pu), log_t, 1, 5, P, fc.ctypes.data_as(pu))
        fe = np.zeros(1 << L, dtype=np.uint64)
        corc.orc_lde(fc.ctypes.data_as(pu), ln, L, 5, 5, P, fe.ctypes.data_as(pu))
        ch = oracle.Channel()
        ch.send(oracle.merkle_levels([int(v) for v in fe])[-1][0].hex().encode())
        alphas = [ch.receive_random_field_element() for _ in range(3)]
        assert list(al) == alphas
        cp = oracle.fibsq_cp_evals_np(fe, log_t, lb, 5, trace[-1], alphas)
        cc = np.zeros(1 << L, dtype=np.uint64)
        cl = corc.orc_interpolate_coset(np.ascontiguousarray(cp).ctypes.data_as(pu), L, 5, 5, P,
                                        cc.ctypes.data_as(pu))
        assert cl == (1 << log_t) + 1                               # deg CP = T
        r = oracle.fri_commit([int(v) for v in cc[:cl]], L, ch)
        assert [bytes(res.roots[k]) for k in range(res.n_layers)] == r.roots
        assert och.state.decode() == ch.state


# ---- verify_fibsq (host mirror, fri_amd) on oracle transcripts -------------
def test_verify_fibsq_accepts_golden_transcripts(oracle, golden):
    import fri_amd
    for c in golden["fibsq"]:
        ch = oracle.Channel(state=c["channel_in"])
        oracle.fibsq_prove(c["a1"], c["log_t"], c["log_blowup"], c["queries"], ch)
        assert fri_amd.verify_fibsq(ch.proof, c["a_last"], c["log_t"], c["log_blowup"], c["queries"],
                                    c["n_layers"], channel_state=c["channel_in"]), c["name"]


def test_verify_fibsq_rejects_every_flipped_message(oracle):
    import fri_amd
    log_t, lb, q = 4, 2, 2
    ch = oracle.Channel()
    pr = oracle.fibsq_prove(99, log_t, lb, q, ch)
    a_last = oracle.fibsq_trace(99, 1 << log_t)[-1]
    args = (a_last, log_t, lb, q, len(pr.fri.roots))
    msgs = ch.proof
    assert fri_amd.verify_fibsq(msgs, *args)
    for i, m in enumerate(msgs):
        if not m:
            continue
        b = bytearray(m)
        b[len(b) // 2] ^= 1
        assert not fri_amd.verify_fibsq(msgs[:i] + [bytes(b)] + msgs[i + 1:], *args), i
    assert not fri_amd.verify_fibsq(msgs, (a_last + 1) % P, *args[1:])      # other public output
    assert not fri_amd.verify_fibsq(msgs[:-1], *args)


def test_verify_fibsq_rejects_a_forged_composition(oracle):
    """A prover that commits a low-degree polynomial unrelated to the trace
    passes FRI but fails the composition check at the queried points."""
    import fri_amd
    log_t, lb, q = 4, 2, 3
    L = log_t + lb
    T, B, n = 1 << log_t, 1 << lb, 1 << L
    trace = oracle.fibsq_trace(99, T)
    f = oracle.interpolate_lagrange_polynomials(oracle.coset_domain(log_t, offset=1), trace, P)
    fe = [oracle.poly_evaluate(f, x, P) for x in oracle.coset_domain(L)]
    lv = oracle.merkle_levels(fe)
    ch = oracle.Channel()
    ch.send(lv[-1][0].hex().encode())
    [ch.receive_random_field_element() for _ in range(3)]
    r = oracle.fri_commit(oracle.splitmix64_field(3, T + 1), L, ch)      # not the composition
    for _ in range(q):
        idx = ch.receive_random_int(0, n - 2 * B - 1, True)
        for j in range(3):
            ch.send(oracle.fe_to_bytes(fe[idx + j * B]))
            ch.send(oracle.merkle_proof(lv, idx + j * B))
        oracle.decommit_fri_layers(idx, r.layers, r.trees, ch)
    assert not fri_amd.verify_fibsq(ch.proof, trace[-1], log_t, lb, q, len(r.roots))
