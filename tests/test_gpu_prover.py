"""GPU: the prover slice (BASELINE configs[3]) — fri_trace_commit +
fri_fibsq_composition_commit + fri_trace_decommit + fri_decommit_query,
driven by fri_amd.prove_fibsq — against the oracle bit for bit: the golden
transcripts (faithful restatement, small T), and at T = 2^10 and 2^16 the C
oracle's commit phase (orc_fibsq_prove_commit: NTT, batch inverse, fast FRI)
plus the Python twin's decommitment over the oracle's own layers and trees.
The composition polynomial itself is parity-unpinned against the reference
(its src/prover is empty); see tests/test_prover_oracle.py."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 3221225473


def _proof_sha(msgs):
    return hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m for m in msgs)).hexdigest()


def _levels(nodes: bytes, m: int):
    """orc_merkle_build layout (leaves first, power-of-two m) -> list of levels."""
    out, off = [], 0
    while True:
        out.append([nodes[32 * (off + i): 32 * (off + i + 1)] for i in range(m)])
        off += m
        if m == 1:
            return out
        m //= 2


def test_prove_matches_golden_transcripts(ctx, golden):
    import fri_amd
    for c in golden["fibsq"]:
        ch = fri_amd.Channel(state=c["channel_in"])
        pr = fri_amd.prove_fibsq(c["a1"], c["log_t"], c["log_blowup"], c["queries"], ch, ctx=ctx)
        assert pr.trace_root.hex() == c["trace_root"], c["name"]
        assert pr.alphas == c["alphas"] and pr.fri.betas == c["betas"], c["name"]
        assert [r.hex() for r in pr.fri.roots] == c["roots"], c["name"]
        assert pr.fri.final_value == c["final_value"] and pr.queries == c["query_indices"], c["name"]
        assert ch.state == c["channel_out"], c["name"]
        assert len(ch.proof) == c["messages"] and _proof_sha(ch.proof) == c["proof_sha256"], c["name"]


@pytest.mark.parametrize("log_t,lb,queries", [(10, 3, 4), (16, 3, 3), (12, 1, 2), (9, 4, 2)])
def test_prove_matches_c_oracle(ctx, corc, oracle, log_t, lb, queries):
    """The whole transcript at scale (configs[3] is log_t = 16, blowup 8)."""
    import fri_amd
    a1 = 3141592
    L = log_t + lb
    n, B = 1 << L, 1 << lb
    ch = fri_amd.Channel()
    pr = fri_amd.prove_fibsq(a1, log_t, lb, queries, ch, ctx=ctx)
    # oracle: commit phase in C, keeping trace LDE / trace tree / FRI layers / trees
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    root = ctypes.create_string_buffer(32)
    al = (ctypes.c_uint64 * 3)()
    res = oracle.OrcFriResult()
    fe = np.zeros(n, dtype=np.uint64)
    ftree = ctypes.create_string_buffer(32 * (2 * n - 1))
    lay = np.zeros(2 * n, dtype=np.uint64)
    tsz = sum(2 * (n >> k) - 1 for k in range(L + 1))
    trees = ctypes.create_string_buffer(32 * tsz)
    pu = ctypes.POINTER(ctypes.c_uint64)
    assert corc.orc_fibsq_prove_commit(a1, log_t, lb, 5, 5, P, ctypes.byref(och), root, al, ctypes.byref(res),
                                       fe.ctypes.data_as(pu), ftree, lay.ctypes.data_as(pu), trees) == 0
    assert pr.trace_root == root.raw and pr.alphas == list(al)
    assert pr.fri.roots == [bytes(res.roots[k]) for k in range(res.n_layers)]
    assert pr.fri.betas == [int(res.betas[k]) for k in range(res.n_rounds)]
    assert pr.fri.final_value == res.final_value and pr.fri.final_degree == res.final_degree
    # deg CP = T: the folds end at a constant after log_t + 1 rounds
    assert res.n_rounds == log_t + 1
    # decommitment over the oracle's data, channel continued from the oracle state
    flev = _levels(ftree.raw, n)
    layers, tlev, lo, to = [], [], 0, 0
    for k in range(res.n_layers):
        m = n >> k
        layers.append([int(v) for v in lay[lo:lo + m]])
        tlev.append(_levels(trees.raw[32 * to: 32 * (to + 2 * m - 1)], m))
        lo += m
        to += 2 * m - 1
    ref = oracle.Channel(state=och.state.decode())
    for _ in range(queries):
        idx = ref.receive_random_int(0, n - 2 * B - 1, True)
        for j in range(3):
            ref.send(oracle.fe_to_bytes(int(fe[idx + j * B])))
            ref.send(oracle.merkle_proof(flev, idx + j * B))
        oracle.decommit_fri_layers(idx, layers, tlev, ref)
    assert ch.state == ref.state
    assert ch.proof[-len(ref.proof):] == ref.proof
    assert fri_amd.verify_fibsq(ch.proof, fri_amd.fibsq_trace(a1, 1 << log_t)[-1], log_t, lb, queries,
                                len(pr.fri.roots))


def test_prove_verify_rejects_tampering(ctx):
    import fri_amd
    log_t, lb, q = 12, 3, 3
    ch = fri_amd.Channel()
    pr = fri_amd.prove_fibsq(5, log_t, lb, q, ch, ctx=ctx)
    a_last = fri_amd.fibsq_trace(5, 1 << log_t)[-1]
    args = (a_last, log_t, lb, q, len(pr.fri.roots))
    assert fri_amd.verify_fibsq(ch.proof, *args)
    first_query = 2 + 3 + 2 * len(pr.fri.roots)            # trace root, 3 alphas, roots/betas/final, index
    for i in (0, 2, first_query, first_query + 1, first_query + 2, len(ch.proof) - 1):
        b = bytearray(ch.proof[i])
        b[-1] ^= 1
        assert not fri_amd.verify_fibsq(ch.proof[:i] + [bytes(b)] + ch.proof[i + 1:], *args), i


def test_composition_detects_constraint_violation(ctx):
    """A wrong claimed output a_{T-1}: CP is no longer a polynomial of degree
    <= T and the library refuses (FRI_EDEGREE) instead of committing it."""
    import fri_amd
    log_t, lb = 10, 3
    trace = fri_amd.fibsq_trace(3141592, 1 << log_t)
    ctx.trace_commit(trace, lb, readback=False)
    with pytest.raises(fri_amd.FriError) as e:
        ctx.fibsq_composition_commit(log_t, lb, (int(trace[-1]) + 1) % P, [1, 2, 3], channel_state=bytes(32))
    assert e.value.code == fri_amd.FRI_EDEGREE
    # the refused commit's layers are not served afterwards
    assert ctx.commit_info()[1:] == (0, 0)
    buf = np.zeros(16, dtype=np.uint32)
    assert ctx.lib.fri_layer_copy(ctx.h, 0, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                  buf.size) == fri_amd.FRI_ESTATE
    res = ctx.fibsq_composition_commit(log_t, lb, int(trace[-1]), [1, 2, 3], channel_state=bytes(32))
    assert res.n_rounds == log_t + 1


def test_prover_entry_errors(ctx):
    import fri_amd
    trace = fri_amd.fibsq_trace(7, 1 << 8)
    ctx.trace_commit(trace, 3, readback=False)
    with pytest.raises(fri_amd.FriError) as e:          # other (log_t, blowup) than the resident trace
        ctx.fibsq_composition_commit(9, 3, int(trace[-1]), [1, 2, 3])
    assert e.value.code == fri_amd.FRI_ESTATE
    with pytest.raises(fri_amd.FriError) as e:
        ctx.trace_decommit(1 << 11, 8, 3, 11)             # index beyond the LDE
    assert e.value.code == fri_amd.FRI_EINVAL
    with pytest.raises(fri_amd.FriError) as e:
        ctx.trace_decommit(0, 8, 9, 11)                   # count > 8
    assert e.value.code == fri_amd.FRI_EINVAL
    vals = ctx.trace_decommit(5, 8, 3, 11)
    _, _, lde = ctx.trace_commit(trace, 3)
    assert [v for v, _ in vals] == [int(lde[5]), int(lde[13]), int(lde[21])]
