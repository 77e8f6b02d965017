"""CPU: the C oracle against the independent Python twin (hashlib SHA-256)
and against the committed golden vectors (tests/golden/fri_golden.json);
faithful reference algorithm == fast algorithms (NTT LDE, eval-form fold,
batch inverse) on the same inputs."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

P = 3221225473


def u64(vals):
    a = np.ascontiguousarray(np.asarray(vals, dtype=np.uint64))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def test_sha256_matches_hashlib(corc):
    rng = random.Random(3)
    for n in list(range(0, 130)) + [191, 192, 193, 255, 256, 1000]:
        msg = bytes(rng.getrandbits(8) for _ in range(n))
        out = ctypes.create_string_buffer(32)
        corc.orc_sha256(msg, n, out)
        assert out.raw == hashlib.sha256(msg).digest()


def test_sha256_fips_vectors(corc):
    vecs = {b"": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
            b"abc": "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
            b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq":
                "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"}
    for m, h in vecs.items():
        out = ctypes.create_string_buffer(32)
        corc.orc_sha256(m, len(m), out)
        assert out.raw.hex() == h


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 100, 256, 1000])
def test_merkle_c_matches_python(corc, oracle, n):
    vals = [random.Random(n).randrange(P) for _ in range(n)]
    arr, p = u64(vals)
    cnt = corc.orc_merkle_nodes_count(n)
    buf = ctypes.create_string_buffer(32 * cnt)
    assert corc.orc_merkle_build(p, n, buf) == cnt
    levels = oracle.merkle_levels(vals)
    flat = b"".join(b"".join(lv) for lv in levels)
    assert buf.raw == flat


def test_merkle_single_leaf_root_is_leaf_hash(oracle):
    """rs_merkle: a one-leaf tree's root is the leaf itself (mod.rs:24-26)."""
    assert oracle.merkle_root_hex([7]) == hashlib.sha256((7).to_bytes(8, "big")).hexdigest()


def test_channel_c_matches_python(corc, oracle):
    ch = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(ch))
    pc = oracle.Channel()
    rng = random.Random(9)
    for step in range(40):
        if step % 3 == 2:
            a = corc.orc_channel_receive_fe(ctypes.byref(ch), P)
            b = pc.receive_random_field_element(P)
            assert a == b
        elif step % 7 == 6:
            a = corc.orc_channel_receive_int(ctypes.byref(ch), 0, 8191)
            b = pc.receive_random_int(0, 8191, True)
            assert a == b
        else:
            msg = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 70)))
            corc.orc_channel_send(ctypes.byref(ch), msg, len(msg))
            pc.send(msg)
        assert ch.state.decode() == pc.state


def _run_c(corc, oracle, fn, case):
    coeffs = case["coeffs"]
    d = len(coeffs)
    arr, p = u64(coeffs if d else [0])
    ch = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(ch))
    if case["channel_in"]:
        ch.state = case["channel_in"].encode()
        ch.state_len = 64
    fb = None
    if case["forced_betas"] is not None:
        fbarr, fb = u64(case["forced_betas"])
    res = oracle.OrcFriResult()
    n = 1 << case["log_n"]
    total = sum(n >> k for k in range(40) if (n >> k) > 0)
    layers = np.zeros(total, dtype=np.uint64)
    rc = fn(p, d, case["log_n"], case["offset"], 5, P, ctypes.byref(ch), fb, ctypes.byref(res),
            layers.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), None)
    assert rc == 0
    return res, ch, layers


@pytest.mark.parametrize("fn_name", ["orc_fri_commit_faithful", "orc_fri_commit_fast"])
def test_golden_vectors_reproduce(corc, oracle, golden, fn_name):
    fn = getattr(corc, fn_name)
    for case in golden["cases"]:
        res, ch, layers = _run_c(corc, oracle, fn, case)
        assert res.n_layers == len(case["roots"]), case["name"]
        assert [bytes(res.roots[k]).hex() for k in range(res.n_layers)] == case["roots"], case["name"]
        assert [res.betas[r] for r in range(res.n_rounds)] == case["betas"], case["name"]
        assert res.final_value == case["final_value"] and res.final_degree == case["final_degree"]
        assert ch.state.decode() == case["channel_out"]
        off = 0
        n = 1 << case["log_n"]
        for k in range(res.n_layers):
            m = n >> k
            lay = layers[off:off + m].astype("<u4")
            assert hashlib.sha256(lay.tobytes()).hexdigest() == case["layer_sha256"][k], (case["name"], k)
            off += m


@pytest.mark.parametrize("log_n,seed", [(12, 1), (13, 2), (14, 3)])
def test_faithful_equals_fast(corc, oracle, log_n, seed):
    d = (1 << log_n) // 8
    case = {"coeffs": oracle.splitmix64_field(seed, d), "log_n": log_n, "offset": 5, "channel_in": "",
            "forced_betas": None}
    r1, c1, l1 = _run_c(corc, oracle, corc.orc_fri_commit_faithful, case)
    r2, c2, l2 = _run_c(corc, oracle, corc.orc_fri_commit_fast, case)
    assert r1.n_layers == r2.n_layers
    assert all(bytes(r1.roots[k]) == bytes(r2.roots[k]) for k in range(r1.n_layers))
    assert c1.state == c2.state
    assert np.array_equal(l1, l2)


def test_lde_equals_horner(corc, oracle):
    for log_n, d in [(3, 8), (6, 5), (9, 64)]:
        c = oracle.splitmix64_field(log_n, d)
        arr, p = u64(c)
        out = np.zeros(1 << log_n, dtype=np.uint64)
        corc.orc_lde(p, d, log_n, 5, 5, P, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        dom = oracle.coset_domain(log_n)
        assert [int(v) for v in out] == [oracle.poly_evaluate(c, x, P) for x in dom]


def test_coset_interpolation_equals_lagrange(corc, oracle):
    log_n = 4
    ys = oracle.splitmix64_field(77, 1 << log_n)
    arr, p = u64(ys)
    out = np.zeros(1 << log_n, dtype=np.uint64)
    n = corc.orc_interpolate_coset(p, log_n, 5, 5, P, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    want = oracle.interpolate_lagrange_polynomials(oracle.coset_domain(log_n), ys, P)
    assert [int(v) for v in out[:n]] == want


def test_batch_inverse_equals_fermat(corc):
    x = [0, 1, 2, 3, P - 1, 12345, 0, 99]
    arr, p = u64(x)
    out = np.zeros(len(x), dtype=np.uint64)
    corc.orc_batch_inverse(p, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), len(x), P)
    assert [int(v) for v in out] == [corc.orc_fe_inverse(v, P) for v in x]


def test_eval_fold_equals_coefficient_fold(corc, oracle):
    """fri_commit.rs:53-65: fold of the evaluations == evaluations of the folded polynomial."""
    log_m = 6
    c = oracle.splitmix64_field(4, 16)
    beta = 123456789
    layer = np.zeros(1 << log_m, dtype=np.uint64)
    arr, p = u64(c)
    corc.orc_lde(p, len(c), log_m, 5, 5, P, layer.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    out = np.zeros(1 << (log_m - 1), dtype=np.uint64)
    w = corc.orc_fe_pow(5, (P - 1) >> log_m, P)
    corc.orc_fold_eval(layer.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 1 << log_m, 5, w, beta, P,
                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    folded, _ = oracle.next_fri_polynomial(c, len(c) - 1, beta, P)
    dom = [oracle.fe_pow(x, 2, P) for x in oracle.coset_domain(log_m)[: 1 << (log_m - 1)]]
    assert [int(v) for v in out] == [oracle.poly_evaluate(folded, x, P) for x in dom]


def test_degree_bookkeeping_beta_zero(oracle):
    """beta = 0 with an all-zero even part keeps the odd part's degree
    (scalar_mul does not trim, ops.rs:194-198; add_assign early return ops.rs:87-91)."""
    c = [0, 5, 0, 7, 0, 9]
    coeffs, deg = oracle.next_fri_polynomial(c, 5, 0, P)
    assert coeffs == [0, 0, 0] and deg == 2
    coeffs, deg = oracle.next_fri_polynomial(c, 5, 3, P)
    assert deg == 2 and coeffs == [15, 21, 27]


def test_commit_rejects_domain_exhaustion(oracle):
    with pytest.raises(ValueError):
        oracle.fri_commit([1] * 9, 3, oracle.Channel())


# ---- decommitment (fri_commit.rs:137-179) ---------------------------------
def _verify_path(leaf_value, idx, path, n, root):
    """Recompute the root from a leaf and its rs_merkle single-leaf proof."""
    import hashlib
    h = hashlib.sha256(int(leaf_value).to_bytes(8, "big")).digest()
    width, off = n, 0
    while width > 1:
        sib = idx ^ 1
        if sib < width:
            s = path[off:off + 32]
            off += 32
            h = hashlib.sha256(s + h if idx & 1 else h + s).digest()
        idx >>= 1
        width = (width + 1) // 2
    assert off == len(path)
    return h == root


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 64, 100])
def test_merkle_proof_verifies(oracle, n):
    vals = oracle.splitmix64_field(n, n)
    levels = oracle.merkle_levels(vals)
    for idx in range(n):
        assert _verify_path(vals[idx], idx, oracle.merkle_proof(levels, idx), n, levels[-1][0])


def test_golden_decommit_reproduces(oracle, golden):
    import hashlib
    for c in golden["cases"]:
        ch = oracle.Channel(state=c["channel_in"])
        r = oracle.fri_commit(c["coeffs"], c["log_n"], ch, offset=c["offset"], forced_betas=c["forced_betas"])
        n0 = len(ch.proof)
        oracle.decommit_fri(3, (1 << c["log_n"]) - 1, r.layers, r.trees, ch)
        want = c["decommit_q3"]
        assert ch.state == want["state"], c["name"]
        assert len(ch.proof) - n0 == want["messages"]
        got = hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m for m in ch.proof[n0:])).hexdigest()
        assert got == want["proof_sha256"], c["name"]


def test_flat_transcript_helper_matches_python_twin(oracle, corc):
    """tests/oracle_flat.py (the C oracle's layers and trees, decommitted by
    the Python twin through index views) gives the Python twin's own whole
    transcript: commit messages, two queries' openings and the final state."""
    import oracle_flat
    for log_n, seed, state in ((9, 3, ""), (10, 4, "ab" * 32)):
        coeffs = oracle.splitmix64_field(seed, (1 << log_n) // 8)
        msgs, st = oracle_flat.transcript(corc, coeffs, log_n, 2, state=state)
        ch = oracle.Channel(state=state)
        r = oracle.fri_commit(coeffs, log_n, ch)
        oracle.decommit_fri(2, (1 << log_n) - 1, r.layers, r.trees, ch)
        assert msgs == ch.proof and st == ch.state
