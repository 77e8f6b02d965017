"""GPU parity: every C-ABI entry point of libfri_amd.so against the oracle
(C restatement + Python twin) on identical inputs; bit-exact (integer field
arithmetic + SHA-256, no tolerance).  Mirrors the reference's test style
(src/fields/element.rs:149-290, src/polynomial/ops.rs:551-1089,
src/polynomial/interpolation.rs:154-374) for the GPU path."""
import ctypes
import os
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 3221225473


def rng_field(seed, n):
    r = np.random.default_rng(seed)
    return r.integers(0, P, size=n, dtype=np.uint64)


def c_u64(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


# ------------------------------------------------------------------ field --
def test_batch_inverse_matches_fermat(ctx, corc):
    x = rng_field(1, 10007)
    x[::97] = 0                              # inverse(0) = 0 (element.rs:54-57)
    x[1] = 1
    x[2] = P - 1
    got = ctx.batch_inverse(x)
    xs, px = c_u64(x)
    want = np.empty_like(xs)
    corc.orc_batch_inverse(px, want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), xs.size, P)
    assert np.array_equal(got.astype(np.uint64), want)
    for i in (0, 1, 2, 3, 500, 10006):
        assert int(got[i]) == corc.orc_fe_inverse(int(x[i]), P)


def test_batch_inverse_edges(ctx):
    assert ctx.batch_inverse([0]).tolist() == [0]
    assert ctx.batch_inverse([1, 2]).tolist() == [1, (P + 1) // 2]
    assert ctx.batch_inverse([]).tolist() == []


# --------------------------------------------------------------- poly: LDE --
@pytest.mark.parametrize("log_n,d", [(1, 1), (1, 2), (3, 1), (4, 2), (6, 8), (10, 128), (12, 512),
                                     (13, 1024), (14, 2048), (16, 8192), (17, 100), (20, 1 << 17),
                                     (22, 1 << 19), (12, 4096),
                                     # 16-byte load/store phases (k_ntt_pass VEC): full tiles from
                                     # n = 2^13; a first pass of 8 stages whose last loaded vector
                                     # straddles d (d mod 4 = 1, 2, 3), blowup 1, n = one tile
                                     (16, 8189), (16, 8190), (16, 8191), (16, 1 << 16), (13, 8191),
                                     (13, 1 << 13), (24, (1 << 21) - 3),
                                     # first pass of 9..12 stages (k_ntt_first_wide) with 3, 2, 1 and 0
                                     # trivial stages, vectors straddling d, blowup 1
                                     (17, 1 << 14), (17, 16385), (18, 32767), (19, 1 << 16), (19, (1 << 19) - 1),
                                     (20, 1 << 19), (20, 1 << 20), (21, 1 << 18), (23, 12345),
                                     # 2^24 with 2 and 0 trivial stages
                                     (24, 1 << 22), (24, 1 << 24)])
def test_lde_matches_oracle(ctx, corc, log_n, d):
    c = rng_field(log_n * 100 + d, d)
    got = ctx.lde(c, log_n, 5)
    cs, pc = c_u64(c)
    want = np.empty(1 << log_n, dtype=np.uint64)
    assert corc.orc_lde(pc, d, log_n, 5, 5, P, want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    assert np.array_equal(got.astype(np.uint64), want)


def test_lde_matches_horner(ctx, corc):
    """Config 1 analogue (benches/poly_ops.rs:161-181): Horner at every domain point."""
    log_n, d = 10, 1 << 10
    c = rng_field(3333, d)
    got = ctx.lde(c, log_n, 5)
    cs, pc = c_u64(c)
    w = corc.orc_fe_pow(5, (P - 1) >> log_n, P)
    for i in (0, 1, 7, 511, 512, 1023):
        x = corc.orc_fe_mul(5, corc.orc_fe_pow(w, i, P), P)
        assert int(got[i]) == corc.orc_poly_evaluate(pc, d, x, P)


def test_evaluate_matches_horner(ctx, corc):
    c = rng_field(7, 300)
    xs = rng_field(8, 257)
    got = ctx.evaluate(c, xs)
    cs, pc = c_u64(c)
    for i in range(0, 257, 16):
        assert int(got[i]) == corc.orc_poly_evaluate(pc, 300, int(xs[i]), P)
    assert ctx.evaluate([], [5]).tolist() == [0]          # zero poly (ops.rs:561-566)
    assert ctx.evaluate([5], [0]).tolist() == [5]          # constant (ops.rs:568-574)


@pytest.mark.parametrize("d,count", [(1 << 21, 1), (5000, 1), (4096, 3), ((1 << 16) + 3, 100), (1 << 20, 7),
                                     (100000, 2000)])
def test_evaluate_few_points_many_coefficients(ctx, corc, d, count):
    """Polynomial::evaluate (ops.rs:76-83) with the coefficients split over
    lanes (few points, many coefficients: the reference's bench_eval shape,
    benches/poly_ops.rs:161-181, at prover sizes) against Horner in the C oracle;
    x = 0, 1 and p - 1 included."""
    c = rng_field(d + count, d)
    xs = rng_field(count * 7 + 1, count)
    xs[0] = 0
    if count > 2:
        xs[1], xs[2] = 1, P - 1
    got = ctx.evaluate(c, xs)
    cs, pc = c_u64(c)
    for i in range(count) if count <= 8 else list(range(4)) + list(range(count - 4, count)) + [count // 2]:
        assert int(got[i]) == corc.orc_poly_evaluate(pc, d, int(xs[i]), P), i


# ------------------------------------------------------ poly: interpolate --
@pytest.mark.parametrize("log_n", [0, 1, 2, 5, 10, 13, 16, 17, 20, 24])
def test_interpolate_roundtrip(ctx, corc, log_n):
    n = 1 << log_n
    c = rng_field(log_n + 5, n)
    c[-1] = 0
    c[-2 if n > 1 else -1] = 0
    ys = ctx.lde(c, log_n, 5)
    got = ctx.interpolate(ys, 5)
    trimmed = np.trim_zeros(c.astype(np.uint64), "b")
    assert np.array_equal(got.astype(np.uint64), trimmed)
    ys64, py = c_u64(ys)
    want = np.empty(n, dtype=np.uint64)
    ln = corc.orc_interpolate_coset(py, log_n, 5, 5, P, want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert np.array_equal(got.astype(np.uint64), want[:ln])


@pytest.mark.parametrize("n,seed,dups", [(1, 1, 0), (2, 2, 0), (3, 3, 1), (5, 4, 0), (7, 5, 2), (16, 6, 0),
                                         (17, 7, 3), (33, 8, 0), (40, 9, 5)])
def test_interpolate_points_matches_lagrange(ctx, oracle, n, seed, dups):
    """Polynomial::interpolate on arbitrary points (interpolation.rs:121-152,
    fri_interpolate_points) against the twin's restatement of the reference's
    Lagrange sum, duplicate points (whose basis polynomials vanish through
    inverse(0) = 0) and zero values included."""
    r = np.random.default_rng(seed)
    xs = [int(v) for v in r.integers(0, P, n)]
    for i in range(dups):
        xs[int(r.integers(0, n))] = xs[int(r.integers(0, n))]
    ys = [int(v) for v in r.integers(0, P, n)]
    if n > 2:
        ys[1] = 0
    got = ctx.interpolate_points(xs, ys)
    want = oracle.interpolate_lagrange_polynomials(xs, ys, P)
    assert got.tolist() == want


@pytest.mark.parametrize("n", [100, 1000, 4096, 4999, 16387])
def test_interpolate_points_matches_c_oracle(ctx, corc, n):
    """Larger arbitrary point sets against the C oracle's Lagrange sum; the
    result evaluates back to ys at every point."""
    r = np.random.default_rng(n)
    xs = np.unique(r.integers(0, P, n + 64, dtype=np.uint64))[:n]
    r.shuffle(xs)
    ys = r.integers(0, P, n, dtype=np.uint64)
    got = ctx.interpolate_points(xs, ys)
    want = np.empty(n, dtype=np.uint64)
    ln = corc.orc_interpolate_lagrange(xs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                       ys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                       want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), P)
    assert np.array_equal(got.astype(np.uint64), want[:ln])
    assert np.array_equal(ctx.evaluate(got, xs).astype(np.uint64), ys)


def test_interpolate_points_on_coset_equals_intt(ctx):
    """On a coset the O(n^2) path and the iNTT path give the same polynomial."""
    log_n = 10
    c = rng_field(77, 1 << log_n)
    ys = ctx.lde(c, log_n, 5)
    w = pow(5, (P - 1) >> log_n, P)
    xs = [5 * pow(w, i, P) % P for i in range(1 << log_n)]
    assert np.array_equal(ctx.interpolate_points(xs, ys), ctx.interpolate(ys, 5))


def test_interpolate_points_edges(ctx):
    import fri_amd
    assert ctx.interpolate_points([], []).tolist() == []                     # Polynomial::zero()
    assert ctx.interpolate_points([7], [0]).tolist() == []
    assert ctx.interpolate_points([7], [9]).tolist() == [9]
    with pytest.raises(fri_amd.FriError):
        ctx.interpolate_points([1, 2], [3])                                  # interpolation.rs:127 panics
    with pytest.raises(fri_amd.FriError):
        ctx.interpolate_points([P], [1])                                     # not canonical


def test_interpolate_matches_lagrange(ctx, corc, oracle):
    """Same interpolant as the reference's Lagrange path (interpolation.rs:121-152)."""
    log_n = 4
    ys = rng_field(99, 1 << log_n)
    got = ctx.interpolate(ys, 5)
    xs = oracle.coset_domain(log_n)
    want = oracle.interpolate_lagrange_polynomials(xs, [int(v) for v in ys], P)
    assert got.tolist() == want


# ---------------------------------------------------------------- fold ----
@pytest.mark.parametrize("log_m", [1, 2, 5, 11, 16, 20])
def test_fold_matches_coefficient_fold(ctx, corc, oracle, log_m):
    """fri_commit.rs:53-65: coefficient fold + Horner on the squared domain."""
    m = 1 << log_m
    d = max(1, m // 4)
    c = rng_field(log_m, d)
    layer = ctx.lde(c, log_m, 5)
    beta = int(rng_field(log_m + 1000, 1)[0])
    got = ctx.fold(layer, 5, beta)
    lay, pl = c_u64(layer)
    want = np.empty(m // 2, dtype=np.uint64)
    w = corc.orc_fe_pow(5, (P - 1) >> log_m, P)
    corc.orc_fold_eval(pl, m, 5, w, beta, P, want.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert np.array_equal(got.astype(np.uint64), want)
    if log_m <= 11:
        poly, _ = oracle.next_fri_polynomial([int(v) for v in c], len(c) - 1, beta, P)
        sq = corc.orc_fe_mul(5, 5, P)
        ref = ctx.lde(poly if poly else [0], log_m - 1, sq)
        assert np.array_equal(got, ref)


# -------------------------------------------------------------- Merkle ----
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 64, 100, 512, 513, 1024, 4096, 65536, 1 << 20])
def test_merkle_root_matches_oracle(ctx, corc, oracle, n):
    v = rng_field(n, n)
    got = ctx.merkle_root(v)
    vs, pv = c_u64(v)
    cnt = corc.orc_merkle_nodes_count(n)
    buf = ctypes.create_string_buffer(32 * cnt)
    corc.orc_merkle_build(pv, n, buf)
    assert got == buf.raw[32 * (cnt - 1):]
    if n <= 4096:
        assert got.hex() == oracle.merkle_root_hex([int(x) for x in v])


def test_large_merkle_root_releases_scratch(corc, oracle):
    """fri_merkle_root builds its tree in the context's grown scratch; a tree
    past 256 MiB is released after the call, so a large root does not pin HBM
    for the context's life and a large commit on the same context still fits
    (16 GiB pinned after a 2^28 root)."""
    import fri_amd
    big = fri_amd.Context(0, 24)
    try:
        base = big.device_bytes()[0]
        v = rng_field(23, 1 << 23)                    # tree of 2^24 digests: 512 MiB
        got = big.merkle_root(v)
        vs, pv = c_u64(v)
        cnt = corc.orc_merkle_nodes_count(1 << 23)
        buf = ctypes.create_string_buffer(32 * cnt)
        corc.orc_merkle_build(pv, 1 << 23, buf)
        assert got == buf.raw[32 * (cnt - 1):]
        cur, peak = big.device_bytes()
        assert cur == base and peak >= base + (512 << 20)
        small = rng_field(11, 1 << 12)                # small trees keep their scratch (no hipFree per call)
        big.merkle_root(small)
        assert big.device_bytes()[0] > base
        c = oracle.splitmix64_np(42, 1 << 21).astype(np.uint32)
        res = big.commit(c, 24)
        assert res.n_layers == 22
    finally:
        big.close()


def test_merkle_tree_class(oracle):
    import fri_amd
    vals = [1, 2, 3, 4, 5]
    assert fri_amd.MerkleTree(vals).root() == oracle.merkle_root_hex(vals)


# -------------------------------------------------------------- commit ----
def _check_case(ctx, case, graph=True):
    import fri_amd
    st = bytes.fromhex(case["channel_in"]) if case["channel_in"] else None
    res = ctx.commit(case["coeffs"], case["log_n"], case["offset"], channel_state=st,
                     forced_betas=case["forced_betas"], graph=graph)
    assert res.n_layers == len(case["roots"])
    assert [bytes(res.roots[k]).hex() for k in range(res.n_layers)] == case["roots"]
    assert [int(res.betas[r]) for r in range(res.n_rounds)] == case["betas"]
    assert res.final_value == case["final_value"]
    assert res.final_degree == case["final_degree"]
    assert bytes(res.channel_out.digest).hex() == case["channel_out"]
    for k in range(res.n_layers):
        lay = ctx.layer(k, case["log_n"])
        assert hashlib.sha256(lay.astype("<u4").tobytes()).hexdigest() == case["layer_sha256"][k]
    leaves = ctx.tree_level(0, 0, case["log_n"])
    assert [h.hex() for h in leaves[:4]] == case["leaf0_head"]
    return fri_amd


def test_commit_golden_vectors(ctx, golden):
    for case in golden["cases"]:
        _check_case(ctx, case, graph=True)


def test_commit_golden_eager(ctx, golden):
    for case in golden["cases"][::4]:
        _check_case(ctx, case, graph=False)


def test_commit_channel_mirror(ctx, golden, oracle):
    """fri_commit() drives the host Channel exactly like the reference transcript."""
    import fri_amd
    case = [c for c in golden["cases"] if c["name"] == "rand_n9_s42"][0]
    ch = fri_amd.Channel()
    proof = fri_amd.fri_commit(case["coeffs"], case["log_n"], ch, ctx=ctx)
    och = oracle.Channel()
    oracle.fri_commit(case["coeffs"], case["log_n"], och)
    assert ch.state == och.state
    assert ch.proof == och.proof
    assert ch.proof_size() == case["proof_size"]
    assert proof.final_poly == [case["final_value"]]


@pytest.mark.parametrize("log_n,seed", [(12, 1), (14, 2), (16, 3), (18, 4), (20, 42)])
def test_commit_matches_fast_oracle(ctx, corc, oracle, log_n, seed):
    d = (1 << log_n) // 8
    c = np.array(oracle.splitmix64_field(seed, d), dtype=np.uint64)
    res = ctx.commit(c, log_n)
    cs, pc = c_u64(c)
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(pc, d, log_n, 5, 5, P, ctypes.byref(och), None, ctypes.byref(ores),
                                    None, None) == 0
    assert res.n_layers == ores.n_layers
    for k in range(ores.n_layers):
        assert bytes(res.roots[k]) == bytes(ores.roots[k])
    for r in range(ores.n_rounds):
        assert res.betas[r] == ores.betas[r]
    assert res.final_value == ores.final_value
    assert bytes(res.channel_out.digest).hex() == och.state.decode()


@pytest.mark.parametrize("log_n,d,seed", [(16, 1, 7), (16, 4, 8), (14, 2, 9), (18, 16, 10), (21, 64, 11), (12, 2, 12)])
def test_commit_final_layer_outside_tail(ctx, corc, oracle, log_n, d, seed):
    """High blowup: the degree reaches 0 on a layer of >= 2^10 elements, so
    the final send (channel jobs 6, 7) runs in a k_tree_top after the root
    (round 5: every post-level job in one iteration), and the tail kernel and
    later layers are gated off.  Bit-exact against the C oracle."""
    c = np.array(oracle.splitmix64_field(seed, d), dtype=np.uint64)
    res = ctx.commit(c, log_n)
    cs, pc = c_u64(c)
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(pc, d, log_n, 5, 5, P, ctypes.byref(och), None, ctypes.byref(ores),
                                    None, None) == 0
    assert log_n - (ores.n_layers - 1) >= 10          # the last layer is not a tail layer
    assert res.n_layers == ores.n_layers and res.n_rounds == ores.n_rounds
    for k in range(ores.n_layers):
        assert bytes(res.roots[k]) == bytes(ores.roots[k])
    for r in range(ores.n_rounds):
        assert res.betas[r] == ores.betas[r]
    assert res.final_value == ores.final_value
    assert bytes(res.channel_out.digest).hex() == och.state.decode()


def test_commit_2p24_full_parity(ctx, corc, oracle):
    """BASELINE config 3 (codeword 2^24, blowup 8): bit-exact against the
    OpenMP C oracle, plus size-independent properties."""
    log_n = 24
    d = 1 << 21
    c = np.array(oracle.splitmix64_field(42, d), dtype=np.uint64)
    res = ctx.commit(c, log_n)
    assert res.n_rounds == 21 and res.n_layers == 22
    last = ctx.layer(21, log_n)
    assert last.size == 8 and np.all(last == res.final_value)      # final layer constant
    cs, pc = c_u64(c)
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(pc, d, log_n, 5, 5, P, ctypes.byref(och), None, ctypes.byref(ores),
                                    None, None) == 0
    assert [bytes(res.roots[k]) for k in range(22)] == [bytes(ores.roots[k]) for k in range(22)]
    assert [res.betas[r] for r in range(21)] == [ores.betas[r] for r in range(21)]
    assert bytes(res.channel_out.digest).hex() == och.state.decode()


def _large_commit_parity(oracle_commit, oracle, log_n, seed):
    """One commit at 2^log_n on a context of its own vs the OpenMP C oracle:
    every root, beta, final value and the channel state; the last layer is
    the constant final value (size-independent property)."""
    import fri_amd
    d = 1 << (log_n - 3)
    c = oracle.splitmix64_np(seed, d).astype(np.uint32)
    big = fri_amd.Context(0, log_n)
    try:
        res = big.commit(c, log_n)
        assert res.n_rounds == log_n - 3 and res.n_layers == log_n - 2
        last = big.layer(res.n_layers - 1, log_n)
        assert last.size == 8 and np.all(last == res.final_value)
        got = {"roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)],
               "betas": [int(res.betas[r]) for r in range(res.n_rounds)],
               "final_value": int(res.final_value), "final_degree": int(res.final_degree),
               "state": bytes(res.channel_out.digest).hex()}
    finally:
        big.close()
    assert got == oracle_commit(log_n, seed)


def test_commit_2p26_full_parity(oracle_commit, oracle):
    _large_commit_parity(oracle_commit, oracle, 26, 7)


@pytest.mark.timeout(600)
def test_commit_2p28_full_parity(oracle_commit, oracle):
    """BASELINE configs[4]'s codeword (2^28) on ONE GPU, bit-exact (~38 GB
    HBM; the oracle transcript is shared with the 8-rank sharded test)."""
    _large_commit_parity(oracle_commit, oracle, 28, 8)


def test_auth_path_verifies(ctx, oracle):
    log_n = 10
    c = oracle.splitmix64_field(77, 128)
    res = ctx.commit(c, log_n)
    for k in (0, 3):
        for idx in (0, 5, (1 << (log_n - k)) - 1):
            val, path = ctx.auth_path(k, idx, log_n)
            h = hashlib.sha256(int(val).to_bytes(8, "big")).digest()
            i = idx
            for sib in path:
                h = hashlib.sha256(h + sib if i % 2 == 0 else sib + h).digest()
                i //= 2
            assert h == bytes(res.roots[k])


def test_graph_replay_stable(ctx, oracle):
    c = oracle.splitmix64_field(5, 1 << 13)
    a = ctx.commit(c, 16)
    b = ctx.commit(c, 16)
    c2 = oracle.splitmix64_field(6, 1 << 13)
    x = ctx.commit(c2, 16)
    assert bytes(a.roots[0]) == bytes(b.roots[0]) != bytes(x.roots[0])
    assert [a.betas[i] for i in range(13)] == [b.betas[i] for i in range(13)]


def _oracle_commit(oracle, coeffs, log_n):
    ch = oracle.Channel()
    r = oracle.fri_commit(coeffs, log_n, ch, keep=False)
    return [x.hex() for x in r.roots], r.betas, r.final_value, ch.state


def _gpu_commit(ctx, coeffs, log_n):
    res = ctx.commit(coeffs, log_n)
    return ([bytes(res.roots[k]).hex() for k in range(res.n_layers)], [res.betas[r] for r in range(res.n_rounds)],
            res.final_value, bytes(res.channel_out.digest).hex() if res.channel_out.has_state else "")


@pytest.mark.parametrize("log_n", [5, 12, 16, 20])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_noncanonical_input_rejected_on_device(ctx, oracle, oracle_commit, log_n, where):
    """The input coefficients are validated on the device, in layer 0's
    coefficient scan (tail kernel at 2^5, wide leaf + top at 2^12/2^16, quad
    leaf + mids + top at 2^20): a value >= p anywhere gives FRI_EINVAL, with
    nothing served, through the host and the device entry points; the next
    valid commit on the same context equals the C oracle's."""
    import fri_amd
    d = (1 << log_n) >> 3
    seed = 500 + log_n
    coeffs = oracle.splitmix64_np(seed, d).astype(np.uint32)
    bad = coeffs.copy()
    bad[{"first": 0, "middle": d // 2, "last": d - 1}[where]] = P if where != "middle" else 0xFFFFFFFF
    with pytest.raises(fri_amd.FriError) as e:
        ctx.commit(bad, log_n)
    assert e.value.code == fri_amd.FRI_EINVAL
    assert ctx.commit_info()[2] == 0                                    # no layers served
    # the same input through fri_commit_device, from the context's input buffer
    dptr = ctypes.c_void_p(ctx.input_upload(bad))
    res = fri_amd.CommitResult()
    rc = ctx.lib.fri_commit_device(ctx.h, dptr, d, log_n, fri_amd.GENERATOR, None, 0, None, ctypes.byref(res))
    assert rc == fri_amd.FRI_EINVAL
    res = ctx.commit(coeffs, log_n)
    got = {"roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)],
           "betas": [int(res.betas[r]) for r in range(res.n_rounds)],
           "final_value": int(res.final_value), "final_degree": int(res.final_degree),
           "state": bytes(res.channel_out.digest).hex()}
    assert got == oracle_commit(log_n, seed)


@pytest.mark.parametrize("log_n,d", [(1, 1), (1, 2), (2, 1), (2, 4), (3, 3), (3, 8), (4, 16), (5, 7), (5, 32)])
def test_tiny_codewords(ctx, oracle, log_n, d):
    """Smallest domains, including blowup 1 (d = n): the last layer has one element."""
    coeffs = oracle.splitmix64_field(100 + log_n * 10 + d, d)
    assert _gpu_commit(ctx, coeffs, log_n) == _oracle_commit(oracle, coeffs, log_n)


def test_plan_reuse_across_sizes(ctx, corc, oracle):
    """One context, commits of changing size: plans are rebuilt and graphs re-captured."""
    for log_n in (12, 9, 14, 12, 10, 14):
        coeffs = oracle.splitmix64_field(log_n, (1 << log_n) // 8)
        if log_n <= 10:
            want = _oracle_commit(oracle, coeffs, log_n)
        else:
            c = np.array(coeffs, dtype=np.uint64)
            cs, pc = c_u64(c)
            och = oracle.OrcChannel()
            corc.orc_channel_init(ctypes.byref(och))
            ores = oracle.OrcFriResult()
            assert corc.orc_fri_commit_fast(pc, len(coeffs), log_n, 5, 5, P, ctypes.byref(och), None,
                                            ctypes.byref(ores), None, None) == 0
            want = ([bytes(ores.roots[k]).hex() for k in range(ores.n_layers)],
                    [ores.betas[r] for r in range(ores.n_rounds)], ores.final_value, och.state.decode())
        assert _gpu_commit(ctx, coeffs, log_n) == want, log_n


def test_error_codes(ctx):
    import fri_amd
    with pytest.raises(fri_amd.FriError) as e:
        ctx.commit([1] * 33, 5)                              # d > n: reference exhausts the domain
    assert e.value.code == fri_amd.FRI_EDEGREE
    with pytest.raises(fri_amd.FriError) as e:
        ctx.commit([P], 5)                                   # not canonical
    assert e.value.code == fri_amd.FRI_EINVAL
    with pytest.raises(fri_amd.FriError) as e:
        ctx.merkle_root([])                                  # merkle/mod.rs:25 unwrap on empty
    assert e.value.code == fri_amd.FRI_EINVAL
    with pytest.raises(fri_amd.FriError):
        ctx.lde([1, 2], 30)                                  # beyond context capacity


# ---- decommitment: fri_decommit_query + host mirror (fri_commit.rs:137-179) --
def _proof_hash(msgs):
    import hashlib
    return hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m for m in msgs)).hexdigest()


def test_decommit_matches_golden(ctx, golden):
    import fri_amd
    for c in golden["cases"]:
        if c["forced_betas"] is not None:
            continue                      # the reference surface has no forced betas
        ch = fri_amd.Channel(state=c["channel_in"])
        proof = fri_amd.fri_commit(c["coeffs"], c["log_n"], ch, offset=c["offset"], ctx=ctx)
        assert ch.state == c["channel_out"], c["name"]
        n0 = len(ch.proof)
        fri_amd.decommit_fri(3, (1 << c["log_n"]) - 1, proof, ch)
        want = c["decommit_q3"]
        assert ch.state == want["state"], c["name"]
        assert len(ch.proof) - n0 == want["messages"], c["name"]
        assert _proof_hash(ch.proof[n0:]) == want["proof_sha256"], c["name"]


@pytest.mark.parametrize("log_n,seed,queries", [(16, 5, 8), (20, 6, 4)])
def test_decommit_matches_oracle_large(ctx, oracle, log_n, seed, queries):
    """Device gather at scale vs the oracle's rs_merkle proofs, over the same
    (bit-exact, separately tested) layers."""
    import fri_amd
    coeffs = oracle.splitmix64_field(seed, (1 << log_n) // 8)
    ch = fri_amd.Channel()
    proof = fri_amd.fri_commit(coeffs, log_n, ch, ctx=ctx)
    layers = [[int(v) for v in proof.layer(k)] for k in range(proof.n_layers)]
    trees = [oracle.merkle_levels(l) for l in layers]
    assert [t[-1][0] for t in trees] == proof.roots
    och = oracle.Channel(state=ch.state)
    n0 = len(ch.proof)
    fri_amd.decommit_fri(queries, (1 << log_n) - 1, proof, ch)
    oracle.decommit_fri(queries, (1 << log_n) - 1, layers, trees, och)
    assert ch.state == och.state
    assert ch.proof[n0:] == och.proof


def test_decommit_errors(ctx):
    import ctypes

    import fri_amd
    vals = np.zeros(64, dtype=np.uint32)
    ln = ctypes.c_size_t()
    fri_amd.fri_commit(list(range(1, 17)), 7, fri_amd.Channel(), ctx=ctx)
    rc = ctx.lib.fri_decommit_query(ctx.h, 3, vals.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), 64, None, 0,
                                    ctypes.byref(ln))
    assert rc == fri_amd.FRI_EINVAL                            # no paths buffer ...
    assert ln.value == sum(64 * (7 - k) for k in range(5))     # ... but the size is reported (5 layers)


def test_stale_proof_refused(ctx, oracle):
    """A FRIProof reads its layers from the context; once a later commit has
    replaced them (here a smaller codeword) its read-backs raise instead of
    serving the other commit's data (fri_commit_info generation)."""
    import fri_amd
    c12 = oracle.splitmix64_field(12, 512)
    p1 = fri_amd.fri_commit(c12, 12, fri_amd.Channel(), ctx=ctx)
    l1 = p1.layer(1)
    assert l1.size == 2048
    g1 = ctx.commit_info()
    p2 = fri_amd.fri_commit(oracle.splitmix64_field(10, 128), 10, fri_amd.Channel(), ctx=ctx)
    assert ctx.commit_info()[0] > g1[0] and ctx.commit_info()[1:] == (10, p2.n_layers)
    with pytest.raises(fri_amd.FriError) as e:
        p1.layer(0)
    assert e.value.code == fri_amd.FRI_ESTATE
    with pytest.raises(fri_amd.FriError) as e:
        fri_amd.decommit_fri(1, 4095, p1, fri_amd.Channel())
    assert e.value.code == fri_amd.FRI_ESTATE
    with pytest.raises(fri_amd.FriError) as e:
        ctx.layer(0, 12)                                     # wrong codeword size for the resident commit
    assert e.value.code == fri_amd.FRI_ESTATE
    assert p2.layer(0).size == 1024
    # the same polynomial again: the new proof serves, the old one stays refused
    p3 = fri_amd.fri_commit(c12, 12, fri_amd.Channel(), ctx=ctx)
    assert np.array_equal(p3.layer(1), l1)
    with pytest.raises(fri_amd.FriError):
        p2.layer(0)



# ---- trace side of the prover: fri_trace_commit -------
def _stark101_trace(n):
    """STARK-101's FibonacciSq trace: a0 = 1, a1 = 3141592, a_{i+2} = a_{i+1}^2 + a_i^2 (mod p)."""
    a = [1, 3141592]
    while len(a) < n:
        a.append((a[-1] * a[-1] + a[-2] * a[-2]) % P)
    return a[:n]


def test_trace_commit_small_vs_reference_algorithms(ctx, oracle):
    """Lagrange interpolation + Horner evaluation + rs_merkle tree (the
    reference's own algorithms, restated) at 2^6 -> 2^9."""
    log_t, lb = 6, 3
    trace = oracle.splitmix64_field(77, 1 << log_t)
    root, coeffs, lde = ctx.trace_commit(trace, lb)
    xs = oracle.coset_domain(log_t, offset=1)
    want_c = oracle.interpolate_lagrange_polynomials(xs, trace, P)
    assert [int(c) for c in coeffs] == want_c
    want_lde = [oracle.poly_evaluate(want_c, x, P) for x in oracle.coset_domain(log_t + lb)]
    assert [int(v) for v in lde] == want_lde
    assert root == oracle.merkle_levels(want_lde)[-1][0]


@pytest.mark.parametrize("log_t,lb,kind", [(10, 3, "stark101"), (16, 3, "random"), (16, 2, "stark101")])
def test_trace_commit_vs_fast_oracle(ctx, corc, oracle, log_t, lb, kind):
    """BASELINE configs[3]'s trace length (2^16) and the STARK-101 trace, vs
    the C oracle's coset interpolation, LDE and Merkle build, plus a round
    trip: every 2^lb-th LDE point lies on offset*<w_t>, and interpolating
    those values gives the trace polynomial back."""
    nt = 1 << log_t
    trace = _stark101_trace(nt) if kind == "stark101" else oracle.splitmix64_field(log_t, nt)
    root, coeffs, lde = ctx.trace_commit(trace, lb)
    ys = np.ascontiguousarray(np.array(trace, dtype=np.uint64))
    oc = np.zeros(nt, dtype=np.uint64)
    ln = corc.orc_interpolate_coset(ys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), log_t, 1, 5, P,
                                    oc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
    assert ln == len(coeffs) and np.array_equal(oc[:ln].astype(np.uint32), coeffs)
    ol = np.zeros(nt << lb, dtype=np.uint64)
    c64 = np.ascontiguousarray(oc[:max(ln, 1)])
    assert corc.orc_lde(c64.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ln, log_t + lb, 5, 5, P,
                        ol.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) == 0
    assert np.array_equal(ol.astype(np.uint32), lde)
    cnt = corc.orc_merkle_nodes_count(nt << lb)
    buf = ctypes.create_string_buffer(32 * cnt)
    corc.orc_merkle_build(ol.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nt << lb, buf)
    assert root == buf.raw[32 * (cnt - 1):]
    # every 2^lb-th LDE point is offset * w_t^i: interpolating those values on
    # that coset gives the trace polynomial back
    back = ctx.interpolate(lde[:: 1 << lb], 5)
    assert np.array_equal(back, coeffs)


def test_verify_fri_on_device_transcript(ctx):
    """End to end at 2^20: GPU commit + GPU decommitment gather verify."""
    import fri_amd
    log_n = 20
    coeffs = np.array(__import__("fri_oracle").splitmix64_field(11, 1 << 17), dtype=np.uint64)
    ch = fri_amd.Channel()
    proof = fri_amd.fri_commit(coeffs, log_n, ch, ctx=ctx)
    fri_amd.decommit_fri(8, (1 << log_n) - 1, proof, ch)
    assert fri_amd.verify_fri(ch.proof, log_n, proof.n_layers, 8, (1 << log_n) - 1)
    bad = list(ch.proof)
    bad[-3] = bytes([bad[-3][0] ^ 1]) + bad[-3][1:]          # a sibling value of the last query
    assert not fri_amd.verify_fri(bad, log_n, proof.n_layers, 8, (1 << log_n) - 1)


def test_concurrent_contexts_match_oracle(corc, oracle):
    """Serving pattern (INTEGRATION.md "Threading and serving"): one context
    per host thread on one GPU, commits in flight together, every transcript
    bit-exact against the C oracle."""
    import threading

    import fri_amd
    log_n, C, reps = 18, 3, 4
    d = (1 << log_n) // 8
    polys = [np.array(oracle.splitmix64_field(900 + c, d), dtype=np.uint64) for c in range(C)]
    want = []
    for p in polys:
        cs, pc = c_u64(p)
        och = oracle.OrcChannel()
        corc.orc_channel_init(ctypes.byref(och))
        ores = oracle.OrcFriResult()
        assert corc.orc_fri_commit_fast(pc, d, log_n, 5, 5, P, ctypes.byref(och), None, ctypes.byref(ores),
                                        None, None) == 0
        want.append(([bytes(ores.roots[k]) for k in range(ores.n_layers)],
                     [int(ores.betas[k]) for k in range(ores.n_rounds)], int(ores.final_value)))
    ctxs = [fri_amd.Context(0, log_n) for _ in range(C)]
    got = [[] for _ in range(C)]

    def run(c):
        for _ in range(reps):
            got[c].append(ctxs[c].commit(polys[c], log_n))

    th = [threading.Thread(target=run, args=(c,)) for c in range(C)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in range(C):
        assert len(got[c]) == reps
        for r in got[c]:
            assert ([bytes(r.roots[k]) for k in range(r.n_layers)], [int(r.betas[k]) for k in range(r.n_rounds)],
                    int(r.final_value)) == want[c]
        ctxs[c].close()
