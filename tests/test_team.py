"""Single-process multi-GPU context (fri_ctx_create_multi, include/fri_amd.h):
ONE call of fri_commit (src/fri/fri_commit.rs:72-76) commits a codeword
coset-sharded over a team of ranks driven from this one host thread.

On the 1-GPU box every rank sits on GPU 0 and the team uses the peer
transport (device copies between the ranks' buffers, ordered by events), the
same kernels and schedule as on G devices; only the xGMI reads become local
ones.  Every transcript is compared with the C oracle's (bit-exact), every
read-back of a sharded layer with a 1-GPU commit of the same polynomial, and
every rank's transport log with the deadlock-freedom condition of DESIGN.md §7."""
import ctypes
import hashlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _transcript(res):
    return {"roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)],
            "betas": [int(res.betas[r]) for r in range(res.n_rounds)],
            "final_value": int(res.final_value), "final_degree": int(res.final_degree),
            "state": bytes(res.channel_out.digest).hex()}


def _coeffs(oracle, seed, log_n, blowup_log=3):
    return oracle.splitmix64_np(seed, (1 << log_n) >> blowup_log).astype(np.uint32)


@pytest.fixture(scope="module")
def team4():
    import fri_amd
    c = fri_amd.Context.multi([0, 0, 0, 0], 23, transport="peer")
    yield c
    c.close()


@pytest.fixture(scope="module")
def one24():
    import fri_amd
    c = fri_amd.Context(0, 24)
    yield c
    c.close()


def test_team_info_and_selftest(team4):
    assert team4.dist_info() == (0, 4, "peer")
    for r in range(4):
        assert team4.team_rank(r).dist_info() == (r, 4, "peer")
    team4.dist_selftest(4096)
    for r in range(4):
        ops = [op for _, op, _, _ in team4.team_rank(r).transport_log()]
        assert ops == ["alltoall", "allgather", "sendrecv"]


@pytest.mark.parametrize("log_n,seed", [(20, 5), (22, 42), (23, 7)])
def test_team4_commit_matches_oracle(team4, oracle, oracle_commit, log_n, seed):
    """fri_commit on the team context: the whole transcript equals the C
    oracle's (one call; ranks 1-3 on the context's worker threads)."""
    from test_dist import check_transport_schedule
    res = team4.commit(_coeffs(oracle, seed, log_n), log_n)
    assert _transcript(res) == oracle_commit(log_n, seed)
    logs = [team4.team_rank(r).transport_log() for r in range(4)]
    check_transport_schedule(logs)
    assert sum(1 for e in logs[0] if e[1] == "alltoall") == 1


@pytest.mark.parametrize("G,log_n", [(2, 21), (8, 24)])
def test_team_sizes_match_oracle(oracle, oracle_commit, G, log_n):
    """G = 2 (radix-2 layer 0, no all-to-all) and G = 8 (a shard-sized 2^21
    rank context), on one GPU over the peer transport."""
    import fri_amd
    cx = fri_amd.Context.multi([0] * G, log_n, transport="peer")
    try:
        for seed in (42, 43):
            assert _transcript(cx.commit(_coeffs(oracle, seed, log_n), log_n)) == oracle_commit(log_n, seed)
        # each rank holds about 1/G of the plan: rank 1's HBM well below the
        # 1-GPU plan's layers + trees + x^-1 tables (host-side layout)
        r1 = cx.team_rank(1).device_bytes()[1]
        full = fri_amd.plan_layout((1 << log_n) >> 3, log_n)["bytes"]
        assert r1 < full * (0.5 if G == 8 else 0.8), (r1, full)
    finally:
        cx.close()


def test_team_readbacks_equal_single_gpu(team4, one24, oracle):
    """Every read-back of the team commit (layers, tree levels below and
    above the block roots, authentication paths, whole decommitments) equals
    the 1-GPU commit's of the same polynomial."""
    L = 22
    cf = _coeffs(oracle, 99, L)
    r1 = one24.commit(cf, L)
    rt = team4.commit(cf, L)
    assert _transcript(rt) == _transcript(r1)
    n_layers = rt.n_layers
    for k in (0, 1, 2, 3, n_layers - 1):
        assert np.array_equal(team4.layer(k, L), one24.layer(k, L)), k
    for k in (0, 2):
        Lk = L - k
        for lvl in (0, 1, Lk - 3, Lk - 2, Lk - 1, Lk):
            assert team4.tree_level(k, lvl, L) == one24.tree_level(k, lvl, L), (k, lvl)
    for k, idx in ((0, 12345), (1, (1 << 21) - 1), (2, 777)):
        assert team4.auth_path(k, idx, L) == one24.auth_path(k, idx, L)
    for idx in (0, 31337, (1 << 22) - 5):
        assert team4.decommit_query(idx, n_layers, L) == one24.decommit_query(idx, n_layers, L)
    g, ln, nl = team4.commit_info()
    assert (ln, nl) == (L, n_layers)
    assert team4.commit_degrees() == one24.commit_degrees()


def test_team_python_mirror_unchanged(team4, one24, oracle, oracle_commit):
    """The reference-shaped surface (fri_amd.fri_commit / decommit_fri /
    verify_fri, the Python twin of the Rust shim in INTEGRATION.md) takes the
    team context unchanged: the commit's messages equal the C oracle's, and
    the whole transcript with two decommitments equals a 1-GPU context's."""
    import fri_amd
    L = 21
    coeffs = _coeffs(oracle, 3, L)
    chans = []
    for cx in (team4, one24):
        ch = fri_amd.Channel()
        proof = fri_amd.fri_commit(coeffs, L, ch, ctx=cx)
        assert ch.state == oracle_commit(L, 3)["state"]
        fri_amd.decommit_fri(2, (1 << L) - 1, proof, ch)
        assert fri_amd.verify_fri(ch.proof, L, proof.n_layers, 2, (1 << L) - 1)
        chans.append(ch)
    assert chans[0].proof == chans[1].proof and chans[0].state == chans[1].state


def test_team_small_codeword_runs_on_rank0(team4, oracle, oracle_commit):
    """A codeword below the sharding threshold (2^20) runs on rank 0 alone:
    the other ranks issue no collective, and the layers read back whole."""
    team4.commit(_coeffs(oracle, 8, 21), 21)
    before = team4.team_rank(1).transport_log()
    res = team4.commit(_coeffs(oracle, 11, 16), 16)
    assert _transcript(res) == oracle_commit(16, 11)
    assert team4.team_rank(1).transport_log() == before
    assert np.array_equal(team4.layer(0, 16), team4.lde(_coeffs(oracle, 11, 16), 16))


def test_team_errors_then_recovers(team4, oracle, oracle_commit):
    """A non-canonical coefficient fails the team commit with FRI_EINVAL on
    every rank (checked on the device), forced betas reach every rank, and the
    team commits correctly afterwards; the pipelined and attach calls are
    refused on a team context."""
    import fri_amd
    L = 21
    bad = _coeffs(oracle, 5, L)
    bad[1000] = fri_amd.P
    with pytest.raises(fri_amd.FriError) as e:
        team4.commit(bad, L)
    assert e.value.code == fri_amd.FRI_EINVAL
    assert team4.commit_info()[2] == 0
    betas = [(i * 7919 + 11) % fri_amd.P for i in range(fri_amd.MAX_ROUNDS)]
    r = team4.commit(_coeffs(oracle, 5, L), L, forced_betas=betas)
    one = fri_amd.Context(0, L)
    try:
        assert _transcript(r) == _transcript(one.commit(_coeffs(oracle, 5, L), L, forced_betas=betas))
    finally:
        one.close()
    assert _transcript(team4.commit(_coeffs(oracle, 5, L), L)) == oracle_commit(L, 5)
    with pytest.raises(fri_amd.FriError) as e:
        team4.commit_async(_coeffs(oracle, 5, L), L)
    assert e.value.code == fri_amd.FRI_EINVAL
    with pytest.raises(fri_amd.FriError) as e:
        team4.attach_loopback(0, 2)
    assert e.value.code == fri_amd.FRI_EINVAL
    with pytest.raises(fri_amd.FriError) as e:
        team4.detach()
    assert e.value.code == fri_amd.FRI_EINVAL


@pytest.mark.parametrize("rank,op", [(2, 0), (1, 3), (3, 7), (0, 5)])   # 8 collectives at 2^22 x 4
def test_team_rank_failure_does_not_block(team4, oracle, oracle_commit, rank, op):
    """One rank fails at its op-th collective (fri_debug_team_inject_failure,
    as a broken transfer would): the call returns FRI_ERCCL naming that rank
    and op instead of leaving the other ranks waiting at the rendezvous, every
    rank's streams are drained, and the next team commit is right."""
    import time

    import fri_amd
    L = 22
    cf = _coeffs(oracle, 17, L)
    team4.inject_team_failure(rank, op)
    t0 = time.time()
    with pytest.raises(fri_amd.FriError) as e:
        team4.commit(cf, L)
    assert e.value.code == fri_amd.FRI_ERCCL
    assert f"rank {rank}" in str(e.value) and "injected failure" in str(e.value), str(e.value)
    assert time.time() - t0 < 30
    assert _transcript(team4.commit(cf, L)) == oracle_commit(L, 17)


def test_team_commit_device_from_rank0_buffer(team4, oracle, oracle_commit):
    """fri_commit_device on the team: the context's input buffer (rank 0's
    device) is copied by rank 0 locally and by the other ranks over the
    transport.  FRI_FLAG_RANK_INPUTS then reuses the ranks' staged copies,
    verified against rank 0's buffer by a per-rank checksum: a buffer
    rewritten since the staging gives FRI_ESTATE on every rank and commits
    nothing, until a commit without the flag stages it again."""
    import fri_amd
    L = 22
    cf = _coeffs(oracle, 42, L)
    p = ctypes.c_void_p(team4.input_upload(cf))
    out = fri_amd.CommitResult()
    for _ in range(3):
        team4._check(team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None, 0, None,
                                                 ctypes.byref(out)))
        assert _transcript(out) == oracle_commit(L, 42)
    # FRI_FLAG_RANK_INPUTS: every rank reads its own resident copy
    for _ in range(2):
        team4._check(team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None,
                                                 fri_amd.FLAG_RANK_INPUTS, None, ctypes.byref(out)))
        assert _transcript(out) == oracle_commit(L, 42)
    # ... which needs rank 0's buffer and a staged copy of this shape
    for bad in ((p, cf.size // 2), (ctypes.c_void_p(p.value + 64), cf.size)):
        rc = team4.lib.fri_commit_device(team4.h, bad[0], bad[1], L, fri_amd.GENERATOR, None,
                                         fri_amd.FLAG_RANK_INPUTS, None, ctypes.byref(out))
        assert rc == fri_amd.FRI_ESTATE
    # rank 0's buffer rewritten with same-shape coefficients: refused, nothing committed
    g0 = team4.commit_info()[0]
    lay0 = team4.layer(0, L)
    cf2 = _coeffs(oracle, 43, L)
    assert team4.input_upload(cf2) == p.value
    rc = team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None, fri_amd.FLAG_RANK_INPUTS,
                                     None, ctypes.byref(out))
    assert rc == fri_amd.FRI_ESTATE, rc
    assert "differs from rank 0" in team4.lib.fri_last_error(team4.h).decode()
    assert team4.commit_info()[0] == g0                   # the resident commit is untouched
    assert np.array_equal(team4.layer(0, L), lay0)
    # one word changed is enough
    cf3 = cf2.copy()
    cf3[cf3.size // 3] ^= 1
    team4._check(team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None, 0, None,
                                             ctypes.byref(out)))                  # stages cf2
    assert _transcript(out) == oracle_commit(L, 43)
    team4.input_upload(cf3)
    rc = team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None, fri_amd.FLAG_RANK_INPUTS,
                                     None, ctypes.byref(out))
    assert rc == fri_amd.FRI_ESTATE
    team4.input_upload(cf2)
    team4._check(team4.lib.fri_commit_device(team4.h, p, cf.size, L, fri_amd.GENERATOR, None,
                                             fri_amd.FLAG_RANK_INPUTS, None, ctypes.byref(out)))
    assert _transcript(out) == oracle_commit(L, 43)


def test_team_input_in_place_and_tail_graph(team4, oracle, oracle_commit):
    """At 2^20 over 4 ranks the sharded part is layer 0 alone, so the local
    tail (one hipGraph per plan) folds the input coefficients itself: its
    graph names the input pointer.  Commits alternating between host input
    (staged in the plan's buffer) and rank 0's input buffer (read in place)
    re-capture it; every transcript equals the C oracle's."""
    import fri_amd
    L = 20
    cf, cg = _coeffs(oracle, 61, L), _coeffs(oracle, 62, L)
    p = ctypes.c_void_p(team4.input_upload(cg))
    out = fri_amd.CommitResult()
    for _ in range(2):
        assert _transcript(team4.commit(cf, L)) == oracle_commit(L, 61)
        team4._check(team4.lib.fri_commit_device(team4.h, p, cg.size, L, fri_amd.GENERATOR, None, 0, None,
                                                 ctypes.byref(out)))
        assert _transcript(out) == oracle_commit(L, 62)
    team4._check(team4.lib.fri_commit_device(team4.h, p, cg.size, L, fri_amd.GENERATOR, None,
                                             fri_amd.FLAG_RANK_INPUTS, None, ctypes.byref(out)))
    assert _transcript(out) == oracle_commit(L, 62)


def test_team_create_arguments():
    import fri_amd
    with pytest.raises(fri_amd.FriError):
        fri_amd.Context.multi([0, 0, 0], 22)                  # not a power of two
    with pytest.raises(fri_amd.FriError):
        fri_amd.Context.multi([0, 0], 22, transport="rccl")   # ranks share a device: RCCL cannot run them
    with pytest.raises(fri_amd.FriError):
        fri_amd.Context.multi([0, 99], 22)                    # no such device
    c = fri_amd.Context.multi([0], 16)                        # one device: an ordinary context
    try:
        assert c.dist_info()[2] == "none"
        with pytest.raises(fri_amd.FriError) as e:
            c.force_copy(True)                                # a test hook of teams only
        assert e.value.code == fri_amd.FRI_EINVAL
    finally:
        c.close()
    c = fri_amd.Context.multi([0, 0], 21)                     # the default transport is the peer transport
    try:
        assert c.dist_info() == (0, 2, "peer")
    finally:
        c.close()


def test_default_context_follows_fri_devices(monkeypatch, oracle, oracle_commit):
    """fri_ctx_create_default (what the reference-signature bindings open):
    FRI_DEVICES names the ranks ("0,0" -> a two-rank team on GPU 0), unset it
    is every visible GPU (one here: an ordinary context); a malformed value is
    FRI_EINVAL.  The Python mirror's fri_commit without ctx uses it."""
    import fri_amd
    monkeypatch.setenv("FRI_DEVICES", "0,0")
    c = fri_amd.Context.default(21)
    try:
        assert c.n_ranks == 2 and c.dist_info() == (0, 2, "peer")
        assert _transcript(c.commit(_coeffs(oracle, 6, 21), 21)) == oracle_commit(21, 6)
    finally:
        c.close()
    for bad in ("0,0,0", "x", "0,,0"):
        monkeypatch.setenv("FRI_DEVICES", bad)
        with pytest.raises(fri_amd.FriError) as e:
            fri_amd.Context.default(20)
        assert e.value.code == fri_amd.FRI_EINVAL
    monkeypatch.setenv("FRI_DEVICES", "0,0")
    monkeypatch.setenv("FRI_TRANSPORT", "carrier-pigeon")
    with pytest.raises(fri_amd.FriError):
        fri_amd.Context.default(20)
    monkeypatch.delenv("FRI_TRANSPORT")
    monkeypatch.delenv("FRI_DEVICES")
    c = fri_amd.Context.default(16)
    try:
        assert c.n_ranks >= 1 and c.dist_info()[2] == "none"
    finally:
        c.close()


def test_reference_decommit_signature_on_team(team4, oracle):
    """decommit_fri(num_queries, max_index, &fri_layers, &fri_merkles,
    &mut channel) (fri_commit.rs:168-174), Python mirror, on a team commit:
    the same messages as the proof form; layers of another commit and a stale
    proof are refused."""
    import fri_amd
    L = 21
    coeffs = _coeffs(oracle, 31, L)
    ch_a = fri_amd.Channel()
    proof = fri_amd.fri_commit(coeffs, L, ch_a, ctx=team4)
    ch_b = fri_amd.Channel(state=ch_a.state, proof=list(ch_a.proof))
    layers, merkles = proof.fri_layers, proof.fri_merkles
    fri_amd.decommit_fri(2, (1 << L) - 1, layers, merkles, ch_a)
    fri_amd.decommit_fri(2, (1 << L) - 1, proof, ch_b)
    assert ch_a.proof == ch_b.proof and ch_a.state == ch_b.state
    assert merkles[3].get_authentication_path(5) == b"".join(team4.auth_path(3, 5, L)[1])
    wrong = [l.copy() for l in layers]
    wrong[2] = (wrong[2] + 1) % fri_amd.P
    with pytest.raises(fri_amd.FriError):
        fri_amd.decommit_fri(3, (1 << L) - 1, wrong, merkles, fri_amd.Channel(state=ch_a.state))
    fri_amd.fri_commit(_coeffs(oracle, 32, L), L, fri_amd.Channel(), ctx=team4)
    with pytest.raises(fri_amd.FriError) as e:
        fri_amd.decommit_fri(1, (1 << L) - 1, layers, merkles, fri_amd.Channel(state=ch_a.state))
    assert e.value.code == fri_amd.FRI_ESTATE


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("copy", [False, True], ids=["pull", "copy"])
def test_team_2p28_world8_configs4(oracle_commit, copy):
    """BASELINE configs[4]: the 2^28 codeword committed coset-sharded over 8
    ranks by ONE fri_commit call on a team context (peer transport, every
    rank on GPU 0: 8 shard-sized plans, ~50 GB), bit-exact against the C
    oracle; every decommitment layer checks against its root."""
    import fri_amd
    import fri_oracle as fo
    L = 28
    cf = fo.splitmix64_np(42, (1 << L) >> 3).astype(np.uint32)
    cx = fri_amd.Context.multi([0] * 8, L, transport="peer")
    try:
        cx.force_copy(copy)          # copy: hipMemcpyPeerAsync per source (the no-peer-access path)
        res = cx.commit(cf, L)
        want = oracle_commit(L, 42)
        assert _transcript(res) == want
        q = cx.decommit_query(123456789, res.n_layers, L)
        for k, (v, sv, path, spath) in enumerate(q):
            m = 1 << (L - k)
            i = 123456789 % m
            h = hashlib.sha256(int(v).to_bytes(8, "big")).digest()
            for lvl in range(L - k):
                sib = path[32 * lvl:32 * lvl + 32]
                h = hashlib.sha256(sib + h if (i >> lvl) & 1 else h + sib).digest()
            assert h.hex() == want["roots"][k], k
    finally:
        cx.close()


_TF = int(os.environ.get("TEAM_FUZZ_N", "0"))      # > 0: that many cases per team size (longer runs)


@pytest.mark.parametrize("copy", [False, True], ids=["pull", "copy"])
@pytest.mark.parametrize("G,n_cases", [(2, _TF or 8), (4, _TF or 8), (8, _TF or 6)])
def test_team_fuzz_vs_c_oracle(G, n_cases, corc, oracle, copy):
    """Randomised team commits (the sharded fuzz's cases, dist_worker.fuzz_case:
    2^20..2^22, ragged coefficient counts including 0, blowups 1..16, degrees
    that end inside the sharded layers, zero / constant / odd-only polynomials,
    random cosets, prefilled channels, forced betas on every third case) on a
    team of G ranks on GPU 0 (peer transport), one fri_commit call each:
    the whole transcript equals the OpenMP C oracle's 1-node commit
    (orc_fri_commit_fast, src/fri/fri_commit.rs:72-122), and the ranks'
    transport logs pass the cross-rank schedule check.  Run twice: over the pull
kernel and over the hipMemcpyPeerAsync fallback a team takes where peer
access is unavailable (fri_debug_team_force_copy)."""
    import fri_amd
    from dist_worker import fuzz_case, fuzz_forced_betas
    from test_dist import check_transport_schedule
    seed = 1000 * G + 7 + (500 if copy else 0)
    cx = fri_amd.Context.multi([0] * G, 22, transport="peer")
    try:
        cx.force_copy(copy)
        for i in range(n_cases):
            log_n, c, offset, state = fuzz_case(seed + i, G)
            fb = fuzz_forced_betas(seed + i)
            res = cx.commit(np.asarray(c, dtype=np.uint32), log_n, offset=offset, channel_state=state,
                            forced_betas=fb)
            fbp = None
            if fb is not None:
                fba = np.ascontiguousarray(np.array(fb, dtype=np.uint64))
                fbp = fba.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
            cs = np.ascontiguousarray(c, dtype=np.uint64)
            och = oracle.OrcChannel()
            corc.orc_channel_init(ctypes.byref(och))
            if state is not None:
                och.state = state.hex().encode()
                och.state_len = 64
            ores = oracle.OrcFriResult()
            assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, log_n,
                                            offset, 5, oracle.P, ctypes.byref(och), fbp, ctypes.byref(ores), None,
                                            None) == 0
            what = (f"case {seed + i}: G={G} log_n={log_n} d={c.size} offset={offset} "
                    f"prefilled={state is not None} forced={fb is not None}")
            want = {"roots": [bytes(ores.roots[k]).hex() for k in range(ores.n_layers)],
                    "betas": [int(ores.betas[j]) for j in range(ores.n_rounds)],
                    "final_value": int(ores.final_value), "final_degree": int(ores.final_degree),
                    "state": och.state.decode()}
            assert _transcript(res) == want, what
            if log_n >= 20:
                check_transport_schedule([cx.team_rank(r).transport_log() for r in range(G)])
    finally:
        cx.close()
