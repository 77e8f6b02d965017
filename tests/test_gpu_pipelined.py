"""Pipelined commits (fri_commit_device_async / fri_commit_wait): several
commits of device-resident coefficients pending on one context, run back to
back on its stream.  Each result must equal the C oracle's transcript of the
same polynomial (fri_commit, src/fri/fri_commit.rs:72-122), whatever the
order the tickets are collected in; read-backs serve the last enqueued commit;
the limits and errors are those of include/fri_amd.h."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOG_N = 16


def _dev(torch, coeffs_u32):
    """A device copy of the coefficients, through the library's own HIP
    runtime (fri_amd.DeviceBuffer; `torch` is unused, kept for the call sites)."""
    import fri_amd
    return fri_amd.DeviceBuffer(coeffs_u32)


def _transcript(res):
    return {"roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)],
            "betas": [int(res.betas[r]) for r in range(res.n_rounds)],
            "final_value": int(res.final_value), "final_degree": int(res.final_degree),
            "state": bytes(res.channel_out.digest).hex()}


@pytest.fixture(scope="module")
def torch():
    """(Formerly torch, for device buffers; the buffers now come from the
    library's own HIP runtime: fri_amd.DeviceBuffer.)"""
    return None


@pytest.fixture()
def pctx():
    import fri_amd
    c = fri_amd.Context(0, LOG_N)
    yield c
    c.close()


def _polys(oracle, torch, seeds, log_n=LOG_N):
    d = (1 << log_n) >> 3
    return [(s, _dev(torch, oracle.splitmix64_np(s, d).astype(np.uint32))) for s in seeds]


def test_pipelined_results_match_oracle_any_order(pctx, oracle, oracle_commit, torch):
    import fri_amd
    d = (1 << LOG_N) >> 3
    polys = _polys(oracle, torch, [901, 902, 903, 904])
    tickets = [pctx.commit_device_async(buf.data_ptr(), d, LOG_N) for _, buf in polys]
    assert len(set(tickets)) == fri_amd.MAX_INFLIGHT
    for i in (2, 0, 3, 1):                                   # collected out of order
        assert _transcript(pctx.commit_wait(tickets[i])) == oracle_commit(LOG_N, polys[i][0])
    # the slots are free again: a second round through the same graphs
    tickets = [pctx.commit_device_async(buf.data_ptr(), d, LOG_N) for _, buf in polys[::-1]]
    for t, (seed, _) in zip(tickets, polys[::-1]):
        assert _transcript(pctx.commit_wait(t)) == oracle_commit(LOG_N, seed)


def test_pipelined_readbacks_serve_the_last_commit(pctx, oracle, oracle_commit, torch):
    import hashlib
    d = (1 << LOG_N) >> 3
    polys = _polys(oracle, torch, [911, 912, 913])
    g0 = pctx.commit_info()[0]
    tickets = [pctx.commit_device_async(buf.data_ptr(), d, LOG_N) for _, buf in polys]
    # before any wait: the read-backs wait for the stream and see the third commit
    gen, log_n, n_layers = pctx.commit_info()
    assert gen == g0 + 3 and log_n == LOG_N and n_layers == LOG_N - 2
    last = oracle_commit(LOG_N, 913)
    for k in (0, 5):
        val, path = pctx.auth_path(k, 3, LOG_N)
        h = hashlib.sha256(int(val).to_bytes(8, "big")).digest()
        i = 3
        for sib in path:
            h = hashlib.sha256(h + sib if i % 2 == 0 else sib + h).digest()
            i //= 2
        assert h.hex() == last["roots"][k]
    for t, (seed, _) in zip(tickets, polys):
        assert _transcript(pctx.commit_wait(t)) == oracle_commit(LOG_N, seed)


def test_pipelined_limits_and_errors(pctx, oracle, oracle_commit, torch):
    import fri_amd
    d = (1 << LOG_N) >> 3
    (seed, buf), = _polys(oracle, torch, [921])
    tickets = [pctx.commit_device_async(buf.data_ptr(), d, LOG_N) for _ in range(fri_amd.MAX_INFLIGHT)]
    with pytest.raises(fri_amd.FriError) as e:               # FRI_MAX_INFLIGHT pending
        pctx.commit_device_async(buf.data_ptr(), d, LOG_N)
    assert e.value.code == fri_amd.FRI_ESTATE
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_wait(max(tickets) + 1)                   # never issued
    assert e.value.code == fri_amd.FRI_EINVAL
    for t in tickets:
        assert _transcript(pctx.commit_wait(t)) == oracle_commit(LOG_N, seed)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_wait(tickets[0])                         # already collected
    assert e.value.code == fri_amd.FRI_EINVAL
    pctx.set_profiling(True)
    try:
        with pytest.raises(fri_amd.FriError) as e:
            pctx.commit_device_async(buf.data_ptr(), d, LOG_N)
        assert e.value.code == fri_amd.FRI_ESTATE
    finally:
        pctx.set_profiling(False)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_device_async(buf.data_ptr(), (1 << LOG_N) + 1, LOG_N)   # d > n
    assert e.value.code == fri_amd.FRI_EDEGREE


def test_pipelined_noncanonical_input(pctx, oracle, oracle_commit, torch):
    """A coefficient >= p fails that commit alone (FRI_EINVAL at its wait);
    the commits before and after it in the pipeline are unaffected."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    good = oracle.splitmix64_np(931, d).astype(np.uint32)
    bad = good.copy()
    bad[d // 3] = 0xFFFFFFFF
    gb, bb = _dev(torch, good), _dev(torch, bad)
    t0 = pctx.commit_device_async(gb.data_ptr(), d, LOG_N)
    t1 = pctx.commit_device_async(bb.data_ptr(), d, LOG_N)
    assert pctx.commit_info()[2] == 0                        # the resident (last) commit failed
    t2 = pctx.commit_device_async(gb.data_ptr(), d, LOG_N)
    assert _transcript(pctx.commit_wait(t0)) == oracle_commit(LOG_N, 931)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_wait(t1)
    assert e.value.code == fri_amd.FRI_EINVAL
    assert _transcript(pctx.commit_wait(t2)) == oracle_commit(LOG_N, 931)
    assert pctx.commit_info()[2] == LOG_N - 2


def test_pipelined_with_plan_change_and_sync_commits(pctx, oracle, oracle_commit, torch):
    """A commit with another (d, log_n) waits for the pending ones (their
    results stay collectable); a synchronous commit in between too."""
    d16 = (1 << LOG_N) >> 3
    (s1, b1), (s2, b2) = _polys(oracle, torch, [941, 942])
    (s3, b3), = _polys(oracle, torch, [943], log_n=14)
    t1 = pctx.commit_device_async(b1.data_ptr(), d16, LOG_N)
    t2 = pctx.commit_device_async(b2.data_ptr(), d16, LOG_N)
    t3 = pctx.commit_device_async(b3.data_ptr(), (1 << 14) >> 3, 14)      # new plan
    sync = pctx.commit(oracle.splitmix64_np(944, d16).astype(np.uint32), LOG_N)
    assert _transcript(sync) == oracle_commit(LOG_N, 944)
    assert _transcript(pctx.commit_wait(t3)) == oracle_commit(14, s3)
    assert _transcript(pctx.commit_wait(t1)) == oracle_commit(LOG_N, s1)
    assert _transcript(pctx.commit_wait(t2)) == oracle_commit(LOG_N, s2)
    assert pctx.commit_info()[1:] == (LOG_N, LOG_N - 2)      # the sync commit is resident


def test_pipelined_channel_state_and_eager_flag(pctx, oracle, corc, torch):
    """A channel state carried in (fri_commit's &mut Channel after earlier
    sends) and the eager (no-graph) flag go through the pipelined entry point
    too: each transcript equals the C oracle's from the same channel state."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    c = oracle.splitmix64_np(951, d).astype(np.uint32)
    buf = _dev(torch, c)
    state = bytes(range(32))
    och = oracle.OrcChannel()                              # the C oracle's channel, state as hex
    corc.orc_channel_init(ctypes.byref(och))
    och.state = state.hex().encode()
    och.state_len = 64
    cs = np.ascontiguousarray(c.astype(np.uint64))
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, LOG_N, 5, 5,
                                    oracle.P, ctypes.byref(och), None, ctypes.byref(ores), None, None) == 0
    want = {"roots": [bytes(ores.roots[k]).hex() for k in range(ores.n_layers)],
            "betas": [int(ores.betas[r]) for r in range(ores.n_rounds)],
            "final_value": int(ores.final_value), "final_degree": int(ores.final_degree),
            "state": och.state.decode()}
    assert _transcript(pctx.commit(c, LOG_N, channel_state=state)) == want
    t0 = pctx.commit_device_async(buf.data_ptr(), d, LOG_N, channel_state=state)
    ch = fri_amd.ChannelState()
    ctypes.memmove(ch.digest, state, 32)
    ch.has_state = 1
    t1 = ctypes.c_uint64()
    pctx._check(pctx.lib.fri_commit_device_async(pctx.h, buf.data_ptr(), d, LOG_N, fri_amd.GENERATOR,
                                                 ctypes.byref(ch), fri_amd.FLAG_NO_GRAPH, None, ctypes.byref(t1)))
    assert _transcript(pctx.commit_wait(t1.value)) == want
    assert _transcript(pctx.commit_wait(t0)) == want


def test_pipelined_then_sharded_on_one_context(oracle, oracle_commit, torch):
    """Pending pipelined commits and a sharded commit (loopback rehearsal
    transport, world 1 would not shard: world 2) on the same context: the
    sharded plan waits for the pending commits, whose results stay
    collectable; a 1-GPU pipelined commit afterwards is exact again."""
    import fri_amd
    log_n = 21
    d = (1 << log_n) >> 3
    cx = fri_amd.Context(0, log_n)
    try:
        c = oracle.splitmix64_np(961, d).astype(np.uint32)
        buf = _dev(torch, c)
        t = [cx.commit_device_async(buf.data_ptr(), d, log_n) for _ in range(2)]
        cx.attach_loopback(0, 2)
        cx.commit_sharded(c, log_n)          # loopback: not the real transcript, only the plan switch
        cx.detach()
        for ti in t:
            assert _transcript(cx.commit_wait(ti)) == oracle_commit(log_n, 961)
        t2 = cx.commit_device_async(buf.data_ptr(), d, log_n)
        assert _transcript(cx.commit_wait(t2)) == oracle_commit(log_n, 961)
    finally:
        cx.close()


def test_pipelined_host_input(pctx, oracle, oracle_commit):
    """fri_commit_async: host coefficients are copied before the call
    returns, so one host buffer can be refilled for the next commit while the
    earlier ones are still pending; every transcript equals the oracle's."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    buf = np.empty(d, dtype=np.uint32)
    seeds = [971, 972, 973, 974]
    tickets = []
    for s in seeds:
        buf[:] = oracle.splitmix64_np(s, d).astype(np.uint32)
        tickets.append(pctx.commit_async(buf, LOG_N))
    buf[:] = 0                                               # the pending commits do not see this
    for t, s in zip(tickets, seeds):
        assert _transcript(pctx.commit_wait(t)) == oracle_commit(LOG_N, s)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_async(np.zeros((1 << LOG_N) + 1, dtype=np.uint32), LOG_N)    # d > n
    assert e.value.code == fri_amd.FRI_EDEGREE
    bad = oracle.splitmix64_np(975, d).astype(np.uint32)
    bad[7] = P_BAD
    t = pctx.commit_async(bad, LOG_N)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.commit_wait(t)
    assert e.value.code == fri_amd.FRI_EINVAL


P_BAD = 3221225473                                           # p itself: not canonical


def test_python_mirror_pipelined_matches_golden(golden, oracle):
    """fri_amd.fri_commit_pipelined over the golden cases grouped by
    (log_n, offset): every proof and channel equals the golden transcript;
    only the last proof of a group serves read-backs, and its decommitment
    (decommit_fri, fri_commit.rs:168-179) equals the golden one."""
    import fri_amd
    groups = {}
    for c in golden["cases"]:
        if not c["forced_betas"]:
            groups.setdefault((c["log_n"], c["offset"]), []).append(c)
    checked = 0
    for (log_n, offset), cases in groups.items():
        if len(cases) < 2:
            continue
        cx = fri_amd.Context(0, max(log_n, 10))
        try:
            chans = []
            for c in cases:
                ch = fri_amd.Channel()
                ch.state = c["channel_in"]
                chans.append(ch)
            proofs = fri_amd.fri_commit_pipelined([c["coeffs"] for c in cases], log_n, chans, offset, ctx=cx)
            for i, (c, pr, ch) in enumerate(zip(cases, proofs, chans)):
                assert [r.hex() for r in pr.roots] == c["roots"]
                assert pr.betas == c["betas"]
                assert ch.state == c["channel_out"] and ch.proof_size() == c["proof_size"]
                if i + 1 < len(cases):
                    with pytest.raises(fri_amd.FriError):
                        pr.layer(0)                                  # replaced by a later commit
                checked += 1
            last, ch = cases[-1], chans[-1]
            n0 = len(ch.proof)
            fri_amd.decommit_fri(3, (1 << log_n) - 1, proofs[-1], ch)
            assert ch.state == last["decommit_q3"]["state"]
        finally:
            cx.close()
    assert checked >= 4


def test_python_mirror_pipelined_over_contexts(oracle, oracle_commit):
    """Several contexts driven from one host thread (commits dealt
    round-robin, concurrent on their streams): every transcript equals the
    oracle's, and on each context only its last proof is resident."""
    import fri_amd
    log_n = 16
    d = (1 << log_n) >> 3
    seeds = list(range(981, 988))
    ctxs = [fri_amd.Context(0, log_n) for _ in range(3)]
    try:
        chans = [fri_amd.Channel() for _ in seeds]
        proofs = fri_amd.fri_commit_pipelined([oracle.splitmix64_np(s, d).astype(np.uint32) for s in seeds],
                                              log_n, chans, ctx=ctxs)
        for s, pr, ch in zip(seeds, proofs, chans):
            want = oracle_commit(log_n, s)
            assert [r.hex() for r in pr.roots] == want["roots"] and pr.betas == want["betas"]
            assert ch.state == want["state"]
        for i, pr in enumerate(proofs):
            last_on_ctx = i + len(ctxs) >= len(proofs)
            if last_on_ctx:
                assert pr.layer(1).size == 1 << (log_n - 1)
            else:
                with pytest.raises(fri_amd.FriError):
                    pr.layer(0)
    finally:
        for c in ctxs:
            c.close()


def test_commit_lanes(pctx, oracle, oracle_commit, torch):
    """Commit lanes (fri_ctx_set_lanes): a pending commit runs on the lane
    with the fewest pending commits, a stream with its own plan.  With 1..4 lanes every
    transcript equals the oracle's; each lane in use holds one plan of HBM;
    the limits of include/fri_amd.h hold."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    polys = _polys(oracle, torch, [1001, 1002, 1003, 1004, 1005, 1006])
    want = {s: oracle_commit(LOG_N, s) for s, _ in polys}
    pctx.commit(oracle.splitmix64_np(1001, d).astype(np.uint32), LOG_N)      # lane 0's plan
    one_plan = pctx.device_bytes()[0]
    for lanes in (1, 2, 3, 4):
        pctx.set_lanes(lanes)
        pend = []
        for i, (s, buf) in enumerate(polys):
            pend.append((s, pctx.commit_device_async(buf.data_ptr(), d, LOG_N)))
            if len(pend) == lanes + 1 or len(pend) == fri_amd.MAX_INFLIGHT:
                s0, t = pend.pop(0)
                assert _transcript(pctx.commit_wait(t)) == want[s0], (lanes, s0)
        for s0, t in pend:
            assert _transcript(pctx.commit_wait(t)) == want[s0], (lanes, s0)
        # read-backs serve the last commit, whichever lane it ran on
        assert pctx.commit_info()[2] == LOG_N - 2
        assert bytes(pctx.tree_level(0, LOG_N, LOG_N)[0]).hex() == want[polys[-1][0]]["roots"][0]
    cur = pctx.device_bytes()[0]
    assert cur > 3 * one_plan // 2, (cur, one_plan)          # several lanes' plans are resident
    for bad in (0, fri_amd.MAX_INFLIGHT + 1):
        with pytest.raises(fri_amd.FriError) as e:
            pctx.set_lanes(bad)
        assert e.value.code == fri_amd.FRI_EINVAL
    t = pctx.commit_device_async(polys[0][1].data_ptr(), d, LOG_N)
    with pytest.raises(fri_amd.FriError) as e:
        pctx.set_lanes(2)                                    # commits pending
    assert e.value.code == fri_amd.FRI_ESTATE
    assert _transcript(pctx.commit_wait(t)) == want[polys[0][0]]


def test_lanes_sync_commit_and_input_buffer(pctx, oracle, oracle_commit, torch):
    """A synchronous commit runs on lane 0 while a pipelined commit is still
    pending on lane 1; both transcripts are right and the read-backs then
    serve the synchronous one.  The context's input buffer keeps its pointer,
    holds what the caller uploaded whatever is committed in between, and
    pipelined commits on every lane read it in place."""
    d = (1 << LOG_N) >> 3
    (s1, b1), (s2, b2) = _polys(oracle, torch, [1011, 1012])
    c3 = oracle.splitmix64_np(1013, d).astype(np.uint32)
    pctx.set_lanes(4)
    p0 = pctx.input_upload(c3)                                       # the caller's buffer holds c3
    t1 = pctx.commit_device_async(b1.data_ptr(), d, LOG_N)          # lane 0
    t2 = pctx.commit_device_async(b2.data_ptr(), d, LOG_N)          # lane 1
    assert _transcript(pctx.commit_wait(t1)) == oracle_commit(LOG_N, s1)
    sync = pctx.commit(c3, LOG_N)                                    # lane 0, beside lane 1's pending commit
    assert _transcript(sync) == oracle_commit(LOG_N, 1013)
    assert _transcript(pctx.commit_wait(t2)) == oracle_commit(LOG_N, s2)
    assert pctx.layer(2, LOG_N).size == 1 << (LOG_N - 2)
    val, _ = pctx.auth_path(0, 5, LOG_N)
    assert int(val) == int(pctx.lde(c3[:d], LOG_N)[5])               # the sync commit's layer 0
    assert pctx.input_buffer(d) == p0
    ta = pctx.commit_device_async(b1.data_ptr(), d, LOG_N)          # another pointer: staged privately
    pctx.commit_wait(ta)
    pctx.commit(oracle.splitmix64_np(1014, d).astype(np.uint32), LOG_N)   # host input: staged privately
    ts = [pctx.commit_device_async(p0, d, LOG_N) for _ in range(4)]       # lanes 0-3 read the buffer in place
    for t in ts:
        assert _transcript(pctx.commit_wait(t)) == oracle_commit(LOG_N, 1013)


@pytest.mark.parametrize("log_n,lanes", [(LOG_N, 3), (20, 3), (LOG_N, 1)])
def test_input_buffer_independent_of_lane_deal(oracle, oracle_commit, torch, log_n, lanes):
    """The input buffer belongs to the caller (fri_commit.rs:72-76: the
    caller owns poly): with four commits pending, commits from it are mixed
    with commits from other device buffers and from host coefficients (which
    the library stages privately), dealt to whichever lane; every commit from
    the buffer commits what the caller last uploaded there, and an upload
    (fri_ctx_input_upload) waits for the pending commits that still read the
    old contents.  Every transcript equals the C oracle's."""
    import fri_amd
    d = (1 << log_n) >> 3
    seeds_dev, seeds_host, seeds_buf = [1301, 1302], [1303, 1304], [1305, 1306, 1307]
    devs = {s: _dev(torch, oracle.splitmix64_np(s, d).astype(np.uint32)) for s in seeds_dev}
    host = {s: oracle.splitmix64_np(s, d).astype(np.uint32) for s in seeds_host}
    cx = fri_amd.Context(0, log_n)
    try:
        cx.set_lanes(lanes)
        p0 = cx.input_upload(oracle.splitmix64_np(seeds_buf[0], d).astype(np.uint32))
        in_buf = seeds_buf[0]
        pend, checked, uploads = [], 0, 0
        rng = np.random.default_rng(log_n * 10 + lanes)
        for i in range(40):
            if len(pend) == fri_amd.MAX_INFLIGHT:
                s0, t0 = pend.pop(0)
                assert _transcript(cx.commit_wait(t0)) == oracle_commit(log_n, s0), (i, s0)
                checked += 1
            k = i % 5 if i < 20 else int(rng.integers(0, 5))
            if k in (0, 3):                                          # the caller's buffer, read in place
                pend.append((in_buf, cx.commit_device_async(p0, d, log_n)))
            elif k == 1:                                             # another device buffer
                s = seeds_dev[i % 2]
                pend.append((s, cx.commit_device_async(devs[s].data_ptr(), d, log_n)))
            elif k == 2:                                             # host coefficients
                s = seeds_host[i % 2]
                pend.append((s, cx.commit_async(host[s], log_n)))
            else:                                                    # new contents, while commits of the old pend
                in_buf = seeds_buf[(seeds_buf.index(in_buf) + 1) % len(seeds_buf)]
                assert cx.input_upload(oracle.splitmix64_np(in_buf, d).astype(np.uint32)) == p0
                uploads += 1
        for s0, t0 in pend:
            assert _transcript(cx.commit_wait(t0)) == oracle_commit(log_n, s0), s0
            checked += 1
        assert uploads >= 4 and checked >= 20 and checked + uploads == 40
        # a synchronous commit from the buffer, and one from the host: neither changes it
        assert _transcript(cx.commit(host[seeds_host[0]], log_n)) == oracle_commit(log_n, seeds_host[0])
        res = fri_amd.CommitResult()
        cx._check(cx.lib.fri_commit_device(cx.h, p0, d, log_n, fri_amd.GENERATOR, None, 0, None, ctypes.byref(res)))
        assert _transcript(res) == oracle_commit(log_n, in_buf)
    finally:
        cx.close()


def test_input_buffer_grows_and_keeps_contents(oracle, oracle_commit):
    """fri_ctx_input_buffer with a larger d moves the buffer (contents kept);
    commits from the new pointer re-capture their graphs, and no commit needs
    a plan before the buffer exists."""
    import fri_amd
    cx = fri_amd.Context(0, 18)
    try:
        d14, d16 = (1 << 14) >> 3, (1 << 16) >> 3
        c14 = oracle.splitmix64_np(1401, d14).astype(np.uint32)
        p14 = cx.input_upload(c14)                                   # before any commit on the context
        res = fri_amd.CommitResult()
        cx._check(cx.lib.fri_commit_device(cx.h, p14, d14, 14, fri_amd.GENERATOR, None, 0, None, ctypes.byref(res)))
        assert _transcript(res) == oracle_commit(14, 1401)
        p16 = cx.input_buffer(d16)                                   # larger: moved, first d14 words kept
        cx._check(cx.lib.fri_commit_device(cx.h, p16, d14, 14, fri_amd.GENERATOR, None, 0, None, ctypes.byref(res)))
        assert _transcript(res) == oracle_commit(14, 1401)
        cx.input_upload(oracle.splitmix64_np(1601, d16).astype(np.uint32))
        t = cx.commit_device_async(p16, d16, 16)
        assert _transcript(cx.commit_wait(t)) == oracle_commit(16, 1601)
        assert cx.input_buffer(d14) == p16                           # smaller: the same buffer
        with pytest.raises(fri_amd.FriError) as e:
            cx.input_buffer((1 << 18) + 1)                           # beyond the context's codeword bound
        assert e.value.code == fri_amd.FRI_EINVAL
    finally:
        cx.close()


def test_lanes_balanced_at_depth_four(pctx, oracle, oracle_commit, torch):
    """Four commits pending on three lanes: each new commit goes to the lane
    with the fewest pending commits (ties: the lane dealt a commit longest
    ago), so no lane holds two while another holds none, and the lanes rotate
    instead of lane 0 taking two of every four (the slot-mod-lanes deal).
    Every transcript equals the oracle's."""
    d = (1 << LOG_N) >> 3
    polys = _polys(oracle, torch, [1101, 1102, 1103])
    want = {s: oracle_commit(LOG_N, s) for s, _ in polys}
    pctx.set_lanes(3)
    pend, lanes = [], []
    for i in range(16):
        s, buf = polys[i % 3]
        t = pctx.commit_device_async(buf.data_ptr(), d, LOG_N)
        pend.append((s, t))
        load = [0, 0, 0]
        for _, tt in pend:
            load[pctx.ticket_lane(tt)] += 1
        assert max(load) - min(load) <= 1, (i, load)
        lanes.append(pctx.ticket_lane(t))
        if len(pend) == 4:
            s0, t0 = pend.pop(0)
            assert _transcript(pctx.commit_wait(t0)) == want[s0]
    for s0, t0 in pend:
        assert _transcript(pctx.commit_wait(t0)) == want[s0]
    # after the first four, every window of three consecutive commits uses all three lanes
    for i in range(4, len(lanes) - 2):
        assert sorted(lanes[i:i + 3]) == [0, 1, 2], lanes


def test_rejected_sync_commit_keeps_pending_lane_commit_resident(pctx, oracle, oracle_commit, torch):
    """A pipelined commit pending on lane 1, then a synchronous fri_commit
    rejected for its arguments: the read-backs still serve the lane-1 commit
    (its generation, its layers), not lane 0's older plan."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    (s0, b0), (s1, b1) = _polys(oracle, torch, [1111, 1112])
    pctx.set_lanes(2)
    pctx.commit(oracle.splitmix64_np(s0, d).astype(np.uint32), LOG_N)    # lane 0 resident: s0
    t0 = pctx.commit_device_async(b0.data_ptr(), d, LOG_N)              # lane 0 (both idle: lower index)
    t1 = pctx.commit_device_async(b1.data_ptr(), d, LOG_N)              # lane 1 (fewest pending)
    assert {pctx.ticket_lane(t0), pctx.ticket_lane(t1)} == {0, 1}
    gen = pctx.commit_info()[0]
    for bad in (dict(log_n=LOG_N + 1), dict(offset=0)):
        with pytest.raises(fri_amd.FriError) as e:
            pctx.commit(oracle.splitmix64_np(s0, d).astype(np.uint32), bad.get("log_n", LOG_N),
                        offset=bad.get("offset", fri_amd.GENERATOR))
        assert e.value.code == fri_amd.FRI_EINVAL
        g, ln, nl = pctx.commit_info()
        assert (g, ln, nl) == (gen, LOG_N, LOG_N - 2)
        root0 = bytes(pctx.tree_level(0, LOG_N, LOG_N)[0]).hex()
        assert root0 == oracle_commit(LOG_N, s1)["roots"][0]            # the last enqueued commit
        lay = pctx.layer(1, LOG_N)
        val, _ = pctx.auth_path(1, 7, LOG_N)
        assert int(val) == int(lay[7])
    assert _transcript(pctx.commit_wait(t0)) == oracle_commit(LOG_N, s0)
    assert _transcript(pctx.commit_wait(t1)) == oracle_commit(LOG_N, s1)


def test_lane_without_memory_falls_back_and_keeps_input_buffer(oracle, oracle_commit, torch):
    """A lane that gets no HBM for its plan (a device-memory cap on the
    context) drops out of the rotation: the commits run on lane 0, lane 0's
    plan and the input buffer stay valid (only the partial plan is released),
    and every transcript is right.  Lifting the cap and setting the lanes
    again brings the lanes back."""
    import fri_amd
    d = (1 << LOG_N) >> 3
    c0 = oracle.splitmix64_np(1201, d).astype(np.uint32)
    polys = _polys(oracle, torch, [1202, 1203, 1204])
    cx = fri_amd.Context(0, LOG_N)
    try:
        cx.commit(c0, LOG_N)
        p0 = cx.input_upload(c0)
        cur = cx.device_bytes()[0]
        cx.set_device_cap(cur + (1 << 16))                   # lane state yes, a second plan no
        cx.set_lanes(3)
        ts = [(s, cx.commit_device_async(b.data_ptr(), d, LOG_N)) for s, b in polys]
        assert [cx.ticket_lane(t) for _, t in ts] == [0, 0, 0]
        for s, t in ts:
            assert _transcript(cx.commit_wait(t)) == oracle_commit(LOG_N, s)
        assert cx.input_buffer(d) == p0
        t = cx.commit_device_async(p0, d, LOG_N)             # the buffer still holds c0
        assert _transcript(cx.commit_wait(t)) == oracle_commit(LOG_N, 1201)
        cx.set_device_cap(0)
        cx.set_lanes(3)
        ts = [(s, cx.commit_device_async(b.data_ptr(), d, LOG_N)) for s, b in polys]
        assert sorted(cx.ticket_lane(t) for _, t in ts) == [0, 1, 2]
        for s, t in ts:
            assert _transcript(cx.commit_wait(t)) == oracle_commit(LOG_N, s)
    finally:
        cx.close()
