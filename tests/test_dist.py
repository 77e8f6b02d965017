"""Multi-rank (N > 1) coverage of the coset-sharded commit.

CPU (gloo, world 2 and 4): the sharded protocol modelled with the C oracle
(tests/dist_model.py) reproduces the single-node transcript bit for bit.
GPU (gloo host transport, 2 and 4 ranks sharing GPU 0): libfri_amd.so's
fri_commit_sharded reproduces the single-GPU fri_commit transcript."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


sys.path.insert(0, os.path.join(ROOT, "tests"))
from dist_worker import make_coeffs  # noqa: E402


def run_ranks(mode, world, log_n, seed, timeout, env_extra=None, blowup_log=3, stream_stderr=False, kind="random"):
    out = tempfile.mkdtemp(prefix=f"fri_{mode}_")
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["POLY_KIND"] = kind
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), mode, str(log_n), str(seed), out, str(blowup_log)]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=None if stream_stderr else subprocess.PIPE,
                       text=True, timeout=timeout)
    if r.returncode != 0:
        errs = "".join(open(os.path.join(out, f)).read() for f in sorted(os.listdir(out)) if f.endswith(".err"))
        raise AssertionError(f"ranks failed:\n{errs[-6000:]}\n--- stderr tail ---\n{(r.stderr or '')[-2000:]}")
    res = [json.load(open(os.path.join(out, f"rank{i}.json"))) for i in range(world)]
    return res


def single_node(oracle, log_n, seed, kind="random"):
    coeffs = [int(x) for x in make_coeffs(kind, seed, (1 << log_n) // 8)]
    ch = oracle.Channel()
    r = oracle.fri_commit(coeffs, log_n, ch, keep=False)
    return {"roots": [x.hex() for x in r.roots], "betas": r.betas, "final_value": r.final_value,
            "final_degree": r.final_degree, "state": ch.state}


def check_transport_schedule(logs):
    """The RCCL deadlock-freedom condition on the logged
    schedules of every rank (fri_debug_transport_log): per channel (0: main
    communicator, 1: exchange communicator) every rank issues the same
    sequence of (op, bytes), and every pair exchange at position i with peer q
    is matched by q's pair exchange at position i with this rank as peer."""
    world = len(logs)
    for chan in (0, 1):
        seqs = [[tuple(e) for e in lg if e[0] == chan] for lg in logs]
        assert len({len(q) for q in seqs}) == 1, f"chan {chan}: ranks issue different numbers of collectives"
        for i in range(len(seqs[0])):
            assert len({(q[i][1], q[i][3]) for q in seqs}) == 1, f"chan {chan} position {i}: {[q[i] for q in seqs]}"
            if seqs[0][i][1] == "sendrecv":
                for r in range(world):
                    peer = seqs[r][i][2]
                    assert 0 <= peer < world and peer != r
                    assert seqs[peer][i][2] == r, f"chan {chan} position {i}: rank {r} -> {peer} unmatched"
            else:
                assert all(q[i][2] == -1 for q in seqs)
    return [len([e for e in logs[0] if e[0] == c]) for c in (0, 1)]


@pytest.mark.parametrize("world,kind", [(2, "random"), (4, "random"), (8, "random"),
                                        (4, "odd_only"), (8, "odd_only"), (4, "low_degree"),
                                        (8, "low_degree"), (4, "tail_heavy")])
def test_sharded_protocol_model_gloo(oracle, world, kind):
    """The sharded protocol, the sharded coefficient fold and its degree
    records included, modelled over gloo with the C oracle doing the per-block
    work: the transcript equals the single-node oracle's."""
    log_n = 10
    want = single_node(oracle, log_n, 42, kind)
    got = run_ranks("model", world, log_n, 42, timeout=600, env_extra={"SHARD_MIN": "7"}, kind=kind)
    for r in got:
        assert r == want


def test_transport_schedule_check_rejects_mismatch():
    """The schedule check itself: a reordered collective, a size mismatch and
    an unmatched pair exchange are each caught."""
    ok = [[(0, "alltoall", -1, 64), (1, "sendrecv", 1, 32), (0, "allgather", -1, 64)],
          [(0, "alltoall", -1, 64), (1, "sendrecv", 0, 32), (0, "allgather", -1, 64)]]
    assert check_transport_schedule(ok) == [2, 1]
    bad_order = [ok[0], [ok[1][2], ok[1][1], ok[1][0]]]
    bad_size = [ok[0], [ok[1][0], (1, "sendrecv", 0, 16), ok[1][2]]]
    bad_peer = [[(1, "sendrecv", 1, 8)], [(1, "sendrecv", 1, 8)]]
    for bad in (bad_order, bad_size, bad_peer):
        with pytest.raises(AssertionError):
            check_transport_schedule(bad)


@pytest.mark.gpu
@pytest.mark.parametrize("world,log_n,blowup_log,kind", [
    (2, 22, 3, "random"), (4, 22, 3, "random"),    # several sharded layers, then local
    (2, 20, 3, "random"), (2, 21, 3, "random"),    # switch to local right after layer 0 / 1
    (2, 21, 1, "random"), (4, 22, 0, "random"),    # d > n/G: the coset reduction folds several chunks
    (8, 23, 3, "random"),                          # the driver's N = 8 shape: 3-level top, block permutations
    (4, 22, 3, "odd_only"),                        # add_assign's early return in a sharded round
    (8, 23, 3, "low_degree"),                      # the commit ends in a sharded layer (final value: rank 0)
    (4, 22, 3, "tail_heavy"),                      # the degree comes from the last rank's chunk
])
def test_sharded_commit_gpu_matches_single(world, log_n, blowup_log, kind, corc, oracle):
    import ctypes

    import numpy as np
    seed = 7
    got = run_ranks("gpu", world, log_n, seed, timeout=900, blowup_log=blowup_log, kind=kind)
    d = (1 << log_n) >> blowup_log
    c = np.ascontiguousarray(make_coeffs(kind, seed, d).astype(np.uint64))
    och = oracle.OrcChannel()
    corc.orc_channel_init(ctypes.byref(och))
    ores = oracle.OrcFriResult()
    assert corc.orc_fri_commit_fast(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, log_n, 5, 5, oracle.P,
                                    ctypes.byref(och), None, ctypes.byref(ores), None, None) == 0
    want_roots = [bytes(ores.roots[k]).hex() for k in range(ores.n_layers)]
    for r in got:
        assert r["roots"] == want_roots
        assert r["betas"] == [ores.betas[i] for i in range(ores.n_rounds)]
        assert r["final_value"] == ores.final_value
        assert r["state"] == och.state.decode()
        assert r["layer0_refused"] and r["tail_matches_single"] and r["auth_matches_single"]
        if kind != "low_degree":
            assert r["tail_matches_single"] is True and r["auth_matches_single"] is True
        assert r["decommit_matches_single"]
        assert r["noncanonical_rejected"]
        assert r["single_root0"] == want_roots[0]
    n_main, n_x = check_transport_schedule([r["transport_log"] for r in got])
    assert n_main >= 1 and (n_x >= 1 or kind == "low_degree" or log_n - 1 < 20)


_SF = int(os.environ.get("SHARD_FUZZ_N", "0"))      # > 0: that many cases per world size (longer runs)


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_cases", [(2, _SF or 10), (4, _SF or 10), (8, _SF or 8)])
def test_sharded_fuzz_vs_c_oracle(world, n_cases, corc, oracle):
    """Randomised sharded commits (dist_worker.fuzz_case: 2^20..2^22, ragged
    coefficient counts including 0, blowups 1..16, degrees that end the commit
    inside the sharded layers, zero / constant / odd-only / trailing-zero
    polynomials, random cosets, prefilled channels, and for every third case
    forced betas with zeros among them) on W ranks sharing GPU 0:
    every root, beta, the final value and degree and the channel state equal
    the OpenMP C oracle's 1-node commit (orc_fri_commit_fast, which follows
    src/fri/fri_commit.rs:72-122), on every rank, and every case's transport
    schedule passes the cross-rank check."""
    import ctypes

    import numpy as np
    from dist_worker import fuzz_case, fuzz_forced_betas
    seed = 100 * world
    got = run_ranks("gpu_fuzz", world, n_cases, seed, timeout=900)
    for i in range(n_cases):
        log_n, c, offset, state = fuzz_case(seed + i, world)
        fb = fuzz_forced_betas(seed + i)
        fbp = None
        if fb is not None:
            fba = np.ascontiguousarray(np.array(fb, dtype=np.uint64))
            fbp = fba.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        d = c.size
        cs = np.ascontiguousarray(c, dtype=np.uint64)
        och = oracle.OrcChannel()
        corc.orc_channel_init(ctypes.byref(och))
        if state is not None:
            och.state = state.hex().encode()
            och.state_len = 64
        ores = oracle.OrcFriResult()
        assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, log_n, offset, 5,
                                        oracle.P, ctypes.byref(och), fbp, ctypes.byref(ores), None, None) == 0
        what = (f"case {seed + i}: world={world} log_n={log_n} d={d} offset={offset} prefilled={state is not None} "
                f"forced={fb is not None}")
        want = {"roots": [bytes(ores.roots[k]).hex() for k in range(ores.n_layers)],
                "betas": [ores.betas[j] for j in range(ores.n_rounds)],
                "final_value": ores.final_value, "final_degree": ores.final_degree, "state": och.state.decode()}
        for r in got:
            case = r["cases"][i]
            assert "error" not in case, (what, case)
            assert {k: case[k] for k in want} == want, what
        check_transport_schedule([r["cases"][i]["transport_log"] for r in got])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_and_local_commits_mixed(world):
    """One context per rank alternating at random between sharded commits
    (2^20 / 2^21, collective) and the rank's own synchronous and pipelined
    1-GPU commits (2^14 / 2^16, three commit lanes): every plan switch between
    the sharded and the 1-GPU shapes frees the lanes' plans behind the
    pending commits, and every transcript, on every rank, must still equal
    the C oracle's (src/fri/fri_commit.rs:72-122)."""
    got = run_ranks("gpu_soak", world, 300, 4242 + world, timeout=900)
    for r in got:
        assert r["bad"] == [], r["bad"][:5]
        assert r["counts"]["sharded"] > 40 and r["counts"]["sync"] > 40 and r["counts"]["async"] > 40, r["counts"]


@pytest.mark.gpu
def test_loopback_rehearsal_transport(oracle):
    """fri_debug_attach_loopback (tools/shard_projection.py): one rank's share
    of a sharded commit runs on one device with every round of the real
    commit. The degree progression comes from the replicated coefficient fold,
    so the layer and round counts equal the 1-GPU commit's. The roots are not
    the real ones. Detaching ends the rehearsal."""
    import fri_amd
    import numpy as np
    log_n, world = 22, 8
    c = oracle.splitmix64_np(11, (1 << log_n) >> 3).astype(np.uint32)
    one = fri_amd.Context(0, log_n)
    try:
        ref = one.commit(c, log_n)
        degrees = one.commit_degrees()
    finally:
        one.close()
    assert len(degrees) == ref.n_layers and degrees[0] == c.size - 1 and degrees[-1] == 0
    ctx = fri_amd.Context(0, log_n - 3)
    try:
        ctx.attach_loopback(0, world)
        assert ctx.dist_info() == (0, world, "loopback")
        ctx.loopback_degrees(degrees)
        r = ctx.commit_sharded(c, log_n)
        assert (r.n_layers, r.n_rounds) == (ref.n_layers, ref.n_rounds) == (log_n - 2, log_n - 3)
        assert ctx.commit_degrees() == degrees
        ops = [e[1] for e in ctx.transport_log()]
        assert ops.count("alltoall") == 1 and "sendrecv" in ops
        ctx.detach()
        assert ctx.dist_info()[2] == "none"
        with pytest.raises(fri_amd.FriError) as e:
            ctx.decommit_query(0, r.n_layers, log_n, sharded=True)
        assert e.value.code == fri_amd.FRI_ESTATE
    finally:
        ctx.close()


@pytest.mark.gpu
def test_rccl_transport_selftest_world1():
    """The RCCL data path's calls (grouped send/recv all-to-all, all-gather,
    pair exchange on the split communicator + exchange stream) on the real
    device, as self-communication: multi-rank RCCL needs one GPU per rank."""
    import fri_amd
    ctx = fri_amd.Context(0, 12)
    try:
        ctx.attach_rccl(0, 1, fri_amd.Context.unique_id())
        ctx.dist_selftest(4096)
        ctx.detach()
    finally:
        ctx.close()


def _run_child(code, timeout=180, rccl_timeout=True):
    """Run `code` in a fresh interpreter (its own HIP context and RCCL state:
    a rendezvous thread abandoned there cannot leak into other tests) and
    return the JSON object it prints last."""
    env = dict(os.environ)
    if rccl_timeout:
        env["FRI_RCCL_TIMEOUT_S"] = "3"
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "stark-prover_amd", "python"),
                                         os.path.join(ROOT, "oracle"), env.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


_ATTACH_TIMEOUT_CHILD = r"""
import json, os, time
import fri_amd, fri_oracle as fo
ctx = fri_amd.Context(0, 20)
t0 = time.monotonic()
try:
    ctx.attach_rccl(0, 2, fri_amd.Context.unique_id())
    out = {"raised": False}
except fri_amd.FriError as e:
    out = {"raised": True, "code": e.code, "msg": str(e)}
out["seconds"] = time.monotonic() - t0
out["n_layers"] = int(ctx.commit(fo.splitmix64_field(3, 128), 10).n_layers)
print(json.dumps(out), flush=True)
os._exit(0)   # the abandoned setup thread is still blocked in RCCL's bootstrap
"""


@pytest.mark.gpu
def test_rccl_attach_times_out_without_peer():
    """A rendezvous that never completes (rank 0 of 2, rank 1 absent) ends in
    FRI_ERCCL after FRI_RCCL_TIMEOUT_S instead of hanging, and the context
    stays usable for 1-GPU commits.  Runs in a child process: the abandoned
    setup thread stays blocked in RCCL's bootstrap until that process exits."""
    import fri_amd
    r = _run_child(_ATTACH_TIMEOUT_CHILD)
    assert r["raised"] and r["code"] == fri_amd.FRI_ERCCL and "rendezvous" in r["msg"]
    assert r["seconds"] < 60
    assert r["n_layers"] == 8


_STALL_CHILD = r"""
import json, os, time
import fri_amd, fri_oracle as fo
ctx = fri_amd.Context(0, 16)
ctx.attach_rccl(0, 1, fri_amd.Context.unique_id())       # default deadline: a first RCCL init can take seconds
ctx.dist_selftest(1024)                                   # the transport works
os.environ["FRI_RCCL_TIMEOUT_S"] = "3"                    # read by the library at every deadline
ctx._check(ctx.lib.fri_debug_inject_stall(ctx.h, 1))      # next all-to-all never completes
out = {}
t0 = time.monotonic()
try:
    ctx.dist_selftest(1024)
    out["first"] = None
except fri_amd.FriError as e:
    out["first"] = [e.code, str(e)]
out["seconds"] = time.monotonic() - t0
try:
    ctx.dist_selftest(1024)
    out["second"] = None
except fri_amd.FriError as e:
    out["second"] = [e.code, str(e)]
c = fo.splitmix64_field(3, 1 << 11)
out["commit_layers"] = int(ctx.commit(c, 14).n_layers)     # the context still commits on one GPU
ctx.close()
print(json.dumps(out), flush=True)
"""


@pytest.mark.gpu
def test_rccl_collective_stall_aborts():
    """A collective that never completes (injected: the all-to-all replaced
    by a kernel that waits like one whose peer is gone) ends in FRI_ERCCL
    within FRI_RCCL_TIMEOUT_S: the deadline polls the stream, aborts the
    communicators (which releases the waiting kernel) and drains the stream;
    the next sharded call finds no transport (FRI_ESTATE); 1-GPU commits on
    the same context still work."""
    import fri_amd
    r = _run_child(_STALL_CHILD, rccl_timeout=False)
    assert r["first"] is not None and r["first"][0] == fri_amd.FRI_ERCCL, r
    assert "no progress" in r["first"][1] and "still busy" not in r["first"][1]
    assert 2.5 < r["seconds"] < 30
    assert r["second"] is not None and r["second"][0] == fri_amd.FRI_ESTATE
    assert r["commit_layers"] == 12


@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_sharded_2p28_world8_configs4(oracle_commit):
    """BASELINE configs[4]: a 2^28 codeword (d = 2^25) committed coset-sharded
    by 8 ranks (host transport over gloo, all 8 sharing GPU 0), each rank on a
    shard-sized context (log_n_max 25): every root, beta, the final value and
    the channel state equal the OpenMP C oracle's 1-node commit, on every rank,
    and each rank holds well under 1/8 of the ~38 GB a 1-GPU 2^28 commit needs."""
    got = run_ranks("gpu_shard", 8, 28, 8, timeout=1100, stream_stderr=True)
    check_transport_schedule([r["transport_log"] for r in got])
    want = oracle_commit(28, 8)
    for r in got:
        assert r["roots"] == want["roots"]
        assert r["betas"] == want["betas"]
        assert r["final_value"] == want["final_value"] and r["final_degree"] == want["final_degree"]
        assert r["state"] == want["state"]
        assert r["layer0_refused"] and r["last_layer_constant"]
        assert r["verify_fri"] and r["transcript_sha"] == got[0]["transcript_sha"]
        assert r["hbm_peak_bytes"] < 8 * 2**30, r["hbm_peak_bytes"]
    print("per-rank HBM (GiB):", [round(r["hbm_peak_bytes"] / 2**30, 2) for r in got])


@pytest.mark.gpu
@pytest.mark.parametrize("world,log_n,blowup_log", [(2, 22, 3), (4, 23, 3), (8, 24, 3),
                                                    (2, 21, 0), (4, 22, 1), (8, 23, 2)])
def test_sharded_shard_sized_context(world, log_n, blowup_log, oracle_commit):
    """Shard-sized contexts (log_n_max = log_n - log2 world) at smaller sizes,
    blowups 1..8 (d up to n: the coset reduction folds several chunks, and the
    two-rank decimation takes d/2 coefficients per half): the same transcript
    as the oracle, and per-rank HBM well below what the whole-codeword plan
    needed (layers + trees alone are ~130 * 2^log_n bytes)."""
    got = run_ranks("gpu_shard", world, log_n, 11, timeout=900, blowup_log=blowup_log)
    check_transport_schedule([r["transport_log"] for r in got])
    want = oracle_commit(log_n, 11, blowup_log)
    d = (1 << log_n) >> blowup_log
    for r in got:
        assert {k: r[k] for k in want} == want
        assert r["layer0_refused"] and r["last_layer_constant"]
        assert r["verify_fri"] and r["transcript_sha"] == got[0]["transcript_sha"]
        # the input (full: the coset LDE reads it) and the coefficient-fold
        # chunks (two buffers of d / (2 world) words, or the local tail's poly)
        d_bytes = 4 * d + 8 * max(d // (2 * world), d >> 9)
        assert r["hbm_peak_bytes"] < 130 * (1 << log_n) / world + d_bytes + (512 << 20), r["hbm_peak_bytes"]
