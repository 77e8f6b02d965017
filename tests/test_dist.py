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


def run_ranks(mode, world, log_n, seed, timeout, env_extra=None, blowup_log=3):
    out = tempfile.mkdtemp(prefix=f"fri_{mode}_")
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), mode, str(log_n), str(seed), out, str(blowup_log)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open(os.path.join(out, f"rank{i}.json"))) for i in range(world)]
    return res


def single_node(oracle, log_n, seed):
    coeffs = oracle.splitmix64_field(seed, (1 << log_n) // 8)
    ch = oracle.Channel()
    r = oracle.fri_commit(coeffs, log_n, ch, keep=False)
    return {"roots": [x.hex() for x in r.roots], "betas": r.betas, "final_value": r.final_value,
            "final_degree": r.final_degree, "state": ch.state}


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_protocol_model_gloo(oracle, world):
    log_n = 10
    want = single_node(oracle, log_n, 42)
    got = run_ranks("model", world, log_n, 42, timeout=600, env_extra={"SHARD_MIN": "7"})
    for r in got:
        assert r == want


@pytest.mark.gpu
@pytest.mark.parametrize("world,log_n,blowup_log", [
    (2, 22, 3), (4, 22, 3),          # several sharded layers, then local
    (2, 20, 3), (2, 21, 3),          # switch to local right after layer 0 / 1
    (2, 21, 1), (4, 22, 0),          # d > n/G: the coset reduction folds several chunks
    (8, 23, 3),                      # the driver's N = 8 shape: 3-level top, block permutations
])
def test_sharded_commit_gpu_matches_single(world, log_n, blowup_log, corc, oracle):
    import ctypes

    import numpy as np
    seed = 7
    got = run_ranks("gpu", world, log_n, seed, timeout=900, blowup_log=blowup_log)
    d = (1 << log_n) >> blowup_log
    c = np.ascontiguousarray(np.array(oracle.splitmix64_field(seed, d), dtype=np.uint64))
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
        assert r["single_root0"] == want_roots[0]


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


@pytest.mark.gpu
def test_rccl_attach_times_out_without_peer(monkeypatch, oracle):
    """A rendezvous that never completes (rank 0 of 2, rank 1 absent) ends in
    FRI_ERCCL after FRI_RCCL_TIMEOUT_S instead of hanging, and the context
    stays usable for 1-GPU commits.  (The abandoned setup thread stays blocked
    in RCCL's bootstrap for the rest of the process: keep this test last among
    the RCCL tests.)"""
    import time
    import fri_amd
    monkeypatch.setenv("FRI_RCCL_TIMEOUT_S", "3")
    ctx = fri_amd.Context(0, 20)
    try:
        t0 = time.monotonic()
        with pytest.raises(fri_amd.FriError, match="rendezvous"):
            ctx.attach_rccl(0, 2, fri_amd.Context.unique_id())
        assert time.monotonic() - t0 < 60
        coeffs = oracle.splitmix64_field(3, 128)
        res = ctx.commit(coeffs, 10)
        assert res.n_layers == 8
    finally:
        ctx.close()
