"""Team contexts over DISTINCT devices (fri_ctx_create_multi, fri_ctx_create_default).

These are the lines DESIGN.md §7 "Never executed" lists: peer access between
two devices (hipDeviceEnablePeerAccess), k_peer_pull reading another GPU's
HBM over xGMI, the hipMemcpyPeerAsync fallback between devices, and the
in-process RCCL team (ncclCommInitAll).  They need a box with at least two
GPUs and are skipped on a one-GPU box (the same protocol over ranks sharing
GPU 0 is tests/test_team.py).  Every transcript is compared with the C
oracle's, every read-back with a one-GPU commit of the same polynomial."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _ndev():
    import torch
    return torch.cuda.device_count()          # (counting devices does not initialise them)


def _need(n):
    have = _ndev()
    if have < n:
        pytest.skip(f"needs {n} distinct GPUs, {have} visible")


def _transcript(res):
    return {"roots": [bytes(res.roots[k]).hex() for k in range(res.n_layers)],
            "betas": [int(res.betas[r]) for r in range(res.n_rounds)],
            "final_value": int(res.final_value), "final_degree": int(res.final_degree),
            "state": bytes(res.channel_out.digest).hex()}


def _coeffs(oracle, seed, log_n, blowup_log=3):
    return oracle.splitmix64_np(seed, (1 << log_n) >> blowup_log).astype(np.uint32)


@pytest.fixture(scope="module")
def one23():
    import fri_amd
    _need(2)
    c = fri_amd.Context(0, 23)
    yield c
    c.close()


def _check_team(cx, one, oracle, oracle_commit, L=22, seed=42):
    from test_dist import check_transport_schedule
    cf = _coeffs(oracle, seed, L)
    rt = cx.commit(cf, L)
    assert _transcript(rt) == oracle_commit(L, seed)
    check_transport_schedule([cx.team_rank(r).transport_log() for r in range(cx.n_ranks)])
    r1 = one.commit(cf, L)
    for k in (0, 1, rt.n_layers - 1):
        assert np.array_equal(cx.layer(k, L), one.layer(k, L)), k
    for idx in (0, 12345, (1 << L) - 3):
        assert cx.decommit_query(idx, rt.n_layers, L) == one.decommit_query(idx, r1.n_layers, L), idx


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("path", ["pull", "copy"])
def test_peer_team_on_distinct_devices(one23, oracle, oracle_commit, G, path):
    """Ranks on GPUs 0..G-1 over the peer transport: the pull kernel reads
    the other devices' buffers through peer access (`pull`), or one
    hipMemcpyPeerAsync per source (`copy`, fri_debug_team_force_copy)."""
    import fri_amd
    _need(G)
    cx = fri_amd.Context.multi(list(range(G)), 23, transport="peer")
    try:
        assert cx.dist_info() == (0, G, "peer")
        cx.force_copy(path == "copy")
        _check_team(cx, one23, oracle, oracle_commit)
        _check_team(cx, one23, oracle, oracle_commit, seed=43)
    finally:
        cx.close()


@pytest.mark.parametrize("G", [2, 4, 8])
def test_rccl_team_on_distinct_devices(one23, oracle, oracle_commit, G):
    """The in-process RCCL team (ncclCommInitAll, one communicator per rank
    for each stream): opt-in, refused for ranks sharing a device."""
    import fri_amd
    _need(G)
    cx = fri_amd.Context.multi(list(range(G)), 23, transport="rccl")
    try:
        assert cx.dist_info() == (0, G, "rccl")
        _check_team(cx, one23, oracle, oracle_commit)
    finally:
        cx.close()


def test_mixed_ordinals(one23, oracle, oracle_commit):
    """Two ranks on each of two devices: same-device pulls and xGMI pulls in
    one collective; RCCL refuses the shared devices."""
    import fri_amd
    _need(2)
    cx = fri_amd.Context.multi([0, 0, 1, 1], 23, transport="peer")
    try:
        _check_team(cx, one23, oracle, oracle_commit)
    finally:
        cx.close()
    with pytest.raises(fri_amd.FriError) as e:
        fri_amd.Context.multi([0, 0, 1, 1], 23, transport="rccl")
    assert e.value.code == fri_amd.FRI_EINVAL


def test_default_context_spans_the_visible_devices(monkeypatch, one23, oracle, oracle_commit):
    """fri_ctx_create_default with FRI_DEVICES unset: a team over the largest
    power-of-two prefix of the visible GPUs (what the reference-signature
    bindings open), committing the oracle's transcript."""
    import fri_amd
    _need(2)
    monkeypatch.delenv("FRI_DEVICES", raising=False)
    monkeypatch.delenv("FRI_TRANSPORT", raising=False)
    n = _ndev()
    want = 1
    while want * 2 <= min(n, 64):
        want *= 2
    cx = fri_amd.Context.default(23)
    try:
        assert cx.n_ranks == want and cx.dist_info() == (0, want, "peer")
        _check_team(cx, one23, oracle, oracle_commit)
    finally:
        cx.close()
