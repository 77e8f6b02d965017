"""Shared fixtures.  `-m gpu` tests need a gfx950 GPU and the built
libfri_amd.so; everything else runs on CPU (oracle, host logic, ABI exports,
gloo multi-process)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


@pytest.fixture(scope="session")
def oracle():
    import fri_oracle
    return fri_oracle


@pytest.fixture(scope="session")
def corc():
    import fri_oracle
    return fri_oracle.load_c_oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "fri_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    import fri_amd
    c = fri_amd.Context(0, 24)
    yield c
    c.close()


@pytest.fixture(scope="session")
def oracle_commit(corc):
    """Transcript of the OpenMP C oracle's fri_commit (orc_fri_commit_fast) of
    splitmix64(seed) % p coefficients, d = 2^log_n >> blowup_log: roots (hex),
    betas, final value / degree and channel state.  Cached per session: the
    2^28 transcript (BASELINE configs[4]) is shared by the single-GPU and the
    sharded parity tests."""
    import ctypes
    import functools

    import numpy as np

    import fri_oracle as fo

    @functools.lru_cache(maxsize=None)
    def run(log_n, seed, blowup_log=3):
        d = (1 << log_n) >> blowup_log
        c = np.ascontiguousarray(fo.splitmix64_np(seed, d))
        och = fo.OrcChannel()
        corc.orc_channel_init(ctypes.byref(och))
        r = fo.OrcFriResult()
        assert corc.orc_fri_commit_fast(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), d, log_n, 5, 5, fo.P,
                                        ctypes.byref(och), None, ctypes.byref(r), None, None) == 0
        return {"roots": [bytes(r.roots[k]).hex() for k in range(r.n_layers)],
                "betas": [int(r.betas[i]) for i in range(r.n_rounds)],
                "final_value": int(r.final_value), "final_degree": int(r.final_degree),
                "state": och.state.decode()}
    return run

