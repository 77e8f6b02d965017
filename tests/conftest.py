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
