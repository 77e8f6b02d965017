"""Soak of one context under a random mix of commit entry points
(tools/soak.py): synchronous commits from host and device input, pipelined
commits of device buffers, host coefficients and the context's own input
buffer, with lane-count and shape changes.  Every transcript must equal the C
oracle's (src/fri/fri_commit.rs:72-122); an ordering race between lanes,
stagings or result slots shows up as a wrong transcript."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed", [11, 12])
def test_soak_mixed_entry_points(seed):
    spec = importlib.util.spec_from_file_location("soak", os.path.join(ROOT, "tools", "soak.py"))
    soak = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(soak)
    n_ok, kinds = soak.main(["--commits", "3000", "--seed", str(seed)])
    assert n_ok == 3000
    assert all(kinds.get(k, 0) > 200 for k in range(5)), kinds
