"""Soak of one context under a random mix of commit entry points
(tools/soak.py): synchronous commits from host and device input, pipelined
commits of device buffers, host coefficients and the context's own input
buffer, refills of that buffer (fri_ctx_input_upload), lane-count and shape
changes.  Every transcript must equal the C oracle's
(src/fri/fri_commit.rs:72-122); an ordering race between lanes, stagings or
result slots shows up as a wrong transcript.  The soak's model of the input
buffer asks the library nothing (no fri_debug_ticket_lane): the buffer holds
what the caller last uploaded."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("seed,contexts", [(11, 1), (12, 1), (13, 3)])
def test_soak_mixed_entry_points(seed, contexts):
    """One context, and three contexts driven round-robin at random from one
    thread (their host-input uploads share the device's upload stream)."""
    spec = importlib.util.spec_from_file_location("soak", os.path.join(ROOT, "tools", "soak.py"))
    soak = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(soak)
    n_ok, kinds = soak.main(["--commits", "3000", "--seed", str(seed), "--contexts", str(contexts)])
    assert sum(kinds.get(k, 0) for k in range(5)) <= n_ok <= 3000
    assert all(kinds.get(k, 0) > 200 for k in range(6)), kinds
