"""bench.py's host logic on the CPU: the agreement step of the sharded
setup (every rank learns which step failed on which rank before the next
collective, and the fallback note names them)."""
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_setup_failure_names_step_and_rank():
    out = tempfile.mkdtemp(prefix="bench_agree_")
    world = 4
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "bench_agree_worker.py"), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open(os.path.join(out, f"rank{i}.json"))) for i in range(world)]
    for x in res:
        assert x["ok"] == [True, False, False]
        assert x["notes"][0] is None
        assert x["notes"][1] == "setup step 'attach (rccl)' failed on rank(s) [1]: " \
                                "RuntimeError: ncclCommInitRank: invalid usage"
        assert x["notes"][2].startswith("setup step 'first sharded commit 2^28 (strong_primary)' failed on rank(s) "
                                        "[0, 1, 2, 3]: sharded transcript differed")
