"""CPU: how `bench.py --gpus N` becomes N ranks (launch_plan), decided
before anything touches the GPU, and the relay of rank 0's JSON line when
bench.py spawns the ranks itself."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,transport,want", [
    (1, {}, "rccl", "run"),                              # the default 1-GPU line
    (2, {}, "rccl", "spawn"),                            # plain `bench.py --gpus 2`: spawn the ranks
    (8, {}, "host", "spawn"),
    (8, {"WORLD_SIZE": "8"}, "rccl", "run"),             # torchrun --nproc-per-node 8 bench.py --gpus 8
    (8, {"WORLD_SIZE": "1"}, "rccl", "mismatch"),        # a 1-rank job must not be labelled 8 GPUs
    (1, {"WORLD_SIZE": "4"}, "rccl", "mismatch"),
    (4, {}, "p2p", "run"),                               # one process drives the 4 GPUs (team context)
    (4, {"WORLD_SIZE": "4"}, "p2p", "run"),
])
def test_launch_plan(gpus, env, transport, want):
    assert bench.launch_plan(gpus, env, transport) == want


def test_spawn_command_is_a_local_launcher():
    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "3"], 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--master-port=29512" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def test_spawn_relays_rank0_line(monkeypatch, capsys):
    """The parent prints exactly the child's JSON line on stdout (other stdout
    text goes to stderr) and returns the child's exit status."""
    line = {"metric": bench.METRIC, "value": 1.0, "n_gpus": 2}
    prog = ("import json,sys; print('gloo banner'); print(json.dumps(%r)); sys.exit(0)" % line)
    monkeypatch.setattr(bench, "spawn_command", lambda g, a, p: [sys.executable, "-c", prog])
    assert bench._spawn_ranks(2, []) == 0
    out, err = capsys.readouterr()
    assert [json.loads(x) for x in out.splitlines()] == [line]
    assert "gloo banner" in err
    monkeypatch.setattr(bench, "spawn_command", lambda g, a, p: [sys.executable, "-c", "import sys; sys.exit(3)"])
    assert bench._spawn_ranks(2, []) == 3
    monkeypatch.setattr(bench, "spawn_command", lambda g, a, p: [sys.executable, "-c", "pass"])
    assert bench._spawn_ranks(2, []) == 1                 # no line: a failure, even with status 0
