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


def test_pmc_traffic_only_for_the_same_sources(tmp_path):
    """roofline.traffic comes from profiles/pmc_traffic.json only when the
    figure was collected on the sources of this build (source_hash)."""
    ent = {"merkle_layer0_leaf": {"hbm_bytes_per_launch": 1.25e9}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"24": dict(ent, source_hash=bench.source_hash())}))
    val, note = bench._pmc_traffic(24, str(p))
    assert val == 1.25e9 and bench.source_hash()[:12] in note
    p.write_text(json.dumps({"24": dict(ent, source_hash="0" * 64)}))
    val, note = bench._pmc_traffic(24, str(p))
    assert val is None and "re-collect" in note
    val, note = bench._pmc_traffic(20, str(p))
    assert val is None


def test_source_hash_covers_the_kernels():
    import glob
    files = [f for pat in bench.SOURCE_GLOBS for f in glob.glob(os.path.join(ROOT, pat))]
    names = {os.path.basename(f) for f in files}
    assert {"fri_layer.hip", "fri_kernels.hip", "fri_commit.hip", "fri_host.hpp", "sha256_fast.hpp", "fri_amd.h", "Makefile"} <= names
    assert len(bench.source_hash()) == 64


@pytest.mark.parametrize("team,world,ndev,ranks,want", [
    (None, 1, 1, 1, (1, False)),                 # the default 1-GPU line
    (None, 8, 8, 8, (8, False)),                 # torchrun x8 on an 8-GPU node
    (None, 2, 1, 2, (1, True)),                  # 2 ranks on the 1-GPU box: a rehearsal
    ([0, 1, 2, 3], 1, 8, 4, (4, False)),         # p2p team over 4 GPUs
    ([0, 0], 1, 1, 2, (1, True)),                # p2p team, 2 ranks on one GPU
])
def test_devices_used_reports_distinct_gpus(team, world, ndev, ranks, want):
    """n_gpus in the line is the number of distinct devices; ranks sharing a
    device mark the run oversubscribed (such a run is not an
    N-GPU scaling point)."""
    assert bench.devices_used(team, world, ndev, ranks) == want
