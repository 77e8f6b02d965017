"""Runs the C++ host-mirror tests (tests/cpp/test_stark101.cpp) — the
reference-shaped C++ API (stark-prover_amd/host/stark101.hpp) over
libfri_amd.so.  The CPU group needs no device; the GPU group drives the
device through the C ABI and compares with tests/golden bit for bit."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "stark-prover_amd")
BIN = os.path.join(PKG, "build", "test_stark101")


def _build():
    subprocess.run(["make", "-s", "-C", PKG, "test_host"], check=True, timeout=600)


def _run(group):
    _build()
    p = subprocess.run([BIN, group], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert " 0 failures" in p.stdout
    return p.stdout


def test_golden_include_is_current():
    """golden_cases.inc is generated from fri_golden.json; it must not drift."""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fri_golden.json")))
    inc = open(os.path.join(ROOT, "tests", "cpp", "golden_cases.inc")).read()
    for c in g["cases"]:
        assert f'"{c["name"]}"' in inc and f'"{c["channel_out"]}"' in inc, c["name"]


def test_cpp_host_mirror_cpu():
    out = _run("cpu")
    assert "ok   cpu::channel_replays_golden_commits" in out
    assert "ok   cpu::verify_fri_rejects_tampering" in out
    assert "ok   cpu::verify_fibsq_accepts_and_rejects" in out


def test_device_field_arithmetic_on_host(tmp_path):
    """csrc/field.hpp (redc / add / sub / Montgomery conversions used by every
    kernel) is host-callable: check it against __int128 arithmetic on edge
    values (0, 1, p-1, 2^31, ...) and 2M random operand pairs
    (tests/cpp/test_field.cpp)."""
    exe = tmp_path / "test_field"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-o", str(exe),
                    os.path.join(ROOT, "tests", "cpp", "test_field.cpp")], check=True, timeout=300)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and " 0 failures" in p.stdout, p.stdout


def test_host_library_exports_reference_api():
    _build()
    syms = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(PKG, "lib", "libstark101.so")],
                          capture_output=True, text=True, check=True).stdout
    for name in ("stark101::fri_commit(", "stark101::decommit_fri(", "stark101::decommit_fri_layers(",
                 "stark101::verify_fri(", "stark101::MerkleTree::MerkleTree(", "stark101::interpolate(",
                 "stark101::batch_inverse(", "stark101::evaluate_on_coset(", "stark101::prove_fibsq(",
                 "stark101::verify_fibsq("):
        assert name in syms, name
    needed = subprocess.run(["readelf", "-d", os.path.join(PKG, "lib", "libstark101.so")],
                            capture_output=True, text=True, check=True).stdout
    assert "libfri_amd.so" in needed                      # the device path, no CPU fallback
    assert "oracle" not in needed


@pytest.mark.gpu
def test_cpp_host_mirror_gpu():
    out = _run("gpu")
    assert "ok   gpu::fri_commit_and_decommit_match_golden" in out
    assert "ok   gpu::fri_commit_pipelined_matches_golden" in out
    assert "ok   gpu::prove_fibsq_matches_golden" in out


@pytest.mark.gpu
def test_cpp_reference_signatures_on_default_team(tmp_path, corc):
    """The reference's own signatures, no context named anywhere:
    fri_commit(poly, domain, &mut channel) and decommit_fri(num_queries,
    max_index, &fri_layers, &fri_merkles, &mut channel)
    (fri_commit.rs:72-76,168-174) through the C++ mirror, whose per-thread
    default context is a team over FRI_DEVICES ("0,0,0,0": four ranks on the
    one GPU of the box; on an 8-GPU node, unset, it would be all eight).  At
    2^22 the commit is coset-sharded; the whole transcript -- every root, beta,
    the final value and two queries' openings -- equals the C oracle's, a
    later commit makes the old proof's decommitment panic, and layers of
    another commit are refused (tests/cpp/test_stark101.cpp refsig)."""
    import numpy as np

    import fri_oracle as fo
    import oracle_flat
    _build()
    out = tmp_path / "refsig.txt"
    env = dict(os.environ, FRI_DEVICES="0,0,0,0")
    p = subprocess.run([BIN, "refsig", "22", str(out)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = out.read_text().split("\n")
    assert lines[0] == "ranks 4", lines[0]
    state = lines[1].split()[1]
    msgs = [bytes.fromhex(ln.split()[1]) if len(ln.split()) > 1 else b"" for ln in lines[2:] if ln.startswith("msg")]
    want_msgs, want_state = oracle_flat.transcript(corc, fo.splitmix64_np(42, (1 << 22) >> 3), 22, 2)
    assert len(msgs) == len(want_msgs)
    assert msgs == want_msgs
    assert state == want_state
