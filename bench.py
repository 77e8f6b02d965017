#!/usr/bin/env python3
"""bench.py — FRI commit throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log-n 24]

One step = one full FRI commit (src/fri/fri_commit.rs:72-122) of a synthetic
random polynomial with d = 2^21 coefficients (blowup 8) onto the codeword
2^24 = BASELINE.json configs[2]: coset LDE (NTT), 22 SHA-256 Merkle trees
(all levels kept), 21 Fiat-Shamir rounds and folds, final value — inputs
resident in HBM when the timed region starts, result (roots, betas, final
value, channel state) read back to the host at the end of every step.

N > 1 (torchrun, one process per GPU): by default strong scaling of ONE
2^28 codeword (BASELINE.json configs[4]) committed coset-sharded across the
ranks (fri_commit_sharded_device over the library's RCCL communicator), with
the weak 2^24-per-GPU and the strong 2^24 points as secondary keys
(`scaling_points`); `--log-n L` alone selects weak scaling, 2^L per GPU.
The sharded transcript is checked against the C oracle's golden transcript
(tests/golden/bench_transcripts.json) before timing; on any mismatch/error
every rank falls back to --mode replicas (N independent commits) and
`config.parallelism` says so.  value = codeword elements committed per second
by the whole job, timed by the slowest rank.

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))

METRIC = "FRI commit field-elems/sec at codeword 2^24; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TOPS = 78.6            # 256 CU x 128 int32 lane-ops/clk x 2.4 GHz
VALU_MEASURED_TOPS = 64.0        # full-rate v_xor/v_bitop3 streams over the whole chip (valu_cal.hip, lone_wave.hip)
DOMINANT = "merkle_layer0_leaf"  # dominant kernel class (DESIGN.md "Roofline")


def algorithmic_bytes(log_n, d):
    """B_field = 4d + 8n + 8n, B_tree = 32 * (all tree nodes)."""
    n = 1 << log_n
    rounds = max(0, (d - 1).bit_length())
    rounds = min(rounds, log_n)
    nodes = sum((2 << (log_n - k)) - 1 for k in range(rounds + 1))
    layers = sum(1 << (log_n - k) for k in range(rounds + 1))
    b_field = 4 * d + 4 * layers + 4 * layers
    return b_field, 32 * nodes


# VALU issue units per SHA-256 compression as the kernels run them (DESIGN.md
# §5): a leaf hash (one block, message mostly zeros) 2009, an internal node
# (its block plus the constant padding block) 3592; v_alignbit / v_add3 are
# half rate on gfx950 and count twice.
LEAF_ISSUE_UNITS = 2009.0
NODE_ISSUE_UNITS = 3592.0


def valu_issue_units(log_n, d):
    """Issue units of every leaf and node hash of a whole commit (all R+1
    layers' trees): the VALU work the commit cannot avoid (1.879e11 at 2^24).
    NTT, folds and the channel add well under 1%."""
    rounds = min(max(0, (d - 1).bit_length()), log_n)
    leaves = sum(1 << (log_n - k) for k in range(rounds + 1))
    nodes = sum((1 << (log_n - k)) - 1 for k in range(rounds + 1))
    return leaves * LEAF_ISSUE_UNITS + nodes * NODE_ISSUE_UNITS


def whole_commit_valu(log_n, d, ms_per_commit, n_commits=1, n_dev=1):
    """valu_issue_units of n_commits commits over ms_per_commit on n_dev GPUs,
    against the nominal VALU peak and the measured issue ceiling of those GPUs
    (the chain's idle chip shows here, where the dominant kernel's own
    roofline cannot see it)."""
    units = valu_issue_units(log_n, d)
    t = n_commits * units / (ms_per_commit * 1e-3) / 1e12
    out = {"issue_units_per_commit": units, "ms_per_commit": round(ms_per_commit, 4), "achieved": round(t, 2),
           "unit": "T int32 lane-ops/s", "peak": VALU_PEAK_TOPS * n_dev, "frac": round(t / (VALU_PEAK_TOPS * n_dev), 4),
           "measured_ceiling": VALU_MEASURED_TOPS * n_dev,
           "frac_of_measured_ceiling": round(t / (VALU_MEASURED_TOPS * n_dev), 4)}
    if n_commits != 1 or n_dev != 1:
        out.update(commits=n_commits, n_gpus=n_dev)
    return out


def sha_compressions(log_n, d):
    rounds = min(max(0, (d - 1).bit_length()), log_n)
    leaves = sum(1 << (log_n - k) for k in range(rounds + 1))
    nodes = sum((1 << (log_n - k)) - 1 for k in range(rounds + 1))
    return leaves + 2 * nodes


def _coeffs(seed, d, P):
    """splitmix64(seed) % p, SURVEY.md §8(d) (same stream as oracle.splitmix64_field)."""
    import numpy as np
    idx = np.arange(1, d + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z % np.uint64(P)).astype(np.uint32)


def _same(a, b):
    return (a.n_layers == b.n_layers and a.n_rounds == b.n_rounds and a.final_value == b.final_value
            and a.final_degree == b.final_degree
            and all(bytes(a.roots[k]) == bytes(b.roots[k]) for k in range(a.n_layers))
            and list(a.betas)[: a.n_rounds] == list(b.betas)[: b.n_rounds]
            and bytes(a.channel_out.digest) == bytes(b.channel_out.digest))


def agree_step(dist, world, rank, step, what):
    """Run one step of the sharded setup; every rank learns whether ALL ranks
    succeeded before anyone enters the next collective (a rank that failed
    alone must not leave the others blocked inside RCCL), and which step
    failed on which ranks with what error (gloo all-gather), so the fallback
    line names them on every rank.  Returns (ok, note)."""
    ok, msg = 1, None
    try:
        if step() is False:
            ok, msg = 0, "sharded transcript differed from the C oracle's"
    except Exception as e:  # noqa: BLE001 - any failure (FriError or other) must reach the other ranks
        ok, msg = 0, str(e) if type(e).__name__ == "FriError" else f"{type(e).__name__}: {e}"
    every = [None] * world
    dist.all_gather_object(every, (ok, msg))
    bad = [r for r, (o, _) in enumerate(every) if not o]
    if not bad:
        return True, None
    note = f"setup step '{what}' failed on rank(s) {bad}: {every[bad[0]][1]}"
    print(f"[bench] rank {rank}: {note}", file=sys.stderr, flush=True)
    return False, note


def _host_transport_check(fri_amd, ctx, dist, world, rank, logG, args, agree, timed):
    """After an RCCL setup failure: the 2^24 codeword (and 2^(24 + log2 N)
    when it fits the context) committed coset-sharded over the host-staged
    gloo transport, checked against the oracle's transcript and timed for a
    few steps (bench.py's own N > 1 protocol, every step agreed over gloo).
    Returns the record for scaling_points (or the step that failed)."""
    out = {"transport": "host-staged gloo (the RCCL run failed)", "what": "correctness of the coset-sharded path "
           "across these GPUs; every collective goes through host memory, so the time is not a scaling figure"}
    ok, msg = agree(dist, world, rank, lambda: ctx.attach_torch(rank, world), "attach (host)")
    if ok:
        ok, msg = agree(dist, world, rank, lambda: ctx.dist_selftest(1024), "host transport self-test")
    if not ok:
        out["error"] = msg
        return out
    points = []
    for L in (24, 24 + logG):
        if L - logG <= ctx.log_n_max and L not in points:
            points.append(L)
    for L in points:
        dL = 1 << (L - args.blowup_log)
        cf = _coeffs(42, dL, fri_amd.P)
        exp = _expected(L, args.blowup_log)
        got = {}

        def first():
            got["r"] = ctx.commit_sharded(cf, L)
            return True if exp is None else _matches(got["r"], exp)

        ok, msg = agree(dist, world, rank, first, f"host-transport sharded commit 2^{L}")
        if not ok:
            out[f"2^{L}"] = {"error": msg}
            continue
        k = 3
        el = timed(lambda: ctx.commit_sharded(cf, L), k, 0)
        out[f"2^{L}"] = {"codeword_log2": L, "per_gpu_log2": L - logG, "ms_per_step": round(1000 * el / k, 4),
                         "steps": k, "oracle_verified": exp is not None}
    try:
        ctx.detach()
    except fri_amd.FriError:
        pass
    return out


def _expected(log_n, blowup_log):
    """Oracle transcript of the bench workload (tests/golden/bench_transcripts.json,
    written by tests/golden/make_bench_transcripts.py from the C oracle), or None."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_transcripts.json")) as f:
            return json.load(f).get(f"{log_n}/42/{blowup_log}")
    except (OSError, ValueError):
        return None


def _matches(res, exp):
    return (res.n_layers == len(exp["roots"]) and res.n_rounds == len(exp["betas"])
            and [bytes(res.roots[k]).hex() for k in range(res.n_layers)] == exp["roots"]
            and [int(res.betas[i]) for i in range(res.n_rounds)] == exp["betas"]
            and int(res.final_value) == exp["final_value"] and int(res.final_degree) == exp["final_degree"]
            and bytes(res.channel_out.digest).hex() == exp["state"])


def launch_plan(gpus, env, transport="rccl"):
    """How `bench.py --gpus N` runs, decided before anything touches the GPU:
      "run"      - this process is the whole job (N == 1, or --transport p2p:
                   one process drives the N GPUs as a team context) or one
                   rank of a launcher's job whose WORLD_SIZE is N;
      "spawn"    - N > 1 and no launcher: start the N ranks as
                   `python -m torch.distributed.run` (a child process) and
                   relay rank 0's JSON line;
      "mismatch" - a launcher started WORLD_SIZE ranks but --gpus says N:
                   refuse (a 1-rank job must not be reported as N GPUs)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "spawn" if gpus > 1 and transport != "p2p" else "run"
    return "run" if int(ws) == gpus else "mismatch"


def spawn_command(gpus, argv, port):
    """The child launcher of launch_plan's "spawn": one rank per GPU over
    127.0.0.1 (the container hostname may not resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _spawn_ranks(gpus, argv):
    """Run the N ranks under torch.distributed.run as a child process (this
    process never initialises HIP), pass their stderr through and print rank
    0's JSON line on stdout; exit with the child's status."""
    cmd = spawn_command(gpus, argv, _free_port())
    print(f"[bench] --gpus {gpus} without a launcher: {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout.splitlines():
        try:
            if "metric" in json.loads(ln):
                line = ln
        except ValueError:
            print(ln, file=sys.stderr)
    if line is not None:
        print(line, flush=True)
    return proc.returncode if line is not None or proc.returncode else 1


def main():
    # The contract's ONE JSON line goes to the original stdout; everything
    # else written to fd 1 by native libraries (gloo connection messages, the
    # RCCL banner) or by Python is redirected to stderr.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=None,
                    help="N=1: codeword log2 (default 24).  N>1: with --scaling strong the fixed codeword "
                         "(default 28 = configs[4]); with --scaling weak the log2 per GPU (default 24)")
    ap.add_argument("--scaling", choices=("auto", "strong", "weak"), default="auto",
                    help="N>1: strong = one fixed codeword over the N ranks; weak = 2^log_n per GPU. "
                         "auto: strong at 2^28 (BASELINE configs[4]), or weak when --log-n is given")
    ap.add_argument("--blowup-log", type=int, default=3)
    ap.add_argument("--mode", choices=("sharded", "replicas"), default="sharded",
                    help="N>1: one coset-sharded codeword (default), or N independent 2^24 commits")
    ap.add_argument("--transport", choices=("rccl", "host", "p2p"), default="rccl",
                    help="sharded data path: the library's RCCL communicator (one process per GPU), host-staged "
                         "gloo (rehearsal only), or p2p: ONE process drives the N GPUs as a team context "
                         "(fri_ctx_create_multi, peer transport over xGMI); under a launcher rank 0 runs the team")
    ap.add_argument("--no-p2p-fallback", action="store_true",
                    help="N>1 rccl: when the RCCL run fails, go to replicas without trying the p2p team first")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N>1: skip the secondary scaling points (weak 2^24 per GPU, strong 2^24)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the side measurements (PCIe-inclusive, serving, prover, 2^28): A/B timing runs")
    args = ap.parse_args()
    plan = launch_plan(args.gpus, os.environ, args.transport)
    if plan == "spawn":
        os.dup2(json_fd, 1)                         # the relayed line goes to the real stdout
        raise SystemExit(_spawn_ranks(args.gpus, sys.argv[1:]))
    if plan == "mismatch":
        msg = f"--gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks"
        os.write(json_fd, (json.dumps({"metric": METRIC, "value": None, "error": msg}) + "\n").encode())
        print(f"[bench] {msg}", file=sys.stderr, flush=True)
        raise SystemExit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local_rank
    if world > 1:
        # one node: RCCL's bootstrap over the loopback interface (the data path
        # is P2P over xGMI either way; the container's other interfaces and
        # its hostname may not be routable / resolvable), unless set already.
        # A job spread over several nodes keeps RCCL's own interface choice.
        if int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) == world:
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        # a rendezvous or collective that makes no progress ends in FRI_ERCCL
        # after this many seconds (fri_amd.h; library default 120): the
        # fallbacks after a failed RCCL run then still fit a bench run's budget
        os.environ.setdefault("FRI_RCCL_TIMEOUT_S", "60")
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()          # does not initialise HIP
        device = local_rank % max(ndev, 1)        # rehearsal with more ranks than GPUs shares devices
        torch.cuda.set_device(device)
        # control plane (unique-id broadcast, barriers, max-over-ranks) on gloo;
        # the data path runs on the library's own RCCL communicator.
        dist.init_process_group("gloo")

    import numpy as np
    import fri_amd

    pg = dist                    # the job's process group (kept when the team runs on rank 0 alone)
    # --transport p2p: one process drives the N GPUs (a team context); under
    # a launcher rank 0 drives them all and the other ranks wait for it
    team_n = (world if world > 1 else args.gpus) if args.transport == "p2p" else 0
    if team_n and world > 1:
        if rank != 0:
            _team_wait(pg)
            return
        dist = None
    ndev_all = _device_count()
    logG = (team_n or world).bit_length() - 1
    mode = args.mode if (team_n or world) > 1 else "single"
    if (team_n or world) > 1 and (1 << logG) != (team_n or world):
        mode = "replicas"                                   # sharding needs a power-of-two world
        team_n = 0
    scaling = "weak"
    if mode == "sharded":
        scaling = args.scaling if args.scaling != "auto" else ("weak" if args.log_n is not None else "strong")
    note = None
    fallback = None

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(step, steps, warmup):
        for _ in range(warmup):
            step()
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        barrier_sync()
        return max_over_ranks(time.perf_counter() - t0)

    res = fri_amd.CommitResult()
    secondary = {}
    dist_report = None
    team_devices = None
    if mode == "sharded" and team_n:
        log_n = (args.log_n or 28) if scaling == "strong" else (args.log_n or 24) + logG
        team_devices = [r % max(ndev_all, 1) for r in range(team_n)]
        ts = _team_stage(fri_amd, team_devices, _shard_points(args, scaling, log_n, logG), args, timed)
        ctx, step, res0, res, d, coeffs, verified = (ts[k] for k in ("ctx", "step", "res0", "res", "d", "coeffs",
                                                                     "verified"))
        secondary.update(ts["secondary"])
        dist_report = ts["dist_report"]
    elif mode == "sharded":
        import torch
        log_n = (args.log_n or 28) if scaling == "strong" else (args.log_n or 24) + logG
        points = _shard_points(args, scaling, log_n, logG)
        ctx = fri_amd.Context(device, max(L for _, L in points) - logG)   # shard-sized (fri_amd.h)
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(fri_amd.Context.unique_id()), dtype=torch.uint8).clone()
        dist.broadcast(uid, 0)

        failed_step = None

        def agreed(step, what):
            nonlocal note, failed_step
            ok, msg = agree_step(dist, world, rank, step, what)
            if not ok:
                note = msg
                failed_step = failed_step or what
            return ok

        attached = False

        def attach():
            nonlocal attached
            if args.transport == "host":
                ctx.attach_torch(rank, world)
            else:
                ctx.attach_rccl(rank, world, bytes(uid.numpy()))
            attached = True

        ok = (agreed(attach, f"attach ({args.transport})")
              and agreed(lambda: ctx.dist_selftest(4096), "transport self-test"))   # transport sanity first
        if ok:
            r_rank, r_world, r_kind = ctx.dist_info()
            dist_report = {"transport": r_kind, "world_reported": r_world, "rank_reported": r_rank}
        for name, L in points:
            if not ok:
                break
            dL = 1 << (L - args.blowup_log)
            cf = _coeffs(42, dL, fri_amd.P)                     # one polynomial for the whole job
            exp = _expected(L, args.blowup_log)
            first = fri_amd.CommitResult()

            def first_commit():
                first_ = ctx.commit_sharded(cf, L)
                ctypes.memmove(ctypes.byref(first), ctypes.byref(first_), ctypes.sizeof(first))
                return True if exp is None else _matches(first_, exp)

            if not agreed(first_commit, f"first sharded commit 2^{L} ({name})"):
                if name.endswith("_primary"):
                    ok = False
                else:
                    secondary[name] = {"error": note}
                    note = None
                    ok = ctx.dist_info()[2] != "none"              # an aborted transport ends the sharded run
                continue
            dptr = ctypes.c_void_p(ctx.input_upload(cf))      # inputs resident: this rank's input buffer
            out = fri_amd.CommitResult() if not name.endswith("_primary") else res

            def sstep(dptr=dptr, dL=dL, L=L, out=out):
                ctx._check(ctx.lib.fri_commit_sharded_device(ctx.h, dptr, dL, L, fri_amd.GENERATOR, None, 0, None,
                                                              ctypes.byref(out)))

            if name.endswith("_primary"):
                res0, d, coeffs, step = first, dL, cf, sstep
                verified = exp is not None
                break
            k = max(3, args.steps // 4)
            el = timed(sstep, k, 1)
            secondary[name] = {"codeword_log2": L, "per_gpu_log2": L - logG, "ms_per_step": round(1000 * el / k, 4),
                               "value": round((1 << L) * k / el, 1), "unit": "field-elems/s", "steps": k,
                               "oracle_verified": exp is not None and _same(out, first) and _matches(out, exp)}
        if not ok and args.transport == "rccl" and failed_step is not None:
            # The RCCL run failed (setup, self-test or the first commit):
            # before the replicas, run the sharded commit once more over the
            # host-staged gloo transport (slow: every collective goes through
            # host memory), so the line still shows whether the coset-sharded
            # path reproduces the oracle's transcript across these GPUs, i.e.
            # whether the failure is RCCL's or the protocol's.  Never `value`.
            if attached:
                try:
                    ctx.detach()
                except fri_amd.FriError:
                    pass
                attached = False
            if "still busy" in (note or ""):
                # a stream that did not drain after the RCCL abort: no more work on this device
                secondary["sharded_host_transport"] = {"skipped": "a stream stayed busy after the RCCL abort"}
            else:
                log_n_max = ctx.log_n_max
                ctx.close()                        # a fresh context for the check (its own streams)
                ctx = fri_amd.Context(device, log_n_max)
                secondary["sharded_host_transport"] = _host_transport_check(
                    fri_amd, ctx, dist, world, rank, logG, args, agree_step, timed)
        if not ok:
            fallback = note or "the sharded setup failed"
            if attached:
                try:
                    ctx.detach()
                except fri_amd.FriError:
                    pass
            ctx.close()
            secondary = {k: v for k, v in secondary.items() if k == "sharded_host_transport"}
            team_status = None
            if args.transport == "rccl" and not args.no_p2p_fallback:
                # Before the replicas: the same coset-sharded commit driven by
                # rank 0 alone as a team context over every GPU of the job
                # (peer transport: device copies over xGMI, no RCCL).  The
                # other ranks wait for its verdict; on success they wait for
                # the end of the job, otherwise everyone goes to replicas.
                print(f"[bench] rank {rank}: {fallback}; trying the p2p team on rank 0", file=sys.stderr, flush=True)
                ts = None
                if rank == 0:
                    team_devices = [r % max(ndev_all, 1) for r in range(world)]
                    try:
                        ts = _team_stage(fri_amd, team_devices, _shard_points(args, scaling, log_n, logG), args,
                                         lambda st, k, w: _plain_timed(st, k, w))
                        team_status = "ok"
                    except Exception as e:  # noqa: BLE001 - reported in the line, then replicas
                        team_status = f"{type(e).__name__}: {e}"
                box = [team_status]
                dist.broadcast_object_list(box, src=0)
                team_status = box[0]
                if team_status == "ok":
                    if rank != 0:
                        _team_wait(pg)
                        return
                    dist = None
                    team_n = world
                    ctx, step, res0, res, d, coeffs, verified = (ts[k] for k in ("ctx", "step", "res0", "res", "d",
                                                                                 "coeffs", "verified"))
                    secondary.update(ts["secondary"])
                    dist_report = ts["dist_report"]
                    fallback = f"RCCL run failed ({fallback}); the p2p team on rank 0 ran the sharded commit instead"
                else:
                    secondary["sharded_p2p_team"] = {"error": team_status}
            if team_status != "ok":
                print(f"[bench] rank {rank}: {fallback}; falling back to replicas", file=sys.stderr, flush=True)
                mode = "replicas"
                scaling = "weak"
    if mode != "sharded":
        log_n = args.log_n or 24
        d = 1 << (log_n - args.blowup_log)
        ctx = fri_amd.Context(device, log_n)
        coeffs = _coeffs(42 + (rank if mode == "replicas" else 0), d, fri_amd.P)   # replicas: a codeword per rank
        res0 = ctx.commit(coeffs, log_n)
        exp = _expected(log_n, args.blowup_log) if mode == "single" else None
        verified = exp is not None and _matches(res0, exp)
        if exp is not None and not verified:
            raise SystemExit("1-GPU transcript differs from the C oracle's (tests/golden/bench_transcripts.json)")
        # inputs resident in HBM: the context's input buffer, filled once
        # before the timed region (fri_ctx_input_upload) and read in place
        dptr = ctypes.c_void_p(ctx.input_upload(coeffs))

        def step():
            ctx._check(ctx.lib.fri_commit_device(ctx.h, dptr, d, log_n, fri_amd.GENERATOR, None, 0, None,
                                                 ctypes.byref(res)))

    solo = world == 1 and not team_n        # one process, one GPU: the side stages run
    elapsed = timed(step, args.steps, args.warmup)
    if args.warmup:
        assert _same(res, res0)

    n = 1 << log_n
    ms_per_step = 1000.0 * elapsed / args.steps
    units_per_step = n if mode == "sharded" else world * n
    value = units_per_step * args.steps / elapsed
    blk_log = log_n - (logG if mode == "sharded" else 0)     # layer-0 elements hashed by one GPU
    # ---- roofline of the dominant kernel: HIP events on the context stream,
    # recorded around every launch of that kernel during profiled steps.
    roofline = None
    breakdown = None
    if not args.no_profile:
        ctx.reset_profile()
        ctx.set_profiling(True)
        prof_steps = max(3, min(args.steps, 10))
        for _ in range(prof_steps):
            step()
        ctx.set_profiling(False)
        ms, launches, nbytes = ctx.profile(DOMINANT)
        if launches:
            avg_ms = ms / launches
            per_launch = nbytes / launches
            hbm_gbs = per_launch / (avg_ms * 1e-3) / 1e9
            # SHA-256 Merkle work is bound by int32 VALU issue:
            # leaf hash 2009 issue units, node hash 3592 (v_alignbit/v_add3
            # are half rate on gfx950).  The leaf kernel hashes 2^L leaves and
            # (15/16) 2^L nodes (levels 1..4).
            nleaf = 1 << blk_log
            units = nleaf * 2009.0 + (15.0 / 16.0) * nleaf * 3592.0
            valu_t = units / (avg_ms * 1e-3) / 1e12
            hbm = {"achieved": round(hbm_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": per_launch}
            valu = {"achieved": round(valu_t, 2), "peak": VALU_PEAK_TOPS, "unit": "T int32 lane-ops/s",
                    "frac": round(valu_t / VALU_PEAK_TOPS, 4), "issue_units_per_launch": units,
                    "measured_ceiling": VALU_MEASURED_TOPS,
                    "frac_of_measured_ceiling": round(valu_t / VALU_MEASURED_TOPS, 4)}
            # the bound is whichever resource the kernel uses the larger share of
            bound, top = ("valu", valu) if valu["frac"] >= hbm["frac"] else ("hbm", hbm)
            roofline = {"bound": bound, "kernel": "k_layer_leaf (layer 0: leaves + tree levels 1-4)",
                        "achieved": top["achieved"], "peak": top["peak"], "unit": top["unit"], "frac": top["frac"],
                        "traffic": None, "avg_launch_ms": round(avg_ms, 4), "launches": launches,
                        "hbm": hbm, "valu": valu}
            # the HBM-shaped kernel of the path: the coset-LDE NTT (algorithmic
            # bytes 4d read + 4n written per commit).  Its passes move more:
            # the first reads 4d and writes 4n, every later pass reads and
            # writes 4n (8-stage passes); PMC puts them at about
            # 0.85 VALU instructions per quad-cycle per SIMD.
            lms, ll, lbytes = ctx.profile("lde")
            if ll:
                lde_s = lms / ll * 1e-3
                lde_gbs = (lbytes / ll) / lde_s / 1e9
                npass = (log_n + 7) // 8 if mode != "sharded" else None
                pass_bytes = (4 * d + 4 * n + 8 * n * (npass - 1)) if npass else None
                roofline["lde_ntt"] = {"bound": "hbm", "limiter": "valu issue (PMC)", "achieved": round(lde_gbs, 2),
                                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(lde_gbs / HBM_PEAK_GBS, 4),
                                       "bytes_per_launch": lbytes / ll, "avg_launch_ms": round(lms / ll, 4),
                                       "passes": npass, "pass_bytes_per_launch": pass_bytes,
                                       "pass_GBs": round(pass_bytes / lde_s / 1e9, 2) if pass_bytes else None}
        breakdown = {}
        for cls in ("lde", "alltoall", "merkle_layer0_leaf", "layer0", "layers", "gather"):
            cms, cl, _ = ctx.profile(cls)
            if cl:
                breakdown[cls] = round(cms / prof_steps, 4)
        traffic, traffic_note = _pmc_traffic(blk_log)
        if roofline is not None:
            roofline["traffic"] = traffic
            roofline["traffic_note"] = traffic_note

    # A second multi-GPU point from the same job: after the RCCL run, rank 0
    # drives every GPU of the job as one team context (peer transport over
    # xGMI) on the primary codeword while the other ranks wait.  Beside
    # `value`, never it.
    if mode == "sharded" and not team_n and world > 1 and not args.no_secondary and pg is not None:
        barrier_sync()
        if rank == 0:
            try:
                ts = _team_stage(fri_amd, [r % max(ndev_all, 1) for r in range(world)],
                                 [("strong_primary", log_n)], args, _plain_timed)
                k = max(3, args.steps // 4)
                el = _plain_timed(ts["step"], k, 1)
                secondary["p2p_team"] = {"codeword_log2": log_n, "ranks": world, "ms_per_step": round(1000 * el / k, 4),
                                         "value": round((1 << log_n) * k / el, 1), "unit": "field-elems/s",
                                         "steps": k, "oracle_verified": bool(ts["verified"]),
                                         "transport": ts["dist_report"],
                                         "what": "the same codeword from ONE process: fri_ctx_create_multi over "
                                                 "the job's GPUs, one fri_commit_device call per step"}
                ts["ctx"].close()
            except Exception as e:  # noqa: BLE001 - reported beside the line
                secondary["p2p_team"] = {"error": f"{type(e).__name__}: {e}"}
        barrier_sync()

    b_field, b_tree = algorithmic_bytes(log_n, d)
    whole = {"B_alg_bytes": b_field + b_tree, "B_field_bytes": b_field, "B_tree_bytes": b_tree,
             "achieved_GBs": round((b_field + b_tree) / (ms_per_step * 1e-3) / 1e9, 2),
             "frac_of_hbm_peak": round((b_field + b_tree) / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
             "sha256_compressions": sha_compressions(log_n, d)}

    # (run before any stage that creates streams of its own: each context's
    # stream should get a hardware queue of its own, GPU_MAX_HW_QUEUES = 4)
    # Queue sharing explains the round-3 gap between the bench and
    # tools/multi_ctx_probe.py, see DESIGN.md §8.
    # Serving throughput: C independent commits in flight on one GPU (one
    # context + stream per host thread, the documented multi-context use).
    # The tree tops of one commit (one workgroup on the serial Fiat-Shamir
    # chain) overlap the leaf hashing of the others.  Beside `value`, never it.
    # The multi-context stages run first (their contexts are destroyed after
    # them), then the commit lanes of the one-context pipelined stage: every
    # active stream then has a hardware queue of its own.
    concurrent = None
    pipelined = None
    if solo and mode == "single" and log_n >= 20 and not args.no_extras:
        single = _concurrent_async_stage(fri_amd, ctx, dptr, d, log_n, res0, K=4, steps=max(12, args.steps))
        concurrent = _concurrent_stage(fri_amd, ctx, dptr, d, log_n, res0, C=3, steps=max(5, args.steps // 2))
        concurrent["single_thread_async"] = single
    if solo and mode == "single" and log_n >= 20 and not args.no_extras:
        pipelined = _pipelined_stage(fri_amd, ctx, dptr, d, log_n, res0, steps=args.steps)
    # the whole commit in VALU terms (verdict r05 item 4): the hash work of
    # every layer over ms_per_step -- what the serial Fiat-Shamir chain costs
    # shows here, not in the dominant kernel's roofline -- and the same work
    # over the pipelined per-commit time (commit lanes fill the idle chip)
    # (on the distinct GPUs the work ran on; replicas: one commit per rank)
    n_ranks_all = (dist_report or {}).get("world_reported", world) if mode == "sharded" else world
    n_dev, oversub = devices_used(team_devices if team_n else None, world, ndev_all, n_ranks_all)
    whole["valu"] = whole_commit_valu(log_n, d, ms_per_step, n_commits=world if mode == "replicas" else 1,
                                      n_dev=n_dev)
    if pipelined and pipelined.get("ms_per_commit"):
        whole["valu_pipelined"] = dict(whole_commit_valu(log_n, d, pipelined["ms_per_commit"]),
                                       lanes=pipelined.get("best_lanes"),
                                       what="the same work over the per-commit time of the best pipelined_commits "
                                            "configuration (commits overlapping on commit lanes)")

    # PCIe-inclusive rate (host coefficients in, result out): never `value`
    pcie = None
    if solo and not args.no_extras:
        k = max(3, min(args.steps, 10))
        t0 = time.perf_counter()
        for _ in range(k):
            ctx.commit(coeffs, log_n)
        pcie = {"ms_per_step": round(1000.0 * (time.perf_counter() - t0) / k, 4),
                "what": f"fri_commit from a pageable host buffer of {d} u32 coefficients (H2D inside the call)"}
        if mode == "single":
            # the same host input through fri_commit_async, two commits in
            # flight: the pinned copy and the upload (copy engine) of commit
            # i+1 overlap commit i
            outs = [fri_amd.CommitResult() for _ in range(k)]
            for t in [ctx.commit_async(coeffs, log_n) for _ in range(2)]:    # warm-up: slot buffers and graphs
                ctx.commit_wait(t)
            t0 = time.perf_counter()
            pend = []
            for i in range(k):
                pend.append(ctx.commit_async(coeffs, log_n))
                if len(pend) == 2:
                    ctx.commit_wait(pend.pop(0), outs[i - 1])
            ctx.commit_wait(pend.pop(0), outs[k - 1])
            pcie["pipelined_ms_per_step"] = round(1000.0 * (time.perf_counter() - t0) / k, 4)
            pcie["pipelined_transcripts_ok"] = all(_same(o, res0) for o in outs)
            pcie["pipelined_what"] = "fri_commit_async from the same host buffer, 2 commits in flight"

    # Decommitment (fri_commit.rs:137-179) on the commit
    # just made: one fri_decommit_query per query index gathers both values and
    # both authentication paths of every layer.  Beside `value`, never it.
    decommit = None
    if solo and mode == "single" and not args.no_extras:
        decommit = _decommit_stage(fri_amd, ctx, res, log_n)

    # Trace side of the prover (BASELINE configs[3] trace length): 2^16 trace
    # -> iNTT -> coset LDE 2^19 -> Merkle commit, device-resident (reported
    # beside the metric, never `value`).
    trace_stage = None
    if solo and log_n >= 19 and not args.no_extras:
        tr = _coeffs(7, 1 << 16, fri_amd.P)
        ctx.trace_commit(tr, 3)
        k = 10
        t0 = time.perf_counter()
        for _ in range(k):
            ctx.trace_commit(tr, 3)
        trace_stage = {"ms_per_call": round(1000.0 * (time.perf_counter() - t0) / k, 4),
                       "what": "fri_trace_commit: 2^16 trace -> iNTT -> LDE on 5*<w_2^19> -> SHA-256 Merkle "
                               "(host trace in, root + coefficients + LDE read back)"}

    # Whole prover slice, BASELINE configs[3]: STARK-101 FibonacciSq trace of
    # 2^16 rows -> LDE 2^19 + Merkle -> alphas -> composition polynomial ->
    # FRI commit -> 3 queries (trace + FRI decommitments); host trace in,
    # transcript out.  Reported beside the metric, never `value`.
    prover = None
    if solo and log_n >= 19 and not args.no_extras:
        prover = _prover_stage(ctx, fri_amd, with_cpu=(rank == 0 and not args.no_cpu_baseline))

    # The 1-GPU point of the 2^28 strong-scaling curve (BASELINE configs[4]'s
    # codeword on one GPU, ~38 GB of HBM), checked against the oracle's
    # transcript.  Beside `value`, never it.
    if solo and mode == "single" and log_n < 28 and not args.no_extras:
        secondary["single_2p28"] = _single_point(fri_amd, device, 28, args.blowup_log, steps=5)

    if team_n:                               # a team: the largest rank's HBM
        hbm_max = float(max(ctx.team_rank(r).device_bytes()[1] for r in range(team_n)))
    else:
        hbm_max = max_over_ranks(float(ctx.device_bytes()[1]))

    cpu = None
    configs0 = None
    if rank == 0 and solo and not args.no_cpu_baseline:
        cpu = _cpu_baseline(coeffs, d, log_n)
        configs0 = _configs0_stage(ctx)

    if rank == 0:
        # the sharded run's size as its communicator (or the team) reports it;
        # n_dev: the GPUs the job actually ran on, fewer than the ranks when
        # ranks share a device (a rehearsal on a box with fewer GPUs than
        # --gpus): such a run reports n_gpus = the distinct devices and keeps
        # its points out of scaling_points
        n_ranks = n_ranks_all
        if mode == "sharded":
            workload = (f"fri_commit codeword 2^{log_n}, blowup {1 << args.blowup_log} (d=2^{log_n - args.blowup_log}), "
                        f"coset-sharded over {n_ranks} {'GPUs' if not oversub else f'ranks on {n_dev} GPU(s)'} "
                        f"(2^{blk_log} per rank), SHA-256 Merkle per layer, "
                        f"{res.n_rounds} rounds")
            if team_n:
                nd = len(set(team_devices or []))
                par = (f"coset-sharded x{n_ranks} in ONE process (team context, peer transport: each collective "
                       f"one pull kernel over xGMI) on {nd} distinct device(s); inputs resident on every rank "
                       f"(FRI_FLAG_RANK_INPUTS)")
                if fallback:
                    par += f" (FALLBACK: {fallback})"
            else:
                par = (f"coset-sharded x{n_ranks} (RCCL all-to-all + pair exchange)" if args.transport == "rccl"
                       else f"coset-sharded x{n_ranks} (host-staged gloo transport, rehearsal)")
        else:
            workload = (f"fri_commit codeword 2^{log_n}, blowup {1 << args.blowup_log} (d=2^{log_n - args.blowup_log}), "
                        f"SHA-256 Merkle per layer, {res.n_rounds} rounds" + (", per GPU" if world > 1 else ""))
            par = f"replicas x{world}" if world > 1 else "single GPU"
            if fallback:
                par += f" (FALLBACK: the coset-sharded path failed: {fallback})"
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "field-elems/s", "n_gpus": n_dev,
            "n_ranks": n_ranks,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (splitmix64 % p coefficients" + (", seed 42)" if mode != "replicas" else ", seed 42+rank)"),
            "config": {"workload": workload, "codeword_log2": log_n, "per_gpu_log2": blk_log,
                       "blowup": 1 << args.blowup_log, "field": "p=3*2^30+1", "parallelism": par,
                       "transport": dist_report},
            "oracle_verified": bool(verified),
            "hbm_bytes_per_rank_max": int(hbm_max),
            "roofline": roofline,
            "whole_commit": whole,
            "scaling_points": (secondary or None) if not oversub else None,
            "breakdown_ms_per_step": breakdown,
            "pcie_inclusive": pcie,
            "decommit": decommit,
            "prover_trace_commit": trace_stage,
            "pipelined_commits": pipelined,
            "concurrent_commits": concurrent,
            "prover_fibsq": prover,
            "cpu_baseline": cpu,
            "configs0_cpu": configs0,
        }
        if fallback:
            line["note"] = fallback
        if oversub:
            line["oversubscribed"] = True
            line["rehearsal_points"] = secondary or None
            line["note"] = ((line.get("note") + "; ") if line.get("note") else "") + (
                f"OVERSUBSCRIBED: {n_ranks} ranks on {n_dev} device(s): a correctness/rehearsal run, "
                f"not a {n_ranks}-GPU scaling point")
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if mode == "sharded" and not team_n:
        ctx.detach()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    elif pg is not None:
        _team_wait(pg)                   # the ranks that waited for this team run


def devices_used(team_devices, world, ndev, n_ranks):
    """(distinct GPUs the job ran on, whether ranks share them): a team's
    device list, else one process per rank on local_rank % ndev."""
    if team_devices is not None:
        n_dev = len(set(team_devices)) or 1
    else:
        n_dev = min(world, max(ndev, 1)) if world > 1 else 1
    return n_dev, n_ranks > n_dev


def _device_count():
    """GPUs visible to this process, without initialising HIP (torch's count
    does not; 1 when torch is unavailable)."""
    try:
        import torch
        return max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 1


def _team_wait(pg):
    """A rank that is not driving the p2p team: wait for rank 0's run to end."""
    pg.barrier()
    pg.destroy_process_group()


def _plain_timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    return time.perf_counter() - t0


def _shard_points(args, scaling, log_n, logG):
    """The sharded run's codewords: the primary (strong 2^28 / weak 2^24 per
    GPU) last, so its plan stays resident, after the secondary points."""
    points = [(f"{scaling}_primary", log_n)]
    if not args.no_secondary:
        for name, L in (("weak_2p24_per_gpu", 24 + logG), ("strong_2p24", 24)):
            if L != log_n:
                points.insert(0, (name, L))
    return points


def _team_stage(fri_amd, devices, points, args, timed):
    """The coset-sharded commit over `devices` from THIS process: one team
    context (fri_ctx_create_multi, peer transport), one fri_commit_device
    call per step (the single-call surface of fri_commit.rs:72-76).  Inputs
    resident on every rank, as in the one-process-per-GPU run: the first
    (checked) commit stages the coefficients into every rank's input buffer
    and the timed steps pass FRI_FLAG_RANK_INPUTS.  Each point's first
    transcript is checked against the C oracle's golden transcript; a
    mismatch raises."""
    G = len(devices)
    logG = G.bit_length() - 1
    ctx = fri_amd.Context.multi(devices, max(L for _, L in points), transport="peer")
    r_rank, r_world, r_kind = ctx.dist_info()
    out = {"ctx": ctx, "secondary": {},
           "dist_report": {"transport": r_kind, "world_reported": r_world, "rank_reported": r_rank,
                           "process": "one process drives every rank (team context)", "devices": devices,
                           "distinct_devices": len(set(devices))}}
    for name, L in points:
        dL = 1 << (L - args.blowup_log)
        cf = _coeffs(42, dL, fri_amd.P)
        exp = _expected(L, args.blowup_log)
        first = ctx.commit(cf, L)          # host input: every rank stages it (ranks 1..G-1: their copies)
        if exp is not None and not _matches(first, exp):
            raise RuntimeError(f"team transcript of 2^{L} differs from the C oracle's")
        # rank 0's input buffer gets the same coefficients; the timed steps
        # reuse the ranks' staged copies (FRI_FLAG_RANK_INPUTS, verified by a
        # per-rank checksum against this buffer on every step)
        dptr = ctypes.c_void_p(ctx.input_upload(cf))
        res = fri_amd.CommitResult()

        def step(dptr=dptr, dL=dL, L=L, res=res):
            ctx._check(ctx.lib.fri_commit_device(ctx.h, dptr, dL, L, fri_amd.GENERATOR, None,
                                                 fri_amd.FLAG_RANK_INPUTS, None, ctypes.byref(res)))

        if name.endswith("_primary"):
            out.update(step=step, res0=first, res=res, d=dL, coeffs=cf, verified=exp is not None, log_n=L)
            break
        k = max(3, args.steps // 4)
        el = timed(step, k, 1)
        out["secondary"][name] = {"codeword_log2": L, "per_gpu_log2": L - logG, "ms_per_step": round(1000 * el / k, 4),
                                  "value": round((1 << L) * k / el, 1), "unit": "field-elems/s", "steps": k,
                                  "oracle_verified": exp is not None and _same(res, first) and _matches(res, exp)}
    return out


def _decommit_stage(fri_amd, ctx, res, log_n, nq=64):
    """fri_decommit_query through the C ABI (preallocated buffers) for nq
    pseudo-random indices of the resident commit (transcript `res`); every
    path of the first query is checked against the committed roots on the
    host (hashlib)."""
    import hashlib
    import numpy as np
    n_layers = ctx.commit_info()[2]
    vals = np.empty(2 * n_layers, dtype=np.uint32)
    total = sum(64 * (log_n - k) for k in range(n_layers))
    buf = ctypes.create_string_buffer(total)
    got = ctypes.c_size_t()
    vptr = vals.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    idx = [(0x9E3779B97F4A7C15 * (i + 1)) % (1 << log_n) for i in range(nq)]

    def query(i):
        ctx._check(ctx.lib.fri_decommit_query(ctx.h, i, vptr, vals.size, buf, total, ctypes.byref(got)))

    query(idx[0])
    ok, off, raw = True, 0, buf.raw
    for k in range(n_layers):
        depth, m = log_n - k, 1 << (log_n - k)
        for v, j, path in ((int(vals[2 * k]), idx[0] % m, raw[off:off + 32 * depth]),
                           (int(vals[2 * k + 1]), (idx[0] % m + m // 2) % m, raw[off + 32 * depth:off + 64 * depth])):
            h = hashlib.sha256(v.to_bytes(8, "big")).digest()
            for lvl in range(depth):
                sib = path[32 * lvl:32 * lvl + 32]
                h = hashlib.sha256(h + sib if j % 2 == 0 else sib + h).digest()
                j //= 2
            ok = ok and h == bytes(res.roots[k])
        off += 64 * depth
    for i in idx[:16]:                      # warm: GPU out of its idle clocks
        query(i)
    ts = []
    for i in idx:
        t0 = time.perf_counter()
        query(i)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    us = 1e6 * ts[len(ts) // 2]
    return {"us_per_query": round(us, 1), "statistic": "median", "queries": nq, "layers": n_layers,
            "first_query_paths_verified": ok,
            "what": "fri_decommit_query: both values and both authentication paths of every layer "
                    "(one gather launch per query, written straight into pinned host memory)"}


def _concurrent_stage(fri_amd, ctx, dptr, d, log_n, res0, C, steps):
    import threading
    ctxs, ptrs, results = [ctx], [dptr], [fri_amd.CommitResult() for _ in range(C)]
    seeds = [42 + (c % 3) for c in range(C)]          # distinct inputs: thread c commits seed 42 + c mod 3
    for c in range(1, C):
        cx = fri_amd.Context(ctx_device(ctx), log_n)
        cx.commit(_coeffs(seeds[c], d, fri_amd.P), log_n)
        p = ctypes.c_void_p(cx.input_upload(_coeffs(seeds[c], d, fri_amd.P)))
        ctxs.append(cx)
        ptrs.append(p)

    def run(c, k):
        for _ in range(k):
            ctxs[c]._check(ctxs[c].lib.fri_commit_device(ctxs[c].h, ptrs[c], d, log_n, fri_amd.GENERATOR, None, 0,
                                                         None, ctypes.byref(results[c])))

    for c in range(C):
        run(c, 1)
    th = [threading.Thread(target=run, args=(c, steps)) for c in range(C)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    exps = [_expected_seed(log_n, sd) for sd in seeds]
    ok = all(exps[c] is not None and _matches(r, exps[c]) for c, r in enumerate(results))
    for cx in ctxs[1:]:
        cx.close()
    return {"commits_in_flight": C, "ms_per_commit": round(1000.0 * wall / (C * steps), 4),
            "value": round(C * steps * (1 << log_n) / wall, 1), "unit": "field-elems/s", "transcripts_ok": ok,
            "what": f"{C} host threads, one fri_ctx + stream each, {steps} commits of 2^{log_n} per thread "
                    "(thread c: seed 42 + c mod 3, transcripts checked against the C oracle's)"}


def _expected_seed(log_n, seed):
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_transcripts.json")) as f:
            return json.load(f).get(f"{log_n}/{seed}/3")
    except (OSError, ValueError):
        return None


def _hip_runtime():
    """The HIP runtime libfri_amd.so is linked against (already loaded in
    this process): device buffers for the bench's extra inputs without a
    second runtime (PyTorch bundles its own libamdhip64)."""
    path = "libamdhip64.so.7"
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64.so" in line and "/torch/" not in line:
                    path = line.split()[-1]
                    break
    except OSError:
        pass
    hip = ctypes.CDLL(path)
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    return hip


def _pipelined_stage(fri_amd, ctx, dptr, d, log_n, res0, steps):
    """ONE context, pipelined: up to `depth` commits pending
    (fri_commit_device_async / fri_commit_wait), each on a commit lane of its
    own (fri_ctx_set_lanes: a stream with its own plan), so one commit's
    serial tree tops overlap the next commit's leaf hashing.  Distinct inputs:
    three polynomials (splitmix64 seeds 42, 43, 44) in device buffers of their
    own, dealt in turn; each buffer stays unchanged while its commits are
    pending (fri_amd.h).  Every collected transcript is checked against the C
    oracle's for its seed (tests/golden/bench_transcripts.json)."""
    seeds = (42, 43, 44)
    exps = [_expected_seed(log_n, sd) for sd in seeds]
    hip = _hip_runtime()
    ptrs = []
    # the uploads go through a stream of their own that is destroyed again:
    # a synchronous hipMemcpy would bring up the null stream, which keeps a
    # hardware queue (GPU_MAX_HW_QUEUES = 4) and leaves one fewer for the lanes
    st = ctypes.c_void_p()
    via_null = os.environ.get("FRI_BENCH_NULL_STREAM_FILL") == "1"
    if not via_null and hip.hipStreamCreate(ctypes.byref(st)) != 0:
        return {"error": "hipStreamCreate failed"}
    for sd in seeds:
        host = _coeffs(sd, d, fri_amd.P)
        p = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(4 * d)) != 0:
            return {"error": "hipMalloc of the input buffers failed"}
        src = host.ctypes.data_as(ctypes.c_void_p)
        rc = (hip.hipMemcpy(p, src, ctypes.c_size_t(4 * d), 1) if via_null else
              hip.hipMemcpyAsync(p, src, ctypes.c_size_t(4 * d), 1, st) or hip.hipStreamSynchronize(st))
        if rc != 0:
            return {"error": "upload of the input buffers failed"}
        ptrs.append(p)
    if not via_null:
        hip.hipStreamDestroy(st)
    out = {}
    steps = max(steps, 60)
    for lanes, depth in ((1, 2), (2, 2), (3, 3), (3, 4), (4, 4)):
        ctx.set_lanes(lanes)
        res = [fri_amd.CommitResult() for _ in range(steps)]

        def run(k):
            pend = []
            for i in range(k):
                pend.append((i, ctx.commit_device_async(ptrs[i % 3], d, log_n)))
                if len(pend) == depth:
                    j, t = pend.pop(0)
                    ctx.commit_wait(t, res[j % steps])
            for j, t in pend:
                ctx.commit_wait(t, res[j % steps])

        run(2 * depth)                                              # warm-up: lane plans and slot graphs
        t0 = time.perf_counter()
        run(steps)
        wall = time.perf_counter() - t0
        ok = all(exps[i % 3] is not None and _matches(r, exps[i % 3]) for i, r in enumerate(res))
        out[f"lanes_{lanes}_depth_{depth}"] = {"lanes": lanes, "depth": depth, "ms_per_commit": round(1000.0 * wall / steps, 4),
                                 "value": round(steps * (1 << log_n) / wall, 1), "unit": "field-elems/s",
                                 "transcripts_ok": ok}
    ctx.set_lanes(fri_amd.DEFAULT_LANES)
    # lane 0's commits from the other buffers staged their inputs in the
    # context's input buffer (dptr, fri_amd.h): put the seed-42 polynomial back
    ctx._check(ctx.lib.fri_commit_device(ctx.h, ptrs[0], d, log_n, fri_amd.GENERATOR, None, 0, None,
                                         ctypes.byref(fri_amd.CommitResult())))
    for p in ptrs:
        hip.hipFree(p)
    best = min(out.values(), key=lambda v: v["ms_per_commit"])
    out.update({"ms_per_commit": best["ms_per_commit"], "value": best["value"], "best_lanes": best["lanes"],
                "transcripts_ok": all(v["transcripts_ok"] for v in out.values() if isinstance(v, dict)),
                "hbm_bytes": ctx.device_bytes()[1],
                "what": f"{steps} commits of 2^{log_n} on ONE fri_ctx, `depth` pending, dealt to `lanes` commit lanes "
                        "(fri_commit_device_async / fri_commit_wait); 3 distinct polynomials (seeds 42-44), "
                        "each transcript checked against the C oracle's"})
    return out


def _concurrent_async_stage(fri_amd, ctx, dptr, d, log_n, res0, K, steps, depth=2):
    """K contexts (one stream each) driven from ONE host thread: commits of
    resident coefficients dealt round-robin with fri_commit_device_async, up
    to `depth` in flight per context, collected with fri_commit_wait."""
    ctxs, ptrs = [ctx], [dptr]
    seeds = [42 + (j % 3) for j in range(K)]          # distinct inputs: context j commits seed 42 + j mod 3
    for j in range(1, K):
        cx = fri_amd.Context(ctx_device(ctx), log_n)
        cx.commit(_coeffs(seeds[j], d, fri_amd.P), log_n)
        p = ctypes.c_void_p(cx.input_upload(_coeffs(seeds[j], d, fri_amd.P)))
        ctxs.append(cx)
        ptrs.append(p)

    def run(n, outs):
        pend = []
        for i in range(n):
            j = i % K
            if len(pend) == depth * K:
                jj, t, k = pend.pop(0)
                ctxs[jj].commit_wait(t, outs[k])
            pend.append((j, ctxs[j].commit_device_async(ptrs[j], d, log_n), i))
        for jj, t, k in pend:
            ctxs[jj].commit_wait(t, outs[k])

    for cx in ctxs:
        cx.set_lanes(1)                               # one stream per context: the concurrency is across contexts
    run(depth * K, [fri_amd.CommitResult() for _ in range(depth * K)])       # warm-up: slot graphs
    outs = [fri_amd.CommitResult() for _ in range(steps)]
    t0 = time.perf_counter()
    run(steps, outs)
    wall = time.perf_counter() - t0
    exps = {sd: _expected_seed(log_n, sd) for sd in set(seeds)}
    ok = all(exps[seeds[i % K]] is not None and _matches(r, exps[seeds[i % K]]) for i, r in enumerate(outs))
    ctx.set_lanes(fri_amd.DEFAULT_LANES)
    for cx in ctxs[1:]:
        cx.close()
    return {"contexts": K, "in_flight_per_context": depth, "ms_per_commit": round(1000.0 * wall / steps, 4),
            "value": round(steps * (1 << log_n) / wall, 1), "unit": "field-elems/s", "transcripts_ok": ok,
            "what": f"one host thread, {K} fri_ctx (one stream each), {steps} commits of 2^{log_n} dealt round-robin "
                    "with fri_commit_device_async / fri_commit_wait; context j commits seed 42 + j mod 3, every "
                    "transcript checked against the C oracle's"}


def ctx_device(ctx):
    return getattr(ctx, "device", 0)


def _prover_stage(ctx, fri_amd, with_cpu, log_t=16, log_b=3, queries=3, a1=3141592):
    ch = fri_amd.Channel()
    pr = fri_amd.prove_fibsq(a1, log_t, log_b, queries, ch, ctx=ctx)        # warm-up + plan build
    ok = fri_amd.verify_fibsq(ch.proof, pr.a_last, log_t, log_b, queries, len(pr.fri.roots))
    k = 5
    t0 = time.perf_counter()
    for _ in range(k):
        fri_amd.prove_fibsq(a1, log_t, log_b, queries, fri_amd.Channel(), ctx=ctx)
    ms = 1000.0 * (time.perf_counter() - t0) / k
    out = {"ms_per_proof": round(ms, 4), "verified": bool(ok), "fri_layers": len(pr.fri.roots),
           "proof_messages": len(ch.proof), "proof_bytes": ch.proof_size(),
           "what": f"STARK-101 FibonacciSq prover: trace 2^{log_t} -> LDE 2^{log_t + log_b} + Merkle -> alphas -> "
                   f"composition polynomial -> FRI commit ({len(pr.fri.roots)} layers) -> {queries} queries; "
                   f"host trace in, transcript out (BASELINE configs[3])"}
    # the same proof through the C++ host mirror (no interpreter in the query
    # loop), when stark-prover_amd/build/prover_native is built
    exe = os.path.join(ROOT, "stark-prover_amd", "build", "prover_native")
    if os.path.exists(exe):
        # its Gpu::thread_default would open every visible GPU
        # (fri_ctx_create_default): pin it to this rank's device
        env = dict(os.environ, FRI_DEVICES=str(ctx_device(ctx)))
        env.pop("FRI_TRANSPORT", None)
        try:
            r = subprocess.run([exe, str(log_t), str(log_b), str(queries), "10"], capture_output=True, text=True,
                               timeout=120, env=env)
            out["native_cpp"] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception as e:  # noqa: BLE001
            out["native_cpp"] = {"error": str(e)}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        try:
            import fri_oracle as fo
            lib = fo.load_c_oracle()
            och = fo.OrcChannel()
            lib.orc_channel_init(ctypes.byref(och))
            root = ctypes.create_string_buffer(32)
            al = (ctypes.c_uint64 * 3)()
            r = fo.OrcFriResult()
            t0 = time.perf_counter()
            lib.orc_fibsq_prove_commit(a1, log_t, log_b, 5, 5, fo.P, ctypes.byref(och), root, al, ctypes.byref(r),
                                       None, None, None, None)
            t = time.perf_counter() - t0
            out["cpu_baseline"] = {"ms_per_proof": round(1000.0 * t, 2), "cores": lib.orc_num_threads(),
                                   "kind": "port", "matches_gpu": root.raw == pr.trace_root and
                                   [bytes(r.roots[j]) for j in range(r.n_layers)] == pr.fri.roots,
                                   "sample": "OpenMP C restatement of the commit phase (trace LDE + Merkle, "
                                             "composition, FRI), queries excluded"}
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": str(e)}
    return out


SOURCE_GLOBS = ("stark-prover_amd/csrc/*.hip", "stark-prover_amd/csrc/*.hpp", "include/fri_amd.h",
                "stark-prover_amd/Makefile")


def source_hash():
    """SHA-256 over the library's sources and build flags (the files of
    SOURCE_GLOBS, sorted by path): what a PMC traffic figure was measured on.
    tools/pmc_traffic.py stores it beside the figure."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for pat in SOURCE_GLOBS:
        for path in sorted(glob.glob(os.path.join(ROOT, pat))):
            h.update(os.path.relpath(path, ROOT).encode() + b"\0")
            with open(path, "rb") as f:
                h.update(f.read())
            h.update(b"\0")
    return h.hexdigest()


def _pmc_traffic(log_n, path=None):
    """HBM bytes per launch of the dominant kernel from the committed
    rocprofv3 PMC summary (profiles/pmc_traffic.json), and a note.  The
    figure is used only when it was collected on the library built from the
    same sources (source_hash); otherwise traffic is null and the note says
    why: a kernel change must not carry a stale figure."""
    path = path or os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            j = json.load(f)
        ent = j.get(str(log_n), {})
        dom = ent.get(DOMINANT)
        if not dom:
            return None, f"no PMC figure for 2^{log_n} in profiles/pmc_traffic.json"
        want = source_hash()
        if ent.get("source_hash") != want:
            return None, (f"profiles/pmc_traffic.json was collected on sources {str(ent.get('source_hash'))[:12]}, "
                          f"this build is {want[:12]}: re-collect (tools/collect_profiles.sh)")
        return dom["hbm_bytes_per_launch"], f"rocprofv3 PMC FETCH_SIZE + WRITE_SIZE, sources {want[:12]}"
    except (OSError, ValueError, KeyError) as e:
        return None, f"profiles/pmc_traffic.json unreadable: {e}"


def _single_point(fri_amd, device, log_n, blowup_log, steps):
    """One more 1-GPU codeword size (its own context), timed over `steps`
    commits on resident inputs and checked against the oracle transcript."""
    d = 1 << (log_n - blowup_log)
    try:
        cx = fri_amd.Context(device, log_n)
    except fri_amd.FriError as e:
        return {"error": str(e)}
    try:
        r0 = cx.commit(_coeffs(42, d, fri_amd.P), log_n)
        exp = _expected(log_n, blowup_log)
        p = ctypes.c_void_p(cx.input_upload(_coeffs(42, d, fri_amd.P)))
        r = fri_amd.CommitResult()

        def st():
            cx._check(cx.lib.fri_commit_device(cx.h, p, d, log_n, fri_amd.GENERATOR, None, 0, None, ctypes.byref(r)))

        st()
        t0 = time.perf_counter()
        for _ in range(steps):
            st()
        el = time.perf_counter() - t0
        return {"codeword_log2": log_n, "n_gpus": 1, "ms_per_step": round(1000 * el / steps, 4),
                "value": round((1 << log_n) * steps / el, 1), "unit": "field-elems/s", "steps": steps,
                "hbm_bytes": cx.device_bytes()[1],
                "oracle_verified": exp is not None and _matches(r0, exp) and _same(r, r0)}
    except fri_amd.FriError as e:
        return {"error": str(e)}
    finally:
        cx.close()


def _host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "nproc": avail, "sched_getaffinity": avail, "cpu_count": os.cpu_count(),
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
            "share_rule": "the GPU pool allots 16 host CPUs per GPU and asks jobs to size worker pools to that share "
                          "(OMP_NUM_THREADS=16 on the box); nproc / os.cpu_count() show the whole machine"}


def _median_runs(fn, runs, warmup=1):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2], ts


def _cpu_baseline(coeffs, d, log_n):
    """Oracle timed on the host (checker only, never the product path),
    following BASELINE.md's CPU-baseline plan:
      * fast: the OpenMP C restatement (NTT LDE, eval-form fold, SHA-256
        Merkle, channel) of the same 2^log_n commit on all host threads,
        median of 5 runs after one warm-up (kind "port": `value`);
      * faithful: the reference algorithm itself (Horner LDE at every
        domain point, coefficient fold + Horner re-evaluation; ops.rs:76-83,
        fri_commit.rs:32-65), one thread like the reference, measured at
        2^10..2^16 and extrapolated to 2^20 / 2^24 by a least-squares fit
        t = a*n*d + b*n (labelled extrapolated)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import fri_oracle as fo
    try:
        lib = fo.load_c_oracle()
    except Exception as e:  # noqa: BLE001
        return {"value": None, "error": f"oracle unavailable: {e}"}
    host = _host_info()
    c64 = np.ascontiguousarray(coeffs.astype(np.uint64))
    pc = c64.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    r = fo.OrcFriResult()

    def fast():
        ch = fo.OrcChannel()
        lib.orc_channel_init(ctypes.byref(ch))
        lib.orc_fri_commit_fast(pc, d, log_n, 5, 5, fo.P, ctypes.byref(ch), None, ctypes.byref(r), None, None)

    t_fast, runs = _median_runs(fast, 5)
    nthreads = lib.orc_num_threads()
    exp = _expected(log_n, 3)
    fast_ok = exp is not None and [bytes(r.roots[k]).hex() for k in range(r.n_layers)] == exp["roots"]
    # Thread scaling of the same restatement at 2^20 (1 .. the allotted
    # share), fitted with Amdahl's t(p) = s + w/p: the whole host's rate is
    # that fit's extrapolation, labelled as such.  The GPU box allots each GPU
    # a share of its host CPUs (OMP_NUM_THREADS, 16 per GPU) and asks jobs to
    # stay within it, so nothing here runs on more threads than that.
    L_s = min(log_n, 20)
    cs20 = np.ascontiguousarray(fo.splitmix64_np(42, 1 << (L_s - 3)))
    p20 = cs20.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))

    def fast20():
        ch = fo.OrcChannel()
        lib.orc_channel_init(ctypes.byref(ch))
        lib.orc_fri_commit_fast(p20, cs20.size, L_s, 5, 5, fo.P, ctypes.byref(ch), None, ctypes.byref(r), None, None)

    scal = []
    for th in sorted({1, 2, 4, 8, nthreads}):
        if th > nthreads:
            continue
        lib.orc_set_num_threads(th)
        scal.append((th, _median_runs(fast20, 3)[0]))
    lib.orc_set_num_threads(nthreads)
    As = np.array([[1.0, 1.0 / th] for th, _ in scal])
    ys = np.array([t for _, t in scal])
    (ser, par), *_ = np.linalg.lstsq(As / ys[:, None], np.ones_like(ys), rcond=None)
    t_share = ser + par / nthreads
    t_all = ser + par / max(1, host["nproc"] or 1)
    all_cores = {"cores": host["nproc"], "extrapolated": True,
                 "value": round((1 << log_n) / (t_fast * t_all / t_share), 1),
                 "model": "Amdahl t(p) = s + w/p fitted to the 2^%d commit at p = %s threads; "
                          "the 2^%d rate scaled by t(share)/t(nproc)" % (L_s, [th for th, _ in scal], log_n),
                 "serial_fraction": round(float(ser / (ser + par)), 4),
                 "measured_2p%d" % L_s: [{"threads": th, "seconds": round(t, 4)} for th, t in scal]}
    # faithful reference algorithm, single thread
    lib.orc_set_num_threads(1)
    pts = []
    for ls in range(10, 17):
        ds = 1 << (ls - 3)
        cs = np.ascontiguousarray(fo.splitmix64_np(42, ds))
        pcs = cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))

        def faithful():
            ch2 = fo.OrcChannel()
            lib.orc_channel_init(ctypes.byref(ch2))
            lib.orc_fri_commit_faithful(pcs, ds, ls, 5, 5, fo.P, ctypes.byref(ch2), None, ctypes.byref(r), None,
                                        None)

        t, _ = _median_runs(faithful, 3 if ls <= 14 else 1, warmup=1 if ls <= 14 else 0)
        pts.append((ls, ds, t))
    lib.orc_set_num_threads(nthreads)
    A = np.array([[(1 << ls) * ds, 1 << ls] for ls, ds, _ in pts], dtype=np.float64)
    y = np.array([t for _, _, t in pts])
    w = 1.0 / y                                       # relative least squares
    (a, b), *_ = np.linalg.lstsq(A * w[:, None], y * w, rcond=None)

    def extrap(L):
        n_, d_ = 1 << L, 1 << (L - 3)
        t = a * n_ * d_ + b * n_
        return {"codeword_log2": L, "seconds": float(f"{t:.4g}"), "value": round(n_ / t, 1), "extrapolated": True}

    return {"value": round((1 << log_n) / t_fast, 1), "unit": "field-elems/s", "cores": nthreads,
            "kind": "port", "host": host, "oracle_verified": fast_ok,
            "cpu_share": {"threads": nthreads, "source": "OMP_NUM_THREADS (the GPU box's host-CPU share per GPU)"},
            "sha256": ("x86 SHA extensions (as the reference's sha2 0.10.8 selects at run time)"
                       if lib.orc_sha_backend() else "portable FIPS 180-4 code (no SHA extensions on this CPU)"),
            "all_cores": all_cores,
            "sample": f"full workload: OpenMP C restatement (NTT LDE, eval-form fold, SHA-256 Merkle, channel) "
                      f"at codeword 2^{log_n} on the box's {nthreads}-thread CPU share, median of 5 runs after "
                      f"1 warm-up: {t_fast:.3f} s (runs {', '.join(f'{t:.3f}' for t in runs)})",
            "faithful": {"kind": "port", "cores": 1,
                         "what": "reference algorithm (Horner LDE + coefficient fold + Horner re-evaluation, "
                                 "SHA-256 rs_merkle tree, hex channel), one thread",
                         "measured": [{"codeword_log2": ls, "d": ds, "seconds": round(t, 5),
                                       "value": round((1 << ls) / t, 1)} for ls, ds, t in pts],
                         "fit": {"model": "t = a*n*d + b*n", "a_ns_per_horner_step": round(a * 1e9, 4),
                                 "b_ns_per_element": round(b * 1e9, 2)},
                         "at_2p20": extrap(20), "at_2p24": extrap(24)}}


def _configs0_stage(ctx):
    """BASELINE configs[0] (benches/poly_ops.rs / poly_lang.rs shape, CPU-only
    in the reference): the reference's two LDE/interpolation primitives at the
    published sizes, restated in the C oracle over p = 3*2^30+1 (one thread),
    printed beside the reference's own criterion numbers (macOS laptop,
    moduli 17 / 7), plus this repo's NTT / iNTT at degree 2^10 on
    the host (oracle) and through the GPU library (host buffers in and out)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import fri_oracle as fo
    lib = fo.load_c_oracle()
    nth = lib.orc_num_threads()
    lib.orc_set_num_threads(1)
    P = fo.P
    p64 = ctypes.POINTER(ctypes.c_uint64)

    def per_call(fn, target_s=0.2):
        k = 1
        while True:
            t0 = time.perf_counter()
            for _ in range(k):
                fn()
            t = time.perf_counter() - t0
            if t >= target_s or k >= 1 << 20:
                return t / k
            k *= 4

    out = {"reference_published": {
        "Eval_17_ns": {"10": 33.752, "100": 603.66, "1000": 6488.7, "5000": 32277.0},
        "interpolate_lagrange_us": {"10": 28.956, "50": 95.849, "100": 215.36, "200": 526.25, "500": 2383.3},
        "source": "criterion screenshots, macOS laptop (results/12:08/..., results/base/langrange_bench.png); "
                  "benches/poly_ops.rs:161-181, benches/poly_lang.rs:33-51; moduli 17 and 7"}}
    ev = {}
    for deg in (10, 100, 1000, 5000):
        c = np.ascontiguousarray(fo.splitmix64_np(3333, deg + 1))
        x = int(fo.splitmix64_np(7, 1)[0])
        reps = max(1, 2_000_000 // (deg + 1))              # one FFI call per 2M Horner steps
        ev[str(deg)] = round(1e9 * per_call(lambda: lib.orc_bench_evaluate(c.ctypes.data_as(p64), deg + 1, x, P,
                                                                           reps)) / reps, 1)
    out["evaluate_horner_ns"] = ev
    lg = {}
    for n in (10, 50, 100, 200, 500):
        xs = np.ascontiguousarray(fo.splitmix64_np(11, n))
        ys = np.ascontiguousarray(fo.splitmix64_np(12, n))
        o = np.zeros(n + 1, dtype=np.uint64)
        lg[str(n)] = round(1e6 * per_call(lambda: lib.orc_interpolate_lagrange(
            xs.ctypes.data_as(p64), ys.ctypes.data_as(p64), n, o.ctypes.data_as(p64), P)), 2)
    out["interpolate_lagrange_us"] = lg
    # degree 2^10: NTT LDE (blowup 8) and coset iNTT interpolate
    c = np.ascontiguousarray(fo.splitmix64_np(42, 1 << 10))
    ev_out = np.zeros(1 << 13, dtype=np.uint64)
    ys = np.ascontiguousarray(fo.splitmix64_np(43, 1 << 10))
    co = np.zeros(1 << 10, dtype=np.uint64)
    out["ntt_lde_2p10_to_2p13_us"] = round(1e6 * per_call(lambda: lib.orc_lde(
        c.ctypes.data_as(p64), 1 << 10, 13, 5, 5, P, ev_out.ctypes.data_as(p64))), 2)
    out["intt_interpolate_2p10_us"] = round(1e6 * per_call(lambda: lib.orc_interpolate_coset(
        ys.ctypes.data_as(p64), 10, 5, 5, P, co.ctypes.data_as(p64))), 2)
    lib.orc_set_num_threads(nth)
    c32, y32 = c.astype(np.uint32), ys.astype(np.uint32)
    gl = ctx.lde(c32, 13)
    gi = ctx.interpolate(y32)
    out["gpu_matches_oracle"] = bool(np.array_equal(gl, ev_out.astype(np.uint32))
                                     and np.array_equal(gi, co[:gi.size].astype(np.uint32)))
    out["gpu_lde_2p10_to_2p13_us"] = round(1e6 * per_call(lambda: ctx.lde(c32, 13)), 2)
    out["gpu_interpolate_2p10_us"] = round(1e6 * per_call(lambda: ctx.interpolate(y32)), 2)
    out["host"] = _host_info()
    out["what"] = ("C oracle over p=3*2^30+1, one thread: Horner evaluate (ops.rs:76-83) at the Eval_17 degrees, "
                   "Lagrange interpolate (interpolation.rs:121-152) at the poly_lang sizes, NTT LDE / iNTT at "
                   "degree 2^10; GPU: fri_lde / fri_interpolate with host buffers (launch + copies dominate)")
    return out


if __name__ == "__main__":
    main()
