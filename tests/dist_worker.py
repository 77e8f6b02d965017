"""Worker for the multi-rank tests (launched by torch.distributed.run, gloo).

    python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
        --master-port P tests/dist_worker.py MODE LOG_N SEED OUT_DIR

MODE "model": CPU model of the sharded commit (tests/dist_model.py) with the
              C oracle doing the per-block work and gloo doing the exchanges.
MODE "gpu":   libfri_amd.so fri_commit_sharded on GPU 0 (every rank shares
              the one GPU), collectives staged through the host over gloo.
MODE "gpu_soak": LOG_N operations on one context per rank: sharded commits
              (collective, the same sequence on every rank) mixed with this
              rank's own synchronous and pipelined 1-GPU commits, every
              transcript checked against the C oracle's.
MODE "gpu_fuzz": LOG_N random sharded commits (fuzz_case(SEED + i, W): ragged
              coefficient counts, blowups 1..16, early-ending and zero
              polynomials, random cosets, prefilled channels), one result per
              case, plus each case's transport schedule.
MODE "gpu_shard": the same on a context sized for one rank's shard only
              (log_n_max = log_n - log2 W; BASELINE configs[4] is 2^28 over
              8 ranks); reports the rank's HBM bytes, no 1-GPU re-commit.
Each rank writes OUT_DIR/rank<r>.json with its transcript-visible result.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "stark-prover_amd", "python"))
sys.path.insert(0, HERE)


def make_coeffs(kind, seed, d):
    """Coefficient vectors of the multi-rank tests (numpy uint32).  Beyond
    random full-degree polynomials they steer the sharded degree bookkeeping
    (next_fri_polynomial, fri_commit.rs:32-50) through its other branches:
      odd_only   every even coefficient zero: round 1 takes add_assign's early
                 return (the degree of beta*odd, untrimmed);
      low_degree only the first 3 coefficients nonzero (degree 2, two rounds):
                 the commit ends while the layers are still sharded, and the
                 final value comes from the rank holding coefficient 0;
      tail_heavy the top coefficient nonzero, a zero run below it: the degree
                 maxima come from the last rank's chunk."""
    import numpy as np

    import fri_oracle as fo
    c = fo.splitmix64_np(seed, d).astype(np.uint32)
    if kind == "odd_only":
        c[0::2] = 0
    elif kind == "low_degree":
        c[3:] = 0
    elif kind == "tail_heavy":
        c[d // 3:d - 1] = 0
    elif kind != "random":
        raise ValueError(kind)
    return c


def fuzz_case(i, world):
    """Case i of the sharded fuzz (the same on every rank and in the test):
    (log_n, coefficients as uint64, offset, prefilled channel state or None).
    log_n >= 20 so that the commit really shards (SHARD_MIN_LOG)."""
    import numpy as np
    P = 3221225473
    r = np.random.default_rng(50000 + i)
    log_n = int(r.integers(20, 23))
    n = 1 << log_n
    kind = int(r.integers(0, 7))
    if kind == 0:
        d = n >> int(r.integers(0, 5))                 # blowup 1..16 (d > n/G: chunked coset reduction)
    elif kind == 1:
        d = int(r.integers(0, n + 1))                  # any count, 0 included
    elif kind == 2:
        d = int(r.integers(1, 65))                     # ends inside the sharded layers
    else:
        d = n >> 3
    c = r.integers(0, P, size=d, dtype=np.uint64)
    if d and kind == 3:
        c[int(r.integers(0, d)):] = 0                  # trailing zeros: the degree from some rank's chunk
    elif d and kind == 4:
        c[:] = 0                                       # zero polynomial
    elif d and kind == 5:
        c[1:] = 0                                      # constant
    elif d and kind == 6:
        c[0::2] = 0                                    # add_assign's early return in round 1
    offset = int(r.integers(1, P))
    state = r.bytes(32) if r.integers(0, 2) else None
    return log_n, c, offset, state


def fuzz_forced_betas(i):
    """Forced betas (the FRI_FLAG_FORCE_BETAS test hook) for every third
    fuzz case, a third of them zero: beta = 0 keeps the odd part's degree in
    the reference's untrimmed scalar_mul (src/polynomial/ops.rs:87-98), which
    the sharded degree bookkeeping must reproduce from the chunk maxima."""
    import numpy as np
    if i % 3:
        return None
    r = np.random.default_rng(90000 + i)
    fb = r.integers(1, 3221225473, size=32, dtype=np.uint64)
    fb[r.random(32) < 0.34] = 0
    return [int(x) for x in fb]


def main():
    mode, log_n, seed, out_dir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    blowup_log = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    kind = os.environ.get("POLY_KIND", "random")
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import numpy as np

    import fri_oracle as fo
    if mode == "gpu_soak":
        # LOG_N = number of operations; the operation sequence is drawn from
        # SEED on every rank alike (sharded commits are collective), the
        # polynomials of the local commits from SEED + rank (they differ per rank)
        import ctypes
        import fri_amd
        corc = fo.load_c_oracle()

        def oracle_t(c, L):
            cs = np.ascontiguousarray(c, dtype=np.uint64)
            och = fo.OrcChannel()
            corc.orc_channel_init(ctypes.byref(och))
            res = fo.OrcFriResult()
            assert corc.orc_fri_commit_fast(cs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), c.size, L, 5, 5, fo.P,
                                            ctypes.byref(och), None, ctypes.byref(res), None, None) == 0
            return [bytes(res.roots[k]).hex() for k in range(res.n_layers)], och.state.decode()

        def got_t(r):
            return [bytes(r.roots[k]).hex() for k in range(r.n_layers)], bytes(r.channel_out.digest).hex()

        polys = {}
        for L in (20, 21, 14, 16):
            for j in range(2):
                c = fo.splitmix64_np(8000 + 10 * L + j + (0 if L >= 20 else 100 * (rank + 1)), (1 << L) >> 3)
                polys[(L, j)] = (c.astype(np.uint32), oracle_t(c, L))
        ctx = fri_amd.Context(0, 21)
        ctx.attach_torch(rank, world)
        ctx.set_lanes(3)
        seq = np.random.default_rng(seed)            # same on every rank
        loc = np.random.default_rng(seed + 1 + rank)  # this rank's local choices
        pend, counts, bad = [], {"sharded": 0, "sync": 0, "async": 0}, []

        def wait_one():
            t, key = pend.pop(0)
            if got_t(ctx.commit_wait(t)) != polys[key][1]:
                bad.append(("async", key))

        for i in range(log_n):
            if seq.random() < 0.3:
                L, j = int(seq.choice([20, 21])), int(seq.integers(0, 2))
                r = ctx.commit_sharded(polys[(L, j)][0], L)
                counts["sharded"] += 1
                if got_t(r) != polys[(L, j)][1]:
                    bad.append(("sharded", L, j))
            else:
                L, j = int(loc.choice([14, 16])), int(loc.integers(0, 2))
                if loc.random() < 0.5:
                    counts["sync"] += 1
                    if got_t(ctx.commit(polys[(L, j)][0], L)) != polys[(L, j)][1]:
                        bad.append(("sync", L, j))
                else:
                    if len(pend) == fri_amd.MAX_INFLIGHT:
                        wait_one()
                    pend.append((ctx.commit_async(polys[(L, j)][0], L), (L, j)))
                    counts["async"] += 1
        while pend:
            wait_one()
        ctx.detach()
        ctx.close()
        with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"counts": counts, "bad": bad}, f)
        dist.barrier()
        dist.destroy_process_group()
        return
    if mode == "gpu_fuzz":
        import fri_amd
        ctx = fri_amd.Context(0, 22)
        ctx.attach_torch(rank, world)
        cases = []
        for i in range(log_n):                         # LOG_N = number of cases
            ln, c, offset, state = fuzz_case(seed + i, world)
            fb = fuzz_forced_betas(seed + i)
            try:
                r = ctx.commit_sharded(c.astype(np.uint32), ln, offset, channel_state=state, forced_betas=fb)
            except fri_amd.FriError as e:
                cases.append({"error": f"{e.code}: {e}"})
                continue
            cases.append({"roots": [bytes(r.roots[k]).hex() for k in range(r.n_layers)],
                          "betas": [int(r.betas[j]) for j in range(r.n_rounds)],
                          "final_value": int(r.final_value), "final_degree": int(r.final_degree),
                          "state": bytes(r.channel_out.digest).hex(), "transport_log": ctx.transport_log()})
        ctx.detach()
        ctx.close()
        with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
            json.dump({"cases": cases}, f)
        dist.barrier()
        dist.destroy_process_group()
        return
    d = (1 << log_n) >> blowup_log
    coeffs = make_coeffs(kind, seed, d)
    if mode == "model":
        coeffs = [int(x) for x in coeffs]
    if mode == "gpu_shard":
        import time
        import fri_amd
        logw = world.bit_length() - 1
        t0 = time.monotonic()
        ctx = fri_amd.Context(0, log_n - logw)
        ctx.attach_torch(rank, world)
        ctx.dist_selftest(1024)
        r = ctx.commit_sharded(coeffs, log_n)
        tlog = ctx.transport_log()
        cur, peak = ctx.device_bytes()
        res = {"roots": [bytes(r.roots[k]).hex() for k in range(r.n_layers)],
               "betas": [int(r.betas[i]) for i in range(r.n_rounds)],
               "final_value": int(r.final_value), "final_degree": int(r.final_degree),
               "state": bytes(r.channel_out.digest).hex(), "hbm_bytes": cur, "hbm_peak_bytes": peak,
               "ctx_log_n_max": log_n - logw, "seconds": round(time.monotonic() - t0, 2),
               "transport_log": tlog}
        try:
            ctx.layer(0, log_n)
            res["layer0_refused"] = False
        except fri_amd.FriError:
            res["layer0_refused"] = True
        last = r.n_layers - 1
        res["last_layer_constant"] = bool((ctx.layer(last, log_n) == r.final_value).all())
        # decommit_fri over the sharded proof (collective), then verify_fri on
        # the whole transcript: paths to the roots, folds, final value
        ch = fri_amd.Channel()
        proof = fri_amd.fri_commit_sharded(coeffs, log_n, ch, ctx)
        fri_amd.decommit_fri(3, (1 << log_n) - 1, proof, ch)
        res["transcript_sha"] = __import__("hashlib").sha256(b"".join(ch.proof)).hexdigest()
        res["verify_fri"] = bool(fri_amd.verify_fri(ch.proof, log_n, proof.n_layers, 3, (1 << log_n) - 1))
        print(f"[rank {rank}] 2^{log_n} sharded over {world}: {res['seconds']} s, HBM {peak / 2**30:.2f} GiB",
              file=sys.stderr, flush=True)
        ctx.detach()
        ctx.close()
    elif mode == "model":
        import dist_model
        res = dist_model.sharded_commit(coeffs, log_n, rank, world, shard_min_log=int(os.environ.get("SHARD_MIN", "8")))
    else:
        import fri_amd
        ctx = fri_amd.Context(0, log_n)
        ctx.attach_torch(rank, world)
        ctx.dist_selftest(1024)
        # a coefficient >= p: rejected on the device by every rank (layer 0's
        # replicated top), after the collectives ran in step on all ranks
        bad = np.array(coeffs, dtype=np.uint32)      # a copy: coeffs stays canonical
        bad[len(bad) // 3] = fo.P
        try:
            ctx.commit_sharded(bad, log_n)
            rejected = False
        except fri_amd.FriError as e:
            rejected = e.code == fri_amd.FRI_EINVAL
        r = ctx.commit_sharded(coeffs, log_n)
        tlog = ctx.transport_log()
        res = {"noncanonical_rejected": rejected, "transport_log": tlog,
               "roots": [bytes(r.roots[k]).hex() for k in range(r.n_layers)],
               "betas": [int(r.betas[i]) for i in range(r.n_rounds)],
               "final_value": int(r.final_value), "final_degree": int(r.final_degree),
               "state": bytes(r.channel_out.digest).hex()}
        # read-back: sharded layers are refused, the locally finished tail is served
        try:
            ctx.layer(0, log_n)
            res["layer0_refused"] = False
        except fri_amd.FriError:
            res["layer0_refused"] = True
        last = r.n_layers - 1
        try:
            tail = ctx.layer(last, log_n)
        except fri_amd.FriError as e:          # the commit ended inside the sharded layers
            assert e.code == fri_amd.FRI_ESTATE and kind == "low_degree", e
            tail = None
        if tail is not None:
            qi = min(1, tail.size - 1)        # a 1-element last layer (blowup 1) has only index 0
            _, path = ctx.auth_path(last, qi, log_n)
        qidx = [0, 1, (1 << log_n) - 1, 0x9E3779B97F4A7C15 % (1 << log_n)]
        dq_sharded = [ctx.decommit_query(i, r.n_layers, log_n, sharded=True) for i in qidx]
        ctx.detach()
        single = ctx.commit(coeffs, log_n)
        res["decommit_matches_single"] = dq_sharded == [ctx.decommit_query(i, single.n_layers, log_n) for i in qidx]
        if tail is None:                      # nothing local to compare: the decommitment covers the layers
            res["tail_matches_single"] = res["auth_matches_single"] = "sharded"
        else:
            res["tail_matches_single"] = bool(np.array_equal(tail, ctx.layer(last, log_n)))
            res["auth_matches_single"] = path == ctx.auth_path(last, qi, log_n)[1]
        res["single_root0"] = bytes(single.roots[0]).hex()
        ctx.close()
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except BaseException:
        # the test reads this file: torchrun's own summary hides the traceback
        import traceback
        rank = os.environ.get("RANK", "x")
        with open(os.path.join(sys.argv[4], f"rank{rank}.err"), "w") as f:
            f.write(traceback.format_exc())
        raise
