// fri_sharded.hip — one rank's coset-sharded commit (fri_commit_sharded*,
// SURVEY.md §8(e)) and the collective decommitment after it.
#include "fri_host.hpp"

int fri::run_commit_sharded(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                              uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                              const uint32_t* forced_betas, fri_commit_result* out) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    const uint32_t G = (uint32_t)ctx->tp.world;
    const uint32_t rank = (uint32_t)ctx->tp.rank;
    uint32_t logG = 0;
    while ((1u << logG) < G) logG++;
    if (G == 1 || log_n < SHARD_MIN_LOG || log_n < logG + 12)
        return run_commit(ctx, host_coeffs, dev_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
    if (!ctx->tp.host && !ctx->tp.comm && !ctx->tp.loop && !ctx->tp.peer)
        return fail(ctx, FRI_ESTATE, "no transport attached (detached or aborted)");
    // a rank holds 1/G of the codeword: its NTT, twiddles and scratch are block-sized
    if (log_n - logG > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n - log2(world) out of range for context");
    const size_t n = (size_t)1 << log_n;
    if (d > n) return fail(ctx, FRI_EDEGREE, "more coefficients than domain points (domain would be exhausted)");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    if ((flags & FRI_FLAG_FORCE_BETAS) && !forced_betas) return fail(ctx, FRI_EINVAL, "forced betas missing");
    if (forced_betas && (flags & FRI_FLAG_FORCE_BETAS) && !check_canonical(forced_betas, MAXR))
        return fail(ctx, FRI_EINVAL, "forced beta not canonical");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rc = use_lane(ctx, 0);            // sharded commits run on lane 0, like every synchronous commit
    if (rc) return rc;
    rc = plan_build(ctx, d, log_n, offset, G, rank);
    if (rc) return rc;
    Plan& p = ctx->plan;
    hipStream_t s = ctx->stream;
    const size_t M = n / G;                                   // coset / block size of layer 0
    rc = dist_buffers(ctx, M, G, (size_t)1 << (log_n - (uint32_t)p.k_sw));   // the layer gathered at the switch
    if (rc) return rc;
    DistBuf& db = ctx->db;
    ctx->tp.log.clear();
    ctx->sharded_layers = (uint32_t)p.rmax + 1;      // lowered when the tail goes local
    init_state(ctx, ctx->h_sync, chan_in, flags, forced_betas);
    FRI_HIP(ctx, hipMemcpyAsync(ctx->d_state, ctx->h_state, sizeof(DevState), hipMemcpyHostToDevice, s));
    // the input: this context's own input buffer (fri_ctx_input_buffer) is
    // read in place, anything else is staged into the plan's private buffer
    // (a team rank copies rank 0's buffer over xGMI; FRI_FLAG_RANK_INPUTS
    // hands it the copy staged there before)
    if (dev_coeffs && d && ctx->user_in && dev_coeffs == ctx->user_in) {
        p.src = ctx->user_in;
    } else {
        if (host_coeffs && d)
            FRI_HIP(ctx, hipMemcpyAsync(p.d_in, host_coeffs, d * 4, hipMemcpyHostToDevice, s));
        else if (dev_coeffs && dev_coeffs != p.d_in && d)   // (Default: a team rank reads rank 0's device buffer)
            FRI_HIP(ctx, hipMemcpyAsync(p.d_in, dev_coeffs, d * 4, hipMemcpyDefault, s));
        p.src = p.d_in;
    }

    size_t sp;
    if (G == 2) {
        // ---- layer 0, two ranks: radix-2 decimation, no exchange ---------
        // P(offset w_n^(bM+j)) = E(offset^2 w_M^j) + (-1)^b offset w_n^j O(offset^2 w_M^j):
        // both size-M NTTs on every rank, then this rank's block.
        sp = span_begin(ctx, "lde", d * 4 + M * 12);
        const size_t de = (d + 1) / 2, dod = d / 2;
        launch_decimate(p.src, d, ctx->scratch_a, ctx->scratch_b, s);
        launch_pow_table(db.pre_lo, db.pre_hi, log_n - 1, mul_std(offset, offset), 1u, s);
        NttPlan np{};
        np.log_n = log_n - 1;
        np.tw = ctx->tw_fwd;
        np.pre_lo = db.pre_lo;
        np.pre_hi = db.pre_hi;
        launch_ntt(np, ctx->scratch_a, de, db.cyc, s);
        launch_ntt(np, ctx->scratch_b, dod, db.recv, s);
        launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_n - 1, root_of_unity(log_n), offset, s);   // offset * w_n^j
        launch_radix2_block(db.cyc, db.recv, ctx->pow_lo, ctx->pow_hi, p.layers + p.layer_off[0], M, rank, s);
        span_end(ctx, sp);
    } else {
        // ---- layer 0: coset LDE slice evals[rank + G*m] -------------------
        const uint32_t sft = mul_std(offset, pow_std(root_of_unity(log_n), rank));   // s = offset * w_n^rank
        sp = span_begin(ctx, "lde", d * 4 + M * 8);
        // P mod (x^M - s^M) has P's own coefficients when d <= M (blowup >= G):
        // the NTT then reads the input directly (and skips its zero rows)
        const bool fold_chunks = d > M;
        if (fold_chunks) launch_coset_coeffs(p.src, d, db.recv, M, pow_std(sft, M), s);
        launch_pow_table(db.pre_lo, db.pre_hi, log_n - logG, sft, 1u, s);
        NttPlan np{};
        np.log_n = log_n - logG;
        np.tw = ctx->tw_fwd;
        np.pre_lo = db.pre_lo;
        np.pre_hi = db.pre_hi;
        launch_ntt(np, fold_chunks ? db.recv : p.src, fold_chunks ? M : d, db.cyc, s);
        span_end(ctx, sp);
        sp = span_begin(ctx, "alltoall", M * 4);
        rc = tp_alltoall(ctx, db.cyc, db.recv, (M / G) * 4, s);                       // coset slices -> blocks
        if (rc) return rc;
        launch_cyclic_to_block(db.recv, p.layers + p.layer_off[0], M, G, s);
        span_end(ctx, sp);
    }

    // per-layer coefficient-task grid (workgroups over this rank's chunk S_k)
    auto coef_grid = [&](int kk) {
        const size_t S = (size_t)1 << (p.cs0 - (uint32_t)kk);
        return (uint32_t)std::min<size_t>(2048, std::max<size_t>(1, (S + 8191) / 8192));
    };
    // what the sharded top kernels read per layer (ShardTop), for every layer
    // this commit may run sharded: the block -> rank map follows the folds
    {
        std::vector<uint32_t> bo(G), ro(G);
        for (uint32_t r = 0; r < G; r++) bo[r] = ro[r] = r;
        std::vector<ShardTop> sh(MAXR + 1);
        const bool sched = ctx->tp.loop && !db.sched_h.empty();
        for (int kk = 0; kk <= p.k_sw && kk <= MAXR; kk++) {
            ShardTop& t = sh[kk];
            t.rec_out = db.rec;
            t.rec_mx = p.wgmax;
            t.rec_c0 = kk ? coef_buf(p, kk) : p.src;
            t.rec_R = coef_grid(kk);
            t.G = G;
            t.recs_in = db.rec + REC_WORDS;
            t.sched_on = sched ? 1u : 0u;
            t.sched_deg = (sched && (size_t)kk < db.sched_h.size()) ? db.sched_h[kk] : -1;
            for (uint32_t b2 = 0; b2 < G; b2++) t.rank_of_block[b2] = (uint8_t)ro[b2];
            advance_blocks(bo, ro, G);
        }
        // the table depends only on the plan, the input pointer and the
        // loopback schedule, so it is uploaded when it changes, from a copy
        // that outlives the call: no host sync in front of the commit's first
        // launch.  The previous
        // sharded call ended with a stream sync, so its upload has completed.
        if (db.shtop_h.size() != sh.size() || memcmp(db.shtop_h.data(), sh.data(), sh.size() * sizeof(ShardTop))) {
            db.shtop_h = sh;
            FRI_HIP(ctx, hipMemcpyAsync(db.shtop, db.shtop_h.data(), sh.size() * sizeof(ShardTop),
                                        hipMemcpyHostToDevice, s));
        }
    }
    std::vector<uint32_t> block_of(G), rank_of(G);
    for (uint32_t r = 0; r < G; r++) block_of[r] = rank_of[r] = r;
    // The fold of sharded layer k-1 into this rank's block of layer k runs
    // inside layer k's leaf kernel (fold, leaves, levels 1-4 in one pass, as
    // on one GPU): its operands, the local and the partner's half-blocks.
    // (It was a separate k_pair_fold launch with a write and a re-read of
    // every folded block.)
    const uint32_t* f_first = nullptr;
    const uint32_t* f_second = nullptr;
    const uint32_t* f_xi = nullptr;
    int k = 0;
    for (;; k++) {
        const uint32_t Lk = log_n - (uint32_t)k;        // full layer size 2^Lk
        const size_t B = (size_t)1 << (Lk - logG);       // block size
        uint32_t* vals = p.layers + p.layer_off[k];     // my block at the start of the layer slot
        const bool last = (k == p.rmax);
        const bool next_sharded = next_layer_sharded(log_n, logG, k, p.rmax);
        const bool fused = f_first != nullptr;          // this layer's block is folded by its leaf kernel
        // exchange of the half-block the partner needs for the next fold
        // (overlaps the rest of the layer's tree); its receive buffer
        // alternates with the layer, because layer k+1's leaf kernel still
        // reads the partner half of exchange k while exchange k+1 lands
        const uint32_t b = block_of[rank];
        const bool isA = b < G / 2;
        const uint32_t partner = isA ? rank_of[b + G / 2] : rank_of[b - G / 2];
        uint32_t* half_in = (k & 1) ? db.half2 : db.half;
        auto exchange = [&]() -> int {
            if (!ctx->tp.host) {
                FRI_HIP(ctx, hipEventRecord(ctx->ev_vals, s));
                FRI_HIP(ctx, hipStreamWaitEvent(ctx->xstream, ctx->ev_vals, 0));
                const int r2 = tp_sendrecv(ctx, isA ? vals + B / 2 : vals, half_in, (B / 2) * 4, (int)partner,
                                           ctx->xstream, 1);
                if (r2) return r2;
                FRI_HIP(ctx, hipEventRecord(ctx->ev_xchg, ctx->xstream));
                return FRI_OK;
            }
            return tp_sendrecv(ctx, isA ? vals + B / 2 : vals, half_in, (B / 2) * 4, (int)partner, s, 1);
        };
        // layer 0's block is complete before its tree starts: exchange first;
        // a fused layer's block is made by its leaf kernel: the exchange goes
        // between the launch of the half it sends and the other half's
        int xrc = FRI_OK;
        if (next_sharded && !fused && (rc = exchange())) return rc;
        std::function<void()> after_part1;
        if (next_sharded && fused) after_part1 = [&]() { xrc = exchange(); };
        // block-local tree (levels 0 .. log2 B), gated on round k-1
        LayerTask tl{};
        tl.values = vals;
        tl.tree = p.trees + p.tree_off[k];
        tl.L = Lk - logG;
        tl.gst = ctx->d_state;
        tl.gidx = k > 0 ? k - 1 : -1;
        if (fused) {
            // the partner's half-block of layer k-1 (exchange k-1) has landed
            if (!ctx->tp.host) FRI_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_xchg, 0));
            tl.prev = f_first;
            tl.prev2 = f_second;
            tl.xinv = f_xi;
            tl.send_half = isA ? 1u : 0u;
        }
        uint64_t leaf_nodes = 0;
        for (uint32_t j = 0; j <= 4 && j <= tl.L; j++) leaf_nodes += (uint64_t)1 << (tl.L - j);
        size_t spl = (k == 0 && tl.L >= 19) ? span_begin(ctx, "merkle_layer0_leaf", ((uint64_t)4 << tl.L) + 32 * leaf_nodes)
                                            : (size_t)-1;
        size_t spk = span_begin(ctx, k == 0 ? "layer0" : "layers", 0);
        // coefficient task of this layer, sharded (next_fri_polynomial,
        // fri_commit.rs:32-50): this rank folds coefficients [rank*S_k,
        // (rank+1)*S_k) of poly_k (k == 0: scans that range of the input) into
        // its chunk buffer, on its own stream, concurrent with the block tree.
        // It needs only round k-1's beta and degree (replicated DevState).
        const size_t Sk = (size_t)1 << (p.cs0 - (uint32_t)k);
        LayerTask tc{};
        tc.k = k;
        tc.coef_in = (k <= 1) ? p.src : coef_buf(p, k - 1);
        tc.ibase = (k <= 1) ? 0 : (size_t)rank * (Sk << 1);
        tc.coef_out = k ? coef_buf(p, k) : nullptr;
        tc.obase = (size_t)rank * Sk;
        tc.jlo = (size_t)rank * Sk;
        tc.jhi = (size_t)(rank + 1) * Sk;
        tc.d0 = d;
        tc.wgmax = p.wgmax;
        tc.st = ctx->d_state;
        const uint32_t Gc = coef_grid(k);
        const bool side = !ctx->profiling;   // (profiled commits keep one stream for the spans)
        // The coefficient task starts when the block tree's leaf kernel has
        // ended, beside its latency-bound mids: next to the VALU-bound leaf
        // kernel it took 4x longer and slowed the leaves
        // (tools/shard_projection.py).  The block top waits for it: it writes
        // this rank's record (block root, the maxima of the coefficient
        // slice, the slice's first coefficient) for the all-gather.
        if (!side) launch_coef(tc, Gc, s);
        // (the ordering calls' errors are returned: without the wait the
        // coefficient task is not ordered after the leaf kernel, without the
        // record the block top's wait binds to an older one and reads stale maxima)
        hipError_t beside_err = hipSuccess;
        auto coef_beside = [&]() {
            beside_err = hipStreamWaitEvent(ctx->cstream, ctx->ev_pre, 0);
            if (beside_err != hipSuccess) return;
            launch_coef(tc, Gc, ctx->cstream);
            beside_err = hipEventRecord(ctx->ev_coef, ctx->cstream);
        };
        tl.shard = db.shtop + k;
        launch_layer(tl, s, side ? ctx->ev_pre : (spl == (size_t)-1 ? nullptr : ctx->spans[spl].e),
                     side ? std::function<void()>(coef_beside) : std::function<void()>(),
                     side ? ctx->ev_coef : nullptr, after_part1);
        if (xrc) return xrc;
        FRI_HIP(ctx, beside_err);
        FRI_HIP(ctx, hipGetLastError());
        // all ranks' records; the replicated top reads the block roots (in
        // block order), the maxima and rank 0's first coefficient from them
        rc = tp_allgather(ctx, db.rec, db.rec + REC_WORDS, REC_WORDS * 4, s);
        if (rc) return rc;
        LayerTask tt = tc;
        tt.tree = db.top + (size_t)k * 2 * 64 * 8;
        tt.L = logG;
        tt.shard = db.shtop + k;
        launch_top(tt, 0, nullptr, G, s);
        span_end(ctx, spk);
        if (last) break;
        if (next_sharded) {
            // fold pairs (i, i + m/2): this rank's first operands are its own
            // block's first half (A) or the partner's (B), the second ones the
            // partner's second half (A) or its own (B); layer k+1's leaf kernel folds them
            f_first = isA ? vals : half_in;
            f_second = isA ? half_in : vals + B / 2;
            // the plan's slot k holds exactly this rank's x^-1 half-block slice
            if (fold_xinv_start(b, G, B) != p.xinv_start[k])
                return fail(ctx, FRI_ESTATE, "shard plan out of step with the block schedule");
            f_xi = p.xinv + p.xinv_off[k];
            advance_blocks(block_of, rank_of, G);
            continue;
        }
        // switch to local: gather layer k in block order, then the 1-GPU pipeline from k+1
        ctx->sharded_layers = (uint32_t)k + 1;   // layer k keeps its block-local tree; k+1.. are local
        sp = span_begin(ctx, "gather", B * 4 * G + Sk * 4 * G);
        rc = tp_allgather(ctx, vals, db.gath, B * 4, s);
        if (rc) return rc;
        // poly_k whole for the local coefficient fold (chunks in rank order
        // are poly_k in coefficient order); at k == 0 every rank has the input
        if (k >= 1) {
            if (p.coefF_cap < G * Sk) return fail(ctx, FRI_ESTATE, "shard plan out of step (coefficient gather)");
            rc = tp_allgather(ctx, tc.coef_out, p.coefF, Sk * 4, s);
            if (rc) return rc;
        }
        // layer kk of the local tail; the first one folds the gathered poly_k
        auto tail_task = [&](int kk) {
            LayerTask t = commit_task(ctx, kk);
            if (kk == k + 1 && k >= 1) t.coef_in = p.coefF;
            return t;
        };
        // the gathered blocks into place and the local layers: the same
        // launches on every commit of this plan (block_of at the switch is
        // fixed by (G, rank)), so they replay as one hipGraph captured on the
        // first commit, without a launch gap per kernel
        auto local_tail = [&]() -> int {
            launch_place_blocks(db.gath, p.layers + p.layer_off[k], B, G, block_of.data(), s);
            FRI_HIP(ctx, hipGetLastError());
            for (int kk = k + 1; kk <= p.rmax; kk++) {
                if (log_n - (uint32_t)kk <= TAIL_LOG) {      // small layers: one launch
                    LayerTask ts[TAIL_LOG + 1];
                    uint32_t nt = 0;
                    for (int k2 = kk; k2 <= p.rmax; k2++) ts[nt++] = tail_task(k2);
                    launch_tail(ts, nt, s);
                    break;
                }
                launch_layer(tail_task(kk), s);
            }
            return FRI_OK;
        };
        // peer transport: every rank has issued its last collective's waits
        // before any rank starts capturing the tail graph on its stream (HIP
        // refuses a wait on an event of a stream that is capturing, even when
        // the event was recorded before the capture began)
        if (ctx->tp.peer && !team_barrier(ctx->tp.team))
            return fail(ctx, FRI_ERCCL, "peer transport: another rank failed (" + ctx->tp.team->why + ")");
        if (ctx->profiling || (flags & FRI_FLAG_NO_GRAPH)) {
            if ((rc = local_tail())) return rc;
        } else {
            // (a tail that begins at layer 1 folds the input itself: its
            // graph names the input pointer, captured again when it changes)
            if (p.tail_exec && p.tail_src != p.src) {
                hipGraphExecDestroy(p.tail_exec);
                hipGraphDestroy(p.tail_graph);
                p.tail_exec = nullptr;
                p.tail_graph = nullptr;
            }
            if (!p.tail_exec) {
                FRI_HIP(ctx, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                rc = local_tail();
                hipGraph_t g = nullptr;
                const hipError_t ec = hipStreamEndCapture(s, &g);
                if (rc || ec != hipSuccess) {
                    if (g) hipGraphDestroy(g);
                    if (rc) return rc;
                    FRI_HIP(ctx, ec);
                }
                p.tail_graph = g;
                FRI_HIP(ctx, hipGraphInstantiate(&p.tail_exec, g, nullptr, nullptr, 0));
                p.tail_src = p.src;
            }
            FRI_HIP(ctx, hipGraphLaunch(p.tail_exec, s));
        }
        span_end(ctx, sp);
        break;
    }
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(ctx->h_state, ctx->d_state, sizeof(DevState), hipMemcpyDeviceToHost, s));
    if ((rc = sync_sharded(ctx, s))) {
        ctx->h_state->n_layers = 0;
        return rc;
    }
    if (ctx->profiling) spans_collect(ctx);
    ctx->commit_log_n = log_n;
    return commit_finish(ctx, ctx->h_state, log_n, out);
}

// decommit_fri_layers (fri_commit.rs:137-163) after a sharded commit: the
// opened elements of a sharded layer live in one rank's block (value and the
// lower levels of the path in its block-local tree; the top log G levels in
// the replicated top tree).  Every rank gathers the openings it holds and
// zeros elsewhere (k_decommit_gather), the G outputs are all-gathered and
// combined by a word-wise max (exactly one rank holds each non-zero word; the
// replicated local layers are equal everywhere).  Collective: every rank
// calls it with the same index and gets the same bytes, which equal
// fri_decommit_query's for a 1-GPU commit of the same codeword.

extern "C" int fri_decommit_query_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap,
                                          uint8_t* paths, size_t paths_cap, size_t* paths_len) {
    if (!ctx || !values || !paths_len) return fail(ctx, FRI_EINVAL, "null argument");
    if (ctx->team_root) {
        settle(ctx);
        if (!ctx->sharded_layers) return fail(ctx, FRI_ESTATE, "last commit was not sharded: use fri_decommit_query");
        return team_decommit(ctx, index, values, values_cap, paths, paths_cap, paths_len);
    }
    return decommit_sharded(ctx, index, values, values_cap, paths, paths_cap, paths_len);
}

int fri::decommit_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                            size_t paths_cap, size_t* paths_len) {
    if (!ctx || !values || !paths_len) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const Plan& p = ctx->plan;
    if (!p.valid || ctx->h_state->n_layers == 0) return fail(ctx, FRI_ESTATE, "no committed layers");
    if (!ctx->sharded_layers || !p.sharded) return fail(ctx, FRI_ESTATE, "last commit was not sharded: use fri_decommit_query");
    if (!ctx->tp.host && !ctx->tp.comm && !ctx->tp.loop && !ctx->tp.peer)
        return fail(ctx, FRI_ESTATE, "no transport attached (detached or aborted)");
    const uint32_t G = p.G;
    if ((uint32_t)ctx->tp.world != G) return fail(ctx, FRI_ESTATE, "transport world differs from the commit's");
    uint32_t logG = 0;
    while ((1u << logG) < G) logG++;
    DecommitPlan dp{};
    dp.index = index;
    dp.log_n = p.log_n;
    dp.n_layers = ctx->h_state->n_layers;
    dp.logG = logG;
    const bool local_tail = p.k_sw < p.rmax;
    uint32_t words = 0;
    for (uint32_t k = 0; k < dp.n_layers; k++) {
        dp.layer_off[k] = p.layer_off[k];
        dp.tree_off[k] = p.tree_off[k];
        dp.path_off[k] = words;
        words += 16 * (p.log_n - k);
        if (k < ctx->sharded_layers) {
            dp.shard_lb1[k] = (uint8_t)(p.log_n - k - logG + 1);
            dp.val_block[k] = ((int)k == p.k_sw && local_tail) ? 0 : 1;   // the switch layer's slot was gathered whole
            dp.owned[k] = (uint64_t)1 << p.block[k];
            dp.top_off[k] = (uint64_t)k * 2 * 64 * 8;
        }
    }
    *paths_len = (size_t)words * 4;
    if (values_cap < 2 * (size_t)dp.n_layers) return fail(ctx, FRI_EINVAL, "values buffer too small (2 per layer)");
    if (!paths || paths_cap < (size_t)words * 4) return fail(ctx, FRI_EINVAL, "paths buffer too small (see paths_len)");
    const size_t tw = 2 * (size_t)dp.n_layers + words;
    if (tw * 4 > 65536) return fail(ctx, FRI_EINVAL, "decommitment too large");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    DistBuf& db = ctx->db;
    constexpr size_t SLOT = 16384;                          // words per rank slot (64 KiB)
    if (!db.dq) FRI_HIP(ctx, dalloc(ctx, &db.dq, (size_t)(64 + 1) * SLOT * 4));
    ctx->tp.log.clear();
    int rc = tp_host_stage(ctx, G * SLOT * 4);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    launch_decommit_gather(p.layers, p.trees, dp, db.dq, s, db.top);
    FRI_HIP(ctx, hipGetLastError());
    if ((rc = tp_allgather(ctx, db.dq, db.dq + SLOT, SLOT * 4, s))) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(ctx->tp.hs, db.dq + SLOT, G * SLOT * 4, hipMemcpyDeviceToHost, s));
    if ((rc = sync_sharded(ctx, s))) return rc;
    const uint32_t* all = reinterpret_cast<const uint32_t*>(ctx->tp.hs);
    std::vector<uint32_t> o(tw, 0u);
    for (uint32_t r = 0; r < G; r++)
        for (size_t i = 0; i < tw; i++) o[i] = std::max(o[i], all[(size_t)r * SLOT + i]);
    memcpy(values, o.data(), 2 * dp.n_layers * 4);
    memcpy(paths, o.data() + 2 * dp.n_layers, (size_t)words * 4);
    return FRI_OK;
}

extern "C" int fri_commit_sharded(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n, uint32_t offset,
                                  const fri_channel_state* chan_in, uint32_t flags, const uint32_t* forced_betas,
                                  fri_commit_result* out) {
    if (d && !coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    if (ctx && ctx->team_root) return team_commit(ctx, coeffs, nullptr, d, log_n, offset, chan_in, flags, forced_betas, out);
    return run_commit_sharded(ctx, coeffs, nullptr, d, log_n, offset, chan_in, flags, forced_betas, out);
}

extern "C" int fri_commit_sharded_device(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                                         uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                                         const uint32_t* forced_betas, fri_commit_result* out) {
    if (d && !d_coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    if (ctx && ctx->team_root)
        return team_commit(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
    return run_commit_sharded(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
}
