// fri_commit.hip — the commit plan (layout and allocation, 1-GPU and
// shard-sized) and the 1-GPU commit of src/fri/fri_commit.rs:72-122: a
// static launch sequence (LDE, then one launch_layer per layer, gated on the
// device) captured once into a hipGraph and replayed per commit.
#include "fri_host.hpp"

// G == 1: the whole-codeword plan of fri_commit.  G > 1: the shard-sized plan
// of rank `rank` (see Plan::sharded); its x^-1 slots hold only the slices the
// rank's folds read, computed directly as (offset^(2^k) w_{n_k}^i)^-1 (the
// same values the whole-domain squaring chain gives: D_k = D_0^(2^k)).
// The plan's layout (offsets and sizes, no allocation): also what
// fri_debug_plan_layout reports, so the shard schedule is checkable on a host.
void fri::plan_layout(Plan& p, size_t d, uint32_t log_n, uint32_t G, uint32_t rank, size_t& lay, size_t& tre,
                        size_t& xin) {
    const bool sharded = G > 1;
    uint32_t logG = 0;
    while ((1u << logG) < G) logG++;
    p.log_n = log_n;
    p.d = d;
    p.rmax = rounds_bound(d, log_n);
    p.sharded = sharded;
    p.G = G;
    p.rank = rank;
    p.k_sw = sharded ? switch_layer(log_n, logG, p.rmax) : -1;
    const bool local_tail = sharded && p.k_sw < p.rmax;
    // coefficient chunks: G * S_0 >= d, and S_k = S_0 / 2^k >= 1 up to k_sw
    // (a pair 2j, 2j+1 of poly_{k-1} then never straddles two ranks' chunks)
    p.cs0 = 0;
    if (sharded) {
        const size_t per = (d + G - 1) / G;
        while (((size_t)1 << p.cs0) < per) p.cs0++;
        if ((int)p.cs0 < p.k_sw) p.cs0 = (uint32_t)p.k_sw;
    }
    std::vector<uint32_t> block_of(G), rank_of(G);
    for (uint32_t r = 0; r < G; r++) block_of[r] = rank_of[r] = r;
    lay = tre = xin = 0;
    for (int k = 0; k <= p.rmax; k++) {
        const uint32_t L = log_n - (uint32_t)k;
        const bool blk = sharded && k <= p.k_sw;               // block-local tree
        const uint32_t Lt = blk ? L - logG : L;
        p.layer_off[k] = lay;
        p.tree_off[k] = tre;
        p.xinv_off[k] = xin;
        p.xinv_start[k] = 0;
        p.block[k] = blk ? block_of[rank] : 0u;
        lay += (blk && !(k == p.k_sw && local_tail)) ? ((size_t)1 << Lt) : ((size_t)1 << L);
        tre += 8 * (((size_t)2 << Lt) - 1);
        if (k < p.rmax) {
            if (sharded && k < p.k_sw) {                        // sharded fold: this rank's half-block slice
                const size_t B = (size_t)1 << Lt;
                p.xinv_start[k] = fold_xinv_start(block_of[rank], G, B);
                xin += B / 2;
                advance_blocks(block_of, rank_of, G);
            } else {
                xin += ((size_t)1 << L) / 2;
            }
        }
    }
    p.layer_off[p.rmax + 1] = lay;
    p.tree_off[p.rmax + 1] = tre;
    p.xinv_off[p.rmax + 1] = xin;
}

int fri::plan_build(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t G, uint32_t rank) {
    Plan& p = ctx->plan;
    const bool sharded = G > 1;
    auto same = [&](const Plan& q) {
        return q.d == d && q.log_n == log_n && q.offset == offset && q.sharded == sharded && q.G == G && q.rank == rank;
    };
    if (p.valid && same(p)) return FRI_OK;
    // another shape: every lane's plan goes (after its pending commits); the
    // same shape on other lanes: only this lane's plan is built
    bool stale = p.valid;
    for (const Lane& ln : ctx->lanes) stale = stale || (ln.plan.valid && !same(ln.plan));
    if (stale) plan_free(ctx);
    const size_t n = (size_t)1 << log_n;
    size_t lay, tre, xin;
    plan_layout(p, d, log_n, G, rank, lay, tre, xin);
    p.offset = offset;
    p.in_cap = d ? d : 1;
    p.coef_cap = d / 2 + 1;
    p.coefF_cap = 0;
    if (sharded) {
        // chunks of poly_1 .. poly_k_sw, then the local tail's full poly_{k_sw+1} ..
        const size_t S1 = p.cs0 >= 1 ? ((size_t)1 << (p.cs0 - 1)) : 1;
        const size_t Ssw = (size_t)1 << (p.cs0 - (uint32_t)p.k_sw);
        const bool local_tail = p.k_sw < p.rmax;
        p.coef_cap = std::max(S1, local_tail ? G * Ssw / 2 : (size_t)0) + 1;
        if (local_tail && p.k_sw >= 1) p.coefF_cap = G * Ssw;
    }
    const size_t nhi = log_n > POW_LO_LOG ? ((size_t)1 << (log_n - POW_LO_LOG)) : 1;
    if (dalloc(ctx, &p.d_in, p.in_cap * 4) != hipSuccess || dalloc(ctx, &p.coefA, p.coef_cap * 4) != hipSuccess ||
        dalloc(ctx, &p.coefB, p.coef_cap * 4) != hipSuccess ||
        (p.coefF_cap && dalloc(ctx, &p.coefF, p.coefF_cap * 4) != hipSuccess) ||
        dalloc(ctx, &p.layers, lay * 4) != hipSuccess ||
        dalloc(ctx, &p.trees, tre * 4) != hipSuccess || dalloc(ctx, &p.xinv, (xin ? xin : 1) * 4) != hipSuccess ||
        dalloc(ctx, &p.pre_lo, ((size_t)1 << POW_LO_LOG) * 4) != hipSuccess ||
        dalloc(ctx, &p.pre_hi, nhi * 4) != hipSuccess ||
        dalloc(ctx, &p.wgmax, 6 * ((log_n > 8 ? ((size_t)1 << (log_n - 8)) : 1) + 16) * 4) != hipSuccess) {
        // only the partial plan goes: the other lanes' plans (and lane 0's
        // input buffer, which fri_ctx_input_buffer handed out) stay valid
        plan_release(ctx, p);
        return fail(ctx, FRI_ENOMEM, "device allocation failed for commit plan");
    }
    hipStream_t s = ctx->stream;
    launch_pow_table(p.pre_lo, p.pre_hi, log_n, offset, 1u, s);
    if (sharded) {
        // every slot from its own points; the layer buffer (rewritten by every
        // commit, and at least as large as any slot) holds the points
        uint32_t offk = offset;                               // offset^(2^k)
        for (int k = 0; k < p.rmax; k++) {
            const uint32_t L = log_n - (uint32_t)k;
            const size_t cnt = p.xinv_off[k + 1] - p.xinv_off[k];
            const uint32_t first = mul_std(offk, pow_std(root_of_unity(L), (uint64_t)p.xinv_start[k]));
            launch_coset_points(p.layers, cnt, first, L, s);
            launch_batch_inverse(p.layers, p.xinv + p.xinv_off[k], cnt, 1, s);
            offk = mul_std(offk, offk);
        }
    } else if (p.rmax > 0) {
        // Domain inverses for every fold, built with the batch-inverse kernel:
        // xinv_0[i] = (offset*w_n^i)^-1, xinv_k[i] = xinv_{k-1}[i]^2 (D_k = D_{k-1}^2).
        launch_coset_points(ctx->scratch_a, n / 2, offset, log_n, s);
        launch_batch_inverse(ctx->scratch_a, p.xinv + p.xinv_off[0], n / 2, 1, s);
        for (int k = 1; k < p.rmax; k++)
            launch_square_mont(p.xinv + p.xinv_off[k - 1], p.xinv + p.xinv_off[k], ((size_t)1 << (log_n - k)) / 2, s);
    }
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipStreamSynchronize(s));
    p.valid = true;
    return FRI_OK;
}

// poly_r coefficient buffer: poly_0 is the commit's input (p.src, only ever
// read), then A/B alternate.
uint32_t* fri::coef_buf(Plan& p, int r) {
    if (r == 0) return const_cast<uint32_t*>(p.src);
    return (r % 2 == 1) ? p.coefA : p.coefB;
}

// Layer k of the resident plan as a commit-mode LayerTask.
LayerTask fri::commit_task(fri_ctx* ctx, int k) {
    Plan& p = ctx->plan;
    LayerTask t{};
    t.prev = k ? p.layers + p.layer_off[k - 1] : nullptr;
    t.xinv = k ? p.xinv + p.xinv_off[k - 1] : nullptr;
    t.values = p.layers + p.layer_off[k];
    t.tree = p.trees + p.tree_off[k];
    t.L = p.log_n - (uint32_t)k;
    t.k = k;
    t.coef_in = coef_buf(p, k ? k - 1 : 0);
    t.coef_out = k ? coef_buf(p, k) : nullptr;
    t.d0 = p.d;
    t.wgmax = p.wgmax;
    t.st = ctx->d_state;
    return t;
}

// Enqueue the whole commit on ctx->stream (captured into a graph or eager):
// LDE, then per layer k = 0..rmax one launch_layer (gated on the device).
static void enqueue_commit(fri_ctx* ctx) {
    Plan& p = ctx->plan;
    hipStream_t s = ctx->stream;
    const uint32_t log_n = p.log_n;
    const size_t n = (size_t)1 << log_n;
    NttPlan np = lde_plan(ctx, log_n);
    np.pre_lo = p.pre_lo;
    np.pre_hi = p.pre_hi;
    np.scratch = p.trees;                 // free until layer 0's leaf kernel (>= 16n words)
    size_t sp = span_begin(ctx, "lde", p.d * 4 + n * 4);
    launch_ntt(np, p.src, p.d, p.layers + p.layer_off[0], s);
    span_end(ctx, sp);
    for (int k = 0; k <= p.rmax; k++) {
        const uint32_t L = log_n - (uint32_t)k;
        if (L <= TAIL_LOG) {
            // the remaining small layers: one single-workgroup launch
            LayerTask ts[TAIL_LOG + 1];
            uint32_t nt = 0;
            for (int kk = k; kk <= p.rmax; kk++) ts[nt++] = commit_task(ctx, kk);
            size_t spk = span_begin(ctx, k == 0 ? "layer0" : "layers", 0);
            launch_tail(ts, nt, s);
            span_end(ctx, spk);
            break;
        }
        const LayerTask t = commit_task(ctx, k);
        // Algorithmic bytes of layer 0's leaf kernel: read the values and the
        // input coefficients (degree scan), write tree levels 0..4.
        uint64_t leaf_nodes = 0;
        for (uint32_t j = 0; j <= 4 && j <= L; j++) leaf_nodes += (uint64_t)1 << (L - j);
        const uint64_t leaf_bytes = ((uint64_t)4 << L) + 4 * (uint64_t)p.d + 32 * leaf_nodes;
        size_t spl = (k == 0 && L >= 19) ? span_begin(ctx, "merkle_layer0_leaf", leaf_bytes) : (size_t)-1;
        size_t spk = span_begin(ctx, k == 0 ? "layer0" : "layers", 0);
        launch_layer(t, s, spl == (size_t)-1 ? nullptr : ctx->spans[spl].e);
        span_end(ctx, spk);
    }
}

// Reset `h` (the pinned DevState a commit starts from and copies out to) and
// make it the resident commit's state.
void fri::init_state(fri_ctx* ctx, DevState* h, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas) {
    ctx->h_state = h;
    ctx->res_lane = ctx->cur_lane;
    memset(h, 0, sizeof(DevState));      // n_layers = 0: nothing readable until this commit succeeds
    ctx->commit_gen++;
    if (chan_in && chan_in->has_state) {
        for (int i = 0; i < 8; i++)
            h->chan[i] = ((uint32_t)chan_in->digest[4 * i] << 24) | ((uint32_t)chan_in->digest[4 * i + 1] << 16) |
                         ((uint32_t)chan_in->digest[4 * i + 2] << 8) | chan_in->digest[4 * i + 3];
        h->chan_has = 1;
    }
    h->deg0max = -1;
    h->final_degree = -1;
    for (int r = 0; r < MAXR; r++) { h->newmax[r] = -1; h->evenmax[r] = -1; h->oddmax[r] = -1; }
    for (int r = 0; r <= MAXR; r++) h->deg[r] = -1;
    if ((flags & FRI_FLAG_FORCE_BETAS) && forced_betas) {
        h->forced = 1;
        for (int r = 0; r < MAXR; r++) h->forced_beta[r] = forced_betas[r];
    }
}
// Validate, build the plan and enqueue one commit on the context stream with
// its DevState in `hs` (h_sync, or slot `slot` of the pipelined commits: each
// slot replays its own graph, whose copy-out node targets that slot).
// The argument checks of a 1-GPU commit (everything but the coefficients,
// which the device validates): run before anything is copied or enqueued.
int fri::commit_validate(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t flags,
                           const uint32_t* forced_betas) {
    if (log_n < 1 || log_n > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n out of range for context");
    const size_t n = (size_t)1 << log_n;
    if (d > n) return fail(ctx, FRI_EDEGREE, "more coefficients than domain points (domain would be exhausted)");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    if ((flags & FRI_FLAG_FORCE_BETAS) && !forced_betas) return fail(ctx, FRI_EINVAL, "forced betas missing");
    if (forced_betas && (flags & FRI_FLAG_FORCE_BETAS) && !check_canonical(forced_betas, MAXR))
        return fail(ctx, FRI_EINVAL, "forced beta not canonical");
    return FRI_OK;
}

int fri::commit_enqueue(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                          uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                          const uint32_t* forced_betas, int slot) {
    int rv = commit_validate(ctx, d, log_n, offset, flags, forced_betas);
    if (rv) return rv;
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rc = plan_build(ctx, d, log_n, offset);     // a new plan waits for the pending commits (plan_free)
    if (rc) return rc;
    Plan& p = ctx->plan;
    hipStream_t s = ctx->stream;
    ctx->sharded_layers = 0;
    DevState* hs = slot < 0 ? ctx->h_sync : ctx->h_slot[slot];
    init_state(ctx, hs, chan_in, flags, forced_betas);
    ctx->commit_log_n = log_n;
    // The input.  The context's input buffer (fri_ctx_input_buffer) is read
    // in place, on whichever lane: nothing but the caller (or
    // fri_ctx_input_upload) writes it, so a commit reads what the caller put
    // there, whatever was committed before.  Any other input is staged into
    // this plan's private buffer on this lane's stream.
    if (dev_coeffs && d && ctx->user_in && dev_coeffs == ctx->user_in) {
        p.src = ctx->user_in;
    } else {
        if (host_coeffs && d)
            FRI_HIP(ctx, hipMemcpyAsync(p.d_in, host_coeffs, d * 4, hipMemcpyHostToDevice, s));
        else if (dev_coeffs && d && dev_coeffs != p.d_in)
            FRI_HIP(ctx, hipMemcpyAsync(p.d_in, dev_coeffs, d * 4, hipMemcpyDeviceToDevice, s));
        p.src = p.d_in;
    }
    const bool use_graph = !(flags & FRI_FLAG_NO_GRAPH) && !ctx->profiling;
    if (use_graph) {
        // the DevState copies in (from the pinned state just written) and out
        // are nodes of the graph: no host API call between the commits' kernels.
        // One graph per (result slot, input): the input pointer is baked into
        // the LDE and coefficient launches.
        const int gs = slot < 0 ? FRI_MAX_INFLIGHT : slot;
        const int gv = p.src == p.d_in ? 0 : 1;
        hipGraph_t& pg = p.graph[gs][gv];
        hipGraphExec_t& px = p.exec[gs][gv];
        if (px && p.graph_src[gs][gv] != p.src) {       // the caller's buffer moved (a larger d)
            FRI_HIP(ctx, hipStreamSynchronize(s));         // (the old graph may still be running)
            hipGraphExecDestroy(px);
            hipGraphDestroy(pg);
            px = nullptr;
            pg = nullptr;
        }
        if (!px) {
            FRI_HIP(ctx, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            // a failure inside the capture still ends it (the stream must not
            // stay in capture mode) and drops the partial graph
            hipError_t e1 = hipMemcpyAsync(ctx->d_state, hs, sizeof(DevState), hipMemcpyHostToDevice, s);
            if (e1 == hipSuccess) enqueue_commit(ctx);
            const hipError_t e2 =
                e1 == hipSuccess ? hipMemcpyAsync(hs, ctx->d_state, sizeof(DevState), hipMemcpyDeviceToHost, s) : e1;
            hipGraph_t g = nullptr;
            const hipError_t e3 = hipStreamEndCapture(s, &g);
            if (e2 != hipSuccess || e3 != hipSuccess) {
                if (g) hipGraphDestroy(g);
                FRI_HIP(ctx, e2);
                FRI_HIP(ctx, e3);
            }
            pg = g;
            FRI_HIP(ctx, hipGraphInstantiate(&px, g, nullptr, nullptr, 0));
            p.graph_src[gs][gv] = p.src;
        }
        FRI_HIP(ctx, hipGraphLaunch(px, s));
    } else {
        FRI_HIP(ctx, hipMemcpyAsync(ctx->d_state, hs, sizeof(DevState), hipMemcpyHostToDevice, s));
        enqueue_commit(ctx);
        FRI_HIP(ctx, hipGetLastError());
        FRI_HIP(ctx, hipMemcpyAsync(hs, ctx->d_state, sizeof(DevState), hipMemcpyDeviceToHost, s));
    }
    return FRI_OK;
}

// The result of a finished commit from its copied-out DevState.
int fri::commit_finish(fri_ctx* ctx, DevState* h, uint32_t log_n, fri_commit_result* out) {
    if (h->status) {
        h->n_layers = 0;                 // the failed commit's layers are not served by the read-backs
        return fail(ctx, (int)h->status, status_message(h->status));
    }
    memset(out, 0, sizeof *out);
    out->n_layers = h->n_layers;
    out->n_rounds = h->n_rounds;
    out->log_n = log_n;
    out->final_value = h->final_value;
    out->final_degree = h->final_degree;
    for (uint32_t k = 0; k < h->n_layers && k <= (uint32_t)MAXR; k++) digest_to_bytes(h->roots[k], out->roots[k]);
    for (uint32_t r = 0; r < h->n_rounds && r < (uint32_t)MAXR; r++) out->betas[r] = h->beta[r];
    digest_to_bytes(h->chan, out->channel_out.digest);
    out->channel_out.has_state = h->chan_has;
    ctx->err.clear();
    return FRI_OK;
}

int fri::run_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                      uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                      const uint32_t* forced_betas, fri_commit_result* out) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    // (the argument checks before the lane switch; a failure after it leaves
    // the resident commit on its own lane, see settle)
    int rc = commit_validate(ctx, d, log_n, offset, flags, forced_betas);
    if (rc) return rc;
    // synchronous commits run on lane 0 (always built: the fallback lane of
    // the pipelined commits, fri_lanes.hip)
    rc = use_lane(ctx, 0);
    if (rc) return rc;
    rc = commit_enqueue(ctx, host_coeffs, dev_coeffs, d, log_n, offset, chan_in, flags, forced_betas, -1);
    if (rc) return rc;
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->async_unsettled = false;         // pending pipelined commits ran before this one
    if (ctx->profiling) spans_collect(ctx);
    return commit_finish(ctx, ctx->h_state, log_n, out);
}

extern "C" int fri_commit(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n, uint32_t offset,
                          const fri_channel_state* chan_in, uint32_t flags, const uint32_t* forced_betas,
                          fri_commit_result* out) {
    if (d && !coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    if (ctx && ctx->team_root) return team_commit(ctx, coeffs, nullptr, d, log_n, offset, chan_in, flags, forced_betas, out);
    return run_commit(ctx, coeffs, nullptr, d, log_n, offset, chan_in, flags, forced_betas, out);
}

extern "C" int fri_commit_device(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                                 uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                                 const uint32_t* forced_betas, fri_commit_result* out) {
    if (d && !d_coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    if (ctx && ctx->team_root)
        return team_commit(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
    return run_commit(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
}
extern "C" int fri_debug_plan_layout(size_t d, uint32_t log_n, uint32_t world, uint32_t rank, uint64_t* out,
                                     size_t cap) {
    if (!out || log_n < 1 || log_n > 30 || world < 1 || world > 64 || (world & (world - 1)) || rank >= world)
        return FRI_EINVAL;
    uint32_t logG = 0;
    while ((1u << logG) < world) logG++;
    if (world > 1 && log_n < logG + 12) return FRI_EINVAL;
    if (cap < 4 + 5 * (size_t)(MAXR + 1)) return FRI_EINVAL;
    Plan p;
    size_t lay, tre, xin;
    plan_layout(p, d, log_n, world, rank, lay, tre, xin);
    out[0] = (uint64_t)p.rmax;
    out[1] = (uint64_t)(int64_t)p.k_sw;
    out[2] = 4 * (uint64_t)(lay + tre + xin);                 // bytes of layers + trees + x^-1 tables
    out[3] = p.cs0;                                            // sharded: log2 of the coefficient chunk S_0
    for (int k = 0; k <= p.rmax; k++) {
        uint64_t* o = out + 4 + 5 * (size_t)k;
        o[0] = p.layer_off[k + 1] - p.layer_off[k];            // words in layer slot k
        o[1] = p.tree_off[k + 1] - p.tree_off[k];              // words in tree slot k
        o[2] = p.xinv_off[k + 1] - p.xinv_off[k];              // x^-1 entries of fold k
        o[3] = p.xinv_start[k];                                // domain index of the first
        o[4] = p.block[k];                                     // block held of sharded layer k
    }
    return FRI_OK;
}
