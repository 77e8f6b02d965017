// fri_readback.hip — what a commit leaves in HBM, read back: layers and
// tree levels (FRIProof, fri_commit.rs:9-13), authentication paths and whole
// query decommitments (decommit_fri_layers, fri_commit.rs:137-163), and the
// prover entry points built on them (trace commit, FibonacciSq composition
// commit, trace decommitment).
#include "fri_host.hpp"

extern "C" int fri_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out, size_t cap) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const Plan& p = ctx->plan;
    if (!p.valid || layer >= ctx->h_state->n_layers) return fail(ctx, FRI_ESTATE, "no such committed layer");
    if (layer < ctx->sharded_layers && !ctx->team_root)
        return fail(ctx, FRI_ESTATE, "layer was committed sharded: this rank holds only its block (fri_commit_sharded)");
    size_t m = (size_t)1 << (p.log_n - layer);
    if (cap < m) return fail(ctx, FRI_EINVAL, "output buffer too small");
    if (layer < ctx->sharded_layers) return team_layer_copy(ctx, layer, out);     // the ranks' blocks
    // on the context stream: the null stream would hold a hardware queue of
    // its own (GPU_MAX_HW_QUEUES) for the rest of the process, one fewer for
    // the commit lanes and other contexts
    FRI_HIP(ctx, hipMemcpyAsync(out, p.layers + p.layer_off[layer], m * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

extern "C" int fri_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint8_t* out, size_t cap) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const Plan& p = ctx->plan;
    if (!p.valid || layer >= ctx->h_state->n_layers) return fail(ctx, FRI_ESTATE, "no such committed layer");
    if (layer < ctx->sharded_layers && !ctx->team_root)
        return fail(ctx, FRI_ESTATE, "layer was committed sharded: this rank holds only its block (fri_commit_sharded)");
    uint32_t L = p.log_n - layer;
    if (level > L) return fail(ctx, FRI_EINVAL, "level above root");
    size_t cnt = (size_t)1 << (L - level);
    if (cap < cnt * 32) return fail(ctx, FRI_EINVAL, "output buffer too small");
    std::vector<uint32_t> w(cnt * 8);
    if (layer < ctx->sharded_layers) {
        const int rc = team_tree_level_copy(ctx, layer, level, w.data());    // block trees + top tree
        if (rc) return rc;
    } else {
        FRI_HIP(ctx, hipMemcpyAsync(w.data(), p.trees + p.tree_off[layer] + 8 * level_offset(L, level), cnt * 32,
                                    hipMemcpyDeviceToHost, ctx->stream));   // (not the null stream: fri_layer_copy)
        FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    for (size_t i = 0; i < cnt; i++) digest_to_bytes(&w[8 * i], out + 32 * i);
    return FRI_OK;
}

// One query's value and path through the decommitment gather kernel (a
// one-layer DecommitPlan): one launch that writes the big-endian path
// straight into the pinned host buffer, instead of one blocking copy per
// tree level.

extern "C" int fri_auth_path(fri_ctx* ctx, uint32_t layer, uint64_t index, uint32_t* value_out, uint8_t* path,
                             uint32_t* depth_out) {
    if (!ctx || !value_out || !depth_out) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const Plan& p = ctx->plan;
    if (!p.valid || layer >= ctx->h_state->n_layers) return fail(ctx, FRI_ESTATE, "no such committed layer");
    if (layer < ctx->sharded_layers && !ctx->team_root)
        return fail(ctx, FRI_ESTATE, "layer was committed sharded: this rank holds only its block (fri_commit_sharded)");
    uint32_t L = p.log_n - layer;
    if (index >> L) return fail(ctx, FRI_EINVAL, "index out of range");
    if (layer < ctx->sharded_layers) {
        // a team commit: the decommitment of `index` (idx_k = index mod m_k =
        // index for this layer) through the ranks, then this layer's part
        const uint32_t nl = ctx->h_state->n_layers;
        size_t total = 0, off = 0;
        for (uint32_t k = 0; k < nl; k++) {
            if (k == layer) off = total;
            total += (size_t)64 * (p.log_n - k);
        }
        std::vector<uint32_t> vals(2 * (size_t)nl);
        std::vector<uint8_t> pb(total);
        size_t plen = 0;
        const int rc = team_decommit(ctx, index, vals.data(), vals.size(), pb.data(), pb.size(), &plen);
        if (rc) return rc;
        *value_out = vals[2 * layer];
        if (path) memcpy(path, pb.data() + off, (size_t)32 * L);
        *depth_out = L;
        return FRI_OK;
    }
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rc = dq_alloc(ctx);
    if (rc) return rc;
    DecommitPlan dp{};
    dp.index = index;
    dp.log_n = L;
    dp.n_layers = 1;
    dp.layer_off[0] = p.layer_off[layer];
    dp.tree_off[0] = p.tree_off[layer];
    launch_decommit_gather(p.layers, p.trees, dp, ctx->dq_dev, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *value_out = ctx->dq_host[0];
    if (path) memcpy(path, ctx->dq_host + 2, (size_t)32 * L);     // [value, sibling value, path(index), ...]
    *depth_out = L;
    return FRI_OK;
}

// The gather kernel writes a query's values and paths (<= 64 KiB) straight
// into coherent pinned host memory: no device-to-host copy per query (a copy
// of that size took either ~25 or ~130 us per query, varying from process to
// process; the zero-copy write does not go through the copy engines).
int fri::dq_alloc(fri_ctx* ctx) {
    if (!ctx->dq_host) FRI_HIP(ctx, hipHostMalloc(&ctx->dq_host, 65536, hipHostMallocMapped | hipHostMallocCoherent));
    if (!ctx->dq_dev) {
        void* d = nullptr;
        FRI_HIP(ctx, hipHostGetDevicePointer(&d, ctx->dq_host, 0));
        ctx->dq_dev = static_cast<uint32_t*>(d);
    }
    return FRI_OK;
}

extern "C" int fri_decommit_query(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap,
                                  uint8_t* paths, size_t paths_cap, size_t* paths_len) {
    if (!ctx || !values || !paths_len) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const Plan& p = ctx->plan;
    if (!p.valid || ctx->h_state->n_layers == 0) return fail(ctx, FRI_ESTATE, "no committed layers");
    if (ctx->sharded_layers && ctx->team_root)
        return team_decommit(ctx, index, values, values_cap, paths, paths_cap, paths_len);
    if (ctx->sharded_layers)
        return fail(ctx, FRI_ESTATE, "last commit was sharded: each rank holds only its blocks of the large layers");
    DecommitPlan dp{};
    dp.index = index;
    dp.log_n = p.log_n;
    dp.n_layers = ctx->h_state->n_layers;
    uint32_t words = 0;
    for (uint32_t k = 0; k < dp.n_layers; k++) {
        dp.layer_off[k] = p.layer_off[k];
        dp.tree_off[k] = p.tree_off[k];
        dp.path_off[k] = words;
        words += 16 * (p.log_n - k);
    }
    *paths_len = (size_t)words * 4;
    if (values_cap < 2 * (size_t)dp.n_layers) return fail(ctx, FRI_EINVAL, "values buffer too small (2 per layer)");
    if (!paths || paths_cap < (size_t)words * 4) return fail(ctx, FRI_EINVAL, "paths buffer too small (see paths_len)");
    const size_t total = (2 * (size_t)dp.n_layers + words) * 4;
    if (total > 65536) return fail(ctx, FRI_EINVAL, "decommitment too large");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rc = dq_alloc(ctx);
    if (rc) return rc;
    launch_decommit_gather(p.layers, p.trees, dp, ctx->dq_dev, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    memcpy(values, ctx->dq_host, 2 * dp.n_layers * 4);
    memcpy(paths, ctx->dq_host + 2 * dp.n_layers, (size_t)words * 4);
    return FRI_OK;
}
extern "C" int fri_commit_degrees(fri_ctx* ctx, int32_t* out, size_t cap, uint32_t* n_out) {
    if (!ctx || !n_out) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const uint32_t n = ctx->h_state->n_layers;
    *n_out = n;
    if (n && (!out || cap < n)) return fail(ctx, FRI_EINVAL, "degree buffer too small (n_layers entries)");
    for (uint32_t k = 0; k < n; k++) out[k] = ctx->h_state->deg[k];
    return FRI_OK;
}
// Trace side of the prover (the reference's
// src/trace and src/prover are empty): interpolate the trace on its subgroup
// <w_t> (Polynomial::interpolate, ops.rs:239 -> interpolation.rs:121-152),
// evaluate it on the blown-up coset offset*<w_n> (the LDE, as
// fri_commit.rs:78 evaluates), and Merkle-commit the LDE (merkle/mod.rs:10-26),
// all device-resident.  The LDE tree stays in the context (trace_tree).
extern "C" int fri_trace_commit(fri_ctx* ctx, const uint32_t* trace, uint32_t log_t, uint32_t log_blowup,
                                uint32_t offset, uint8_t root32[32], uint32_t* coeffs_out, size_t* coeff_len,
                                uint32_t* lde_out) {
    if (!ctx || !trace || !root32) return fail(ctx, FRI_EINVAL, "null argument");
    const uint32_t L = log_t + log_blowup;
    if (L > ctx->log_n_max || L < 1) return fail(ctx, FRI_EINVAL, "log_t + log_blowup out of range for context");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    const size_t nt = (size_t)1 << log_t, n = (size_t)1 << L;
    if (!check_canonical(trace, nt)) return fail(ctx, FRI_EINVAL, "trace value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    ctx->trace_valid = false;
    if (ctx->trace_tree_cap < n) {
        dfree(ctx, ctx->trace_tree);
        dfree(ctx, ctx->trace_lde);
        ctx->trace_tree = nullptr;
        ctx->trace_lde = nullptr;
        ctx->trace_tree_cap = 0;
        FRI_HIP(ctx, dalloc(ctx, &ctx->trace_tree, (n * 2) * 32));
        FRI_HIP(ctx, dalloc(ctx, &ctx->trace_lde, n * 4));
        ctx->trace_tree_cap = n;
    }
    hipStream_t s = ctx->stream;
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, trace, nt * 4, hipMemcpyHostToDevice, s));
    // coefficients: c_j = nt^-1 sum_i trace_i w_t^-ij
    NttPlan ip{};
    ip.log_n = log_t;
    ip.tw = ctx->tw_inv;
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_t, 1u, inv_std((uint32_t)(nt % P)), s);
    ip.post_lo = ctx->pow_lo;
    ip.post_hi = ctx->pow_hi;
    launch_ntt(ip, ctx->scratch_a, nt, ctx->scratch_b, s);
    // LDE on offset * <w_n>
    NttPlan lp = lde_plan(ctx, L);
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, L, offset, 1u, s);
    lp.pre_lo = ctx->pow_lo;
    lp.pre_hi = ctx->pow_hi;
    launch_ntt(lp, ctx->scratch_b, nt, ctx->trace_lde, s);
    // Merkle tree of the LDE, every level kept
    LayerTask t{};
    t.values = ctx->trace_lde;
    t.tree = ctx->trace_tree;
    t.L = L;
    launch_layer(t, s);
    FRI_HIP(ctx, hipGetLastError());
    uint32_t w[8];
    FRI_HIP(ctx, hipMemcpyAsync(w, ctx->trace_tree + 8 * level_offset(L, L), 32, hipMemcpyDeviceToHost, s));
    if (coeffs_out) FRI_HIP(ctx, hipMemcpyAsync(coeffs_out, ctx->scratch_b, nt * 4, hipMemcpyDeviceToHost, s));
    if (lde_out) FRI_HIP(ctx, hipMemcpyAsync(lde_out, ctx->trace_lde, n * 4, hipMemcpyDeviceToHost, s));
    FRI_HIP(ctx, hipStreamSynchronize(s));
    digest_to_bytes(w, root32);
    ctx->trace_valid = true;
    ctx->trace_log_t = log_t;
    ctx->trace_log_b = log_blowup;
    ctx->trace_offset = offset;
    if (coeffs_out && coeff_len) {
        size_t len = nt;
        while (len > 0 && coeffs_out[len - 1] == 0) len--;      // Polynomial::new trim (ops.rs:19-37)
        *coeff_len = len;
    }
    ctx->err.clear();
    return FRI_OK;
}
// ------------------------------------------------------------- prover ----
// STARK-101 FibonacciSq composition + FRI commit of the composition
// polynomial (fri_prover.hip has the constraint system).  Reads the trace LDE
// kept by the last fri_trace_commit; CP evaluations -> coset iNTT -> the
// commit of fri_commit_device (layer 0 re-extends exactly those evaluations).
extern "C" int fri_fibsq_composition_commit(fri_ctx* ctx, uint32_t log_t, uint32_t log_blowup, uint32_t offset,
                                            uint32_t a_last, const uint32_t alphas[3],
                                            const fri_channel_state* chan_in, uint32_t flags,
                                            fri_commit_result* out) {
    if (!ctx || !alphas || !out) return fail(ctx, FRI_EINVAL, "null argument");
    if (!ctx->trace_valid || ctx->trace_log_t != log_t || ctx->trace_log_b != log_blowup ||
        ctx->trace_offset != offset)
        return fail(ctx, FRI_ESTATE, "no resident trace commit with this (log_t, log_blowup, offset)");
    if (log_blowup < 1 || ((uint32_t)1 << log_blowup) > FIBSQ_MAX_B)
        return fail(ctx, FRI_EINVAL, "log_blowup must be 1..4 (deg CP = T needs n > T)");
    if (log_t < 2) return fail(ctx, FRI_EINVAL, "trace needs at least 4 rows");
    if (a_last >= P || alphas[0] >= P || alphas[1] >= P || alphas[2] >= P)
        return fail(ctx, FRI_EINVAL, "a_last / alphas not canonical");
    if (flags & FRI_FLAG_FORCE_BETAS) return fail(ctx, FRI_EINVAL, "forced betas are not supported here");
    const uint32_t L = log_t + log_blowup;
    const size_t n = (size_t)1 << L, T = (size_t)1 << log_t;
    const uint32_t B = 1u << log_blowup;
    FibsqParams q{};
    q.log_n = L;
    q.B = B;
    q.offset_m = to_mont(offset);
    const uint32_t w = root_of_unity(L), g = root_of_unity(log_t), wB = root_of_unity(log_blowup);
    q.w_m = to_mont(w);
    q.winv_m = to_mont(inv_std(w));
    q.glast_m = to_mont(pow_std(g, T - 1));
    q.gprev_m = to_mont(pow_std(g, T - 2));
    q.a_last = a_last;
    for (int j = 0; j < 3; j++) q.alpha_m[j] = to_mont(alphas[j]);
    const uint32_t offT = pow_std(offset, T);
    for (uint32_t j = 0; j < B; j++) {
        const uint32_t z = sub(mul_std(offT, pow_std(wB, j)), 1u);
        if (z == 0) return fail(ctx, FRI_EINVAL, "offset^T lies in <w_B>: the coset meets the trace domain");
        q.zinv_m[j] = to_mont(inv_std(z));
    }
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rl = use_lane(ctx, 0);            // the commit below runs on lane 0: so does its input
    if (rl) return rl;
    hipStream_t s = ctx->stream;
    size_t sp = span_begin(ctx, "composition", (uint64_t)n * 8);
    launch_fibsq_cp(ctx->trace_lde, ctx->scratch_c, q, s);
    // coefficients: c_j = n^-1 offset^-j sum_i cp_i w^-ij   (fri_interpolate)
    NttPlan ip{};
    ip.log_n = L;
    ip.tw = ctx->tw_inv;
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, L, inv_std(offset), inv_std((uint32_t)(n % P)), s);
    ip.post_lo = ctx->pow_lo;
    ip.post_hi = ctx->pow_hi;
    launch_ntt(ip, ctx->scratch_c, n, ctx->scratch_b, s);
    span_end(ctx, sp);
    FRI_HIP(ctx, hipGetLastError());
    int rc = run_commit(ctx, nullptr, ctx->scratch_b, n, L, offset, chan_in, flags, nullptr, out);
    if (rc) return rc;
    if (ctx->h_state->deg[0] > (int32_t)T) {
        ctx->h_state->n_layers = 0;      // no proof of a violated trace is served
        return fail(ctx, FRI_EDEGREE, "composition polynomial degree exceeds T: the trace violates the constraints");
    }
    return FRI_OK;
}

// STARK-101 FibonacciSq trace.  The recurrence is one serial dependency
// chain (each row needs the previous two), so it runs on the host: ~2
// 64-bit mulmods per row, far below one kernel launch for any T here.
extern "C" int fri_fibsq_trace(uint32_t a1, uint32_t log_t, uint32_t* out) {
    if (!out || log_t > 30) return FRI_EINVAL;
    if (a1 >= P) return FRI_EINVAL;
    const size_t T = (size_t)1 << log_t;
    uint64_t x = 1, y = a1;
    out[0] = 1;
    if (T > 1) out[1] = a1;
    for (size_t i = 2; i < T; i++) {
        const uint64_t z = (x * x % P + y * y % P) % P;
        out[i] = (uint32_t)z;
        x = y;
        y = z;
    }
    return FRI_OK;
}

extern "C" int fri_trace_decommit(fri_ctx* ctx, uint64_t index, uint64_t stride, uint32_t count, uint32_t* values,
                                  uint8_t* paths, size_t paths_cap) {
    if (!ctx || !values || !paths) return fail(ctx, FRI_EINVAL, "null argument");
    if (!ctx->trace_valid) return fail(ctx, FRI_ESTATE, "no resident trace commit");
    if (count < 1 || count > 8) return fail(ctx, FRI_EINVAL, "count must be 1..8");
    const uint32_t L = ctx->trace_log_t + ctx->trace_log_b;
    if (index >> L) return fail(ctx, FRI_EINVAL, "index out of range");
    const size_t words = (size_t)count * 8 * L;
    if (paths_cap < words * 4) return fail(ctx, FRI_EINVAL, "paths buffer too small (32 bytes per level per value)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rc = dq_alloc(ctx);
    if (rc) return rc;
    launch_trace_gather(ctx->trace_lde, ctx->trace_tree, L, index, stride, count, ctx->dq_dev, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    memcpy(values, ctx->dq_host, count * 4);
    memcpy(paths, ctx->dq_host + count, words * 4);
    return FRI_OK;
}
