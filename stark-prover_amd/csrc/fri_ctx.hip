// fri_ctx.hip — context lifetime (fri_ctx_create / fri_ctx_destroy), the
// timed spans of profiled commits, and the diagnostics of include/fri_amd.h
// (profiling, device-byte accounting, phase stamps).
#include "fri_host.hpp"

static hipEvent_t pool_event(fri_ctx* ctx) {
    if (ctx->event_next == ctx->event_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ctx->event_pool.push_back(e);
    }
    return ctx->event_pool[ctx->event_next++];
}

// Record the begin of a timed span (only while profiling).
size_t fri::span_begin(fri_ctx* ctx, const char* cls, uint64_t bytes) {
    if (!ctx->profiling) return (size_t)-1;
    TimedSpan sp{cls, pool_event(ctx), pool_event(ctx), bytes};
    hipEventRecord(sp.b, ctx->stream);
    ctx->spans.push_back(sp);
    return ctx->spans.size() - 1;
}
void fri::span_end(fri_ctx* ctx, size_t id) {
    if (id == (size_t)-1) return;
    hipEventRecord(ctx->spans[id].e, ctx->stream);
}
void fri::spans_collect(fri_ctx* ctx) {
    for (auto& sp : ctx->spans) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, sp.b, sp.e) == hipSuccess) {
            auto& pe = ctx->prof[sp.cls];
            pe.ms += ms;
            pe.launches += 1;
            pe.bytes += sp.bytes;
        }
    }
    ctx->spans.clear();
    ctx->event_next = 0;
}

// ------------------------------------------------------------ context ----
extern "C" int fri_ctx_create(int device, uint32_t log_n_max, fri_ctx** out) {
    if (!out) return FRI_EINVAL;
    *out = nullptr;
    if (log_n_max < 1 || log_n_max > 30) return FRI_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return FRI_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return FRI_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FRI_ENODEV;
    fri_ctx* ctx = new fri_ctx();
    ctx->device = device;
    ctx->log_n_max = log_n_max;
    const size_t N = (size_t)1 << log_n_max;
    const size_t nhi = log_n_max > POW_LO_LOG ? ((size_t)1 << (log_n_max - POW_LO_LOG)) : 1;
#define CK(expr)                                                    \
    if ((expr) != hipSuccess) { fri_ctx_destroy(ctx); return FRI_ENOMEM; }
    CK(hipSetDevice(device));
    CK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    CK(dalloc(ctx, &ctx->tw_fwd, N * 4));
    CK(dalloc(ctx, &ctx->tw_inv, N * 4));
    CK(dalloc(ctx, &ctx->scratch_a, N * 4));
    CK(dalloc(ctx, &ctx->scratch_b, N * 4));
    CK(dalloc(ctx, &ctx->scratch_c, N * 4));
    CK(dalloc(ctx, &ctx->pow_lo, ((size_t)1 << POW_LO_LOG) * 4));
    CK(dalloc(ctx, &ctx->pow_hi, nhi * 4));
    CK(dalloc(ctx, &ctx->d_state, sizeof(DevState)));
    CK(hipHostMalloc(&ctx->h_sync, sizeof(DevState), hipHostMallocDefault));
    ctx->h_state = ctx->h_sync;
#undef CK
    launch_twiddles(ctx->tw_fwd, log_n_max, false, ctx->stream);
    launch_twiddles(ctx->tw_inv, log_n_max, true, ctx->stream);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) { fri_ctx_destroy(ctx); return FRI_EHIP; }
    *out = ctx;
    return FRI_OK;
}
extern "C" int fri_ctx_destroy(fri_ctx* ctx) {
    if (!ctx) return FRI_EINVAL;
    if (ctx->tp.team && !ctx->team_root) return fail(ctx, FRI_EINVAL, "a rank of a team: destroy the team's context");
    if (ctx->team_root) team_destroy(ctx);       // the other ranks, their workers and communicators
    hipSetDevice(ctx->device);
    if (ctx->stuck) {
        // a stream that stayed busy after the RCCL abort: poll it with the
        // deadline instead of an unbounded synchronize; if it is still busy,
        // leak the context (its kernels may still touch its memory)
        const auto t0 = std::chrono::steady_clock::now();
        const double lim = rccl_timeout_s();
        bool idle = false;
        while (!(idle = (hipStreamQuery(ctx->stream) != hipErrorNotReady &&
                         (!ctx->xstream || hipStreamQuery(ctx->xstream) != hipErrorNotReady) &&
                         (!ctx->cstream || hipStreamQuery(ctx->cstream) != hipErrorNotReady))) &&
               seconds_since(t0) < lim)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (!idle) return FRI_ERCCL;
        ctx->stuck = false;
    }
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    // an upload whose commit was never enqueued (it failed) may still read
    // this context's pinned input buffers on the shared upload stream
    if (ctx->h2d_stream) hipStreamSynchronize(ctx->h2d_stream);
    plan_free(ctx);
    for (Lane& ln : ctx->lanes) {
        if (ln.stream) hipStreamDestroy(ln.stream);
        dfree(ctx, ln.d_state);
        ln = Lane();
    }
    for (auto e : ctx->event_pool) hipEventDestroy(e);
    fri_dist_detach(ctx);
    dfree(ctx, ctx->db.cyc); dfree(ctx, ctx->db.recv); dfree(ctx, ctx->db.half); dfree(ctx, ctx->db.half2);
    dfree(ctx, ctx->db.top); dfree(ctx, ctx->db.pre_lo); dfree(ctx, ctx->db.pre_hi); dfree(ctx, ctx->db.gath);
    dfree(ctx, ctx->db.dq); dfree(ctx, ctx->db.rec); dfree(ctx, ctx->db.shtop);
    if (ctx->xstream) hipStreamDestroy(ctx->xstream);
    if (ctx->ev_vals) hipEventDestroy(ctx->ev_vals);
    if (ctx->ev_xchg) hipEventDestroy(ctx->ev_xchg);
    if (ctx->cstream) hipStreamDestroy(ctx->cstream);
    if (ctx->ev_pre) hipEventDestroy(ctx->ev_pre);
    if (ctx->ev_coef) hipEventDestroy(ctx->ev_coef);
    dfree(ctx, ctx->tw_fwd); dfree(ctx, ctx->tw_inv);
    dfree(ctx, ctx->scratch_a); dfree(ctx, ctx->scratch_b); dfree(ctx, ctx->scratch_c);
    dfree(ctx, ctx->pow_lo); dfree(ctx, ctx->pow_hi);
    dfree(ctx, ctx->d_state);
    if (ctx->dq_host) hipHostFree(ctx->dq_host);
    if (ctx->stall_flag) hipHostFree(ctx->stall_flag);
    if (ctx->interp_tmp) dfree(ctx, ctx->interp_tmp);
    dfree(ctx, ctx->trace_tree);
    dfree(ctx, ctx->trace_lde);
    dfree(ctx, ctx->user_in);
    dfree(ctx, ctx->d_csum);
    if (ctx->h_csum) hipHostFree(ctx->h_csum);
    if (ctx->h_sync) hipHostFree(ctx->h_sync);
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++) {
        if (ctx->h_slot[i]) hipHostFree(ctx->h_slot[i]);
        if (ctx->ev_slot[i]) hipEventDestroy(ctx->ev_slot[i]);
        if (ctx->h_in[i]) hipHostFree(ctx->h_in[i]);
        dfree(ctx, ctx->d_slot_in[i]);
        if (ctx->ev_in[i]) hipEventDestroy(ctx->ev_in[i]);
    }
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
    return FRI_OK;
}

extern "C" const char* fri_last_error(const fri_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }
extern "C" const char* fri_version(void) { return "fri_amd 0.1 (gfx950, p=3*2^30+1)"; }
// Diagnostic: per-layer top-kernel phase stamps of the last commit
// (100 MHz ticks), only in the -DFRI_STAMPS build.
extern "C" int fri_debug_stamps(fri_ctx* ctx, uint64_t* out, size_t cap) {
    if (!ctx || !out) return FRI_EINVAL;
    settle(ctx);
#ifdef FRI_STAMPS
    const size_t n = sizeof(ctx->h_state->stamps) / sizeof(uint64_t);
    if (cap < n) return fail(ctx, FRI_EINVAL, "buffer too small");
    memcpy(out, ctx->h_state->stamps, sizeof(ctx->h_state->stamps));
    return FRI_OK;
#else
    (void)cap;
    return fail(ctx, FRI_ESTATE, "library built without FRI_STAMPS");
#endif
}

extern "C" int fri_set_profiling(fri_ctx* ctx, int enabled) {
    if (!ctx) return FRI_EINVAL;
    ctx->profiling = enabled != 0;
    return FRI_OK;
}
extern "C" int fri_get_profile(fri_ctx* ctx, const char* cls, double* total_ms, uint64_t* launches,
                               uint64_t* bytes) {
    if (!ctx || !cls) return FRI_EINVAL;
    auto it = ctx->prof.find(cls);
    if (it == ctx->prof.end()) {
        if (total_ms) *total_ms = 0;
        if (launches) *launches = 0;
        if (bytes) *bytes = 0;
        return FRI_OK;
    }
    if (total_ms) *total_ms = it->second.ms;
    if (launches) *launches = it->second.launches;
    if (bytes) *bytes = it->second.bytes;
    return FRI_OK;
}
extern "C" int fri_reset_profile(fri_ctx* ctx) {
    if (!ctx) return FRI_EINVAL;
    ctx->prof.clear();
    return FRI_OK;
}
extern "C" int fri_debug_set_device_cap(fri_ctx* ctx, uint64_t cap_bytes) {
    if (!ctx) return FRI_EINVAL;
    ctx->dev_cap = (size_t)cap_bytes;
    return FRI_OK;
}

extern "C" int fri_ctx_device_bytes(fri_ctx* ctx, uint64_t* current, uint64_t* peak) {
    if (!ctx || !current || !peak) return fail(ctx, FRI_EINVAL, "null argument");
    *current = ctx->dev_bytes;
    *peak = ctx->dev_peak;
    if (ctx->team_root)                        // a team: every rank's (fri_debug_team_rank for one)
        for (uint32_t r = 1; r < ctx->team_root->G; r++) {
            *current += ctx->team_root->rk[r]->dev_bytes;
            *peak += ctx->team_root->rk[r]->dev_peak;
        }
    return FRI_OK;
}
