// fri_lanes.hip — commit lanes (a stream + plan each), pipelined commits
// (fri_commit_async / fri_commit_device_async / fri_commit_wait), the
// context's input buffer, and which commit the read-backs serve.
#include "fri_host.hpp"

// Free one plan's buffers and graphs (its lane's stream must be idle).
void fri::plan_release(fri_ctx* ctx, Plan& p) {
    for (int i = 0; i <= FRI_MAX_INFLIGHT; i++)
        for (int v = 0; v < 2; v++) {
            if (p.exec[i][v]) hipGraphExecDestroy(p.exec[i][v]);
            if (p.graph[i][v]) hipGraphDestroy(p.graph[i][v]);
        }
    if (p.tail_exec) hipGraphExecDestroy(p.tail_exec);
    if (p.tail_graph) hipGraphDestroy(p.tail_graph);
    dfree(ctx, p.d_in); dfree(ctx, p.coefA); dfree(ctx, p.coefB); dfree(ctx, p.coefF); dfree(ctx, p.layers);
    dfree(ctx, p.trees); dfree(ctx, p.xinv); dfree(ctx, p.pre_lo); dfree(ctx, p.pre_hi); dfree(ctx, p.wgmax);
    p = Plan();
}

// Every lane's plan: pipelined commits may still use them, so every lane's
// stream is drained first.
void fri::plan_free(fri_ctx* ctx) {
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    for (Lane& ln : ctx->lanes)
        if (ln.stream) hipStreamSynchronize(ln.stream);
    plan_release(ctx, ctx->plan);
    for (Lane& ln : ctx->lanes) plan_release(ctx, ln.plan);
    ctx->lanes_ok = FRI_MAX_INFLIGHT;     // memory is back: every lane may build a plan again
}

// Install lane j in fri_ctx::{plan, stream, d_state} (creating its stream and
// device state on first use); the lane installed before goes back to its slot.
int fri::use_lane(fri_ctx* ctx, int j) {
    if (j == ctx->cur_lane) return FRI_OK;
    Lane& dst = ctx->lanes[j];
    // (each part on its own: a lane whose state allocation failed once gets
    // it on the next use, instead of being installed with a null state)
    if (!dst.stream) FRI_HIP(ctx, hipStreamCreateWithFlags(&dst.stream, hipStreamNonBlocking));
    if (!dst.d_state && dalloc(ctx, &dst.d_state, sizeof(DevState)) != hipSuccess) {
        dst.d_state = nullptr;
        return fail(ctx, FRI_ENOMEM, "lane state");
    }
    Lane& park = ctx->lanes[ctx->cur_lane];
    std::swap(park.plan, ctx->plan);
    std::swap(park.stream, ctx->stream);
    std::swap(park.d_state, ctx->d_state);
    std::swap(dst.plan, ctx->plan);
    std::swap(dst.stream, ctx->stream);
    std::swap(dst.d_state, ctx->d_state);
    ctx->cur_lane = j;
    return FRI_OK;
}
// Pipelined commits may still be running: a call that reads the resident
// commit (its pinned state, layers or trees) drains the stream first.  The
// resident commit's lane is installed first: a call that switched lanes and
// then failed before it enqueued anything (a rejected argument, a plan that
// got no memory) leaves the resident commit on the lane it ran on, so its
// stream, plan and state are the ones the read-backs must use.
void fri::settle(fri_ctx* ctx) {
    if (ctx->res_lane != ctx->cur_lane) (void)use_lane(ctx, ctx->res_lane);   // (a used lane: cannot fail)
    if (!ctx->async_unsettled) return;
    (void)hipStreamSynchronize(ctx->stream);
    ctx->async_unsettled = false;
    if (ctx->h_state->status) ctx->h_state->n_layers = 0;   // a failed commit serves nothing
}
// One upload stream per device, shared by every context of the process: a
// context per host thread or several contexts driven from one thread (one
// commit stream each) then add one stream in all, not one each, and stay
// within the device's hardware queues (GPU_MAX_HW_QUEUES, 4 by default).
// Created on first use and kept for the life of the process.
static hipError_t upload_stream(int device, hipStream_t* out) {
    static std::mutex m;
    static std::map<int, hipStream_t> streams;
    std::lock_guard<std::mutex> g(m);
    auto it = streams.find(device);
    if (it != streams.end()) { *out = it->second; return hipSuccess; }
    hipStream_t st = nullptr;
    const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) streams[device] = *out = st;
    return e;
}

// The lane of the next pipelined commit: the one with the fewest pending
// (un-waited) commits, ties to the lane dealt a ticket longest ago (never
// used first, lowest index first).  A deal by result slot (slot mod lanes)
// put two of every four commits on lane 0 at depth 4 over 3 lanes, because
// the slot a wait frees is reused at once (BENCH_r04: 3.80 ms per commit
// against 3.32 at depth 3).  Deterministic: no device query.
static int pick_lane(fri_ctx* ctx) {
    const int nl = std::max(1, std::min(ctx->max_lanes, ctx->lanes_ok));
    int best = 0, best_n = FRI_MAX_INFLIGHT + 1;
    uint64_t best_t = 0;
    for (int j = 0; j < nl; j++) {
        int n = 0;
        for (int i = 0; i < FRI_MAX_INFLIGHT; i++) n += (ctx->slot_pending[i] && ctx->slot_lane[i] == j) ? 1 : 0;
        if (n < best_n || (n == best_n && ctx->lane_ticket[j] < best_t)) {
            best = j;
            best_n = n;
            best_t = ctx->lane_ticket[j];
        }
    }
    return best;
}

// Pipelined commits: a free result slot, the commit enqueued with its state
// in that slot, an event after its copy-out.  Host coefficients are first
// copied into the slot's pinned buffer, so the caller may reuse its buffer at
// once and the host-to-device copy is a true async copy on the stream.
static int async_enqueue(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* d_coeffs, size_t d,
                         uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                         const uint32_t* forced_betas, uint64_t* ticket) {
    if (!ctx || !ticket) return fail(ctx, FRI_EINVAL, "null argument");
    if (d && !host_coeffs && !d_coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    if (ctx->profiling) return fail(ctx, FRI_ESTATE, "profiling: time commits with fri_commit_device");
    if (ctx->team_root) return fail(ctx, FRI_EINVAL, "multi-GPU context: pipelined commits run on one-device contexts");
    int slot = -1;
    for (int i = 0; i < FRI_MAX_INFLIGHT && slot < 0; i++)
        if (!ctx->slot_pending[i]) slot = i;
    if (slot < 0) return fail(ctx, FRI_ESTATE, "FRI_MAX_INFLIGHT commits pending: wait for one first");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    int rv = commit_validate(ctx, d, log_n, offset, flags, forced_betas);
    if (rv) return rv;
    // this commit's lane (its own stream, plan and device state): the
    // commits pending on other lanes run beside it.  Its plan first: a lane
    // that gets no memory for it lowers the lanes in use and the commit goes
    // to one of the others (lane 0 always has one, or the call fails).
    for (;;) {
        const int lane = pick_lane(ctx);
        if ((rv = use_lane(ctx, lane))) return rv;
        rv = plan_build(ctx, d, log_n, offset);
        if (rv != FRI_ENOMEM || lane == 0) break;
        ctx->lanes_ok = lane;
    }
    if (rv) return rv;
    // (each lazily created member on its own: one whose creation failed is
    // created on the next call instead of being used null)
    if (!ctx->h_slot[slot]) FRI_HIP(ctx, hipHostMalloc(&ctx->h_slot[slot], sizeof(DevState), hipHostMallocDefault));
    if (!ctx->ev_slot[slot]) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_slot[slot], hipEventDisableTiming));
    // (every argument check ran before the pinned copy and the upload: a
    // commit refused later would leave the slot free with its upload in flight)
    if (host_coeffs && d) {
        // host input: pinned copy now, upload on h2d_stream (the copy engine,
        // beside the commit still running), the commit stream waits for it and
        // then moves it into the plan's input buffer (a device copy)
        if (!ctx->h2d_stream) FRI_HIP(ctx, upload_stream(ctx->device, &ctx->h2d_stream));
        if (!ctx->ev_in[slot]) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_in[slot], hipEventDisableTiming));
        if (ctx->h_in_cap[slot] < d) {       // the slot is free: its last upload and commit have completed
            if (ctx->h_in[slot]) hipHostFree(ctx->h_in[slot]);
            dfree(ctx, ctx->d_slot_in[slot]);
            ctx->h_in[slot] = ctx->d_slot_in[slot] = nullptr;
            ctx->h_in_cap[slot] = 0;
            FRI_HIP(ctx, hipHostMalloc(&ctx->h_in[slot], d * 4, hipHostMallocDefault));
            if (dalloc(ctx, &ctx->d_slot_in[slot], d * 4) != hipSuccess) return fail(ctx, FRI_ENOMEM, "input slot");
            ctx->h_in_cap[slot] = d;
        }
        memcpy(ctx->h_in[slot], host_coeffs, d * 4);
        FRI_HIP(ctx, hipMemcpyAsync(ctx->d_slot_in[slot], ctx->h_in[slot], d * 4, hipMemcpyHostToDevice,
                                    ctx->h2d_stream));
        FRI_HIP(ctx, hipEventRecord(ctx->ev_in[slot], ctx->h2d_stream));
        FRI_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_in[slot], 0));
        d_coeffs = ctx->d_slot_in[slot];
    }
    int rc = commit_enqueue(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, slot);
    if (rc) {
        // the slot stays free: its upload must be over before the next call
        // refills or frees the slot's buffers
        if (host_coeffs && d) (void)hipEventSynchronize(ctx->ev_in[slot]);
        return rc;
    }
    FRI_HIP(ctx, hipEventRecord(ctx->ev_slot[slot], ctx->stream));
    ctx->slot_pending[slot] = true;
    ctx->slot_user[slot] = ctx->plan.src == ctx->user_in;     // reads the caller's buffer in place
    ctx->slot_lane[slot] = ctx->cur_lane;
    ctx->lane_ticket[ctx->cur_lane] = ctx->next_ticket;
    ctx->slot_ticket[slot] = ctx->next_ticket++;
    ctx->slot_log_n[slot] = log_n;
    ctx->async_unsettled = true;
    *ticket = ctx->slot_ticket[slot];
    return FRI_OK;
}

extern "C" int fri_commit_async(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n, uint32_t offset,
                                const fri_channel_state* chan_in, uint32_t flags, const uint32_t* forced_betas,
                                uint64_t* ticket) {
    if (d && !coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    return async_enqueue(ctx, coeffs, nullptr, d, log_n, offset, chan_in, flags, forced_betas, ticket);
}

extern "C" int fri_commit_device_async(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                                       uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                                       const uint32_t* forced_betas, uint64_t* ticket) {
    if (d && !d_coeffs) return fail(ctx, FRI_EINVAL, "null coefficients");
    return async_enqueue(ctx, nullptr, d_coeffs, d, log_n, offset, chan_in, flags, forced_betas, ticket);
}

extern "C" int fri_commit_wait(fri_ctx* ctx, uint64_t ticket, fri_commit_result* out) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    int slot = -1;
    for (int i = 0; i < FRI_MAX_INFLIGHT && slot < 0; i++)
        if (ctx->slot_pending[i] && ctx->slot_ticket[i] == ticket) slot = i;
    if (slot < 0) return fail(ctx, FRI_EINVAL, "no pending commit with this ticket");
    ctx->slot_pending[slot] = false;
    ctx->slot_user[slot] = false;
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipEventSynchronize(ctx->ev_slot[slot]));
    return commit_finish(ctx, ctx->h_slot[slot], ctx->slot_log_n[slot], out);
}

extern "C" int fri_ctx_set_lanes(fri_ctx* ctx, uint32_t max_lanes) {
    if (!ctx) return FRI_EINVAL;
    if (max_lanes < 1 || max_lanes > FRI_MAX_INFLIGHT) return fail(ctx, FRI_EINVAL, "lanes must be 1..FRI_MAX_INFLIGHT");
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++)
        if (ctx->slot_pending[i]) return fail(ctx, FRI_ESTATE, "pipelined commits pending: wait for them first");
    ctx->max_lanes = (int)max_lanes;
    ctx->lanes_ok = FRI_MAX_INFLIGHT;
    return FRI_OK;
}

extern "C" int fri_debug_ticket_lane(fri_ctx* ctx, uint64_t ticket, int* lane) {
    if (!ctx || !lane) return fail(ctx, FRI_EINVAL, "null argument");
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++)
        if (ctx->slot_pending[i] && ctx->slot_ticket[i] == ticket) {
            *lane = ctx->slot_lane[i];
            return FRI_OK;
        }
    return fail(ctx, FRI_EINVAL, "no pending commit with this ticket");
}

// ---- the caller-owned input buffer --------------------------------------
// The pending pipelined commits that read the input buffer in place have
// finished (before it is refilled by fri_ctx_input_upload or moved).
static int wait_user_readers(fri_ctx* ctx) {
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++)
        if (ctx->slot_pending[i] && ctx->slot_user[i]) FRI_HIP(ctx, hipEventSynchronize(ctx->ev_slot[i]));
    return FRI_OK;
}

// One buffer per context (rank 0's device on a team), independent of the
// commit plans: the reference's caller owns `poly` (fri_commit.rs:72-76), and
// so does the caller here.  No commit writes it; a commit from it reads it in
// place on any lane, so what a commit commits is what the caller last wrote
// there, whatever the lane deal or the commits before it did.
extern "C" int fri_ctx_input_buffer(fri_ctx* ctx, size_t d, uint32_t** d_ptr) {
    if (!ctx || !d_ptr) return fail(ctx, FRI_EINVAL, "null argument");
    if (d > ((size_t)1 << ctx->log_n_max)) return fail(ctx, FRI_EINVAL, "d exceeds the context's codeword bound");
    const size_t want = d ? d : 1;
    if (ctx->user_cap < want) {
        // a larger buffer: the commits still reading the old one finish first
        // (its graphs are captured again on their next use, fri_commit.hip)
        FRI_HIP(ctx, hipSetDevice(ctx->device));
        int rc = wait_user_readers(ctx);
        if (rc) return rc;
        FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
        uint32_t* nb = nullptr;
        if (dalloc(ctx, &nb, want * 4) != hipSuccess) return fail(ctx, FRI_ENOMEM, "input buffer");
        if (ctx->user_in) {
            // the old contents move along (the caller may have filled it for
            // a smaller d); on the context stream, not the null stream
            const hipError_t e1 = hipMemcpyAsync(nb, ctx->user_in, ctx->user_cap * 4, hipMemcpyDeviceToDevice,
                                                 ctx->stream);
            const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(ctx->stream) : e1;
            if (e2 != hipSuccess) {
                dfree(ctx, nb);
                FRI_HIP(ctx, e2);
            }
            dfree(ctx, ctx->user_in);
        }
        ctx->user_in = nb;
        ctx->user_cap = want;
    }
    *d_ptr = ctx->user_in;
    return FRI_OK;
}

extern "C" int fri_ctx_input_upload(fri_ctx* ctx, const uint32_t* coeffs, size_t d) {
    if (!ctx || (d && !coeffs)) return fail(ctx, FRI_EINVAL, "null argument");
    uint32_t* buf = nullptr;
    int rc = fri_ctx_input_buffer(ctx, d, &buf);
    if (rc) return rc;
    if (!d) return FRI_OK;
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if ((rc = wait_user_readers(ctx))) return rc;
    // on the context stream, ordered after every commit queued there.  Not
    // on the upload stream: creating it here would hold a hardware queue
    // from the first upload on, and three commit lanes plus the context
    // stream plus that one exceed GPU_MAX_HW_QUEUES (4), which serialised
    // the 3-lane pipelined commits (4.09 against 3.30 ms per 2^24 commit)
    FRI_HIP(ctx, hipMemcpyAsync(buf, coeffs, d * 4, hipMemcpyHostToDevice, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

int fri::input_checksum(fri_ctx* ctx, const uint32_t* d_src, size_t d, uint64_t* out) {
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if (!ctx->d_csum && dalloc(ctx, &ctx->d_csum, 64) != hipSuccess) {
        ctx->d_csum = nullptr;
        return fail(ctx, FRI_ENOMEM, "checksum word");
    }
    if (!ctx->h_csum) FRI_HIP(ctx, hipHostMalloc(&ctx->h_csum, 64, hipHostMallocDefault));
    launch_checksum(d_src, d, ctx->d_csum, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(ctx->h_csum, ctx->d_csum, sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *out = *ctx->h_csum;
    return FRI_OK;
}

extern "C" int fri_commit_info(fri_ctx* ctx, uint64_t* generation, uint32_t* log_n, uint32_t* n_layers) {
    if (!ctx || !generation || !log_n || !n_layers) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    *generation = ctx->commit_gen;
    *n_layers = ctx->plan.valid ? ctx->h_state->n_layers : 0u;   // (a plan change frees the layers)
    *log_n = *n_layers ? ctx->commit_log_n : 0u;
    return FRI_OK;
}
