// fri_transport.hip — the collective transports of the sharded commit:
// RCCL (xGMI), host-staged callbacks (gloo tests), the loopback rehearsal and
// the in-process peer transport of a team context; attach / detach / info,
// the deadline on RCCL progress, and the transport self-test.
#include "fri_host.hpp"

// =================================================================== multi-GPU
int fri::tp_host_stage(fri_ctx* ctx, size_t bytes) {
    Transport& tp = ctx->tp;
    if (tp.hcap >= bytes) return FRI_OK;
    if (tp.hs) hipHostFree(tp.hs);
    if (tp.hr) hipHostFree(tp.hr);
    tp.hs = tp.hr = nullptr;
    tp.hcap = 0;
    FRI_HIP(ctx, hipHostMalloc(&tp.hs, bytes, hipHostMallocDefault));
    FRI_HIP(ctx, hipHostMalloc(&tp.hr, bytes, hipHostMallocDefault));
    tp.hcap = bytes;
    return FRI_OK;
}

// A rendezvous or collective that never completes (a peer that is gone, a
// fabric that does not come up) ends in FRI_ERCCL after FRI_RCCL_TIMEOUT_S
// seconds (default 120) instead of hanging the caller: the communicator setup
// runs on a helper thread the attach waits for with that deadline, and the
// sharded path's stream syncs poll with it and abort the communicators (which
// ends RCCL kernels spinning on an absent peer).  The sharded bench then
// falls back to independent commits.
// Test hook (fri_debug_inject_stall): the next RCCL all-to-all is replaced by
// a one-lane kernel that waits, like an RCCL kernel whose peer never comes,
// until the abort releases it (or, as a bound every wave reaches, 60 s pass).
__global__ void k_stalled_collective(const uint32_t* flag, uint64_t max_ticks) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
           wall_clock64() - t0 < max_ticks)
        __builtin_amdgcn_s_sleep(127);
}

void fri::rccl_abort(fri_ctx* ctx) {
    Transport& tp = ctx->tp;
    // an injected stall is released first, as ncclCommAbort's abort flag
    // releases a real RCCL kernel before the abort waits for the device
    if (ctx->stall_flag) __atomic_store_n(ctx->stall_flag, 1u, __ATOMIC_SEQ_CST);
    if (tp.xcomm) ncclCommAbort(tp.xcomm);
    if (tp.comm) ncclCommAbort(tp.comm);
    tp.comm = tp.xcomm = nullptr;      // the transport is gone: later sharded calls see FRI_ESTATE
}
#define FRI_NCCL(ctx, expr)                                                                  \
    do {                                                                                     \
        const ncclResult_t _r = (expr);                                                      \
        if (_r != ncclSuccess) return fail((ctx), FRI_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

// Stream sync of the sharded path with the same deadline: RCCL kernels whose
// peer never arrives spin on the device; aborting the communicators ends them.
int fri::sync_sharded(fri_ctx* ctx, hipStream_t s) {
    if (ctx->tp.host || !ctx->tp.comm) {
        FRI_HIP(ctx, hipStreamSynchronize(s));
        return FRI_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const double lim = rccl_timeout_s();
    // spin (yielding) for the first 200 us, which covers a commit's short
    // syncs at full responsiveness, then poll every 50 us so that a rank
    // waiting on its peers does not hold a host core at 100%
    // A rank of an RCCL team whose peer failed stops waiting at once: that
    // rank aborted its communicators (team_run), so the collectives it left
    // behind are never matched; this rank aborts its own as well.
    Team* T = ctx->tp.team;
    auto team_failed = [T]() {
        if (!T) return false;
        std::lock_guard<std::mutex> g(T->bm);
        return T->aborted;
    };
    bool peer_failed = false;
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return FRI_OK;
        if (e != hipErrorNotReady) FRI_HIP(ctx, e);
        const double el = seconds_since(t0);
        if (el > lim) break;
        if ((peer_failed = team_failed())) break;
        if (el < 2e-4) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    rccl_abort(ctx);
    // the abort ends RCCL kernels spinning on an absent peer; the wait for
    // the stream to drain is bounded as well (a stream still busy after it
    // is reported, and the context must then not be reused for commits)
    const auto t1 = std::chrono::steady_clock::now();
    bool drained = false;
    while (!(drained = hipStreamQuery(s) != hipErrorNotReady) && seconds_since(t1) < lim)
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (!drained) ctx->stuck = true;      // fri_ctx_destroy must not wait on it unboundedly
    const std::string why = peer_failed ? std::string("another rank of the team failed")
                                        : "no progress in " + std::to_string((int)lim) + " s";
    return fail(ctx, FRI_ERCCL, "sharded commit: " + why + " (RCCL communicators aborted" +
                                    (drained ? ")" : "; stream still busy: destroy the context)"));
}
static const char* op_name(uint32_t op) {
    return op == FRI_OP_ALLGATHER ? "allgather" : op == FRI_OP_ALLTOALL ? "alltoall" : "sendrecv";
}

// One collective of the peer transport (see Team).  ALLTOALL: recv[p] =
// p's send[r]; ALLGATHER: recv[p] = p's send; SENDRECV: recv = peer's send.
static int peer_op(fri_ctx* ctx, uint32_t op, uint32_t chan, const void* send, void* recv, size_t bytes, int peer,
                   hipStream_t s) {
    Team* T = ctx->tp.team;
    const uint32_t r = (uint32_t)ctx->tp.rank, G = T->G;
    if (bytes % 4) return fail(ctx, FRI_EINVAL, "peer transport: byte count not a multiple of 4");
    if (ctx->tp.fail_at >= 0 && ctx->tp.n_ops++ == ctx->tp.fail_at) {      // test hook: this rank fails here
        ctx->tp.fail_at = -1;
        return fail(ctx, FRI_ERCCL, std::string("injected failure at peer op ") + op_name(op));
    }
    FRI_HIP(ctx, hipEventRecord(T->ev_ready[r], s));
    T->slot[r] = PeerSlot{send, recv, bytes, op, chan, peer};
    if (!team_barrier(T)) return fail(ctx, FRI_ERCCL, "peer transport: another rank failed (" + T->why + ")");
    for (uint32_t p = 0; p < G; p++) {
        const PeerSlot& q = T->slot[p];
        if (q.op != op || q.bytes != bytes || q.chan != chan ||
            (op == FRI_OP_SENDRECV && (q.peer < 0 || q.peer >= (int)G || T->slot[q.peer].peer != (int)p))) {
            const std::string m = std::string("peer transport: schedule mismatch at ") + op_name(op) + " (rank " +
                                  std::to_string(p) + " posted " + op_name(q.op) + " of " + std::to_string(q.bytes) +
                                  " bytes)";
            team_abort(T, m);
            return fail(ctx, FRI_ERCCL, m);
        }
    }
    // (the slots are stable from rendezvous A to B: a rank posts its next op
    // only after B, which waits for this one; so everything read from them is
    // read here)
    std::vector<uint32_t> readers;        // ranks that read this rank's send buffer
    for (uint32_t p = 0; p < G; p++)
        if (p != r && (op != FRI_OP_SENDRECV || T->slot[p].peer == (int)r)) readers.push_back(p);
    PeerPull pp{};
    pp.dst = static_cast<uint32_t*>(recv);
    pp.words = bytes / 4;
    std::vector<uint32_t> srcs;
    if (op == FRI_OP_SENDRECV) {
        srcs.push_back((uint32_t)peer);
    } else {
        for (uint32_t p = 0; p < G; p++) srcs.push_back(p);
    }
    bool vec4 = pp.words % 4 == 0 && (reinterpret_cast<uintptr_t>(recv) & 15) == 0;
    for (size_t i = 0; i < srcs.size(); i++) {
        const uint32_t p = srcs[i];
        const uint8_t* base = static_cast<const uint8_t*>(T->slot[p].send) + (op == FRI_OP_ALLTOALL ? (size_t)r * bytes : 0);
        pp.src[i] = reinterpret_cast<const uint32_t*>(base);
        vec4 = vec4 && (reinterpret_cast<uintptr_t>(base) & 15) == 0;
        if (p != r) FRI_HIP(ctx, hipStreamWaitEvent(s, T->ev_ready[p], 0));
    }
    pp.n = (uint32_t)srcs.size();
    pp.vec4 = vec4 ? 1u : 0u;
    if (T->kernel_pull) {
        launch_peer_pull(pp, s);
        FRI_HIP(ctx, hipGetLastError());
    } else {
        for (uint32_t i = 0; i < pp.n; i++) {
            const uint32_t p = srcs[i];
            FRI_HIP(ctx, hipMemcpyPeerAsync(pp.dst + (size_t)i * pp.words, T->dev[r], pp.src[i], T->dev[p], bytes, s));
        }
    }
    FRI_HIP(ctx, hipEventRecord(T->ev_done[r], s));
    if (!team_barrier(T)) return fail(ctx, FRI_ERCCL, "peer transport: another rank failed (" + T->why + ")");
    // this rank's send buffer may be rewritten only after its readers' pulls
    for (uint32_t p : readers) FRI_HIP(ctx, hipStreamWaitEvent(s, T->ev_done[p], 0));
    return FRI_OK;
}

// Every transport call is logged (fri_debug_transport_log): chan 0 is the main
// communicator on the context stream, 1 the exchange communicator on the
// exchange stream, whatever stream the host transport actually uses.
static void tp_log(fri_ctx* ctx, uint32_t chan, uint32_t op, int peer, size_t bytes) {
    fri_transport_op e{};
    e.chan = chan;
    e.op = op;
    e.peer = peer;
    e.bytes = bytes;
    if (ctx->tp.log.size() < 4096) ctx->tp.log.push_back(e);
}

int fri::tp_allgather(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, hipStream_t s) {
    Transport& tp = ctx->tp;
    tp_log(ctx, 0, FRI_OP_ALLGATHER, -1, bytes);
    if (tp.peer) return peer_op(ctx, FRI_OP_ALLGATHER, 0, dsend, drecv, bytes, -1, s);
    if (tp.loop) {                     // G copies of this rank's bytes, one launch (bytes: whole words)
        launch_replicate(static_cast<const uint32_t*>(dsend), static_cast<uint32_t*>(drecv), bytes / 4,
                         (uint32_t)tp.world, s);
        FRI_HIP(ctx, hipGetLastError());
        return FRI_OK;
    }
    if (!tp.host) {
        FRI_NCCL(ctx, ncclAllGather(dsend, drecv, bytes, ncclUint8, tp.comm, s));
        return FRI_OK;
    }
    int rc = tp_host_stage(ctx, bytes * tp.world);
    if (rc) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(tp.hs, dsend, bytes, hipMemcpyDeviceToHost, s));
    FRI_HIP(ctx, hipStreamSynchronize(s));
    if (tp.ops.allgather(tp.ops.user, tp.hs, tp.hr, bytes)) return fail(ctx, FRI_ERCCL, "allgather callback failed");
    FRI_HIP(ctx, hipMemcpyAsync(drecv, tp.hr, bytes * tp.world, hipMemcpyHostToDevice, s));
    return FRI_OK;
}

int fri::tp_alltoall(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes_per_peer, hipStream_t s) {
    Transport& tp = ctx->tp;
    tp_log(ctx, 0, FRI_OP_ALLTOALL, -1, bytes_per_peer);
    if (tp.peer) return peer_op(ctx, FRI_OP_ALLTOALL, 0, dsend, drecv, bytes_per_peer, -1, s);
    if (tp.loop) {
        FRI_HIP(ctx, hipMemcpyAsync(drecv, dsend, bytes_per_peer * tp.world, hipMemcpyDeviceToDevice, s));
        return FRI_OK;
    }
    if (!tp.host && ctx->inject_stall) {
        ctx->inject_stall = false;
        *ctx->stall_flag = 0u;
        hipLaunchKernelGGL(k_stalled_collective, dim3(1), dim3(64), 0, s, ctx->stall_flag_dev,
                           (uint64_t)60 * 100000000ull);   // wall_clock64 runs at 100 MHz
        FRI_HIP(ctx, hipGetLastError());
        return FRI_OK;
    }
    if (!tp.host) {
        FRI_NCCL(ctx, ncclGroupStart());
        for (int p = 0; p < tp.world; p++) {
            FRI_NCCL(ctx, ncclSend((const uint8_t*)dsend + p * bytes_per_peer, bytes_per_peer, ncclUint8, p, tp.comm, s));
            FRI_NCCL(ctx, ncclRecv((uint8_t*)drecv + p * bytes_per_peer, bytes_per_peer, ncclUint8, p, tp.comm, s));
        }
        FRI_NCCL(ctx, ncclGroupEnd());
        return FRI_OK;
    }
    const size_t tot = bytes_per_peer * tp.world;
    int rc = tp_host_stage(ctx, tot);
    if (rc) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(tp.hs, dsend, tot, hipMemcpyDeviceToHost, s));
    FRI_HIP(ctx, hipStreamSynchronize(s));
    if (tp.ops.alltoall(tp.ops.user, tp.hs, tp.hr, bytes_per_peer)) return fail(ctx, FRI_ERCCL, "alltoall callback failed");
    FRI_HIP(ctx, hipMemcpyAsync(drecv, tp.hr, tot, hipMemcpyHostToDevice, s));
    return FRI_OK;
}

// chan 1: the exchange communicator (RCCL: on ctx->xstream, which `s` must be)
int fri::tp_sendrecv(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, int peer, hipStream_t s,
                       uint32_t chan) {
    Transport& tp = ctx->tp;
    tp_log(ctx, chan, FRI_OP_SENDRECV, peer, bytes);
    if (tp.peer) return peer_op(ctx, FRI_OP_SENDRECV, chan, dsend, drecv, bytes, peer, s);
    if (tp.loop) {
        FRI_HIP(ctx, hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, s));
        return FRI_OK;
    }
    if (!tp.host) {
        ncclComm_t c = chan ? tp.xcomm : tp.comm;
        FRI_NCCL(ctx, ncclGroupStart());
        FRI_NCCL(ctx, ncclSend(dsend, bytes, ncclUint8, peer, c, s));
        FRI_NCCL(ctx, ncclRecv(drecv, bytes, ncclUint8, peer, c, s));
        FRI_NCCL(ctx, ncclGroupEnd());
        return FRI_OK;
    }
    int rc = tp_host_stage(ctx, bytes);
    if (rc) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(tp.hs, dsend, bytes, hipMemcpyDeviceToHost, s));
    FRI_HIP(ctx, hipStreamSynchronize(s));
    if (tp.ops.sendrecv(tp.ops.user, tp.hs, tp.hr, bytes, peer)) return fail(ctx, FRI_ERCCL, "sendrecv callback failed");
    FRI_HIP(ctx, hipMemcpyAsync(drecv, tp.hr, bytes, hipMemcpyHostToDevice, s));
    return FRI_OK;
}

extern "C" int fri_dist_unique_id(uint8_t uid[128]) {
    if (!uid) return FRI_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return FRI_ERCCL;
    memcpy(uid, id.internal, 128);
    return FRI_OK;
}

static int dist_check(fri_ctx* ctx, int rank, int world) {
    if (!ctx || world < 1 || world > 64 || (world & (world - 1)) || rank < 0 || rank >= world)
        return fail(ctx, FRI_EINVAL, "world must be a power of two <= 64 and 0 <= rank < world");
    return FRI_OK;
}

static int team_guard(fri_ctx* ctx) {
    return ctx && ctx->tp.team ? fail(ctx, FRI_EINVAL, "multi-GPU context: its transport is the team's") : FRI_OK;
}

extern "C" int fri_dist_attach_rccl(fri_ctx* ctx, int rank, int world, const uint8_t uid[128]) {
    if (int g = team_guard(ctx)) return g;
    int rc = dist_check(ctx, rank, world);
    if (rc) return rc;
    if (!uid) return fail(ctx, FRI_EINVAL, "null unique id");
    fri_dist_detach(ctx);
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId id;
    memcpy(id.internal, uid, 128);
    // communicator setup on a helper thread, waited for with the deadline; a
    // thread still blocked in the rendezvous after it is abandoned (it frees
    // what it creates if it ever finishes)
    struct Setup {
        std::mutex m;
        std::condition_variable cv;
        bool done = false, abandoned = false;
        ncclComm_t comm = nullptr, xcomm = nullptr;
        ncclResult_t r = ncclSuccess;
        const char* what = "";
    };
    auto su = std::make_shared<Setup>();
    const int dev = ctx->device;
    std::thread([su, dev, world, id, rank]() {
        (void)hipSetDevice(dev);
        ncclComm_t c = nullptr, x = nullptr;
        const char* what = "ncclCommInitRank";
        ncclResult_t r = ncclCommInitRank(&c, world, id, rank);
        if (r == ncclSuccess) {
            what = "ncclCommSplit";
            r = ncclCommSplit(c, 0, rank, &x, nullptr);      // second comm for the exchange stream
            if (r != ncclSuccess) { ncclCommDestroy(c); c = nullptr; x = nullptr; }
        }
        std::lock_guard<std::mutex> g(su->m);
        if (su->abandoned) {
            if (x) ncclCommDestroy(x);
            if (c) ncclCommDestroy(c);
        } else {
            su->comm = c; su->xcomm = x; su->r = r; su->what = what;
        }
        su->done = true;
        su->cv.notify_all();
    }).detach();
    const double lim = rccl_timeout_s();
    std::unique_lock<std::mutex> lk(su->m);
    if (!su->cv.wait_for(lk, std::chrono::duration<double>(lim), [&] { return su->done; })) {
        su->abandoned = true;
        return fail(ctx, FRI_ERCCL, "RCCL rendezvous (rank " + std::to_string(rank) + " of " + std::to_string(world) +
                                        ") did not complete in " + std::to_string((int)lim) + " s");
    }
    if (su->r != ncclSuccess) return fail(ctx, FRI_ERCCL, std::string(su->what) + ": " + ncclGetErrorString(su->r));
    ncclComm_t comm = su->comm, xcomm = su->xcomm;
    ctx->tp.comm = comm;
    ctx->tp.xcomm = xcomm;
    ctx->tp.rank = rank;
    ctx->tp.world = world;
    ctx->tp.host = false;
    return FRI_OK;
}

extern "C" int fri_dist_attach_host(fri_ctx* ctx, int rank, int world, const fri_collectives* ops) {
    if (int g = team_guard(ctx)) return g;
    int rc = dist_check(ctx, rank, world);
    if (rc) return rc;
    if (!ops || !ops->allgather || !ops->alltoall || !ops->sendrecv) return fail(ctx, FRI_EINVAL, "null callback");
    fri_dist_detach(ctx);
    ctx->tp.rank = rank;
    ctx->tp.world = world;
    ctx->tp.host = true;
    ctx->tp.ops = *ops;
    return FRI_OK;
}

// Rehearsal transport for timing one rank's share of a sharded commit on one
// device: collectives are device-to-device copies of this rank's own data on
// the calling stream (the exchange stream included, as with RCCL), so the
// GPU never waits for a host round trip.  The transcript is not the real one.
extern "C" int fri_debug_attach_loopback(fri_ctx* ctx, int rank, int world) {
    if (int g = team_guard(ctx)) return g;
    int rc = dist_check(ctx, rank, world);
    if (rc) return rc;
    fri_dist_detach(ctx);
    ctx->tp.rank = rank;
    ctx->tp.world = world;
    ctx->tp.loop = true;
    return FRI_OK;
}

extern "C" int fri_debug_loopback_degrees(fri_ctx* ctx, const int32_t* deg, uint32_t n) {
    if (!ctx) return FRI_EINVAL;
    if (n > (uint32_t)MAXR + 1) return fail(ctx, FRI_EINVAL, "more degrees than layers");
    ctx->db.sched_h.assign(deg ? deg : nullptr, deg ? deg + n : nullptr);
    return FRI_OK;
}


extern "C" int fri_debug_transport_log(fri_ctx* ctx, fri_transport_op* out, size_t cap, size_t* count) {
    if (!ctx || !count) return fail(ctx, FRI_EINVAL, "null argument");
    const auto& lg = ctx->tp.log;
    *count = lg.size();
    if (!out) return FRI_OK;                       // size query
    if (cap < lg.size()) return fail(ctx, FRI_EINVAL, "log buffer too small (see count)");
    for (size_t i = 0; i < lg.size(); i++) out[i] = lg[i];
    return FRI_OK;
}

extern "C" int fri_dist_detach(fri_ctx* ctx) {
    if (!ctx) return FRI_EINVAL;
    if (int g = team_guard(ctx)) return g;
    Transport& tp = ctx->tp;
    if (tp.xcomm) ncclCommDestroy(tp.xcomm);
    if (tp.comm) ncclCommDestroy(tp.comm);
    if (tp.hs) hipHostFree(tp.hs);
    if (tp.hr) hipHostFree(tp.hr);
    tp = Transport();
    ctx->db.shtop_h.clear();     // the next sharded call uploads its top table again
    return FRI_OK;
}

extern "C" int fri_dist_info(fri_ctx* ctx, int* rank, int* world, int* transport) {
    if (!ctx || !rank || !world || !transport) return fail(ctx, FRI_EINVAL, "null argument");
    const Transport& tp = ctx->tp;
    if (tp.host || tp.loop || tp.peer) {
        *transport = tp.host ? FRI_TRANSPORT_HOST : tp.loop ? FRI_TRANSPORT_LOOPBACK : FRI_TRANSPORT_PEER;
        *rank = tp.rank;
        *world = tp.world;
    } else if (tp.comm) {
        // what the communicator itself reports, not what attach was told
        *transport = FRI_TRANSPORT_RCCL;
        FRI_NCCL(ctx, ncclCommCount(tp.comm, world));
        FRI_NCCL(ctx, ncclCommUserRank(tp.comm, rank));
    } else {
        *transport = FRI_TRANSPORT_NONE;
        *rank = 0;
        *world = 1;
    }
    return FRI_OK;
}

// Transport self-test: all-to-all, all-gather and a pair exchange on both
// streams/communicators, checked on the host.  Rank r sends word
// (r << 24) | (p << 16) | i to peer p; the exchange partner is r ^ 1 (itself
// when world == 1).
static int dist_selftest(fri_ctx* ctx, size_t words_per_peer);
extern "C" int fri_dist_selftest(fri_ctx* ctx, size_t words_per_peer) {
    if (!ctx) return FRI_EINVAL;
    if (ctx->team_root) {
        Team* T = ctx->team_root;
        return team_run(ctx, [&](uint32_t r) { return dist_selftest(T->rk[r], words_per_peer); });
    }
    return dist_selftest(ctx, words_per_peer);
}

static int dist_selftest(fri_ctx* ctx, size_t words_per_peer) {
    if (ctx->tp.world < 1 || (!ctx->tp.host && !ctx->tp.comm && !ctx->tp.peer))
        return fail(ctx, FRI_ESTATE, "no transport attached");
    const uint32_t G = (uint32_t)ctx->tp.world, r = (uint32_t)ctx->tp.rank;
    if (words_per_peer == 0 || words_per_peer > ((size_t)1 << 16)) return fail(ctx, FRI_EINVAL, "1 <= words_per_peer <= 65536");
    const size_t W = words_per_peer, tot = W * G;
    int rc = dist_buffers(ctx, tot, G, tot);
    if (rc) return rc;
    ctx->tp.log.clear();
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    // read-backs land in pinned staging: a copy into pageable memory would
    // block the host behind a stalled collective before sync_sharded's deadline
    if ((rc = tp_host_stage(ctx, tot * 4))) return rc;
    std::vector<uint32_t> h(tot);
    for (uint32_t p = 0; p < G; p++)
        for (size_t i = 0; i < W; i++) h[p * W + i] = (r << 24) | (p << 16) | (uint32_t)i;
    hipStream_t s = ctx->stream;
    DistBuf& db = ctx->db;
    auto check = [&](const char* what, auto expect) -> int {
        FRI_HIP(ctx, hipMemcpyAsync(ctx->tp.hs, db.recv, tot * 4, hipMemcpyDeviceToHost, s));
        if (int rs = sync_sharded(ctx, s)) return rs;
        const uint32_t* got = reinterpret_cast<const uint32_t*>(ctx->tp.hs);
        for (uint32_t p = 0; p < G; p++)
            for (size_t i = 0; i < W; i++)
                if (got[p * W + i] != expect(p, (uint32_t)i))
                    return fail(ctx, FRI_ERCCL, std::string("selftest ") + what + " mismatch");
        return FRI_OK;
    };
    FRI_HIP(ctx, hipMemcpyAsync(db.cyc, h.data(), tot * 4, hipMemcpyHostToDevice, s));
    if ((rc = tp_alltoall(ctx, db.cyc, db.recv, W * 4, s))) return rc;
    if ((rc = check("alltoall", [&](uint32_t p, uint32_t i) { return (p << 24) | (r << 16) | i; }))) return rc;
    if ((rc = tp_allgather(ctx, db.cyc, db.recv, W * 4, s))) return rc;      // each rank's first W words
    if ((rc = check("allgather", [&](uint32_t p, uint32_t i) { return (p << 24) | i; }))) return rc;
    const uint32_t partner = G > 1 ? (r ^ 1u) : r;
    // pair exchange on the exchange stream / split communicator, as the fold uses it
    FRI_HIP(ctx, hipEventRecord(ctx->ev_vals, s));
    FRI_HIP(ctx, hipStreamWaitEvent(ctx->xstream, ctx->ev_vals, 0));
    if ((rc = tp_sendrecv(ctx, db.cyc, db.recv, tot * 4, (int)partner, ctx->tp.host ? s : ctx->xstream, 1))) return rc;
    FRI_HIP(ctx, hipEventRecord(ctx->ev_xchg, ctx->tp.host ? s : ctx->xstream));
    FRI_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_xchg, 0));
    if ((rc = check("sendrecv", [&](uint32_t p, uint32_t i) { return (partner << 24) | (p << 16) | i; }))) return rc;
    ctx->err.clear();
    return FRI_OK;
}

int fri::dist_buffers(fri_ctx* ctx, size_t M, uint32_t G, size_t gwords) {
    DistBuf& b = ctx->db;
    const size_t nhi = 1u << 20;   // pow table hi part, generous (M <= 2^32)
    if (b.cap < M) {
        dfree(ctx, b.cyc); dfree(ctx, b.recv); dfree(ctx, b.half); dfree(ctx, b.half2);
        b.cyc = b.recv = b.half = b.half2 = nullptr;
        b.cap = 0;
        FRI_HIP(ctx, dalloc(ctx, &b.cyc, M * 4));
        FRI_HIP(ctx, dalloc(ctx, &b.recv, M * 4));
        FRI_HIP(ctx, dalloc(ctx, &b.half, (M / 2 + 1) * 4));
        FRI_HIP(ctx, dalloc(ctx, &b.half2, (M / 4 + 1) * 4));   // odd layers: half of a block of layer >= 1
        b.cap = M;
    }
    // (each lazily created member on its own, as in async_enqueue)
    if (!b.top) FRI_HIP(ctx, dalloc(ctx, &b.top, (size_t)(MAXR + 1) * 2 * 64 * 32));
    if (!b.pre_lo) FRI_HIP(ctx, dalloc(ctx, &b.pre_lo, ((size_t)1 << POW_LO_LOG) * 4));
    if (!b.pre_hi) FRI_HIP(ctx, dalloc(ctx, &b.pre_hi, nhi * 4));
    if (!b.rec) FRI_HIP(ctx, dalloc(ctx, &b.rec, (size_t)(64 + 1) * REC_WORDS * 4));
    if (!b.shtop) {
        FRI_HIP(ctx, dalloc(ctx, &b.shtop, (size_t)(MAXR + 1) * sizeof(ShardTop)));
        b.shtop_h.clear();                 // a new table buffer: upload on the next sharded call
    }
    if (b.gcap < gwords) {
        dfree(ctx, b.gath);
        b.gath = nullptr;
        FRI_HIP(ctx, dalloc(ctx, &b.gath, gwords * 4));
        b.gcap = gwords;
    }
    if (!ctx->xstream) FRI_HIP(ctx, hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking));
    if (!ctx->ev_vals) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_vals, hipEventDisableTiming));
    if (!ctx->ev_xchg) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_xchg, hipEventDisableTiming));
    if (!ctx->cstream) FRI_HIP(ctx, hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
    if (!ctx->ev_pre) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_pre, hipEventDisableTiming));
    if (!ctx->ev_coef) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_coef, hipEventDisableTiming));
    (void)G;
    return FRI_OK;
}
extern "C" int fri_debug_inject_stall(fri_ctx* ctx, int enable) {
    if (!ctx) return FRI_EINVAL;
    if (!ctx->stall_flag) {
        FRI_HIP(ctx, hipHostMalloc(&ctx->stall_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
        *ctx->stall_flag = 1u;
    }
    if (!ctx->stall_flag_dev) {
        void* d = nullptr;
        FRI_HIP(ctx, hipHostGetDevicePointer(&d, ctx->stall_flag, 0));
        ctx->stall_flag_dev = static_cast<uint32_t*>(d);
    }
    ctx->inject_stall = enable != 0;
    return FRI_OK;
}
