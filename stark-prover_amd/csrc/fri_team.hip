// fri_team.hip — the single-process multi-GPU team context
// (fri_ctx_create_multi): rank 0 on the calling thread, ranks 1..G-1 on
// worker threads, one call of fri_commit committing coset-sharded over them.
#include "fri_host.hpp"

// ------------------------------------------------ in-process team ----
// fri_ctx_create_multi: one context per device (rank r drives devices[r]),
// rank 0 being the context handed to the caller.  A team call (fri_commit,
// fri_decommit_query, ...) runs the coset-sharded protocol of
// run_commit_sharded on every rank at once: rank 0 on the calling thread,
// ranks 1..G-1 on persistent worker threads of the team (one per rank, so a
// rank's HIP calls stay on its own thread and device).  The collectives go
// over RCCL (communicators from ncclCommInitAll) or over the peer transport:
//   each collective, on rank r:  record ready_r after its producer on the
//   op's stream; post (op, bytes, peer, send, recv); rendezvous A; check that
//   every rank posted the same (op, bytes) and matched peers (the
//   deadlock-freedom condition of DESIGN.md §7, enforced here rather than
//   only logged); the stream waits for the sources' ready events and one
//   k_peer_pull reads every source's bytes (same device, or another device
//   over xGMI through peer access); record done_r; rendezvous B; the stream
//   waits for the done events of the ranks that read r's send buffer.
// Every event waited on was recorded before the rendezvous that precedes the
// wait, so no stream can wait for work that has not been submitted (no
// deadlock, even when ranks share a device and its hardware queues), and a
// rank that fails aborts the rendezvous: the others return FRI_ERCCL
// instead of blocking.  The GPU never waits for the host.
void fri::team_abort(Team* T, const std::string& why) {
    std::lock_guard<std::mutex> g(T->bm);
    if (!T->aborted) T->why = why;
    T->aborted = true;
    T->bcv.notify_all();
}

// All G ranks arrive; false when the team was aborted first.
bool fri::team_barrier(Team* T) {
    std::unique_lock<std::mutex> lk(T->bm);
    if (T->aborted) return false;
    const uint64_t g = T->bgen;
    if (++T->arrived == T->G) {
        T->arrived = 0;
        T->bgen++;
        T->bcv.notify_all();
        return true;
    }
    T->bcv.wait(lk, [&] { return T->bgen != g || T->aborted; });
    return T->bgen != g;
}
// =========================================================== team (multi-GPU)
// Run fn(r) on every rank of the team at once: rank 0 on this thread, the
// others on the team's workers.  The first failing rank aborts the
// rendezvous (the others' collectives then fail instead of blocking); its
// message becomes the context's error.
static void team_worker(Team* T, uint32_t r) {
    uint64_t seen = 0;
    for (;;) {
        std::function<int(uint32_t)> fn;
        {
            std::unique_lock<std::mutex> lk(T->jm);
            T->jcv.wait(lk, [&] { return T->quit || T->seq != seen; });
            if (T->quit) return;
            seen = T->seq;
            fn = T->job;
        }
        (void)hipSetDevice(T->dev[r]);
        const int rc = fn(r);
        if (rc) {
            team_abort(T, "rank " + std::to_string(r) + ": " + T->rk[r]->err);
            // RCCL: this rank's collectives will never be matched; its
            // communicators go now (the others abort theirs when they see the
            // team aborted, sync_sharded), not after FRI_RCCL_TIMEOUT_S
            if (T->kind == FRI_TRANSPORT_RCCL) rccl_abort(T->rk[r]);
        }
        std::lock_guard<std::mutex> g(T->jm);
        T->rc[r] = rc;
        if (--T->left == 0) T->dcv.notify_all();
    }
}

int fri::team_run(fri_ctx* root, const std::function<int(uint32_t)>& fn) {
    Team* T = root->team_root;
    {
        std::lock_guard<std::mutex> g(T->bm);
        T->aborted = false;
        T->arrived = 0;
        T->why.clear();
    }
    for (fri_ctx* c : T->rk) c->tp.n_ops = 0;     // (fri_debug_team_inject_failure counts per call)
    {
        std::lock_guard<std::mutex> g(T->jm);
        T->job = fn;
        T->left = T->G - 1;
        std::fill(T->rc.begin(), T->rc.end(), 0);
        T->seq++;
    }
    T->jcv.notify_all();
    const int rc0 = fn(0);
    if (rc0) {
        team_abort(T, "rank 0: " + root->err);
        if (T->kind == FRI_TRANSPORT_RCCL) rccl_abort(root);
    }
    {
        std::unique_lock<std::mutex> lk(T->jm);
        T->dcv.wait(lk, [&] { return T->left == 0; });
    }
    // fri_debug_team_inject_failure applies to this call only, fired or not
    for (fri_ctx* c : T->rk) c->tp.fail_at = -1;
    int rc = rc0;
    for (uint32_t r = 1; r < T->G && !rc; r++) rc = T->rc[r];
    if (rc) {
        // the failure that aborted the team, and every rank's streams drained
        // (a rank that returned early may have left work queued)
        {
            std::lock_guard<std::mutex> g(T->bm);
            root->err = T->why.empty() ? root->err : T->why;
        }
        for (fri_ctx* c : T->rk) {
            (void)hipSetDevice(c->device);
            if (c->stuck) continue;
            for (hipStream_t st : {c->stream, c->xstream, c->cstream})
                if (st) (void)hipStreamSynchronize(st);
        }
        (void)hipSetDevice(root->device);
    }
    return rc;
}

// Peer access is a per-process property of a device pair, shared by every
// team of the process: reference-counted, enabled by the first team that
// needs it and disabled when the last one is gone (never disabled when it was
// enabled outside the library).
struct PeerRef { int refs = 0; bool ours = false; };
static std::mutex g_peer_m;
static std::map<std::pair<int, int>, PeerRef> g_peer;

static bool peer_acquire(int a, int b) {
    std::lock_guard<std::mutex> g(g_peer_m);
    auto it = g_peer.find({a, b});
    if (it == g_peer.end()) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) return false;
        (void)hipSetDevice(a);
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        (void)hipGetLastError();
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return false;
        it = g_peer.emplace(std::make_pair(a, b), PeerRef{0, e == hipSuccess}).first;
    }
    it->second.refs++;
    return true;
}

static void peer_release(int a, int b) {
    std::lock_guard<std::mutex> g(g_peer_m);
    auto it = g_peer.find({a, b});
    if (it == g_peer.end() || it->second.refs == 0) return;
    if (--it->second.refs == 0) {
        if (it->second.ours) {
            (void)hipSetDevice(a);
            (void)hipDeviceDisablePeerAccess(b);
            (void)hipGetLastError();
        }
        g_peer.erase(it);
    }
}

static void team_free(Team* T) {
    {
        std::lock_guard<std::mutex> g(T->jm);
        T->quit = true;
    }
    T->jcv.notify_all();
    for (auto& t : T->th)
        if (t.joinable()) t.join();
    for (uint32_t r = 0; r < T->G; r++) {
        if (r < T->ev_ready.size() && T->ev_ready[r]) { (void)hipSetDevice(T->dev[r]); hipEventDestroy(T->ev_ready[r]); }
        if (r < T->ev_done.size() && T->ev_done[r]) { (void)hipSetDevice(T->dev[r]); hipEventDestroy(T->ev_done[r]); }
    }
    for (const auto& ab : T->peer_pairs) peer_release(ab.first, ab.second);
    delete T;
}

extern "C" int fri_ctx_create_multi(const int* devices, uint32_t n, uint32_t log_n_max, int transport, fri_ctx** out) {
    if (!out) return FRI_EINVAL;
    *out = nullptr;
    if (n < 1 || n > 64 || (n & (n - 1)) || log_n_max < 1 || log_n_max > 30) return FRI_EINVAL;
    if (transport != FRI_TRANSPORT_NONE && transport != FRI_TRANSPORT_RCCL && transport != FRI_TRANSPORT_PEER)
        return FRI_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return FRI_ENODEV;
    std::vector<int> dev(n);
    for (uint32_t r = 0; r < n; r++) {
        dev[r] = devices ? devices[r] : (int)r;
        if (dev[r] < 0 || dev[r] >= ndev) return FRI_ENODEV;
    }
    if (n == 1) return fri_ctx_create(dev[0], log_n_max, out);
    uint32_t logG = 0;
    while ((1u << logG) < n) logG++;
    // rank contexts are shard-sized; rank 0 also commits < 2^20 codewords alone
    const uint32_t sub = std::max(log_n_max > logG ? log_n_max - logG : 1u, std::min(log_n_max, SHARD_MIN_LOG - 1));
    Team* T = new Team();
    T->G = n;
    T->logG = logG;
    T->dev = dev;
    T->rk.assign(n, nullptr);
    T->rc.assign(n, 0);
    T->slot.assign(n, PeerSlot{});
    T->ev_ready.assign(n, nullptr);
    T->ev_done.assign(n, nullptr);
    int rc = FRI_OK;
    auto undo = [&](int code) {
        // (communicators a later step's failure leaves behind are destroyed,
        // not dropped: Transport() alone would leak them)
        for (uint32_t r = 0; r < n; r++) {
            fri_ctx* c = T->rk[r];
            if (!c) continue;
            (void)hipSetDevice(c->device);
            if (c->tp.xcomm) ncclCommDestroy(c->tp.xcomm);
            if (c->tp.comm) ncclCommDestroy(c->tp.comm);
            c->tp = Transport();
        }
        for (uint32_t r = 1; r < n; r++)
            if (T->rk[r]) fri_ctx_destroy(T->rk[r]);
        if (T->rk[0]) { T->rk[0]->team_root = nullptr; fri_ctx_destroy(T->rk[0]); }
        team_free(T);
        return code;
    };
    for (uint32_t r = 0; r < n; r++)
        if ((rc = fri_ctx_create(dev[r], sub, &T->rk[r]))) return undo(rc);
    for (uint32_t r = 0; r < n; r++) {
        if (hipSetDevice(dev[r]) != hipSuccess ||
            hipEventCreateWithFlags(&T->ev_ready[r], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&T->ev_done[r], hipEventDisableTiming) != hipSuccess)
            return undo(FRI_EHIP);
    }
    // peer access between distinct devices: the pull kernel reads the other
    // ranks' buffers over xGMI; without it, per-source hipMemcpyPeerAsync
    // (fri_transport.hip peer_op; fri_debug_team_force_copy forces that path)
    for (uint32_t a = 0; a < n; a++)
        for (uint32_t b = 0; b < n; b++) {
            if (dev[a] == dev[b]) continue;
            if (std::find(T->peer_pairs.begin(), T->peer_pairs.end(), std::make_pair(dev[a], dev[b])) !=
                T->peer_pairs.end())
                continue;                        // (a device pair repeated by repeated ordinals)
            if (peer_acquire(dev[a], dev[b])) T->peer_pairs.emplace_back(dev[a], dev[b]);
            else T->can_pull = false;
        }
    T->kernel_pull = T->can_pull;
    // transport: the peer transport unless RCCL is asked for (FRI_TRANSPORT_NONE
    // means peer: it is what the tests run; the in-process RCCL team has not
    // yet run on distinct devices).  RCCL: one communicator per
    // rank for the main stream, one for the exchange stream; ranks sharing a
    // device cannot use it.
    bool distinct = true;
    for (uint32_t a = 0; a < n; a++)
        for (uint32_t b = a + 1; b < n; b++) distinct = distinct && dev[a] != dev[b];
    T->kind = FRI_TRANSPORT_PEER;
    if (transport == FRI_TRANSPORT_RCCL) {
        if (!distinct) return undo(FRI_EINVAL);  // ranks share a device: RCCL cannot run them
        std::vector<ncclComm_t> c(n, nullptr), x(n, nullptr);
        ncclResult_t nr = ncclCommInitAll(c.data(), (int)n, dev.data());
        if (nr == ncclSuccess) {
            nr = ncclCommInitAll(x.data(), (int)n, dev.data());
            if (nr != ncclSuccess)
                for (auto cm : c) ncclCommDestroy(cm);
        }
        if (nr != ncclSuccess) {
            T->rk[0]->err = std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
            return undo(FRI_ERCCL);
        }
        T->kind = FRI_TRANSPORT_RCCL;
        for (uint32_t r = 0; r < n; r++) { T->rk[r]->tp.comm = c[r]; T->rk[r]->tp.xcomm = x[r]; }
    }
    for (uint32_t r = 0; r < n; r++) {
        Transport& tp = T->rk[r]->tp;
        tp.rank = (int)r;
        tp.world = (int)n;
        tp.team = T;
        tp.peer = T->kind == FRI_TRANSPORT_PEER;
    }
    try {
        for (uint32_t r = 1; r < n; r++) T->th.emplace_back(team_worker, T, r);
    } catch (...) {
        return undo(FRI_ENOMEM);
    }
    T->rk[0]->team_root = T;
    (void)hipSetDevice(dev[0]);
    *out = T->rk[0];
    return FRI_OK;
}

// The devices a caller that names none gets (fri_ctx_create_default):
// FRI_DEVICES, else the largest power-of-two prefix of the visible devices.
static int default_devices(std::vector<int>& dev, int& transport) {
    dev.clear();
    transport = FRI_TRANSPORT_PEER;
    if (const char* t = getenv("FRI_TRANSPORT")) {
        const std::string ts(t);
        if (ts == "rccl") transport = FRI_TRANSPORT_RCCL;
        else if (!ts.empty() && ts != "peer") return FRI_EINVAL;
    }
    const char* e = getenv("FRI_DEVICES");
    if (e && *e) {
        const std::string v(e);
        size_t i = 0;
        while (i <= v.size()) {
            const size_t j = std::min(v.find(',', i), v.size());
            std::string tok = v.substr(i, j - i);
            while (!tok.empty() && tok.front() == ' ') tok.erase(tok.begin());     // "0, 1" as well as "0,1"
            while (!tok.empty() && tok.back() == ' ') tok.pop_back();
            if (tok.empty() || tok.size() > 4 || tok.find_first_not_of("0123456789") != std::string::npos)
                return FRI_EINVAL;
            dev.push_back(atoi(tok.c_str()));
            i = j + 1;
        }
        const size_t n = dev.size();
        if (n == 0 || n > 64 || (n & (n - 1))) return FRI_EINVAL;
        return FRI_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return FRI_ENODEV;
    int k = 1;
    while (k * 2 <= std::min(ndev, 64)) k *= 2;
    for (int r = 0; r < k; r++) dev.push_back(r);
    return FRI_OK;
}

extern "C" int fri_ctx_create_default(uint32_t log_n_max, fri_ctx** out, uint32_t* n_ranks) {
    if (!out) return FRI_EINVAL;
    *out = nullptr;
    std::vector<int> dev;
    int transport = FRI_TRANSPORT_PEER;
    const int rc = default_devices(dev, transport);
    if (rc) return rc;
    if (n_ranks) *n_ranks = (uint32_t)dev.size();
    if (dev.size() == 1) return fri_ctx_create(dev[0], log_n_max, out);
    return fri_ctx_create_multi(dev.data(), (uint32_t)dev.size(), log_n_max, transport, out);
}

extern "C" int fri_debug_team_inject_failure(fri_ctx* ctx, uint32_t rank, int64_t op_index) {
    if (!ctx) return FRI_EINVAL;
    if (!ctx->team_root || ctx->team_root->kind != FRI_TRANSPORT_PEER)
        return fail(ctx, FRI_EINVAL, "not a multi-GPU context on the peer transport");
    if (rank >= ctx->team_root->G) return fail(ctx, FRI_EINVAL, "rank out of range");
    ctx->team_root->rk[rank]->tp.fail_at = op_index;
    return FRI_OK;
}

extern "C" int fri_debug_team_force_copy(fri_ctx* ctx, int enable) {
    if (!ctx) return FRI_EINVAL;
    if (!ctx->team_root || ctx->team_root->kind != FRI_TRANSPORT_PEER)
        return fail(ctx, FRI_EINVAL, "not a multi-GPU context on the peer transport");
    Team* T = ctx->team_root;
    T->kernel_pull = T->can_pull && !enable;
    return FRI_OK;
}

extern "C" int fri_debug_team_rank(fri_ctx* ctx, uint32_t rank, fri_ctx** out) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    if (!ctx->team_root) {
        if (rank) return fail(ctx, FRI_EINVAL, "not a multi-GPU context: rank 0 only");
        *out = ctx;
        return FRI_OK;
    }
    if (rank >= ctx->team_root->G) return fail(ctx, FRI_EINVAL, "rank out of range");
    *out = ctx->team_root->rk[rank];
    return FRI_OK;
}

// Destroy the ranks of a team (called by fri_ctx_destroy on rank 0 before
// rank 0's own teardown): each rank detaches on its own thread (RCCL
// communicators of one clique are destroyed together), then the workers end.
void fri::team_destroy(fri_ctx* root) {
    Team* T = root->team_root;
    (void)team_run(root, [T](uint32_t r) {
        fri_ctx* c = T->rk[r];
        if (c->tp.xcomm) ncclCommDestroy(c->tp.xcomm);
        if (c->tp.comm) ncclCommDestroy(c->tp.comm);
        c->tp.comm = c->tp.xcomm = nullptr;
        return FRI_OK;
    });
    for (uint32_t r = 1; r < T->G; r++) {
        T->rk[r]->tp.team = nullptr;
        fri_ctx_destroy(T->rk[r]);
    }
    root->tp.team = nullptr;
    root->team_root = nullptr;
    team_free(T);
    (void)hipSetDevice(root->device);
}

// Codewords the team commits sharded (run_commit_sharded's own threshold);
// smaller ones run on rank 0 alone.
static bool team_shards(const Team* T, uint32_t log_n) {
    return log_n >= SHARD_MIN_LOG && log_n >= T->logG + 12;
}

int fri::team_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                       uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas, fri_commit_result* out) {
    Team* T = ctx->team_root;
    if (!out) return fail(ctx, FRI_EINVAL, "null argument");
    if (!team_shards(T, log_n))
        return run_commit(ctx, host_coeffs, dev_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
    // FRI_FLAG_RANK_INPUTS: ranks 1..G-1 commit the copy of rank 0's input
    // buffer their plan staged at an earlier team commit instead of copying
    // it again over xGMI.  Trusted only as far as it is checked: every rank
    // first hashes the input it would commit (rank 0 the caller's buffer,
    // the others their resident copy; k_checksum), and a rank whose copy
    // differs (the caller rewrote the buffer since it was staged) makes the
    // call return FRI_ESTATE on every rank before anything is committed.
    std::vector<const uint32_t*> din(T->G, dev_coeffs);
    const bool rank_inputs = (flags & FRI_FLAG_RANK_INPUTS) != 0;
    if (rank_inputs) {
        if (!d || !ctx->user_in || dev_coeffs != ctx->user_in || d > ctx->user_cap)
            return fail(ctx, FRI_ESTATE, "FRI_FLAG_RANK_INPUTS: pass fri_ctx_input_buffer() (rank 0's input buffer)");
        for (uint32_t r = 1; r < T->G; r++) {
            const fri_ctx* c = T->rk[r];
            const Plan& p = c->cur_lane == 0 ? c->plan : c->lanes[0].plan;
            if (!p.valid || !p.sharded || p.d != d || p.log_n != log_n || p.offset != offset || p.G != T->G)
                return fail(ctx, FRI_ESTATE, "FRI_FLAG_RANK_INPUTS: no staged input of this shape on rank " +
                                                 std::to_string(r) + ": commit these coefficients once without it");
            din[r] = p.d_in;
        }
    }
    const uint32_t fl = flags & ~FRI_FLAG_RANK_INPUTS;
    std::vector<fri_commit_result> res(T->G);
    std::vector<uint64_t> sums(T->G, 0);
    int rc = team_run(ctx, [&](uint32_t r) {
        fri_ctx* c = T->rk[r];
        if (rank_inputs) {
            int rs = input_checksum(c, din[r], d, &sums[r]);
            if (rs) return rs;
            if (!team_barrier(T)) return fail(c, FRI_ERCCL, "another rank failed (" + T->why + ")");
            for (uint32_t q = 1; q < T->G; q++)
                if (sums[q] != sums[0])
                    return fail(c, FRI_ESTATE, "FRI_FLAG_RANK_INPUTS: rank " + std::to_string(q) +
                                                   "'s staged input differs from rank 0's input buffer (rewritten "
                                                   "since it was staged): commit without the flag to stage it");
        }
        return run_commit_sharded(c, host_coeffs, din[r], d, log_n, offset, chan_in, fl, forced_betas, &res[r]);
    });
    if (rc) return rc;
    // the redundant tops give every rank the whole transcript: they must agree
    for (uint32_t r = 1; r < T->G; r++)
        if (memcmp(&res[r], &res[0], sizeof(fri_commit_result)))
            return fail(ctx, FRI_ERCCL, "team ranks disagree on the transcript (rank " + std::to_string(r) + ")");
    *out = res[0];
    ctx->err.clear();
    return FRI_OK;
}

// Sharded layer k of the resident team commit, read back whole: rank r holds
// block p.block[k] of it (the switch layer's slot, gathered when the tail
// went local, holds the whole layer on every rank and is read from rank 0).
int fri::team_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out) {
    Team* T = ctx->team_root;
    const Plan& p0 = ctx->plan;
    const uint32_t L = p0.log_n - layer;
    const bool whole = (int)layer == p0.k_sw && p0.k_sw < p0.rmax;
    const size_t B = (size_t)1 << (L - T->logG);
    for (uint32_t r = 0; r < (whole ? 1u : T->G); r++) {
        fri_ctx* c = T->rk[r];
        const Plan& p = c->plan;
        FRI_HIP(ctx, hipSetDevice(c->device));
        const size_t words = whole ? ((size_t)1 << L) : B;
        FRI_HIP(ctx, hipMemcpyAsync(out + (whole ? 0 : (size_t)p.block[layer] * B), p.layers + p.layer_off[layer],
                                    words * 4, hipMemcpyDeviceToHost, c->stream));
    }
    for (uint32_t r = 0; r < (whole ? 1u : T->G); r++) FRI_HIP(ctx, hipStreamSynchronize(T->rk[r]->stream));
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    return FRI_OK;
}

// Level `level` of sharded layer k's tree: the lower L - log G levels from
// the ranks' block trees (block order), the top log G levels from the top
// tree every rank built (rank 0's).
int fri::team_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint32_t* w) {
    Team* T = ctx->team_root;
    const Plan& p0 = ctx->plan;
    const uint32_t L = p0.log_n - layer, Lb = L - T->logG;
    if (level > Lb) {
        const uint32_t j = level - Lb;
        const uint32_t* top = ctx->db.top + (size_t)layer * 2 * 64 * 8;
        FRI_HIP(ctx, hipMemcpyAsync(w, top + 8 * level_offset(T->logG, j), ((size_t)1 << (T->logG - j)) * 32,
                                    hipMemcpyDeviceToHost, ctx->stream));
        FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
        return FRI_OK;
    }
    const size_t cnt = (size_t)1 << (Lb - level);     // digests of this level per block
    for (uint32_t r = 0; r < T->G; r++) {
        fri_ctx* c = T->rk[r];
        const Plan& p = c->plan;
        FRI_HIP(ctx, hipSetDevice(c->device));
        FRI_HIP(ctx, hipMemcpyAsync(w + 8 * cnt * p.block[layer], p.trees + p.tree_off[layer] + 8 * level_offset(Lb, level),
                                    cnt * 32, hipMemcpyDeviceToHost, c->stream));
    }
    for (uint32_t r = 0; r < T->G; r++) FRI_HIP(ctx, hipStreamSynchronize(T->rk[r]->stream));
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    return FRI_OK;
}

// fri_decommit_query on a team commit: every rank runs the sharded
// decommitment (its openings, the peer all-gather, the max-combine); rank 0's
// output is the caller's.
int fri::team_decommit(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                         size_t paths_cap, size_t* paths_len) {
    Team* T = ctx->team_root;
    std::vector<std::vector<uint32_t>> vals(T->G);
    std::vector<std::vector<uint8_t>> pth(T->G);
    std::vector<size_t> plen(T->G, 0);
    for (uint32_t r = 1; r < T->G; r++) {
        vals[r].assign(values_cap ? values_cap : 1, 0u);
        pth[r].assign(paths_cap ? paths_cap : 1, 0u);
    }
    return team_run(ctx, [&](uint32_t r) {
        if (r == 0) return decommit_sharded(ctx, index, values, values_cap, paths, paths_cap, paths_len);
        return decommit_sharded(T->rk[r], index, vals[r].data(), values_cap, paths ? pth[r].data() : nullptr, paths_cap,
                                &plen[r]);
    });
}
