// fri_api.hip — context, commit plan (static launch sequence + hipGraph) and
// the extern "C" entry points declared in include/fri_amd.h.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/fri_amd.h"
#include "fri_internal.hpp"
#include "sha256.hpp"

using namespace fri;

static_assert(MAXR == FRI_MAX_ROUNDS, "round bound");

namespace {

struct ProfEntry { double ms = 0; uint64_t launches = 0; uint64_t bytes = 0; };

struct Plan {
    bool valid = false;
    uint32_t log_n = 0;
    size_t d = 0;
    uint32_t offset = 0;
    int rmax = 0;
    // Shard-sized plan (fri_commit_sharded): rank `rank` of G holds only its
    // block of layers 0..k_sw (their slots, block-local trees and x^-1 slices
    // are block-sized); layers after k_sw are full-size local layers, and
    // layer k_sw's value slot is full-size when the tail goes local.
    bool sharded = false;
    uint32_t G = 1, rank = 0;
    int k_sw = -1;
    // Sharded coefficient fold: rank r holds coefficients [r*S_k, (r+1)*S_k)
    // of poly_k, S_k = 2^(cs0 - k), for k = 1..k_sw (coefA/B hold chunks);
    // coefF receives poly_{k_sw} whole at the switch to the local tail.
    uint32_t cs0 = 0;
    uint32_t* coefF = nullptr;  size_t coefF_cap = 0;
    uint32_t* d_in = nullptr;   size_t in_cap = 0;
    uint32_t* coefA = nullptr;
    uint32_t* coefB = nullptr;  size_t coef_cap = 0;
    uint32_t* layers = nullptr; size_t layer_off[MAXR + 2] = {0};
    uint32_t* trees = nullptr;  size_t tree_off[MAXR + 2] = {0};
    uint32_t* xinv = nullptr;   size_t xinv_off[MAXR + 2] = {0};
    size_t xinv_start[MAXR + 2] = {0};   // domain index of xinv slot k's first entry (sharded slices)
    uint32_t block[MAXR + 2] = {0};      // block this rank holds of sharded layer k (k <= k_sw)
    uint32_t* pre_lo = nullptr;
    uint32_t* pre_hi = nullptr;
    int32_t* wgmax = nullptr;       // per-workgroup coefficient maxima
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipGraph_t slot_graph[FRI_MAX_INFLIGHT] = {};       // fri_commit_device_async: one graph per result slot
    hipGraphExec_t slot_exec[FRI_MAX_INFLIGHT] = {};    // (the DevState copy-out node targets the slot)
    hipGraph_t tail_graph = nullptr;        // sharded plan: the local layers after the switch
    hipGraphExec_t tail_exec = nullptr;
    bool graph_profiled = false;
};

// One commit lane: a plan (every per-commit buffer: input, coefficient
// buffers, layers, trees, x^-1 tables, graphs), the stream the lane's commits
// run on and their device state.  Pipelined commits on one context are dealt
// to lanes (result slot i -> lane i mod max_lanes, created on first use), so
// consecutive commits run on different streams and one commit's serial tree
// tops overlap the next one's leaf hashing.  The lane of the most recently
// enqueued commit is the one installed in fri_ctx::{plan, stream, d_state}
// (use_lane), so every read-back serves that commit.
struct Lane {
    Plan plan;
    hipStream_t stream = nullptr;
    DevState* d_state = nullptr;
};

struct Team;   // in-process team (defined below)

// Collective transport of the sharded commit: RCCL on the context stream, or
// host-staged callbacks (synchronous; used by the gloo tests), or the peer
// transport of an in-process team (fri_ctx_create_multi: device copies
// between the ranks' buffers, ordered by events, on the same streams RCCL
// would use).
struct Transport {
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;     // main stream collectives
    ncclComm_t xcomm = nullptr;    // exchange stream (separate communicator: no cross-stream ordering hazard)
    bool host = false;
    bool loop = false;          // fri_debug_attach_loopback: every exchange returns this rank's own bytes
    bool peer = false;          // in-process team, peer transport (peer_op)
    Team* team = nullptr;       // the team this rank belongs to (peer or team RCCL transport)
    int64_t fail_at = -1;       // fri_debug_team_inject_failure: peer op index (this call) that fails
    int64_t n_ops = 0;          // peer ops issued by the current team call
    fri_collectives ops{};
    uint8_t* hs = nullptr;      // pinned staging
    uint8_t* hr = nullptr;
    size_t hcap = 0;
    std::vector<fri_transport_op> log;   // schedule of the last sharded call (fri_debug_transport_log)
};

// Scratch of the sharded commit (sized on first use).
struct DistBuf {
    size_t cap = 0;             // words in cyc/recv
    uint32_t* cyc = nullptr;    // coset slice / all-to-all send
    uint32_t* recv = nullptr;   // all-to-all / gather receive
    uint32_t* half = nullptr;   // partner half-block (even layers' exchanges)
    uint32_t* half2 = nullptr;  // partner half-block (odd layers': the fused leaf kernel still reads the other)
    uint32_t* top = nullptr;    // per-layer top trees (2G digests each)
    uint32_t* pre_lo = nullptr; // coset pre-scale tables
    uint32_t* pre_hi = nullptr;
    size_t gcap = 0;            // words in gath
    uint32_t* gath = nullptr;   // all-gathered layer at the switch to local
    uint32_t* dq = nullptr;     // sharded decommitment: this rank's openings + all ranks' (G + 1 slots)
    uint32_t* rec = nullptr;    // per-layer record: this rank's (REC_WORDS) then all ranks' (64 * REC_WORDS)
    ShardTop* shtop = nullptr;  // per layer: what the sharded top kernels read (MAXR + 1)
    std::vector<ShardTop> shtop_h;  // the contents last uploaded to shtop (re-uploaded only on change)
    std::vector<int32_t> sched_h;   // loopback rehearsal: recorded degree per layer (fri_debug_loopback_degrees)
};

// In-process team (fri_ctx_create_multi; see "in-process team" below).
struct PeerSlot {
    const void* send;
    void* recv;
    size_t bytes;
    uint32_t op, chan;
    int peer;
};

struct Team {
    uint32_t G = 1, logG = 0;
    int kind = FRI_TRANSPORT_PEER;          // FRI_TRANSPORT_PEER or FRI_TRANSPORT_RCCL
    std::vector<int> dev;
    std::vector<fri_ctx*> rk;               // rk[0] = the owning context
    bool kernel_pull = true;                // every device can read every other's memory
    // job dispatch to the worker threads (ranks 1..G-1)
    std::vector<std::thread> th;
    std::mutex jm;
    std::condition_variable jcv, dcv;
    uint64_t seq = 0;
    uint32_t left = 0;
    bool quit = false;
    std::function<int(uint32_t)> job;
    std::vector<int> rc;
    // rendezvous of the peer transport
    std::mutex bm;
    std::condition_variable bcv;
    uint64_t bgen = 0;
    uint32_t arrived = 0;
    bool aborted = false;
    std::string why;
    std::vector<PeerSlot> slot;
    std::vector<hipEvent_t> ev_ready, ev_done;   // per rank, created on its device
};

// One timed launch group: events recorded around it on the context stream.
struct TimedSpan { std::string cls; hipEvent_t b, e; uint64_t bytes; };

}  // namespace

struct fri_ctx {
    int device = 0;
    uint32_t log_n_max = 0;
    hipStream_t stream = nullptr;
    std::string err;
    uint32_t* tw_fwd = nullptr;     // stage-packed Montgomery twiddles, 2^log_n_max entries
    uint32_t* tw_inv = nullptr;
    uint32_t* scratch_a = nullptr;  // 2^log_n_max words each
    uint32_t* scratch_b = nullptr;
    uint32_t* scratch_c = nullptr;
    uint32_t* pow_lo = nullptr;
    uint32_t* pow_hi = nullptr;
    DevState* d_state = nullptr;
    DevState* h_state = nullptr;    // the state of the most recently enqueued commit (h_sync or a slot)
    DevState* h_sync = nullptr;     // pinned: synchronous commits
    // pipelined commits (fri_commit_device_async): pinned state per slot, an
    // event after its copy-out, the ticket it holds and whether it is unwaited
    DevState* h_slot[FRI_MAX_INFLIGHT] = {};
    hipEvent_t ev_slot[FRI_MAX_INFLIGHT] = {};
    uint64_t slot_ticket[FRI_MAX_INFLIGHT] = {};
    uint32_t slot_log_n[FRI_MAX_INFLIGHT] = {};
    bool slot_pending[FRI_MAX_INFLIGHT] = {};
    // a pipelined commit on another lane handed lane 0's input buffer: its
    // copy of that buffer, made on lane 0's stream, ends with this event
    hipEvent_t ev_src[FRI_MAX_INFLIGHT] = {};
    uint32_t* h_in[FRI_MAX_INFLIGHT] = {};  // fri_commit_async: pinned copy of the slot's host coefficients,
    uint32_t* d_slot_in[FRI_MAX_INFLIGHT] = {};   // its device copy (uploaded on h2d_stream while the
    size_t h_in_cap[FRI_MAX_INFLIGHT] = {};       // previous commit runs) and the upload's event
    hipEvent_t ev_in[FRI_MAX_INFLIGHT] = {};
    hipStream_t h2d_stream = nullptr;   // the device's shared upload stream (upload_stream())
    uint64_t next_ticket = 1;
    bool async_unsettled = false;   // commits enqueued since the stream was last drained
    Plan plan;
    Lane lanes[FRI_MAX_INFLIGHT];   // lanes[cur_lane] is empty: that lane lives in plan / stream / d_state
    int cur_lane = 0;
    int res_lane = 0;               // lane of the resident commit (init_state): the read-backs serve it
    int max_lanes = FRI_DEFAULT_LANES;
    int lanes_ok = FRI_MAX_INFLIGHT;   // lanes below this got plan memory (lowered on ENOMEM, pick_lane)
    int slot_lane[FRI_MAX_INFLIGHT] = {};            // lane of pending slot i
    uint64_t lane_ticket[FRI_MAX_INFLIGHT] = {};     // last ticket dealt to lane j (0: never)
    bool profiling = false;
    std::map<std::string, ProfEntry> prof;
    std::vector<TimedSpan> spans;      // recorded spans of the current commit
    std::vector<hipEvent_t> event_pool;
    size_t event_next = 0;
    Transport tp;
    DistBuf db;
    hipStream_t xstream = nullptr;  // exchange stream (overlaps the local tree)
    hipEvent_t ev_vals = nullptr, ev_xchg = nullptr;
    hipStream_t cstream = nullptr;  // coefficient-fold stream (overlaps the local tree)
    hipEvent_t ev_pre = nullptr, ev_coef = nullptr;
    uint32_t sharded_layers = 0;    // layers of the last commit held block-wise across ranks
    uint64_t commit_gen = 0;        // bumped by every commit: read-backs of an older proof are refused
    uint32_t commit_log_n = 0;      // codeword log2 of the resident commit
    uint32_t* interp_tmp = nullptr; // partials of fri_interpolate_points / fri_evaluate, fri_merkle_root's tree (grown on use)
    size_t interp_cap = 0;
    uint32_t* dq_host = nullptr;    // decommitment gather output: 64 KiB of coherent pinned host
    uint32_t* dq_dev = nullptr;     // memory the gather kernel writes directly (its device address)
    uint32_t* trace_tree = nullptr; // Merkle tree of the last fri_trace_commit LDE
    uint32_t* trace_lde = nullptr;  // ... and the LDE itself (prover: composition, queries)
    size_t trace_tree_cap = 0;      // leaves they can hold
    bool trace_valid = false;       // a trace commit is resident
    uint32_t trace_log_t = 0, trace_log_b = 0, trace_offset = 0;
    bool stuck = false;               // a stream stayed busy after an RCCL abort (sync_sharded)
    bool inject_stall = false;        // fri_debug_inject_stall: next RCCL all-to-all never completes
    uint32_t* stall_flag = nullptr;   // pinned host word the stalled kernel polls (set by rccl_abort)
    uint32_t* stall_flag_dev = nullptr;
    std::map<const void*, size_t> allocs;   // device allocations owned by the context (fri_ctx_device_bytes)
    size_t dev_bytes = 0, dev_peak = 0;
    size_t dev_cap = 0;             // fri_debug_set_device_cap: allocations beyond it fail (0: none)
    Team* team_root = nullptr;      // fri_ctx_create_multi: this context is rank 0 and owns the team
};

// Device allocations of a context go through these, so that
// fri_ctx_device_bytes can report what one rank / one context holds in HBM.
template <class T>
static hipError_t dalloc(fri_ctx* ctx, T** p, size_t bytes) {
    void* q = nullptr;
    if (ctx->dev_cap && ctx->dev_bytes + bytes > ctx->dev_cap) { *p = nullptr; return hipErrorOutOfMemory; }
    const hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) { *p = nullptr; return e; }
    *p = static_cast<T*>(q);
    ctx->allocs[q] = bytes;
    ctx->dev_bytes += bytes;
    if (ctx->dev_bytes > ctx->dev_peak) ctx->dev_peak = ctx->dev_bytes;
    return hipSuccess;
}
static void dfree(fri_ctx* ctx, const void* p) {
    if (!p) return;
    auto it = ctx->allocs.find(p);
    if (it != ctx->allocs.end()) {
        ctx->dev_bytes -= it->second;
        ctx->allocs.erase(it);
    }
    hipFree(const_cast<void*>(p));
}

#define FRI_HIP(ctx, expr)                                                              \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);             \
            return FRI_EHIP;                                                            \
        }                                                                               \
    } while (0)

static double rccl_timeout_s() {
    const char* e = getenv("FRI_RCCL_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 120.0;
}
static double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
static int fail(fri_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

// Every value < p.  A branch-free max over 64 KiB blocks (the compiler
// vectorises it), with the early exit per block: the per-element early-exit
// loop cost about 1 ms per 2^21 coefficients of fri_commit's host input.
// Device-reported commit failures (DevState.status, set by the layer-0 top
// or tail kernel): the input coefficients are validated on the device, in
// the layer-0 coefficient scan, rather than by a host pass over them.
static const char* status_message(uint32_t status) {
    return status == FRI_EINVAL ? "coefficient not canonical (>= p)"
                                : "degree exceeds the domain (reference would panic)";
}

static bool check_canonical(const uint32_t* v, size_t n) {
    // an OR of compares vectorises on the x86-64 baseline (an unsigned max
    // needs SSE4.1): about 2x faster per 2^21 values
    for (size_t i = 0; i < n; i += 16384) {
        const size_t e = n - i < 16384 ? n : i + 16384;
        uint32_t bad = 0;
        for (size_t j = i; j < e; j++) bad |= (uint32_t)(v[j] >= P);
        if (bad) return false;
    }
    return true;
}

static hipEvent_t pool_event(fri_ctx* ctx) {
    if (ctx->event_next == ctx->event_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        ctx->event_pool.push_back(e);
    }
    return ctx->event_pool[ctx->event_next++];
}

// Record the begin of a timed span (only while profiling).
static size_t span_begin(fri_ctx* ctx, const char* cls, uint64_t bytes) {
    if (!ctx->profiling) return (size_t)-1;
    TimedSpan sp{cls, pool_event(ctx), pool_event(ctx), bytes};
    hipEventRecord(sp.b, ctx->stream);
    ctx->spans.push_back(sp);
    return ctx->spans.size() - 1;
}
static void span_end(fri_ctx* ctx, size_t id) {
    if (id == (size_t)-1) return;
    hipEventRecord(ctx->spans[id].e, ctx->stream);
}
static void spans_collect(fri_ctx* ctx) {
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

extern "C" int fri_dist_detach(fri_ctx* ctx);
// team (fri_ctx_create_multi; defined at the end of this file)
static void team_destroy(fri_ctx* root);
static int team_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                       uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas, fri_commit_result* out);
static int team_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out);
static int team_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint32_t* w);
static int team_decommit(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                         size_t paths_cap, size_t* paths_len);
static int team_run(fri_ctx* root, const std::function<int(uint32_t)>& fn);

// Free one plan's buffers and graphs (its lane's stream must be idle).
static void plan_release(fri_ctx* ctx, Plan& p) {
    if (p.exec) hipGraphExecDestroy(p.exec);
    if (p.graph) hipGraphDestroy(p.graph);
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++) {
        if (p.slot_exec[i]) hipGraphExecDestroy(p.slot_exec[i]);
        if (p.slot_graph[i]) hipGraphDestroy(p.slot_graph[i]);
    }
    if (p.tail_exec) hipGraphExecDestroy(p.tail_exec);
    if (p.tail_graph) hipGraphDestroy(p.tail_graph);
    dfree(ctx, p.d_in); dfree(ctx, p.coefA); dfree(ctx, p.coefB); dfree(ctx, p.coefF); dfree(ctx, p.layers);
    dfree(ctx, p.trees); dfree(ctx, p.xinv); dfree(ctx, p.pre_lo); dfree(ctx, p.pre_hi); dfree(ctx, p.wgmax);
    p = Plan();
}

// Every lane's plan: pipelined commits may still use them, so every lane's
// stream is drained first.
static void plan_free(fri_ctx* ctx) {
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    for (Lane& ln : ctx->lanes)
        if (ln.stream) hipStreamSynchronize(ln.stream);
    plan_release(ctx, ctx->plan);
    for (Lane& ln : ctx->lanes) plan_release(ctx, ln.plan);
    ctx->lanes_ok = FRI_MAX_INFLIGHT;     // memory is back: every lane may build a plan again
}

// Install lane j in fri_ctx::{plan, stream, d_state} (creating its stream and
// device state on first use); the lane installed before goes back to its slot.
static int use_lane(fri_ctx* ctx, int j) {
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
    if (ctx->h_sync) hipHostFree(ctx->h_sync);
    for (int i = 0; i < FRI_MAX_INFLIGHT; i++) {
        if (ctx->h_slot[i]) hipHostFree(ctx->h_slot[i]);
        if (ctx->ev_slot[i]) hipEventDestroy(ctx->ev_slot[i]);
        if (ctx->ev_src[i]) hipEventDestroy(ctx->ev_src[i]);
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

// ------------------------------------------------------- kernel-level ----
extern "C" int fri_batch_inverse(fri_ctx* ctx, const uint32_t* in, uint32_t* out, size_t n) {
    if (!ctx || (!in && n) || (!out && n)) return fail(ctx, FRI_EINVAL, "null argument");
    if (!check_canonical(in, n)) return fail(ctx, FRI_EINVAL, "input not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    const size_t cap = (size_t)1 << ctx->log_n_max;
    for (size_t off = 0; off < n; off += cap) {
        size_t m = n - off < cap ? n - off : cap;
        FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, in + off, m * 4, hipMemcpyHostToDevice, ctx->stream));
        launch_batch_inverse(ctx->scratch_a, ctx->scratch_b, m, 0, ctx->stream);
        FRI_HIP(ctx, hipGetLastError());
        FRI_HIP(ctx, hipMemcpyAsync(out + off, ctx->scratch_b, m * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

static NttPlan lde_plan(fri_ctx* ctx, uint32_t log_n) {
    NttPlan p{};
    p.log_n = log_n;
    p.tw = ctx->tw_fwd;
    return p;
}

extern "C" int fri_lde(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n, uint32_t offset,
                       uint32_t* evals_out) {
    if (!ctx || !evals_out || (d && !coeffs)) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_n > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n exceeds context capacity");
    const size_t n = (size_t)1 << log_n;
    if (d > n) return fail(ctx, FRI_EINVAL, "more coefficients than domain points");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    if (!check_canonical(coeffs, d)) return fail(ctx, FRI_EINVAL, "coefficient not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if (d) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, coeffs, d * 4, hipMemcpyHostToDevice, ctx->stream));
    NttPlan p = lde_plan(ctx, log_n);
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_n, offset, 1u, ctx->stream);
    p.pre_lo = ctx->pow_lo;
    p.pre_hi = ctx->pow_hi;
    p.scratch = ctx->scratch_c;
    launch_ntt(p, ctx->scratch_a, d, ctx->scratch_b, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(evals_out, ctx->scratch_b, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

extern "C" int fri_interpolate(fri_ctx* ctx, const uint32_t* ys, uint32_t log_n, uint32_t offset,
                               uint32_t* coeffs_out, size_t* len_out) {
    if (!ctx || !ys || !coeffs_out || !len_out) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_n > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n exceeds context capacity");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    const size_t n = (size_t)1 << log_n;
    if (!check_canonical(ys, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, ys, n * 4, hipMemcpyHostToDevice, ctx->stream));
    NttPlan p{};
    p.log_n = log_n;
    p.tw = ctx->tw_inv;
    // coeff_j = n^-1 * offset^-j * sum_i ys_i w^-ij
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_n, inv_std(offset), inv_std((uint32_t)(n % P)), ctx->stream);
    p.post_lo = ctx->pow_lo;
    p.post_hi = ctx->pow_hi;
    launch_ntt(p, ctx->scratch_a, n, ctx->scratch_b, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(coeffs_out, ctx->scratch_b, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    size_t len = n;
    while (len > 0 && coeffs_out[len - 1] == 0) len--;          // Polynomial::new trim (ops.rs:19-37)
    *len_out = len;
    return FRI_OK;
}

// Device scratch of at least `words` words for the interpolation / evaluation
// partials (grown on demand, freed with the context).
static int ensure_tmp(fri_ctx* ctx, size_t words) {
    if (words <= ctx->interp_cap) return FRI_OK;
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->interp_tmp) dfree(ctx, ctx->interp_tmp);
    ctx->interp_tmp = nullptr;
    ctx->interp_cap = 0;
    if (dalloc(ctx, &ctx->interp_tmp, words * 4) != hipSuccess) return fail(ctx, FRI_ENOMEM, "partials scratch");
    ctx->interp_cap = words;
    return FRI_OK;
}
// Scratch grown past TMP_KEEP_WORDS is released after the call that grew it,
// so one large fri_merkle_root (the tree of 2^28 values is 16 GiB) does not
// pin HBM for the life of the context and starve a later commit plan; smaller
// scratch is kept (no hipFree, which synchronises the device, per call).
constexpr size_t TMP_KEEP_WORDS = (size_t)1 << 26;   // 256 MiB
static void tmp_trim(fri_ctx* ctx) {
    if (ctx->interp_cap <= TMP_KEEP_WORDS) return;
    (void)hipStreamSynchronize(ctx->stream);
    dfree(ctx, ctx->interp_tmp);
    ctx->interp_tmp = nullptr;
    ctx->interp_cap = 0;
}

// interpolate_lagrange_polynomials (interpolation.rs:121-152) on arbitrary
// points: weights, c_j = y_j w_j, f on the 2^k-th roots of unity, iNTT
// (fri_kernels.hip "arbitrary-point interpolate").
extern "C" int fri_interpolate_points(fri_ctx* ctx, const uint32_t* xs, const uint32_t* ys, size_t n,
                                      uint32_t* coeffs_out, size_t* len_out) {
    if (!ctx || !len_out || (n && (!xs || !ys || !coeffs_out))) return fail(ctx, FRI_EINVAL, "null argument");
    uint32_t log_N = 0;
    while (((size_t)1 << log_N) < n) log_N++;
    if (log_N > 17 || log_N > ctx->log_n_max)
        return fail(ctx, FRI_EINVAL, "arbitrary-point interpolation is O(n^2): n <= 2^17 and <= 2^log_n_max");
    if (!check_canonical(xs, n) || !check_canonical(ys, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    *len_out = 0;
    if (n == 0) return FRI_OK;                                   // Polynomial::zero() (interpolation.rs:133-136)
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t N = (size_t)1 << log_N;
    int rc = ensure_tmp(ctx, interp_tmp_words(n, log_N));
    if (rc) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, xs, n * 4, hipMemcpyHostToDevice, s));
    launch_interp_weights(ctx->scratch_a, n, ctx->scratch_b, ctx->interp_tmp, s);   // prod_{i!=j}(x_j - x_i)
    launch_batch_inverse(ctx->scratch_b, ctx->scratch_c, n, 1, s);          // w_j (Montgomery; 0 -> 0)
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_b, ys, n * 4, hipMemcpyHostToDevice, s));   // after the inverse (stream order)
    launch_interp_coeffs(ctx->scratch_b, ctx->scratch_c, n, s);             // c_j = y_j w_j
    launch_interp_eval(ctx->scratch_a, ctx->scratch_c, n, log_N, ctx->scratch_b, ctx->interp_tmp, s);   // f(w_N^k)
    NttPlan p{};
    p.log_n = log_N;
    p.tw = ctx->tw_inv;
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_N, 1u, inv_std((uint32_t)(N % P)), s);   // N^-1
    p.post_lo = ctx->pow_lo;
    p.post_hi = ctx->pow_hi;
    launch_ntt(p, ctx->scratch_b, N, ctx->scratch_a, s);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(coeffs_out, ctx->scratch_a, n * 4, hipMemcpyDeviceToHost, s));   // deg f < n
    FRI_HIP(ctx, hipStreamSynchronize(s));
    tmp_trim(ctx);
    size_t len = n;
    while (len > 0 && coeffs_out[len - 1] == 0) len--;          // Polynomial::new trim (ops.rs:19-37)
    *len_out = len;
    return FRI_OK;
}

extern "C" int fri_evaluate(fri_ctx* ctx, const uint32_t* coeffs, size_t d, const uint32_t* xs, size_t count,
                            uint32_t* out) {
    if (!ctx || (d && !coeffs) || (count && (!xs || !out))) return fail(ctx, FRI_EINVAL, "null argument");
    const size_t cap = (size_t)1 << ctx->log_n_max;
    if (d > cap || count > cap) return fail(ctx, FRI_EINVAL, "size exceeds context capacity");
    if (!check_canonical(coeffs, d) || !check_canonical(xs, count))
        return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if (d) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, coeffs, d * 4, hipMemcpyHostToDevice, ctx->stream));
    if (count) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_b, xs, count * 4, hipMemcpyHostToDevice, ctx->stream));
    const size_t tw = evaluate_tmp_words(d, count);
    if (tw) {
        const int rc = ensure_tmp(ctx, tw);
        if (rc) return rc;
    }
    launch_evaluate(ctx->scratch_a, d, ctx->scratch_b, count, ctx->scratch_c, ctx->interp_tmp, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    if (count) FRI_HIP(ctx, hipMemcpyAsync(out, ctx->scratch_c, count * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    tmp_trim(ctx);
    return FRI_OK;
}

extern "C" int fri_fold(fri_ctx* ctx, const uint32_t* layer, uint32_t log_m, uint32_t layer_offset, uint32_t beta,
                        uint32_t* out) {
    if (!ctx || !layer || !out) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_m < 1 || log_m > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_m out of range");
    if (layer_offset == 0 || layer_offset >= P || beta >= P) return fail(ctx, FRI_EINVAL, "bad offset/beta");
    const size_t m = (size_t)1 << log_m;
    if (!check_canonical(layer, m)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, layer, m * 4, hipMemcpyHostToDevice, ctx->stream));
    launch_coset_points(ctx->scratch_b, m / 2, layer_offset, log_m, ctx->stream);
    launch_batch_inverse(ctx->scratch_b, ctx->scratch_c, m / 2, 1, ctx->stream);
    launch_fold_plain(ctx->scratch_a, ctx->scratch_b, log_m, ctx->scratch_c, beta, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(out, ctx->scratch_b, (m / 2) * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

static void digest_to_bytes(const uint32_t* w, uint8_t* out) {
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(w[i] >> 24); out[4 * i + 1] = (uint8_t)(w[i] >> 16);
        out[4 * i + 2] = (uint8_t)(w[i] >> 8); out[4 * i + 3] = (uint8_t)w[i];
    }
}

// Non-power-of-two trees (rs_merkle promotes a lone right-most node).
__global__ void k_leaf_generic(const uint32_t* v, uint32_t* out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sha::leaf(v[i], out + 8 * i);
}
__global__ void k_level_generic(const uint32_t* in, uint32_t* out, size_t cnt) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t pc = (cnt + 1) / 2;
    if (j >= pc) return;
    if (2 * j + 1 < cnt) sha::node(in + 16 * j, in + 16 * j + 8, out + 8 * j);
    else for (int i = 0; i < 8; i++) out[8 * j + i] = in[16 * j + i];
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

extern "C" int fri_merkle_root(fri_ctx* ctx, const uint32_t* values, size_t n, uint8_t root32[32]) {
    if (!ctx || !values || !root32) return fail(ctx, FRI_EINVAL, "null argument");
    if (n == 0) return fail(ctx, FRI_EINVAL, "empty tree has no root (merkle/mod.rs:25)");
    const size_t cap = (size_t)1 << ctx->log_n_max;
    if (n > cap) return fail(ctx, FRI_EINVAL, "size exceeds context capacity");
    if (!check_canonical(values, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, values, n * 4, hipMemcpyHostToDevice, ctx->stream));
    // the tree lives in the context's partials scratch (no hipMalloc / hipFree,
    // which synchronises the device, per MerkleTree::new)
    uint32_t* root_dev;
    uint32_t* tree = nullptr;
    bool pow2 = (n & (n - 1)) == 0;
    if (pow2) {
        uint32_t L = 0;
        while (((size_t)1 << L) < n) L++;
        const int rc = ensure_tmp(ctx, ((size_t)2 << L) * 8);
        if (rc) return rc;
        tree = ctx->interp_tmp;
        LayerTask t{};
        t.values = ctx->scratch_a;
        t.tree = tree;
        t.L = L;
        launch_layer(t, ctx->stream);
        root_dev = tree + 8 * level_offset(L, L);
    } else {
        size_t total = 0;
        for (size_t m = n;; m = (m + 1) / 2) { total += m; if (m == 1) break; }
        const int rc = ensure_tmp(ctx, total * 8);
        if (rc) return rc;
        tree = ctx->interp_tmp;
        uint32_t* cur = tree;
        hipLaunchKernelGGL(k_leaf_generic, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                           ctx->scratch_a, cur, n);
        size_t cnt = n;
        while (cnt > 1) {
            size_t pc = (cnt + 1) / 2;
            uint32_t* nxt = cur + 8 * cnt;
            hipLaunchKernelGGL(k_level_generic, dim3((unsigned)((pc + 255) / 256)), dim3(256), 0, ctx->stream, cur,
                               nxt, cnt);
            cur = nxt;
            cnt = pc;
        }
        root_dev = cur;
    }
    FRI_HIP(ctx, hipGetLastError());
    uint32_t w[8];
    hipError_t e1 = hipMemcpyAsync(w, root_dev, 32, hipMemcpyDeviceToHost, ctx->stream);
    hipError_t e2 = hipStreamSynchronize(ctx->stream);
    tmp_trim(ctx);
    FRI_HIP(ctx, e1);
    FRI_HIP(ctx, e2);
    digest_to_bytes(w, root32);
    return FRI_OK;
}

// ------------------------------------------------------------- commit ----
static int rounds_bound(size_t d, uint32_t log_n) {
    if (d <= 1) return 0;
    int b = 0;
    for (size_t v = d - 1; v; v >>= 1) b++;
    return b < (int)log_n ? b : (int)log_n;
}

// ---- coset-sharded schedule (shared by the shard-sized plan and the commit) --
constexpr uint32_t SHARD_MIN_LOG = 20;   // layers of >= 2^20 elements are hashed sharded

// Layer k of a sharded commit hands a sharded layer k+1 on while that layer
// is still large (>= 2^SHARD_MIN_LOG) and its blocks hold >= 2^10 elements;
// otherwise layer k is the last sharded one (k_sw) and the tail goes local.
static bool next_layer_sharded(uint32_t log_n, uint32_t logG, int k, int rmax) {
    const uint32_t Lk = log_n - (uint32_t)k;
    return k < rmax && (Lk - 1) >= SHARD_MIN_LOG && (Lk - 1 - logG) >= 10;
}
static int switch_layer(uint32_t log_n, uint32_t logG, int rmax) {
    int k = 0;
    while (next_layer_sharded(log_n, logG, k, rmax)) k++;
    return k;
}
// The fold pairs block b with block b + G/2 (fold pairs (i, i + m/2)); the
// rank holding b (< G/2) keeps output block 2b, its partner 2b + 1.
static void advance_blocks(std::vector<uint32_t>& block_of, std::vector<uint32_t>& rank_of, uint32_t G) {
    for (uint32_t r = 0; r < G; r++) {
        const uint32_t br = block_of[r];
        block_of[r] = br < G / 2 ? 2 * br : 2 * (br - G / 2) + 1;
    }
    for (uint32_t r = 0; r < G; r++) rank_of[block_of[r]] = r;
}
// Domain index of the first x^-1 a sharded fold of layer k needs on a rank
// holding block b of size B: the half-block [bb*B + (isA ? 0 : B/2), + B/2).
static size_t fold_xinv_start(uint32_t b, uint32_t G, size_t B) {
    const bool isA = b < G / 2;
    return (size_t)(isA ? b : b - G / 2) * B + (isA ? 0 : B / 2);
}

// G == 1: the whole-codeword plan of fri_commit.  G > 1: the shard-sized plan
// of rank `rank` (see Plan::sharded); its x^-1 slots hold only the slices the
// rank's folds read, computed directly as (offset^(2^k) w_{n_k}^i)^-1 (the
// same values the whole-domain squaring chain gives: D_k = D_0^(2^k)).
// The plan's layout (offsets and sizes, no allocation): also what
// fri_debug_plan_layout reports, so the shard schedule is checkable on a host.
static void plan_layout(Plan& p, size_t d, uint32_t log_n, uint32_t G, uint32_t rank, size_t& lay, size_t& tre,
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

static int plan_build(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t G = 1, uint32_t rank = 0) {
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

static const uint32_t* root_ptr(const Plan& p, int k) {
    uint32_t L = p.log_n - (uint32_t)k;
    return p.trees + p.tree_off[k] + 8 * level_offset(L, L);
}

// poly_r coefficient buffer: poly_0 is the input, then A/B alternate.
static uint32_t* coef_buf(Plan& p, int r) {
    if (r == 0) return p.d_in;
    return (r % 2 == 1) ? p.coefA : p.coefB;
}

// Layer k of the resident plan as a commit-mode LayerTask.
static LayerTask commit_task(fri_ctx* ctx, int k) {
    Plan& p = ctx->plan;
    LayerTask t{};
    t.prev = k ? p.layers + p.layer_off[k - 1] : nullptr;
    t.xinv = k ? p.xinv + p.xinv_off[k - 1] : nullptr;
    t.values = p.layers + p.layer_off[k];
    t.tree = p.trees + p.tree_off[k];
    t.L = p.log_n - (uint32_t)k;
    t.k = k;
    t.coef_in = k ? coef_buf(p, k - 1) : p.d_in;
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
    launch_ntt(np, p.d_in, p.d, p.layers + p.layer_off[0], s);
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
        LayerTask t{};
        t.prev = k ? p.layers + p.layer_off[k - 1] : nullptr;
        t.xinv = k ? p.xinv + p.xinv_off[k - 1] : nullptr;
        t.values = p.layers + p.layer_off[k];
        t.tree = p.trees + p.tree_off[k];
        t.L = L;
        t.k = k;
        t.coef_in = k ? coef_buf(p, k - 1) : p.d_in;
        t.coef_out = k ? coef_buf(p, k) : nullptr;
        t.d0 = p.d;
        t.wgmax = p.wgmax;
        t.st = ctx->d_state;
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
static void init_state(fri_ctx* ctx, DevState* h, const fri_channel_state* chan_in, uint32_t flags,
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

// Pipelined commits may still be running: a call that reads the resident
// commit (its pinned state, layers or trees) drains the stream first.  The
// resident commit's lane is installed first: a call that switched lanes and
// then failed before it enqueued anything (a rejected argument, a plan that
// got no memory) leaves the resident commit on the lane it ran on, so its
// stream, plan and state are the ones the read-backs must use.
static void settle(fri_ctx* ctx) {
    if (ctx->res_lane != ctx->cur_lane) (void)use_lane(ctx, ctx->res_lane);   // (a used lane: cannot fail)
    if (!ctx->async_unsettled) return;
    (void)hipStreamSynchronize(ctx->stream);
    ctx->async_unsettled = false;
    if (ctx->h_state->status) ctx->h_state->n_layers = 0;   // a failed commit serves nothing
}

// Validate, build the plan and enqueue one commit on the context stream with
// its DevState in `hs` (h_sync, or slot `slot` of the pipelined commits: each
// slot replays its own graph, whose copy-out node targets that slot).
// The argument checks of a 1-GPU commit (everything but the coefficients,
// which the device validates): run before anything is copied or enqueued.
static int commit_validate(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t flags,
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

// 0 only in a diagnostic build (tests/test_gpu_pipelined.py shows the race it closes)
#ifndef FRI_LANE0_INPUT_ORDERED
#define FRI_LANE0_INPUT_ORDERED 1
#endif

static int commit_enqueue(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
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
    const Lane& l0 = ctx->lanes[0];
    if (FRI_LANE0_INPUT_ORDERED && slot >= 0 && ctx->cur_lane != 0 && d && dev_coeffs && l0.plan.valid &&
        dev_coeffs == l0.plan.d_in) {
        // Lane 0's input buffer (fri_ctx_input_buffer) handed to a commit on
        // another lane.  Every commit on lane 0 from another pointer stages its
        // coefficients into that buffer on lane 0's stream, so the copy is made
        // there too: it reads what the buffer holds in call order (after the
        // stagings of commits enqueued before this one, before those of later
        // ones), and this lane's stream waits for it.
        // The copy overwrites this lane's own input buffer, which the commits
        // already queued on this lane may still read: lane 0's stream first
        // waits for them (the event is re-recorded after the copy; each wait
        // binds to the record before it).
        if (!ctx->ev_src[slot]) FRI_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_src[slot], hipEventDisableTiming));
        FRI_HIP(ctx, hipEventRecord(ctx->ev_src[slot], s));
        FRI_HIP(ctx, hipStreamWaitEvent(l0.stream, ctx->ev_src[slot], 0));
        FRI_HIP(ctx, hipMemcpyAsync(p.d_in, dev_coeffs, d * 4, hipMemcpyDeviceToDevice, l0.stream));
        FRI_HIP(ctx, hipEventRecord(ctx->ev_src[slot], l0.stream));
        FRI_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_src[slot], 0));
    } else if (host_coeffs && d) {
        FRI_HIP(ctx, hipMemcpyAsync(p.d_in, host_coeffs, d * 4, hipMemcpyHostToDevice, s));
    } else if (dev_coeffs && dev_coeffs != p.d_in && d) {
        FRI_HIP(ctx, hipMemcpyAsync(p.d_in, dev_coeffs, d * 4, hipMemcpyDeviceToDevice, s));
    }
    const bool use_graph = !(flags & FRI_FLAG_NO_GRAPH) && !ctx->profiling;
    if (use_graph) {
        // the DevState copies in (from the pinned state just written) and out
        // are nodes of the graph: no host API call between the commits' kernels
        hipGraph_t& pg = slot < 0 ? p.graph : p.slot_graph[slot];
        hipGraphExec_t& px = slot < 0 ? p.exec : p.slot_exec[slot];
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
static int commit_finish(fri_ctx* ctx, DevState* h, uint32_t log_n, fri_commit_result* out) {
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

static int run_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                      uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                      const uint32_t* forced_betas, fri_commit_result* out) {
    if (!ctx || !out) return fail(ctx, FRI_EINVAL, "null argument");
    // (the argument checks before the lane switch; a failure after it leaves
    // the resident commit on its own lane, see settle)
    int rc = commit_validate(ctx, d, log_n, offset, flags, forced_betas);
    if (rc) return rc;
    // synchronous commits run on lane 0, whose input buffer is the one
    // fri_ctx_input_buffer hands out (after any commit pending on that lane)
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

extern "C" int fri_ctx_input_buffer(fri_ctx* ctx, size_t d, uint32_t** d_ptr) {
    if (!ctx || !d_ptr) return fail(ctx, FRI_EINVAL, "null argument");
    // The plan's input buffer is only stable for a fixed (d, log_n, offset);
    // the caller passes the returned pointer back to fri_commit_device, which
    // skips the copy when the pointers match.
    // lane 0's (synchronous commits run there; pipelined commits on other
    // lanes copy from it into their own input buffers)
    const Plan& p0 = ctx->cur_lane == 0 ? ctx->plan : ctx->lanes[0].plan;
    if (!p0.valid || p0.d != d) return fail(ctx, FRI_ESTATE, "build a plan first (commit once with this d)");
    *d_ptr = p0.d_in;
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
static int dq_alloc(fri_ctx* ctx);

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
static int dq_alloc(fri_ctx* ctx) {
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

// =================================================================== multi-GPU
static int tp_host_stage(fri_ctx* ctx, size_t bytes) {
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

static void rccl_abort(fri_ctx* ctx) {
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
static int sync_sharded(fri_ctx* ctx, hipStream_t s) {
    if (ctx->tp.host || !ctx->tp.comm) {
        FRI_HIP(ctx, hipStreamSynchronize(s));
        return FRI_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const double lim = rccl_timeout_s();
    // spin (yielding) for the first 200 us, which covers a commit's short
    // syncs at full responsiveness, then poll every 50 us so that a rank
    // waiting on its peers does not hold a host core at 100%
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return FRI_OK;
        if (e != hipErrorNotReady) FRI_HIP(ctx, e);
        const double el = seconds_since(t0);
        if (el > lim) break;
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
    return fail(ctx, FRI_ERCCL, "sharded commit: no progress in " + std::to_string((int)lim) +
                                    " s (RCCL communicators aborted" +
                                    (drained ? ")" : "; stream still busy: destroy the context)"));
}

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
static void team_abort(Team* T, const std::string& why) {
    std::lock_guard<std::mutex> g(T->bm);
    if (!T->aborted) T->why = why;
    T->aborted = true;
    T->bcv.notify_all();
}

// All G ranks arrive; false when the team was aborted first.
static bool team_barrier(Team* T) {
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

static int tp_allgather(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, hipStream_t s) {
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

static int tp_alltoall(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes_per_peer, hipStream_t s) {
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
static int tp_sendrecv(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, int peer, hipStream_t s,
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

extern "C" int fri_commit_degrees(fri_ctx* ctx, int32_t* out, size_t cap, uint32_t* n_out) {
    if (!ctx || !n_out) return fail(ctx, FRI_EINVAL, "null argument");
    settle(ctx);
    const uint32_t n = ctx->h_state->n_layers;
    *n_out = n;
    if (n && (!out || cap < n)) return fail(ctx, FRI_EINVAL, "degree buffer too small (n_layers entries)");
    for (uint32_t k = 0; k < n; k++) out[k] = ctx->h_state->deg[k];
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

static int dist_buffers(fri_ctx* ctx, size_t M, uint32_t G, size_t gwords);

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

static int dist_buffers(fri_ctx* ctx, size_t M, uint32_t G, size_t gwords) {
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

static int run_commit_sharded(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
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
    if (host_coeffs && d)
        FRI_HIP(ctx, hipMemcpyAsync(p.d_in, host_coeffs, d * 4, hipMemcpyHostToDevice, s));
    else if (dev_coeffs && dev_coeffs != p.d_in && d)   // (Default: a team rank reads rank 0's device buffer)
        FRI_HIP(ctx, hipMemcpyAsync(p.d_in, dev_coeffs, d * 4, hipMemcpyDefault, s));

    size_t sp;
    if (G == 2) {
        // ---- layer 0, two ranks: radix-2 decimation, no exchange ---------
        // P(offset w_n^(bM+j)) = E(offset^2 w_M^j) + (-1)^b offset w_n^j O(offset^2 w_M^j):
        // both size-M NTTs on every rank, then this rank's block.
        sp = span_begin(ctx, "lde", d * 4 + M * 12);
        const size_t de = (d + 1) / 2, dod = d / 2;
        launch_decimate(p.d_in, d, ctx->scratch_a, ctx->scratch_b, s);
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
        if (fold_chunks) launch_coset_coeffs(p.d_in, d, db.recv, M, pow_std(sft, M), s);
        launch_pow_table(db.pre_lo, db.pre_hi, log_n - logG, sft, 1u, s);
        NttPlan np{};
        np.log_n = log_n - logG;
        np.tw = ctx->tw_fwd;
        np.pre_lo = db.pre_lo;
        np.pre_hi = db.pre_hi;
        launch_ntt(np, fold_chunks ? db.recv : p.d_in, fold_chunks ? M : d, db.cyc, s);
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
            t.rec_c0 = kk ? coef_buf(p, kk) : p.d_in;
            t.rec_R = coef_grid(kk);
            t.G = G;
            t.recs_in = db.rec + REC_WORDS;
            t.sched_on = sched ? 1u : 0u;
            t.sched_deg = (sched && (size_t)kk < db.sched_h.size()) ? db.sched_h[kk] : -1;
            for (uint32_t b2 = 0; b2 < G; b2++) t.rank_of_block[b2] = (uint8_t)ro[b2];
            advance_blocks(bo, ro, G);
        }
        // the table depends only on the plan (and the loopback schedule), so
        // it is uploaded when it changes, from a copy that outlives the call:
        // no host sync in front of the commit's first launch.  The previous
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
        tc.coef_in = (k <= 1) ? p.d_in : coef_buf(p, k - 1);
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
static int decommit_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                            size_t paths_cap, size_t* paths_len);

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

static int decommit_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
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
        if (rc) team_abort(T, "rank " + std::to_string(r) + ": " + T->rk[r]->err);
        std::lock_guard<std::mutex> g(T->jm);
        T->rc[r] = rc;
        if (--T->left == 0) T->dcv.notify_all();
    }
}

static int team_run(fri_ctx* root, const std::function<int(uint32_t)>& fn) {
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
    if (rc0) team_abort(T, "rank 0: " + root->err);
    {
        std::unique_lock<std::mutex> lk(T->jm);
        T->dcv.wait(lk, [&] { return T->left == 0; });
    }
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
        for (uint32_t r = 1; r < n; r++)
            if (T->rk[r]) { T->rk[r]->tp = Transport(); fri_ctx_destroy(T->rk[r]); }
        if (T->rk[0]) { T->rk[0]->tp = Transport(); T->rk[0]->team_root = nullptr; fri_ctx_destroy(T->rk[0]); }
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
    for (uint32_t a = 0; a < n; a++)
        for (uint32_t b = 0; b < n; b++) {
            if (dev[a] == dev[b]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, dev[a], dev[b]) != hipSuccess || !can) { T->kernel_pull = false; continue; }
            (void)hipSetDevice(dev[a]);
            const hipError_t e = hipDeviceEnablePeerAccess(dev[b], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) T->kernel_pull = false;
            (void)hipGetLastError();
        }
    // transport: RCCL (one communicator per rank for the main stream, one for
    // the exchange stream) when asked or when automatic and it initialises;
    // ranks sharing a device can only use the peer transport
    bool distinct = true;
    for (uint32_t a = 0; a < n; a++)
        for (uint32_t b = a + 1; b < n; b++) distinct = distinct && dev[a] != dev[b];
    T->kind = FRI_TRANSPORT_PEER;
    if (transport != FRI_TRANSPORT_PEER && distinct) {
        std::vector<ncclComm_t> c(n, nullptr), x(n, nullptr);
        ncclResult_t nr = ncclCommInitAll(c.data(), (int)n, dev.data());
        if (nr == ncclSuccess) {
            nr = ncclCommInitAll(x.data(), (int)n, dev.data());
            if (nr != ncclSuccess)
                for (auto cm : c) ncclCommDestroy(cm);
        }
        if (nr == ncclSuccess) {
            T->kind = FRI_TRANSPORT_RCCL;
            for (uint32_t r = 0; r < n; r++) { T->rk[r]->tp.comm = c[r]; T->rk[r]->tp.xcomm = x[r]; }
        } else if (transport == FRI_TRANSPORT_RCCL) {
            T->rk[0]->err = std::string("ncclCommInitAll: ") + ncclGetErrorString(nr);
            return undo(FRI_ERCCL);
        }
    } else if (transport == FRI_TRANSPORT_RCCL) {
        return undo(FRI_EINVAL);                 // ranks share a device: RCCL cannot run them
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

extern "C" int fri_debug_team_inject_failure(fri_ctx* ctx, uint32_t rank, int64_t op_index) {
    if (!ctx) return FRI_EINVAL;
    if (!ctx->team_root || ctx->team_root->kind != FRI_TRANSPORT_PEER)
        return fail(ctx, FRI_EINVAL, "not a multi-GPU context on the peer transport");
    if (rank >= ctx->team_root->G) return fail(ctx, FRI_EINVAL, "rank out of range");
    ctx->team_root->rk[rank]->tp.fail_at = op_index;
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
static void team_destroy(fri_ctx* root) {
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

static int team_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                       uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas, fri_commit_result* out) {
    Team* T = ctx->team_root;
    if (!out) return fail(ctx, FRI_EINVAL, "null argument");
    if (!team_shards(T, log_n))
        return run_commit(ctx, host_coeffs, dev_coeffs, d, log_n, offset, chan_in, flags, forced_betas, out);
    // FRI_FLAG_RANK_INPUTS: each rank reads its own input buffer (resident
    // since the last team commit that staged these coefficients)
    std::vector<const uint32_t*> din(T->G, dev_coeffs);
    if (flags & FRI_FLAG_RANK_INPUTS) {
        uint32_t logG = T->logG;
        for (uint32_t r = 0; r < T->G; r++) {
            const fri_ctx* c = T->rk[r];
            const Plan& p = c->cur_lane == 0 ? c->plan : c->lanes[0].plan;
            if (!p.valid || !p.sharded || p.d != d || p.log_n != log_n || p.offset != offset || p.G != T->G ||
                (r == 0 && dev_coeffs != p.d_in) || log_n < logG)
                return fail(ctx, FRI_ESTATE, "FRI_FLAG_RANK_INPUTS: commit these coefficients once without it, "
                                             "and pass fri_ctx_input_buffer()");
            din[r] = p.d_in;
        }
    }
    const uint32_t fl = flags & ~FRI_FLAG_RANK_INPUTS;
    std::vector<fri_commit_result> res(T->G);
    int rc = team_run(ctx, [&](uint32_t r) {
        return run_commit_sharded(T->rk[r], host_coeffs, din[r], d, log_n, offset, chan_in, fl, forced_betas, &res[r]);
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
static int team_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out) {
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
static int team_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint32_t* w) {
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
static int team_decommit(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
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
