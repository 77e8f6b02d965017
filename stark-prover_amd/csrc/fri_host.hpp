// fri_host.hpp — host-side state of libfri_amd.so, shared by the translation
// units of the C ABI (include/fri_amd.h).  One file per concern:
//   fri_ctx.hip        context lifetime, profiling spans, diagnostics
//   fri_ops.hip        kernel-level entry points: batch inverse, LDE,
//                      interpolation, evaluation, fold, Merkle root
//   fri_commit.hip     the commit plan (layout, allocation) and the 1-GPU
//                      commit (static launch sequence, hipGraph capture/replay)
//   fri_lanes.hip      commit lanes, pipelined commits, the input buffer and
//                      which commit the read-backs serve (residency)
//   fri_readback.hip   read-backs, decommitment and the prover entry points
//   fri_transport.hip  collective transports (RCCL, host callbacks, loopback,
//                      in-process peer) and their self-test
//   fri_sharded.hip    one rank's coset-sharded commit and decommitment
//   fri_team.hip       the single-process multi-GPU team context
// Device-side layouts and kernel launchers are in fri_internal.hpp.
// Everything declared here has hidden visibility: the library exports the C
// ABI of fri_amd.h and nothing else of its host code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/fri_amd.h"
#include "fri_internal.hpp"

#pragma GCC visibility push(hidden)

namespace fri {

static_assert(MAXR == FRI_MAX_ROUNDS, "round bound");

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
    // The commit's input: d_in is the plan's private staging buffer (host
    // coefficients and other device pointers are copied there); src is what
    // the launch sequence of the commit being enqueued reads: d_in, or the
    // context's caller-owned input buffer (fri_ctx::user_in), read in place.
    uint32_t* d_in = nullptr;   size_t in_cap = 0;
    const uint32_t* src = nullptr;
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
    // Commit graphs: one per (result slot, input), the synchronous commit's
    // as slot FRI_MAX_INFLIGHT (the DevState copy-out node targets the slot);
    // input 0 reads d_in, input 1 the caller's buffer at graph_src (captured
    // again when that buffer moves).
    hipGraph_t graph[FRI_MAX_INFLIGHT + 1][2] = {};
    hipGraphExec_t exec[FRI_MAX_INFLIGHT + 1][2] = {};
    const uint32_t* graph_src[FRI_MAX_INFLIGHT + 1][2] = {};
    hipGraph_t tail_graph = nullptr;        // sharded plan: the local layers after the switch
    hipGraphExec_t tail_exec = nullptr;
    const uint32_t* tail_src = nullptr;     // the input pointer tail_exec was captured with
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
    bool can_pull = true;                   // every device can read every other's memory (peer access)
    bool kernel_pull = true;                // peer_op pulls with k_peer_pull (else hipMemcpyPeerAsync)
    std::vector<std::pair<int, int>> peer_pairs;   // device pairs whose peer access this team holds
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
}  // namespace fri

using namespace fri;

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
    bool slot_user[FRI_MAX_INFLIGHT] = {};   // pending slot i reads user_in (fri_ctx_input_upload waits for it)
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
    // The caller-owned input buffer (fri_ctx_input_buffer): written only by the
    // caller or by fri_ctx_input_upload, never by a commit; commits from it
    // read it in place, on any lane.
    uint32_t* user_in = nullptr;
    size_t user_cap = 0;
    uint64_t* d_csum = nullptr;     // input checksum (FRI_FLAG_RANK_INPUTS): device word ...
    uint64_t* h_csum = nullptr;     // ... and its pinned host copy
};

namespace fri {

// Device allocations of a context go through these, so that
// fri_ctx_device_bytes can report what one rank / one context holds in HBM.
template <class T>
inline hipError_t dalloc(fri_ctx* ctx, T** p, size_t bytes) {
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
inline void dfree(fri_ctx* ctx, const void* p) {
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

inline double rccl_timeout_s() {
    const char* e = getenv("FRI_RCCL_TIMEOUT_S");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 120.0;
}
inline double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
inline int fail(fri_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    return code;
}

// Device-reported commit failures (DevState.status, set by the layer-0 top
// or tail kernel): the input coefficients are validated on the device, in
// the layer-0 coefficient scan, rather than by a host pass over them.
inline const char* status_message(uint32_t status) {
    return status == FRI_EINVAL ? "coefficient not canonical (>= p)"
                                : "degree exceeds the domain (reference would panic)";
}

// Every value < p.  A branch-free max over 64 KiB blocks (the compiler
// vectorises it), with the early exit per block: the per-element early-exit
// loop cost about 1 ms per 2^21 coefficients of fri_commit's host input.
inline bool check_canonical(const uint32_t* v, size_t n) {
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

// ------------------------------------------------------------- commit ----
inline int rounds_bound(size_t d, uint32_t log_n) {
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
inline bool next_layer_sharded(uint32_t log_n, uint32_t logG, int k, int rmax) {
    const uint32_t Lk = log_n - (uint32_t)k;
    return k < rmax && (Lk - 1) >= SHARD_MIN_LOG && (Lk - 1 - logG) >= 10;
}
inline int switch_layer(uint32_t log_n, uint32_t logG, int rmax) {
    int k = 0;
    while (next_layer_sharded(log_n, logG, k, rmax)) k++;
    return k;
}
// The fold pairs block b with block b + G/2 (fold pairs (i, i + m/2)); the
// rank holding b (< G/2) keeps output block 2b, its partner 2b + 1.
inline void advance_blocks(std::vector<uint32_t>& block_of, std::vector<uint32_t>& rank_of, uint32_t G) {
    for (uint32_t r = 0; r < G; r++) {
        const uint32_t br = block_of[r];
        block_of[r] = br < G / 2 ? 2 * br : 2 * (br - G / 2) + 1;
    }
    for (uint32_t r = 0; r < G; r++) rank_of[block_of[r]] = r;
}
// Domain index of the first x^-1 a sharded fold of layer k needs on a rank
// holding block b of size B: the half-block [bb*B + (isA ? 0 : B/2), + B/2).
inline size_t fold_xinv_start(uint32_t b, uint32_t G, size_t B) {
    const bool isA = b < G / 2;
    return (size_t)(isA ? b : b - G / 2) * B + (isA ? 0 : B / 2);
}

inline NttPlan lde_plan(fri_ctx* ctx, uint32_t log_n) {
    NttPlan p{};
    p.log_n = log_n;
    p.tw = ctx->tw_fwd;
    return p;
}

inline void digest_to_bytes(const uint32_t* w, uint8_t* out) {
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(w[i] >> 24); out[4 * i + 1] = (uint8_t)(w[i] >> 16);
        out[4 * i + 2] = (uint8_t)(w[i] >> 8); out[4 * i + 3] = (uint8_t)w[i];
    }
}

// ---- fri_ctx.hip: timed spans of profiled commits (hipEvents on ctx->stream)
size_t span_begin(fri_ctx* ctx, const char* cls, uint64_t bytes);
void span_end(fri_ctx* ctx, size_t id);
void spans_collect(fri_ctx* ctx);

// ---- fri_lanes.hip: plans of the commit lanes and residency
void plan_release(fri_ctx* ctx, Plan& p);     // one plan (its lane's stream idle)
void plan_free(fri_ctx* ctx);                 // every lane's plan, after draining the lanes
int use_lane(fri_ctx* ctx, int j);            // install lane j in ctx->{plan, stream, d_state}
void settle(fri_ctx* ctx);                    // before a read-back: the resident commit's lane, drained

// ---- fri_commit.hip: plan and 1-GPU commit
void plan_layout(Plan& p, size_t d, uint32_t log_n, uint32_t G, uint32_t rank, size_t& lay, size_t& tre,
                 size_t& xin);
int plan_build(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t G = 1, uint32_t rank = 0);
uint32_t* coef_buf(Plan& p, int r);
LayerTask commit_task(fri_ctx* ctx, int k);
void init_state(fri_ctx* ctx, DevState* h, const fri_channel_state* chan_in, uint32_t flags,
                const uint32_t* forced_betas);
int commit_validate(fri_ctx* ctx, size_t d, uint32_t log_n, uint32_t offset, uint32_t flags,
                    const uint32_t* forced_betas);
int commit_enqueue(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                   uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                   const uint32_t* forced_betas, int slot);
int commit_finish(fri_ctx* ctx, DevState* h, uint32_t log_n, fri_commit_result* out);
int run_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d, uint32_t log_n,
               uint32_t offset, const fri_channel_state* chan_in, uint32_t flags, const uint32_t* forced_betas,
               fri_commit_result* out);

// ---- fri_readback.hip
int dq_alloc(fri_ctx* ctx);                   // pinned host buffer the gather kernels write

int input_checksum(fri_ctx* ctx, const uint32_t* d_src, size_t d, uint64_t* out);   // (synchronous)

// ---- fri_transport.hip
int tp_host_stage(fri_ctx* ctx, size_t bytes);
void rccl_abort(fri_ctx* ctx);
int sync_sharded(fri_ctx* ctx, hipStream_t s);
int tp_allgather(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, hipStream_t s);
int tp_alltoall(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes_per_peer, hipStream_t s);
int tp_sendrecv(fri_ctx* ctx, const void* dsend, void* drecv, size_t bytes, int peer, hipStream_t s, uint32_t chan);
int dist_buffers(fri_ctx* ctx, size_t M, uint32_t G, size_t gwords);

// ---- fri_sharded.hip
int run_commit_sharded(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d,
                       uint32_t log_n, uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas, fri_commit_result* out);
int decommit_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                     size_t paths_cap, size_t* paths_len);

// ---- fri_team.hip
void team_abort(Team* T, const std::string& why);
bool team_barrier(Team* T);
int team_run(fri_ctx* root, const std::function<int(uint32_t)>& fn);
void team_destroy(fri_ctx* root);
int team_commit(fri_ctx* ctx, const uint32_t* host_coeffs, const uint32_t* dev_coeffs, size_t d, uint32_t log_n,
                uint32_t offset, const fri_channel_state* chan_in, uint32_t flags, const uint32_t* forced_betas,
                fri_commit_result* out);
int team_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out);
int team_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint32_t* w);
int team_decommit(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap, uint8_t* paths,
                  size_t paths_cap, size_t* paths_len);

}  // namespace fri

#pragma GCC visibility pop
