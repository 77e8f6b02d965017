// fri_layer.hip — per-layer FRI commit pipeline on gfx950.
//
// One FRI layer k (2^L evaluations) is committed by at most three kinds of
// launch, all gated on the device state (no host round trip per round):
//
//   k_layer_leaf  (2^(L-10) workgroups, L >= 11)
//       fold of layer k-1 with beta_{k-1}      (src/fri/fri_commit.rs:53-65)
//       leaf hashes SHA256(u64_be(v))           (src/merkle/mod.rs:14-15)
//       tree levels 1..4 (2048 leaves -> 128 nodes per workgroup)
//       a slice of the coefficient fold of round k-1 (fri_commit.rs:32-50)
//       with per-workgroup maxima (no hot atomics) for the exact degree
//   k_tree_mid    (levels l -> l+4, 1024 nodes in / 64 out per workgroup)
//   k_tree_top    (ONE workgroup): last <= 10 levels -> root, degree of
//       poly_k, Fiat-Shamir step (channel.rs:35-55): send(root_hex),
//       beta_k = U256(state) mod p or the final send (fri_commit.rs:114).
//       For layers of <= 2^10 elements it also does the fold, the leaves and
//       the whole coefficient fold itself (single launch per small layer).
//
// Each thread of the leaf / mid kernels takes 4 consecutive inputs and folds
// them to one level+2 node in registers (no LDS, no barrier, no idle lanes);
// levels +3/+4 pair through LDS.  Loads/stores of values are 16 B per lane.
#include "fri_internal.hpp"
#include "sha256_fast.hpp"
#include "sha256_quad.hpp"

namespace fri {

constexpr uint32_t INV2_M2 = 0x80000000u;   // Montgomery(2^-1) = 2^31 mod p

// Diagnostic build (-DFRI_STAMPS, lib/libfri_amd_stamps.so): thread 0 of a
// top kernel records s_memrealtime at phase boundaries.  Never in the product.
#ifdef FRI_STAMPS
#define TOP_STAMP(i)                                                                     \
    do {                                                                                 \
        if (COMMIT && threadIdx.x == 0) t.st->stamps[t.k][(i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define TOP_CLK(i)                                                                               \
    do {                                                                                           \
        if (COMMIT && threadIdx.x == 0) t.st->stamps[t.k][(i)] = __builtin_amdgcn_s_memtime();     \
    } while (0)
#define TOP_STAMP_T(i, tid_)                                                                       \
    do {                                                                                           \
        if (COMMIT && threadIdx.x == (tid_)) t.st->stamps[t.k][(i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define TOP_STAMP(i) do {} while (0)
#define TOP_CLK(i) do {} while (0)
#define TOP_STAMP_T(i, tid_) do {} while (0)
#endif
// workgroup 0 of a wide leaf kernel: start, leaves done, levels done (60..62)
#ifdef FRI_STAMPS
#define WIDE_STAMP(i)                                                                              \
    do {                                                                                           \
        if (COMMIT && blockIdx.x == 0 && threadIdx.x == 0) t.st->stamps[t.k][(i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define WIDE_STAMP(i) do {} while (0)
#endif
// the same marks for a layer of the tail kernel (t: that layer's task)
#ifdef FRI_STAMPS
#define TAIL_STAMP_T(i, tid_, fn)                                                  \
    do {                                                                           \
        if (threadIdx.x == (tid_)) t.st->stamps[t.k][(i)] = fn();                  \
    } while (0)
#define TAIL_STAMP(i) TAIL_STAMP_T(i, 0, __builtin_amdgcn_s_memrealtime)
#define TAIL_CLK(i) TAIL_STAMP_T(i, 0, __builtin_amdgcn_s_memtime)
#else
#define TAIL_STAMP_T(i, tid_, fn) do {} while (0)
#define TAIL_STAMP(i) do {} while (0)
#define TAIL_CLK(i) do {} while (0)
#endif

__device__ __forceinline__ uint32_t fold1(uint32_t a, uint32_t b, uint32_t xinv_m, uint32_t beta_m) {
    uint32_t s = add(a, b), t = sub(a, b);
    return mmul(add(s, mmul(mmul(t, xinv_m), beta_m)), INV2_M2);
}

// Wave priority of the latency-bound chain kernels (tops, tail, narrow mids):
// s_setprio raises their waves over co-resident throughput waves (another
// commit lane's leaf hashing) in the SIMD's issue arbitration.  0 = off.
// Three commit lanes: 3.50 -> 3.42 ms per 2^24 commit, synchronous commits
// unchanged (3 interleaved rounds, profiles/r04_prio_*.txt).
#ifndef FRI_CHAIN_PRIO
#define FRI_CHAIN_PRIO 3
#endif
__device__ __forceinline__ void chain_prio() {
    if (FRI_CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(FRI_CHAIN_PRIO);
}

struct Dg { uint32_t w[8]; };

__device__ __forceinline__ void dg_load(const uint32_t* p, Dg& d) {
    uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
    d.w[0] = a.x; d.w[1] = a.y; d.w[2] = a.z; d.w[3] = a.w; d.w[4] = b.x; d.w[5] = b.y; d.w[6] = b.z; d.w[7] = b.w;
}
__device__ __forceinline__ void dg_store(uint32_t* p, const Dg& d) {
    reinterpret_cast<uint4*>(p)[0] = make_uint4(d.w[0], d.w[1], d.w[2], d.w[3]);
    reinterpret_cast<uint4*>(p)[1] = make_uint4(d.w[4], d.w[5], d.w[6], d.w[7]);
}
__device__ __forceinline__ void dg_lds_load(const uint4* p, Dg& d) {
    uint4 a = p[0], b = p[1];
    d.w[0] = a.x; d.w[1] = a.y; d.w[2] = a.z; d.w[3] = a.w; d.w[4] = b.x; d.w[5] = b.y; d.w[6] = b.z; d.w[7] = b.w;
}
__device__ __forceinline__ void dg_lds_store(uint4* p, const Dg& d) {
    p[0] = make_uint4(d.w[0], d.w[1], d.w[2], d.w[3]);
    p[1] = make_uint4(d.w[4], d.w[5], d.w[6], d.w[7]);
}
__device__ __forceinline__ void hnode(const Dg& l, const Dg& r, Dg& o) { shaf::node(l.w, r.w, o.w); }
__device__ __forceinline__ void hleaf(uint32_t v, Dg& o) { shaf::leaf(v, o.w); }
// compact (looped) forms for the latency-bound mid / top kernels
__device__ __forceinline__ void cnode(const Dg& l, const Dg& r, Dg& o) { shaf::node_compact(l.w, r.w, o.w); }
__device__ __forceinline__ void cleaf(uint32_t v, Dg& o) { shaf::leaf_compact(v, o.w); }

// One node per pair of lanes (sha256_quad.hpp) for the narrow, latency-bound
// levels: thread `tid` < 2*cnt hashes node tid/2; the even lane writes
// digest words 4..7, the odd lane words 0..3 (LDS for the next level, HBM).
__device__ __forceinline__ void pair_level(const uint4* A, uint4* B, uint32_t* out, uint32_t tid, uint32_t cnt,
                                           const shaq::Role& R) {
    // Below 32 nodes the whole of wave 0 still runs: the spare lane pairs
    // recompute node (q mod cnt) and store nothing. A partly masked wave runs
    // the node 0.7-2.7 K cycles slower than a full one (8.4 K), by an amount
    // that changes from launch to launch (bench/plateau_micro.hip mode 10,
    // profiles/r01_plateau_micro_masked.txt). cnt is a power of two.
    if (tid >= max(2 * cnt, 64u)) return;
    const uint32_t q = (tid >> 1) & (cnt - 1), half = (tid & 1u) ^ 1u;
    const bool real = tid < 2 * cnt;
    Dg a, b;
    dg_lds_load(A + 4 * q, a);
    dg_lds_load(A + 4 * q + 2, b);
    uint32_t o[4];
    shaq::node(a.w, b.w, o, R);
    if (!real) return;
    const uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
    B[2 * q + half] = v;
    reinterpret_cast<uint4*>(out + 8 * q)[half] = v;
}

// Narrow levels (<= 32 nodes, one round wave) with the message schedule made
// by wave 1 of the workgroup (sha256_quad.hpp produce / node_ext): the round
// wave, wave 0, issues 48 x 7 fewer instructions per node.  Wave 1 sits on
// another SIMD (waves are dealt to the SIMDs in turn), and at these levels it
// is otherwise idle.  `ord`: the level's ordinal within the launch, strictly
// increasing (the flag counts 3 per level).  0 = off (A/B builds).
#ifndef FRI_SCHED_PRODUCER
#define FRI_SCHED_PRODUCER 1
#endif
// The channel's root blocks (jobs 3, 4) with their schedule on wave 6
// (chan_produce): within noise, 4.612 vs 4.616 ms per 2^24 commit over 4
// interleaved A/B rounds (profiles/r05_sched_channel_ab.txt), so off.
#ifndef FRI_SCHED_CHANNEL
#define FRI_SCHED_CHANNEL 0
#endif
struct SchedLds {
    uint32_t wk[32 * 48];       // per node W16..W63 + K (16-byte aligned rows of 48 words)
    uint32_t flag;
};
__device__ __forceinline__ void sched_init(SchedLds* sl) {
    if (FRI_SCHED_PRODUCER && threadIdx.x == 0) sl->flag = 0u;    // (before the launch's first barrier)
}
__device__ __forceinline__ void pair_level_s(const uint4* A, uint4* B, uint32_t* out, uint32_t tid, uint32_t cnt,
                                             const shaq::Role& R, SchedLds* sl, uint32_t ord) {
    if (!FRI_SCHED_PRODUCER || cnt > 32) {
        pair_level(A, B, out, tid, cnt, R);
        return;
    }
    const uint32_t wv = tid >> 6;
    if (wv > 1) return;
    const uint32_t lane = tid & 63u;
    const uint32_t q = (lane >> 1) & (cnt - 1), half = (lane & 1u) ^ 1u;
    const bool real = lane < 2 * cnt;            // spare lanes redo node q mod cnt and store nothing (see pair_level)
    Dg a, b;
    dg_lds_load(A + 4 * q, a);
    dg_lds_load(A + 4 * q + 2, b);
    if (wv == 1) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 8; i++) { w[i] = a.w[i]; w[8 + i] = b.w[i]; }
        shaq::produce(w, sl->wk + 48 * q, &sl->flag, 3u * ord, real && (lane & 1u) == 0u, lane == 0u, R);
        return;
    }
    uint32_t o[4];
    shaq::node_ext(a.w, b.w, o, R, sl->wk + 48 * q, &sl->flag, 3u * ord);
    if (!real) return;
    const uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
    B[2 * q + half] = v;
    reinterpret_cast<uint4*>(out + 8 * q)[half] = v;
}

// Barrier that waits only for this wave's LDS traffic: HIP's __syncthreads()
// also drains vmcnt, i.e. waits ~1 us for the level's global digest stores,
// which no other wave of the workgroup reads.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

// Coefficient task of one workgroup (w of G): k == 0 -> max nonzero index
// of the input (deg_0); k >= 1 -> fold slice c'_j = c_2j + beta c_2j+1 with
// maxima of c', even part, odd part.  Results: wgmax[3w .. 3w+2].
// coef_slice: the slice over threads [t0, t0 + nthr) (whole waves), per-wave
// maxima into red[3 * (wave - t0 / 64) ..]; coef_combine (one thread, after a
// barrier): red -> wgmax.
__device__ __forceinline__ void coef_slice(const LayerTask& t, uint32_t w, uint32_t G, int32_t* red, uint32_t t0,
                                           uint32_t nthr) {
    int m0 = -1, m1 = -1, m2 = -1;
    const uint32_t tx = threadIdx.x - t0;
    // this rank's coefficient range (all of poly_k unless sharded), split
    // evenly over the G workgroups; indices j are global
    const size_t jhi_all = t.jhi ? t.jhi : ~(size_t)0;
    if (t.k == 0) {
        // m1 >= 0 flags a coefficient >= p (the input is validated here, on
        // the device, instead of by a host scan before the upload)
        const size_t a = t.jlo, b = min(t.d0, jhi_all), n = b > a ? b - a : 0;
        const size_t cs = (n + G - 1) / G, lo = a + (size_t)w * cs, hi = min(b, lo + cs);
        const uint32_t* in = t.coef_in - t.ibase;
        for (size_t j = lo + tx; j < hi; j += nthr) {
            const uint32_t c = in[j];
            if (c) m0 = max(m0, (int)j);
            if (c >= P) m1 = 0;
        }
    } else {
        const DevState* st = t.st;
        const size_t len = (size_t)(st->deg[t.k - 1] + 1), nlen = (len + 1) / 2;
        const uint32_t beta_m = st->beta_mont[t.k - 1];
        const size_t a = t.jlo, b = min(nlen, jhi_all), n = b > a ? b - a : 0;
        const size_t cs = (n + G - 1) / G, lo = a + (size_t)w * cs, hi = min(b, lo + cs);
        const uint32_t* in = t.coef_in - t.ibase;
        uint32_t* outp = t.coef_out - t.obase;
        for (size_t j = lo + tx; j < hi; j += nthr) {
            uint32_t e = in[2 * j];
            uint32_t o = (2 * j + 1 < len) ? in[2 * j + 1] : 0u;
            uint32_t v = add(e, mmul(o, beta_m));
            outp[j] = v;
            if (v) m0 = (int)j;
            if (e) m1 = (int)j;
            if (o) m2 = (int)j;
        }
    }
    m0 = wave_max_i(m0); m1 = wave_max_i(m1); m2 = wave_max_i(m2);
    const uint32_t wave = tx >> 6;
    if ((tx & 63) == 0) { red[3 * wave] = m0; red[3 * wave + 1] = m1; red[3 * wave + 2] = m2; }
}
__device__ __forceinline__ void coef_combine(const LayerTask& t, uint32_t w, const int32_t* red, uint32_t nw) {
    int a = -1, b = -1, c = -1;
    for (uint32_t i = 0; i < nw; i++) { a = max(a, red[3 * i]); b = max(b, red[3 * i + 1]); c = max(c, red[3 * i + 2]); }
    t.wgmax[3 * w] = a; t.wgmax[3 * w + 1] = b; t.wgmax[3 * w + 2] = c;
}
__device__ __forceinline__ void coef_task(const LayerTask& t, uint32_t w, uint32_t G, int32_t* red /*LDS [3*waves]*/) {
    coef_slice(t, w, G, red, 0, blockDim.x);
    lds_barrier();          // red[] only: the leaf digest stores need not drain here
    if (threadIdx.x == 0) coef_combine(t, w, red, blockDim.x / 64);
}

#ifndef FRI_QUAD_LEAVES_FIRST
#define FRI_QUAD_LEAVES_FIRST 1
#endif
// Four consecutive level-l digests (or leaves) per thread -> level l+2 node.
// lv0/lv1 are this layer's level l+0 / l+1 arrays (lv0 written only for
// leaves: it is the input otherwise).
template <bool LEAVES>
__device__ __forceinline__ void quad(const uint4& vals, const uint32_t* in0, uint32_t* lv0, uint32_t* lv1,
                                     size_t q /*quad index*/, Dg& out) {
    Dg a, b, n0, n1;
#if FRI_QUAD_LEAVES_FIRST
    if (LEAVES) {
        // all four leaves first: the thread's 128 contiguous level-l bytes are
        // written together (no partly written line waits in L2 for its other
        // half), and so are its two level-(l+1) digests
        Dg c, d;
        hleaf(vals.x, a); hleaf(vals.y, b); hleaf(vals.z, c); hleaf(vals.w, d);
        dg_store(lv0 + 8 * (4 * q), a); dg_store(lv0 + 8 * (4 * q + 1), b);
        dg_store(lv0 + 8 * (4 * q + 2), c); dg_store(lv0 + 8 * (4 * q + 3), d);
        hnode(a, b, n0);
        hnode(c, d, n1);
        dg_store(lv1 + 8 * (2 * q), n0);
        dg_store(lv1 + 8 * (2 * q + 1), n1);
        hnode(n0, n1, out);
        return;
    }
#endif
    if (LEAVES) { hleaf(vals.x, a); hleaf(vals.y, b); dg_store(lv0 + 8 * (4 * q), a); dg_store(lv0 + 8 * (4 * q + 1), b); }
    else { dg_load(in0 + 8 * (4 * q), a); dg_load(in0 + 8 * (4 * q + 1), b); }
    hnode(a, b, n0);
    dg_store(lv1 + 8 * (2 * q), n0);
    if (LEAVES) { hleaf(vals.z, a); hleaf(vals.w, b); dg_store(lv0 + 8 * (4 * q + 2), a); dg_store(lv0 + 8 * (4 * q + 3), b); }
    else { dg_load(in0 + 8 * (4 * q + 2), a); dg_load(in0 + 8 * (4 * q + 3), b); }
    hnode(a, b, n1);
    dg_store(lv1 + 8 * (2 * q + 1), n1);
    hnode(n0, n1, out);
}

// Levels l+3, l+4 through LDS: TPB level-(l+2) nodes -> TPB/2 -> TPB/4.
template <uint32_t TPB>
__device__ __forceinline__ void lds_two_levels(uint4* lds, const Dg& mine, uint32_t* lv2, uint32_t* lv3, uint32_t* lv4,
                                               size_t g2 /*first level-(l+2) index of this WG*/) {
    uint4* A = lds;             // TPB digests
    uint4* B = lds + 2 * TPB;   // TPB/2 digests
    const uint32_t t = threadIdx.x;
    dg_store(lv2 + 8 * (g2 + t), mine);
    dg_lds_store(A + 2 * t, mine);
    lds_barrier();
    if (t < TPB / 2) {
        Dg l, r, o;
        dg_lds_load(A + 4 * t, l); dg_lds_load(A + 4 * t + 2, r);
        hnode(l, r, o);
        dg_lds_store(B + 2 * t, o);
        dg_store(lv3 + 8 * (g2 / 2 + t), o);
    }
    lds_barrier();
    if (t < TPB / 4) {
        Dg l, r, o;
        dg_lds_load(B + 4 * t, l); dg_lds_load(B + 4 * t + 2, r);
        hnode(l, r, o);
        dg_store(lv4 + 8 * (g2 / 4 + t), o);
    }
}

__device__ __forceinline__ bool gated_off(const LayerTask& t) {
    return t.gst && t.gidx >= 0 && !t.gst->active[t.gidx];
}

// PAIR: a sharded block tree with the pair fold fused in (LayerTask::prev2),
// launched as a part of the layer's workgroups (wg_base).
__device__ __forceinline__ uint32_t pair_beta(const LayerTask& t) { return t.gst->beta_mont[t.gidx]; }

// TPB threads, 4 leaves each: 4*TPB leaves -> TPB/4 level-4 nodes per WG.
template <bool FOLD, bool COMMIT, uint32_t TPB, bool PAIR = false>
__global__ __launch_bounds__(TPB) void k_layer_leaf(LayerTask t) {
    if (gated_off(t)) return;
    __shared__ uint4 lds[3 * TPB];
    __shared__ int32_t red[3 * (TPB / 64)];
    const uint32_t L = t.L;
    const size_t wg = PAIR ? (size_t)blockIdx.x + t.wg_base : (size_t)blockIdx.x;
    const size_t q = wg * TPB + threadIdx.x;   // quad index: leaves 4q..4q+3
    uint4 v;
    if (FOLD) {
        const size_t half = (size_t)1 << L;
        const uint32_t beta_m = COMMIT ? t.st->beta_mont[t.k - 1] : (PAIR ? pair_beta(t) : t.beta_m);
        uint4 a = reinterpret_cast<const uint4*>(t.prev)[q];
        uint4 b = reinterpret_cast<const uint4*>(PAIR ? t.prev2 : t.prev + half)[q];
        uint4 x = reinterpret_cast<const uint4*>(t.xinv)[q];
        v.x = fold1(a.x, b.x, x.x, beta_m); v.y = fold1(a.y, b.y, x.y, beta_m);
        v.z = fold1(a.z, b.z, x.z, beta_m); v.w = fold1(a.w, b.w, x.w, beta_m);
        reinterpret_cast<uint4*>(t.values)[q] = v;
    } else {
        v = reinterpret_cast<const uint4*>(t.values)[q];
    }
    uint32_t* tr = t.tree;
    Dg top;
    quad<true>(v, nullptr, tr + 8 * level_offset(L, 0), tr + 8 * level_offset(L, 1), q, top);
    if (COMMIT) coef_task(t, blockIdx.x, gridDim.x, red);
    lds_two_levels<TPB>(lds, top, tr + 8 * level_offset(L, 2), tr + 8 * level_offset(L, 3),
                        tr + 8 * level_offset(L, 4), wg * TPB);
}

// Levels of the wide leaf kernel with fewer than WIDE_PAIR_MAX nodes in the
// whole layer are latency-bound: they use the lane-pair node.
#ifndef WIDE_PAIR_MAX
#define WIDE_PAIR_MAX (1u << 16)
#endif

// Tree levels the wide leaf kernel builds: all 8 of its 256-leaf subtree when
// the rest of the layer then fits the single-workgroup top (no mid launch).
__host__ __device__ __forceinline__ uint32_t wide_levels(uint32_t L) { return L <= 8 + TOP_LOG ? 8u : 4u; }

// Wide leaf kernel for narrow layers (2^10 .. 2^18 elements): one leaf per
// lane, 256 leaves per workgroup, levels 1..4 through LDS (one node per lane
// per level): latency 1 leaf + 4 nodes instead of the quad form's 4 + 5.
template <bool FOLD, bool COMMIT, bool PAIR = false>
__global__ __launch_bounds__(256) void k_layer_leaf_wide(LayerTask t) {
    if (gated_off(t)) return;
    WIDE_STAMP(60);
    __shared__ uint4 lds[2 * 256 + 2 * 128];
    __shared__ int32_t red[12];
    __shared__ SchedLds sl;
    sched_init(&sl);
    const uint32_t L = t.L;
    const size_t wg = PAIR ? (size_t)blockIdx.x + t.wg_base : (size_t)blockIdx.x;
    const size_t grid = PAIR ? (size_t)t.wg_total : (size_t)gridDim.x;   // the whole layer's workgroups
    const size_t i = wg * 256 + threadIdx.x;
    uint32_t v;
    if (FOLD) {
        const size_t half = (size_t)1 << L;
        const uint32_t beta_m = COMMIT ? t.st->beta_mont[t.k - 1] : (PAIR ? pair_beta(t) : t.beta_m);
        v = fold1(t.prev[i], PAIR ? t.prev2[i] : t.prev[i + half], t.xinv[i], beta_m);
        t.values[i] = v;
    } else {
        v = t.values[i];
    }
    uint32_t* tr = t.tree;
    Dg d;
    cleaf(v, d);       // looped form: its ~2 KB of code costs less cold than the unrolled leaf saves (A/B -0.6%)
    dg_store(tr + 8 * i, d);
    uint4* A = lds;
    uint4* B = lds + 2 * 256;
    dg_lds_store(A + 2 * threadIdx.x, d);
    lds_barrier();
    WIDE_STAMP(61);
    uint32_t cnt = 256;
    const shaq::Role qr = shaq::role_of(threadIdx.x);
    if (grid * 128 < WIDE_PAIR_MAX) chain_prio();   // from level 1 on, all on lane pairs
    const uint32_t nlev = wide_levels(L);
#pragma unroll 1
    for (uint32_t j = 1; j <= nlev; j++) {
        cnt >>= 1;
        uint32_t* out = tr + 8 * (level_offset(L, j) + (wg << (8 - j)));
        if ((size_t)cnt * grid < WIDE_PAIR_MAX) {
            pair_level_s(A, B, out, threadIdx.x, cnt, qr, &sl, j);   // latency-bound level: node per lane pair
        } else if (threadIdx.x < cnt) {
            Dg a, b, o;
            dg_lds_load(A + 4 * threadIdx.x, a);
            dg_lds_load(A + 4 * threadIdx.x + 2, b);
            hnode(a, b, o);
            dg_lds_store(B + 2 * threadIdx.x, o);
            dg_store(out + 8 * threadIdx.x, o);
        }
        // the coefficient slice (needed only by the layer's top kernel) on
        // waves 2-3, idle from level 2 on: off the tree's critical path
        if (COMMIT && j == 2 && threadIdx.x >= 128) coef_slice(t, blockIdx.x, gridDim.x, red, 128, 128);
        lds_barrier();
        uint4* tmp = A; A = B; B = tmp;
    }
    if (COMMIT && threadIdx.x == 128) coef_combine(t, blockIdx.x, red, 2);   // nlev >= 4: red[] settled
    WIDE_STAMP(62);
}

// Reduce the coefficient-maxima triples of the R producer workgroups of this
// workgroup's inputs (R <= 64) into one triple (wave 0).
__device__ __forceinline__ void reduce_mx(const int32_t* in, int32_t* out, uint32_t w, uint32_t R) {
    if (threadIdx.x >= 64) return;
    const uint32_t i = R * w + threadIdx.x;
    int a = -1, b = -1, c = -1;
    if (threadIdx.x < R) { a = in[3 * i]; b = in[3 * i + 1]; c = in[3 * i + 2]; }
    a = wave_max_i(a); b = wave_max_i(b); c = wave_max_i(c);
    if (threadIdx.x == 0) { out[3 * w] = a; out[3 * w + 1] = b; out[3 * w + 2] = c; }
}

#ifndef MID_PAIR_BY_WG
#define MID_PAIR_BY_WG 0     // 1: k_tree_mid<1024> levels 2-4 on lane pairs whatever the layer width (round-2 form)
#endif

// Mid tree: NIN level-l nodes per workgroup -> NIN/16 level-(l+4) nodes,
// one node per lane per level.  NIN = 1024 (512 threads) for wide levels,
// 256 (128 threads: one wave per SIMD on every level) for narrow ones.
template <uint32_t NIN>
__global__ __launch_bounds__(NIN / 2) void k_tree_mid(uint32_t* tree, uint32_t L, uint32_t l, const DevState* st,
                                                      int gate, const int32_t* mx_in, int32_t* mx_out, uint32_t R) {
    if (st && gate >= 0 && !st->active[gate]) return;
    if (NIN == 256) chain_prio();
    // level 1 reads its two inputs straight from HBM (64 contiguous bytes per
    // thread), so LDS holds only levels 1.. (NIN/2 + NIN/4 digests): more
    // workgroups per CU for the wide instance
    __shared__ uint4 lds[NIN + NIN / 2];
    __shared__ SchedLds sl;
    sched_init(&sl);
    uint4* A = lds;
    uint4* B = lds + NIN;
    const uint32_t t = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * NIN;
    const uint32_t* in = tree + 8 * level_offset(L, l);
    {
        Dg a, b, o;
        dg_load(in + 8 * (base + 2 * t), a);
        dg_load(in + 8 * (base + 2 * t + 1), b);
        if (mx_in) reduce_mx(mx_in, mx_out, blockIdx.x, R);
        hnode(a, b, o);
        dg_lds_store(A + 2 * t, o);
        dg_store(tree + 8 * (level_offset(L, l + 1) + (base >> 1) + t), o);
    }
    lds_barrier();
    const shaq::Role qr = shaq::role_of(t);
    uint32_t cnt = NIN / 2;
#pragma unroll 1
    for (uint32_t j = 2; j <= 4; j++) {
        cnt >>= 1;
        uint32_t* out = tree + 8 * (level_offset(L, l + j) + (base >> j));
        // lane pairs only where the whole level is narrow: a lane-pair node
        // issues 1744 instructions on two lanes, a per-lane node 2290 on one,
        // and the wide instance's levels of >= 2^16 nodes are issue-bound
        const bool narrow = NIN == 1024 && !MID_PAIR_BY_WG ? (size_t)cnt * gridDim.x < WIDE_PAIR_MAX
                                                           : 2 * cnt <= NIN / 2;
        if (narrow) {
            pair_level_s(A, B, out, t, cnt, qr, &sl, j);   // narrow: latency-bound
        } else if (t < cnt) {
            Dg a, b, o;
            dg_lds_load(A + 4 * t, a);
            dg_lds_load(A + 4 * t + 2, b);
            hnode(a, b, o);
            dg_lds_store(B + 2 * t, o);
            dg_store(out + 8 * t, o);
        }
        lds_barrier();
        uint4* tmp = A; A = B; B = tmp;
    }
}

// Eight tree levels in one launch for the narrow part of a large layer:
// 256 level-l digests per workgroup -> 1 level-(l+8) digest, every level on
// lane pairs (level 1 reads its children straight from HBM).  Replaces two
// k_tree_mid<256> launches: one kernel boundary, one HBM round trip of the
// level-(l+4) digests and one cold start less per layer.
__global__ __launch_bounds__(256) void k_tree_mid8(uint32_t* tree, uint32_t L, uint32_t l, const DevState* st,
                                                   int gate, const int32_t* mx_in, int32_t* mx_out, uint32_t R) {
    if (st && gate >= 0 && !st->active[gate]) return;
    chain_prio();
    __shared__ uint4 lds[256 + 128];
    __shared__ SchedLds sl;
    sched_init(&sl);
    uint4* A = lds;
    uint4* B = lds + 256;
    const uint32_t t = threadIdx.x;
    const size_t base = (size_t)blockIdx.x * 256;
    const uint32_t* in = tree + 8 * level_offset(L, l);
    const shaq::Role qr = shaq::role_of(t);
    {
        const uint32_t q = t >> 1, half = (t & 1u) ^ 1u;
        Dg a, b;
        dg_load(in + 8 * (base + 2 * q), a);
        dg_load(in + 8 * (base + 2 * q + 1), b);
        if (mx_in) reduce_mx(mx_in, mx_out, blockIdx.x, R);
        uint32_t o[4];
        shaq::node(a.w, b.w, o, qr);
        const uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
        A[2 * q + half] = v;
        reinterpret_cast<uint4*>(tree + 8 * (level_offset(L, l + 1) + (base >> 1) + q))[half] = v;
    }
    lds_barrier();
    uint32_t cnt = 128;
#pragma unroll 1
    for (uint32_t j = 2; j <= 8; j++) {
        cnt >>= 1;
        pair_level_s(A, B, tree + 8 * (level_offset(L, l + j) + (base >> j)), t, cnt, qr, &sl, j);
        lds_barrier();
        uint4* tmp = A; A = B; B = tmp;
    }
}

// One scalar load per 64-byte line of every __constant__ table the compact
// SHA forms read (KTAB, PAD_KW_C, PAD_KW_1024, PAD_KW_1536, 256 B each):
// fills the CU's scalar cache while the inputs load, instead of cold misses
// inside level 1 and inside the channel send.  Loads land in clobbered SGPRs
// and are drained inside the statement.
__device__ __forceinline__ void ktouch(const void* sym) {
    uint32_t a, b, c, d;
    asm volatile("s_nop 4\n\t"
                 "s_load_dword %0, %4, 0x0\n\ts_load_dword %1, %4, 0x40\n\t"
                 "s_load_dword %2, %4, 0x80\n\ts_load_dword %3, %4, 0xc0\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(b), "=&s"(c), "=&s"(d)
                 : "s"(sym)
                 : "memory");
}
__device__ __forceinline__ void kcache_touch_sha_tables() {
    ktouch(&shaf::KTAB[0]);
    ktouch(&shaf::PAD_KW_C.kw[0]);
    ktouch(&shaf::PAD_KW_1024.kw[0]);
    ktouch(&shaf::PAD_KW_1536.kw[0]);
}

// ------------------------------------------------------------ channel ----
// Frozen spec: messages are built word by word in registers.
__device__ __forceinline__ uint32_t hexch(uint32_t nib) { return nib < 10u ? 0x30u + nib : 0x57u + nib; }
// 4 bytes -> 8 lowercase hex chars -> 2 big-endian message words
__device__ __forceinline__ void hex2(uint32_t x, uint32_t& hi, uint32_t& lo) {
    hi = (hexch(x >> 28) << 24) | (hexch((x >> 24) & 15u) << 16) | (hexch((x >> 20) & 15u) << 8) | hexch((x >> 16) & 15u);
    lo = (hexch((x >> 12) & 15u) << 24) | (hexch((x >> 8) & 15u) << 16) | (hexch((x >> 4) & 15u) << 8) | hexch(x & 15u);
}
// one byte -> hex(hex(byte)) = 4 chars = one message word.  For a nibble n,
// hexch(n) is '0'+n or 'a'+n-10, whose own hex is "3" '0'+n or "6" '0'+n-9:
// 0x3330 + n, plus 0x2F7 when n >= 10 (two 16-bit SWAR lanes).
__device__ __forceinline__ uint32_t hexhex(uint32_t b) {
    const uint32_t x = ((b & 0xF0u) << 12) | (b & 0x0Fu);
    const uint32_t ge = ((x + 0x00060006u) >> 4) & 0x00010001u;
    return 0x33303330u + x + ge * 0x2F7u;
}

// Channel work of one top kernel as a sequence of compression jobs run by
// wave 7 (lane pairs redundant), with ONE lane-pair compress and ONE
// compress_kw call site: the jobs done during the narrow tree levels (off
// the critical path) leave exactly the code the post-root jobs need in the
// I-cache.
//   0  rehash block   X = compress(IV, hex(cs))        channel.rs:75-76, the
//   1  rehash pad     cs = X = pad(X)                  receive's deferred rehash
//   2  midstate       X = compress(IV, hex(cs))        first block of the next send
//   3  root block 1   X = compress(X | IV, hex(hex(root[0..15])))   channel.rs:35-39,
//   4  root block 2   X = compress(X, hex(hex(root[16..31])))       message = root hex
//   5  root pad       cs = X = pad_{1536|1024}(X)      -> S
//   6  final block 1  X = compress(IV, hex(cs))        fri_commit.rs:114,
//   7  final block 2  cs = X = compress(X, hex(be64(fv)) | pad)   send(final.to_bytes())
enum { CJ_REHASH = 0, CJ_MID = 2, CJ_ROOT = 3, CJ_FINAL = 6, CJ_END_ROUND = 6, CJ_END_FINAL = 8 };

// Lane-pair form (sha256_quad.hpp): X is this lane's half of the chaining
// value (even lane words 4..7, odd lane 0..3); cs stays whole on every lane.
// wk (FRI_SCHED_PRODUCER): the two root-message blocks (jobs 3, 4) take their
// rounds 16..63 from rows 0 / 1 of wk, made by chan_produce on wave 6; flags
// base + 1 .. base + 6.
__device__ __forceinline__ void chan_job(int j, uint32_t cs[8], uint32_t X[4], uint32_t has, const uint4* root_lds,
                                         uint32_t fv, const shaq::Role& R, const uint32_t* wk = nullptr,
                                         const uint32_t* flag = nullptr, uint32_t base = 0) {
    // the job and the channel flags are wave-uniform: in SGPRs the job's
    // branches are scalar and its padding table is read by scalar loads
    // (a per-lane table pointer costs a vector-load round trip per 16 rounds)
    j = __builtin_amdgcn_readfirstlane(j);
    has = __builtin_amdgcn_readfirstlane(has);
    uint32_t w[16];
    const bool pad = (j == 1) || (j == 5);
    if (j == 0 || j == 2 || j == 6) {
#pragma unroll
        for (int i = 0; i < 8; i++) hex2(cs[i], w[2 * i], w[2 * i + 1]);
#pragma unroll
        for (int i = 0; i < 4; i++) X[i] = R.iv[i];
    } else if (j == 3 || j == 4) {
        // one root byte per lane (lanes 0..15: this block's 16 bytes), its
        // hex(hex()) word computed once, then read out as the 16 wave-uniform
        // message words: 1 + 16 instructions instead of 16 per-word encodings
        const uint32_t b = (__lane_id() & 15u) + (j == 4 ? 16u : 0u);
        const uint32_t rw = reinterpret_cast<const uint32_t*>(root_lds)[b >> 2];
        const uint32_t hh = hexhex((rw >> (24 - 8 * (b & 3))) & 255u);
#pragma unroll
        for (int jj = 0; jj < 16; jj++) w[jj] = __builtin_amdgcn_readlane(hh, jj);
        if (j == 3 && !has) {
#pragma unroll
            for (int i = 0; i < 4; i++) X[i] = R.iv[i];
        }
    } else if (j == 7) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = 0u;
        w[0] = 0x30303030u; w[1] = 0x30303030u;   // "00000000": high u32 of the u64 is 0
        hex2(fv, w[2], w[3]);
        w[4] = 0x80000000u;
        w[15] = 80u * 8u;                           // hex(state) (64) + 16 chars
    }
    if (pad) shaq::compress_kw(X, j == 1 ? shaf::PAD_KW_C.kw : (has ? shaf::PAD_KW_1536.kw : shaf::PAD_KW_1024.kw), R);
    else if (wk && (j == 3 || j == 4)) shaq::compress_ext(X, w, R, wk + 48 * (j - 3), flag, base + 3 * (j - 3));
    else shaq::compress(X, w, R);
    if (j == 1 || j == 5 || j == 7) {            // cs = X, both halves on every lane
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t o = shaq::swap01(X[i]);
            cs[i] = R.is_a ? X[i] : o;
            cs[4 + i] = R.is_a ? o : X[i];
        }
    }
}

// The schedules of the root message's two blocks (jobs 3 and 4: hex(hex(root))
// in two 64-byte halves), on a producer wave while the channel wave runs the
// rounds: both messages are known once the root is, so the producer makes
// both rows (0, 1) in the iteration of job 3; flags base + 1 .. base + 6.
__device__ __forceinline__ void chan_produce(const uint4* root_lds, SchedLds* sl, uint32_t base, const shaq::Role& R) {
    const uint32_t lane = __lane_id();
#pragma unroll 1
    for (uint32_t jb = 0; jb < 2; jb++) {
        const uint32_t b = (lane & 15u) + 16u * jb;
        const uint32_t rw = reinterpret_cast<const uint32_t*>(root_lds)[b >> 2];
        const uint32_t hh = hexhex((rw >> (24 - 8 * (b & 3))) & 255u);
        uint32_t w[16];
#pragma unroll
        for (int jj = 0; jj < 16; jj++) w[jj] = __builtin_amdgcn_readlane(hh, jj);
        shaq::produce(w, sl->wk + 48 * jb, &sl->flag, base + 3 * jb, lane == 0, lane == 0, R);
    }
}

// channel.rs:47-72: beta = U256(state) mod p  (the rehash is deferred).
// U256(state) = sum_i s_i 2^(32 (7-i)): eight independent products with the
// Montgomery weights 2^(32 (8-i)) mod p and a sum tree, instead of eight
// dependent Horner steps on the critical path after the root.
constexpr uint32_t pow2_32k_mod_p(int k) {
    uint64_t r = 1;
    for (int j = 0; j < k; j++) r = (r << 32) % P;
    return (uint32_t)r;
}
__device__ __forceinline__ uint32_t chan_beta(const uint32_t s[8]) {
    constexpr uint32_t W[8] = {pow2_32k_mod_p(8), pow2_32k_mod_p(7), pow2_32k_mod_p(6), pow2_32k_mod_p(5),
                               pow2_32k_mod_p(4), pow2_32k_mod_p(3), pow2_32k_mod_p(2), pow2_32k_mod_p(1)};
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; i++) t[i] = mmul(s[i] >= P ? s[i] - P : s[i], W[i]);
    return add(add(add(t[0], t[1]), add(t[2], t[3])), add(add(t[4], t[5]), add(t[6], t[7])));
}

// ---------------------------------------------------------------- top ----
// One workgroup.  FROM_LEAVES: the layer has N = 2^L <= 1024 elements and is
// done entirely here (fold, leaves, all levels, whole coefficient task).
// Otherwise: N = 2^(L-l) <= 1024 level-l digests -> root.
// COMMIT: the degree of poly_k is reduced up front (its inputs are complete
// at launch); wave 7 runs the channel jobs (chan_job) during the levels whose
// nodes fit waves 0-2, then after the root, in extra iterations of the level
// loop (uniform barrier count).
// SHARD (coset-sharded layers, run_commit_sharded; never FROM_LEAVES):
//   !COMMIT: the top of this rank's block tree; it also writes the rank's
//            per-layer record (t.shard->rec_out: block root, the maxima of
//            its coefficient slice reduced from rec_R workgroup triples, its
//            first coefficient), which the ranks then all-gather;
//   COMMIT:  the replicated top of the layer: its N = G inputs are the block
//            roots in the all-gathered records (rank order, permuted to block
//            order and stored as the top tree's level 0), the maxima and the
//            final-value candidate (rank 0's first coefficient) too.
template <bool FROM_LEAVES, bool FOLD, bool COMMIT, bool SHARD = false>
__global__ __launch_bounds__(512) void k_tree_top(LayerTask t, uint32_t l, const int32_t* mx, uint32_t G) {
    if (gated_off(t)) return;
    chain_prio();
    __shared__ uint4 lds[2 * 1024 + 2 * 512];
    __shared__ int32_t red[24];
    __shared__ SchedLds sl;
    sched_init(&sl);
    const uint32_t L = t.L;
    const uint32_t N = 1u << (L - l);
    const uint32_t tid = threadIdx.x;

    const bool chan_wave = COMMIT && tid >= 448;
    DevState* st = t.st;
    uint32_t cs[8], X[4];
    uint32_t has = 0, forced = 0, fbeta = 0;
    int job = CJ_END_FINAL;
    if (chan_wave) {
        // every channel field in one round trip: no load waits on another's
        // value (the wave reaches the inputs' barrier after this, so a chain
        // of dependent loads here delays every wave of the launch)
#pragma unroll
        for (int i = 0; i < 8; i++) cs[i] = st->chan[i];
        const uint32_t h = st->chan_has, pend = st->chan_pending;
        // the test hook's beta, loaded now rather than after the root
        const uint32_t fo = COMMIT ? st->forced : 0u, fb = st->forced_beta[t.k < MAXR ? t.k : 0];
        has = h;
        job = !h ? CJ_ROOT : (pend ? CJ_REHASH : CJ_MID);
        forced = fo;
        if (fo && t.k < MAXR) fbeta = fb;
    }
    // wave 6 pulls the compact-SHA constant tables into the scalar cache
    // while the inputs load (cold misses inside level 1 and the channel otherwise)
    if (tid >= 384 && tid < 448) kcache_touch_sha_tables();
    uint4* A = lds;
    uint4* B = lds + 2 * 1024;
    uint32_t* tr = t.tree;
    TOP_STAMP(0);
    if (FROM_LEAVES) {
        const size_t half = (size_t)1 << L;
        const uint32_t beta_m = FOLD ? (COMMIT ? st->beta_mont[t.k - 1] : t.beta_m) : 0u;
        // under 64 leaves the spare lanes of wave 0 hash leaf (i mod N) and
        // store nothing: a partly masked wave is slower (see pair_level)
        for (uint32_t i = tid; i < max(N, 64u); i += blockDim.x) {
            const uint32_t j = i & (N - 1);          // N is a power of two
            const bool real = i < N;
            uint32_t v;
            if (FOLD) {
                v = fold1(t.prev[j], t.prev[j + half], t.xinv[j], beta_m);
                if (real) t.values[j] = v;
            } else {
                v = t.values[j];
            }
            Dg d;
            cleaf(v, d);
            if (real) {
                dg_store(tr + 8 * j, d);
                dg_lds_store(A + 2 * j, d);
            }
        }
        if (COMMIT) coef_task(t, 0, 1, red);       // per-wave maxima in red[], wgmax[0..2]
    } else if (SHARD && COMMIT) {
        const ShardTop& sh = *t.shard;
        for (uint32_t i = tid; i < N; i += blockDim.x) {
            Dg d;
            dg_load(sh.recs_in + REC_WORDS * sh.rank_of_block[i], d);
            dg_lds_store(A + 2 * i, d);
            dg_store(tr + 8 * i, d);               // level 0 of the top tree (decommitment paths)
        }
        int m0 = -1, m1 = -1, m2 = -1;
        if (tid < sh.G) {
            const int32_t* rm = reinterpret_cast<const int32_t*>(sh.recs_in + REC_WORDS * tid + 8);
            m0 = rm[0]; m1 = rm[1]; m2 = rm[2];
            if (sh.sched_on) { m0 = sh.sched_deg; m1 = t.k == 0 ? -1 : 0; m2 = -1; }   // loopback rehearsal
        }
        m0 = wave_max_i(m0); m1 = wave_max_i(m1); m2 = wave_max_i(m2);
        if ((tid & 63) == 0) { red[3 * (tid >> 6)] = m0; red[3 * (tid >> 6) + 1] = m1; red[3 * (tid >> 6) + 2] = m2; }
    } else {
        const uint32_t* in = tr + 8 * level_offset(L, l);
        // the producers' maxima are loaded before the digests are waited
        // for: both round trips overlap (G <= 512 triples, one per thread)
        int p0 = -1, p1 = -1, p2 = -1;
        if (COMMIT && tid < G) { p0 = mx[3 * tid]; p1 = mx[3 * tid + 1]; p2 = mx[3 * tid + 2]; }
        for (uint32_t i = tid; i < N; i += blockDim.x) {
            Dg d;
            dg_load(in + 8 * i, d);
            dg_lds_store(A + 2 * i, d);
        }
        if (SHARD && !COMMIT) {                    // this rank's coefficient-slice maxima
            const ShardTop& sh = *t.shard;
            int m0 = -1, m1 = -1, m2 = -1;
            for (uint32_t i = tid; i < sh.rec_R; i += blockDim.x) {
                m0 = max(m0, sh.rec_mx[3 * i]); m1 = max(m1, sh.rec_mx[3 * i + 1]); m2 = max(m2, sh.rec_mx[3 * i + 2]);
            }
            m0 = wave_max_i(m0); m1 = wave_max_i(m1); m2 = wave_max_i(m2);
            if ((tid & 63) == 0) { red[3 * (tid >> 6)] = m0; red[3 * (tid >> 6) + 1] = m1; red[3 * (tid >> 6) + 2] = m2; }
        }
        if (COMMIT) {                              // producer maxima -> per-wave triples
            int m0 = p0, m1 = p1, m2 = p2;
            for (uint32_t i = tid + blockDim.x; i < G; i += blockDim.x) {
                m0 = max(m0, mx[3 * i]); m1 = max(m1, mx[3 * i + 1]); m2 = max(m2, mx[3 * i + 2]);
            }
            m0 = wave_max_i(m0); m1 = wave_max_i(m1); m2 = wave_max_i(m2);
            if ((tid & 63) == 0) { red[3 * (tid >> 6)] = m0; red[3 * (tid >> 6) + 1] = m1; red[3 * (tid >> 6) + 2] = m2; }
        }
    }
    lds_barrier();
    // ---- degree of poly_k (reference degree field; see DevState), uniform ----
    int deg = -1;
    bool noncanon = false;                         // layer 0: an input coefficient >= p
    if (COMMIT) {
        int m0 = -1, m1 = -1, m2 = -1;
#pragma unroll
        for (int i = 0; i < 8; i++) { m0 = max(m0, red[3 * i]); m1 = max(m1, red[3 * i + 1]); m2 = max(m2, red[3 * i + 2]); }
        deg = (t.k == 0) ? m0 : (m1 < 0 ? m2 : m0);
        noncanon = t.k == 0 && m1 >= 0;
    }
    const bool is_final = COMMIT && deg < 1;
    const int job_end = is_final ? CJ_END_FINAL : CJ_END_ROUND;
    uint32_t fv = 0;                               // fri_commit.rs:109-113
    if (chan_wave && is_final && deg == 0)
        fv = SHARD ? t.shard->recs_in[11] : (t.k == 0 ? t.coef_in : t.coef_out)[0];
    TOP_STAMP(1);
    TOP_CLK(17);
    // iterations: the levels, then one in which wave 7 runs every channel
    // job still left (no barrier between the post-root jobs)
    const uint32_t nlev = L - l;
    const uint32_t total = nlev + (COMMIT ? 1u : 0u);
    const uint32_t it_root = COMMIT ? nlev : ~0u;  // the iteration of job 3 (the root's first block)
    const bool chan_prod = FRI_SCHED_CHANNEL && COMMIT && tid >= 384 && tid < 448;   // wave 6 (SIMD 2)
    const shaq::Role R = shaq::role_of(tid);
    uint32_t cnt = N;
#pragma unroll 1
    for (uint32_t it = 0; it < total; it++) {
        const bool level = it < nlev;
        if (level) {
            cnt >>= 1;
            uint32_t* out = tr + 8 * level_offset(L, l + 1 + it);
            if (cnt <= 128) {                   // waves 0-3, one per SIMD (wave 7: channel)
#ifdef FRI_STAMPS
                if (it < 18 && tid == 0) TOP_CLK(24 + 2 * it);
#endif
                pair_level_s(A, B, out, tid, cnt, R, &sl, it);
#ifdef FRI_STAMPS
                if (it < 18 && tid == 0) TOP_CLK(25 + 2 * it);
#endif
            } else {
#pragma unroll 1
                for (uint32_t q = tid; q < cnt; q += blockDim.x) {
                    Dg a, b, o;
                    dg_lds_load(A + 4 * q, a);
                    dg_lds_load(A + 4 * q + 2, b);
#ifdef FRI_STAMPS
                    if (it < 18 && q == 0) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); TOP_CLK(24 + 2 * it); }
#endif
                    cnode(a, b, o);
#ifdef FRI_STAMPS
                    if (it < 18 && q == 0) TOP_CLK(25 + 2 * it);
#endif
                    dg_lds_store(B + 2 * q, o);
                    dg_store(out + 8 * q, o);
                }
            }
        }
        // channel job: during the narrow levels (SIMD 3 idle) only the
        // pre-root jobs, after the last level anything left
        if (chan_wave && job < job_end && (level ? (cnt <= 192 && job < CJ_ROOT) : true)) {
            do {
#ifdef FRI_STAMPS
                if (job == CJ_ROOT) TOP_STAMP_T(14, 448);           // job 3 / job 5 start (14, 13)
                if (job == CJ_ROOT + 2) TOP_STAMP_T(13, 448);
#endif
                chan_job(job, cs, X, has, A, fv, R, FRI_SCHED_CHANNEL ? sl.wk : nullptr, &sl.flag, 3u * it_root);
#ifdef FRI_STAMPS
                if (job >= CJ_ROOT && job <= CJ_ROOT + 2) TOP_STAMP_T(20 + job - CJ_ROOT, 448);   // done (20..22)
#endif
                job++;
            } while (!level && job < job_end);
        }
        if (chan_prod && it == it_root) chan_produce(A, &sl, 3u * it_root, R);
        lds_barrier();
        if (level) {
            uint4* tmp = A; A = B; B = tmp;
            if (it < 11) TOP_STAMP(2 + it);
            if (it + 1 == nlev) { TOP_CLK(18); TOP_STAMP(19); }
        }
    }
    if (SHARD && !COMMIT && tid == 448) {          // this rank's record
        const ShardTop& sh = *t.shard;
        int m0 = -1, m1 = -1, m2 = -1;
#pragma unroll
        for (int i = 0; i < 8; i++) { m0 = max(m0, red[3 * i]); m1 = max(m1, red[3 * i + 1]); m2 = max(m2, red[3 * i + 2]); }
        Dg root;
        dg_lds_load(A, root);
        uint32_t* rec = sh.rec_out;
        dg_store(rec, root);
        reinterpret_cast<uint4*>(rec)[2] = make_uint4((uint32_t)m0, (uint32_t)m1, (uint32_t)m2, sh.rec_c0[0]);
        reinterpret_cast<uint4*>(rec)[3] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (!COMMIT || tid != 448) return;
    // ---- results (wave 7, one lane) ----
    const int k = t.k;
    if (noncanon) {                                // FRI_EINVAL: nothing of this commit is served
        st->active[k] = 0;
        st->status = 1u;
        return;
    }
    st->deg[k] = deg;
    Dg root;
    dg_lds_load(A, root);
#pragma unroll
    for (int i = 0; i < 8; i++) st->roots[k][i] = root.w[i];
    st->n_layers = (uint32_t)k + 1;
    TOP_STAMP_T(15, 448);
    if (deg >= 1 && k < MAXR && L >= 1) {
        uint32_t beta = chan_beta(cs);
#pragma unroll
        for (int i = 0; i < 8; i++) st->chan[i] = cs[i];
        st->chan_has = 1;
        st->chan_pending = 1;                        // receive's rehash deferred to the next top
        if (forced) beta = fbeta;
        st->beta[k] = beta;
        st->beta_mont[k] = to_mont(beta);
        st->active[k] = 1;
        st->n_rounds = (uint32_t)k + 1;
        TOP_STAMP_T(16, 448);
    } else {
        st->active[k] = 0;
        if (deg >= 1) { st->status = 7u; return; }            // FRI_EDEGREE
#pragma unroll
        for (int i = 0; i < 8; i++) st->chan[i] = cs[i];      // after send(final.to_bytes())
        st->final_value = fv;
        st->final_degree = deg;
        st->chan_has = 1;
        st->chan_pending = 0;
    }
}

// ------------------------------------------------------------- tail ----
// The last layers of a commit (2^L <= 2^TAIL_LOG elements each) in ONE
// workgroup and ONE launch: per layer the body of k_tree_top<true, *, true>
// (fold, leaves, coefficient fold, degree, tree levels, channel step), with
// the layer values, the coefficients, beta, the degree and the gate handed to
// the next layer through LDS.  Saves per layer a kernel boundary, the HBM
// round trip of the folded values and coefficients, and the cold first level
// of a fresh workgroup.  The channel state stays in wave 7's registers.
struct TailTask {
    LayerTask t[TAIL_LOG + 1];  // consecutive layers k0 .. k0 + n - 1 (commit mode)
    uint32_t n;
};

template <bool FOLD0>
__global__ __launch_bounds__(512) void k_tree_tail(TailTask tt) {
    const LayerTask& t0 = tt.t[0];
    if (gated_off(t0)) return;
    chain_prio();
    constexpr uint32_t NMAX = 1u << TAIL_LOG;
    __shared__ uint4 lds[2 * NMAX + NMAX];
    __shared__ uint32_t vals[2][NMAX];         // this / previous layer's values
    __shared__ uint32_t coefs[2][NMAX];        // this / previous round's polynomial
    __shared__ int32_t red[24];
    __shared__ uint32_t s_beta_m, s_active;
    __shared__ int32_t s_deg;
    __shared__ uint32_t s_fbeta[TAIL_LOG + 2];   // the test hook's betas of these layers (0: not forced)
    __shared__ uint32_t xv[2 * NMAX];            // every layer's x^-1 table (prefetched)
    __shared__ SchedLds sl;
    sched_init(&sl);
    uint32_t ord = 0;                            // narrow levels so far (schedule producer flag)
    const uint32_t tid = threadIdx.x;
    const bool chan_wave = tid >= 448;
    DevState* st = t0.st;
    // The x^-1 tables of layers 1.. are loaded into LDS by wave 6 during the
    // first layer's levels (one HBM latency for the launch, off the chain,
    // instead of one per layer fold); layer 0 folds from HBM.
    auto prefetch_x = [&](uint32_t t0p, uint32_t nthr) {
        uint32_t off = 1u << tt.t[0].L;
        for (uint32_t li = 1; li < tt.n; li++) {
            const uint32_t N = 1u << tt.t[li].L;
            for (uint32_t j = tid - t0p; j < N; j += nthr) xv[off + j] = tt.t[li].xinv[j];
            off += N;
        }
    };
    uint32_t cs[8], X[4];
    uint32_t has = 0;
    if (chan_wave) {
#pragma unroll
        for (int i = 0; i < 8; i++) cs[i] = st->chan[i];
        has = st->chan_has;
    }
    uint32_t pending = chan_wave ? st->chan_pending : 0u;
    if (tid >= 384 && tid < 448) kcache_touch_sha_tables();
    // forced betas (test hook) read here, off the per-layer critical path
    if (tid < tt.n + 1) {
        const int kk = t0.k + (int)tid;
        s_fbeta[tid] = (st->forced && kk < MAXR) ? st->forced_beta[kk] + 1u : 0u;   // +1: 0 means not forced
    }
    uint32_t beta_m = FOLD0 ? st->beta_mont[t0.k - 1] : 0u;
    int prev_deg = FOLD0 ? st->deg[t0.k - 1] : -1;
    const shaq::Role R = shaq::role_of(tid);
    uint32_t xoff = 0;
#pragma unroll 1
    for (uint32_t li = 0; li < tt.n; li++) {
        const LayerTask& t = tt.t[li];
        const int k = t.k;
        const uint32_t L = t.L, N = 1u << L;
        const uint32_t* xl = li ? xv + xoff : t.xinv;
        xoff += N;
        const bool fold = FOLD0 || li > 0;
        uint32_t* cur_v = vals[li & 1];
        const uint32_t* prev_v = vals[(li & 1) ^ 1];
        uint32_t* cur_c = coefs[li & 1];
        const uint32_t* prev_c = coefs[(li & 1) ^ 1];
        uint4* A = lds;
        uint4* B = lds + 2 * NMAX;
        uint32_t* tr = t.tree;
        TAIL_STAMP(0);
        // ---- fold + leaves (spare lanes of wave 0 recompute leaf i mod N) ----
        for (uint32_t i = tid; i < max(N, 64u); i += blockDim.x) {
            const uint32_t j = i & (N - 1);
            const bool real = i < N;
            uint32_t v;
            if (fold) {
                const uint32_t a = li ? prev_v[j] : t.prev[j], b = li ? prev_v[j + N] : t.prev[j + N];
                v = fold1(a, b, xl[j], beta_m);
                if (real) t.values[j] = v;
            } else {
                v = t.values[j];
            }
            if (real) cur_v[j] = v;
            Dg d;
            cleaf(v, d);
            if (real) {
                dg_store(tr + 8 * j, d);
                dg_lds_store(A + 2 * j, d);
            }
        }
        // ---- coefficient fold of round k-1 (or the input scan at k == 0) ----
        // Needed only for the degree, i.e. from the root on: it runs on waves
        // 4-5 (threads [256, 384)) during the first level iteration that
        // leaves them idle (coef_it), unless the layer has no such level.
        const uint32_t nlev = L;
        const uint32_t coef_it = N > 256 ? 1u : 0u;   // iteration 0 of a 512-leaf layer uses all waves
        const bool coef_late = nlev > coef_it;
        auto coef_fold = [&](uint32_t t0c, uint32_t nthr) {
            int m0 = -1, m1 = -1, m2 = -1;
            const uint32_t tx = tid - t0c;
            if (k == 0) {
                for (size_t j = tx; j < t.d0; j += nthr) {
                    const uint32_t c = t.coef_in[j];
                    if (c) m0 = max(m0, (int)j);
                    if (c >= P) m1 = 0;                    // not canonical (see coef_task)
                }
            } else {
                const uint32_t len = (uint32_t)(prev_deg + 1), nlen = (len + 1) / 2;
                const bool in_lds = li > 0 && k >= 2;      // poly_{k-1} was folded by this kernel
                for (uint32_t j = tx; j < nlen; j += nthr) {
                    const uint32_t e = in_lds ? prev_c[2 * j] : t.coef_in[2 * j];
                    const uint32_t o = (2 * j + 1 < len) ? (in_lds ? prev_c[2 * j + 1] : t.coef_in[2 * j + 1]) : 0u;
                    const uint32_t v = add(e, mmul(o, beta_m));
                    cur_c[j] = v;
                    if (v) m0 = (int)j;
                    if (e) m1 = (int)j;
                    if (o) m2 = (int)j;
                }
            }
            m0 = wave_max_i(m0); m1 = wave_max_i(m1); m2 = wave_max_i(m2);
            const uint32_t w = tx >> 6;
            if ((tx & 63) == 0) { red[3 * w] = m0; red[3 * w + 1] = m1; red[3 * w + 2] = m2; }
        };
        if (!coef_late) coef_fold(0, blockDim.x);
        if (li == 0 && !coef_late) prefetch_x(0, blockDim.x);
        lds_barrier();
        TAIL_STAMP(1);
        TAIL_CLK(17);
        int deg = 1;
        bool noncanon = false;
        int job_end = CJ_END_ROUND;                    // provisional while the degree is pending
        uint32_t fv = 0;                               // fri_commit.rs:109-113
        // red[] (after a barrier) -> degree of poly_k; is it the last layer?
        auto settle = [&](uint32_t nw) {
            int a = -1, b = -1, c = -1;
            for (uint32_t i = 0; i < nw; i++) { a = max(a, red[3 * i]); b = max(b, red[3 * i + 1]); c = max(c, red[3 * i + 2]); }
            deg = (k == 0) ? a : (b < 0 ? c : a);
            noncanon = k == 0 && b >= 0;
            job_end = deg < 1 ? CJ_END_FINAL : CJ_END_ROUND;
            if (chan_wave && deg == 0) fv = (k == 0) ? t.coef_in[0] : cur_c[0];
        };
        if (!coef_late) settle(8);
        // ---- levels + channel jobs (k_tree_top) ----
        int job = CJ_END_FINAL;
        if (chan_wave) job = !has ? CJ_ROOT : (pending ? CJ_REHASH : CJ_MID);
        // the levels, then one iteration in which wave 7 runs every channel
        // job still left (their number follows the degree, settled by then)
        const uint32_t total = nlev + 1;
        const uint32_t it_root = nlev;                                // iteration of job 3
        uint32_t ch_base = 0;                                         // flag base of this layer's root blocks
        uint32_t cnt = N;
#pragma unroll 1
        for (uint32_t it = 0; it < total; it++) {
            const bool level = it < nlev;
            if (level) {
                cnt >>= 1;
                uint32_t* out = tr + 8 * level_offset(L, 1 + it);
                if (cnt <= 128) {
                    if (it < 18) TAIL_CLK(24 + 2 * it);
                    pair_level_s(A, B, out, tid, cnt, R, &sl, ord++);
                    if (it < 18) TAIL_CLK(25 + 2 * it);
                } else {
#pragma unroll 1
                    for (uint32_t q = tid; q < cnt; q += blockDim.x) {
                        Dg a, b, o;
                        dg_lds_load(A + 4 * q, a);
                        dg_lds_load(A + 4 * q + 2, b);
                        cnode(a, b, o);
                        dg_lds_store(B + 2 * q, o);
                        dg_store(out + 8 * q, o);
                    }
                }
            }
            if (!level && it == it_root) ch_base = 3u * (ord++), ord++;   // two ordinals (uniform)
            if (chan_wave && job < job_end && (level ? (cnt <= 192 && job < CJ_ROOT) : true)) {
                do {
                    chan_job(job, cs, X, has, A, fv, R, FRI_SCHED_CHANNEL ? sl.wk : nullptr, &sl.flag, ch_base);
#ifdef FRI_STAMPS
                    if (job >= CJ_ROOT && job <= CJ_ROOT + 2) TAIL_STAMP_T(20 + job - CJ_ROOT, 448, __builtin_amdgcn_s_memrealtime);
#endif
                    job++;
                } while (!level && job < job_end);
            }
            if (FRI_SCHED_CHANNEL && tid >= 384 && tid < 448 && !level && it == it_root) chan_produce(A, &sl, ch_base, R);
            if (coef_late && it == coef_it && tid >= 256 && tid < 384) coef_fold(256, 128);
            if (li == 0 && coef_late && it == coef_it && tid >= 384 && tid < 448) prefetch_x(384, 64);
            lds_barrier();
            if (coef_late && it == coef_it) settle(2);
            if (level) {
                uint4* tmp = A; A = B; B = tmp;
                if (it < 11) TAIL_STAMP(2 + it);
                if (it + 1 == nlev) { TAIL_CLK(18); TAIL_STAMP(19); }
            }
        }
        // ---- results (one lane of wave 7), hand-off to the next layer ----
        if (tid == 448 && noncanon) {                   // FRI_EINVAL (uniform: the loop ends below)
            st->active[k] = 0;
            st->status = 1u;
            s_active = 0;
        } else if (tid == 448) {
            st->deg[k] = deg;
            Dg root;
            dg_lds_load(A, root);
#pragma unroll
            for (int i = 0; i < 8; i++) st->roots[k][i] = root.w[i];
            st->n_layers = (uint32_t)k + 1;
            uint32_t active = 0, bm = 0;
            if (deg >= 1 && k < MAXR && L >= 1) {
                uint32_t beta = chan_beta(cs);
#pragma unroll
                for (int i = 0; i < 8; i++) st->chan[i] = cs[i];
                st->chan_has = 1;
                st->chan_pending = 1;                    // receive's rehash deferred to the next layer
                if (s_fbeta[li]) beta = s_fbeta[li] - 1u;
                st->beta[k] = beta;
                bm = to_mont(beta);
                st->beta_mont[k] = bm;
                st->active[k] = 1;
                st->n_rounds = (uint32_t)k + 1;
                active = 1;
            } else {
                st->active[k] = 0;
                if (deg >= 1) {
                    st->status = 7u;                     // FRI_EDEGREE
                } else {
#pragma unroll
                    for (int i = 0; i < 8; i++) st->chan[i] = cs[i];   // after send(final.to_bytes())
                    st->final_value = fv;
                    st->final_degree = deg;
                    st->chan_has = 1;
                    st->chan_pending = 0;
                }
            }
            s_beta_m = bm;
            s_active = active;
            s_deg = deg;
            TAIL_STAMP_T(15, 448, __builtin_amdgcn_s_memrealtime);
        }
        if (chan_wave) { has = 1; pending = 1; }
        lds_barrier();
        if (!s_active) break;                            // uniform
        beta_m = s_beta_m;
        prev_deg = s_deg;
    }
}

// ------------------------------------------------------------ launcher ----
// Layer schedule (levels are consumed 4 at a time):
//   L <= 9 : one k_tree_top from the leaves.
//   L >= 19: k_layer_leaf (2048 leaves/WG -> 128);  11..18: k_layer_leaf_wide (256 -> 16)
//   then k_tree_mid<1024> while the level has >= 2^18 nodes, k_tree_mid<256>
//   while it has > 512, and k_tree_top on the last <= 512 nodes.
static LayerTask with_gate(const LayerTask& in) {
    LayerTask t = in;
    if (t.st) { t.gst = t.st; t.gidx = t.k > 0 ? t.k - 1 : -1; }
    return t;
}

#ifndef MID8
#define MID8 1               // k_tree_mid8 for the narrow levels of large layers
#endif
#ifndef QUAD_TPB
#define QUAD_TPB 512         // quad leaf kernel: threads per WG (2048 leaves per WG; A/B: 512 beats 256 by ~0.5-1%, 128 and 1024 slower)
#endif
#ifndef QUAD_MIN_LOG
#define QUAD_MIN_LOG 19      // smaller layers: one leaf per lane (A/B: 19 beats 20 and 21)
#endif

// A fused sharded block tree's leaf kernel (PAIR): the layer's G workgroups
// as two launches of G/2, the half-block the next exchange sends first, with
// after_part1 in between (a single launch without it).
template <typename KernelLaunch>
static void pair_parts(LayerTask t, uint32_t G, hipStream_t s, const std::function<void()>& after_part1,
                       KernelLaunch&& go) {
    t.wg_total = G;
    if (!after_part1) {
        t.wg_base = 0;
        go(t, G);
        return;
    }
    const uint32_t h = G / 2;
    t.wg_base = t.send_half ? h : 0u;
    go(t, h);
    after_part1();
    t.wg_base = t.send_half ? 0u : h;
    go(t, h);
}

void launch_layer(const LayerTask& tin, hipStream_t s, hipEvent_t ev_leaf_end, const std::function<void()>& after_leaf,
                  hipEvent_t ev_before_top, const std::function<void()>& after_part1) {
    const LayerTask t = with_gate(tin);
    const uint32_t L = t.L;
    const bool fold = t.prev != nullptr;
    const bool commit = t.st != nullptr;
    const bool pair = t.prev2 != nullptr;          // sharded block tree, pair fold fused (never commit mode)
    const int32_t* nomx = nullptr;
    if (L <= TOP_LOG) {
        if (fold) {
            if (commit) hipLaunchKernelGGL((k_tree_top<true, true, true>), dim3(1), dim3(512), 0, s, t, 0u, nomx, 1u);
            else hipLaunchKernelGGL((k_tree_top<true, true, false>), dim3(1), dim3(512), 0, s, t, 0u, nomx, 1u);
        } else {
            if (commit) hipLaunchKernelGGL((k_tree_top<true, false, true>), dim3(1), dim3(512), 0, s, t, 0u, nomx, 1u);
            else hipLaunchKernelGGL((k_tree_top<true, false, false>), dim3(1), dim3(512), 0, s, t, 0u, nomx, 1u);
        }
        if (ev_leaf_end) hipEventRecord(ev_leaf_end, s);
        return;
    }
    uint32_t G, out_per_wg;
    if (L >= QUAD_MIN_LOG) {
        constexpr uint32_t TPB = QUAD_TPB;
        G = (uint32_t)(((size_t)1 << L) / (4 * TPB));
        out_per_wg = TPB / 4;
        if (pair) {
            pair_parts(t, G, s, after_part1, [&](const LayerTask& tp, uint32_t g) {
                hipLaunchKernelGGL((k_layer_leaf<true, false, TPB, true>), dim3(g), dim3(TPB), 0, s, tp);
            });
        } else if (fold) {
            if (commit) hipLaunchKernelGGL((k_layer_leaf<true, true, TPB>), dim3(G), dim3(TPB), 0, s, t);
            else hipLaunchKernelGGL((k_layer_leaf<true, false, TPB>), dim3(G), dim3(TPB), 0, s, t);
        } else {
            if (commit) hipLaunchKernelGGL((k_layer_leaf<false, true, TPB>), dim3(G), dim3(TPB), 0, s, t);
            else hipLaunchKernelGGL((k_layer_leaf<false, false, TPB>), dim3(G), dim3(TPB), 0, s, t);
        }
    } else {
        G = 1u << (L - 8);
        out_per_wg = 256u >> wide_levels(L);
        if (pair) {
            pair_parts(t, G, s, after_part1, [&](const LayerTask& tp, uint32_t g) {
                hipLaunchKernelGGL((k_layer_leaf_wide<true, false, true>), dim3(g), dim3(256), 0, s, tp);
            });
        } else if (fold) {
            if (commit) hipLaunchKernelGGL((k_layer_leaf_wide<true, true>), dim3(G), dim3(256), 0, s, t);
            else hipLaunchKernelGGL((k_layer_leaf_wide<true, false>), dim3(G), dim3(256), 0, s, t);
        } else {
            if (commit) hipLaunchKernelGGL((k_layer_leaf_wide<false, true>), dim3(G), dim3(256), 0, s, t);
            else hipLaunchKernelGGL((k_layer_leaf_wide<false, false>), dim3(G), dim3(256), 0, s, t);
        }
    }
    if (ev_leaf_end) hipEventRecord(ev_leaf_end, s);
    if (after_leaf) after_leaf();
    const int gate = t.gidx;
    // coefficient maxima: level 0 at wgmax[0 .. 3G); each mid reduces R producers per WG
    const int32_t* mx = commit ? t.wgmax : nullptr;
    size_t mx_off = 3 * (size_t)G;
    uint32_t l = L >= QUAD_MIN_LOG ? 4u : wide_levels(L);
    while (L - l > TOP_LOG) {
        const size_t nodes = (size_t)1 << (L - l);
        const uint32_t nin = nodes >= ((size_t)1 << 18) ? 1024u : 256u;
        const uint32_t grid = (uint32_t)(nodes / nin);
        const uint32_t R = nin / out_per_wg;
        int32_t* mx_out = commit ? t.wgmax + mx_off : nullptr;
        // eight narrow levels in one launch when four would leave more than
        // the top takes (L - l >= 14: two k_tree_mid<256> otherwise)
        const bool eight = nin == 256 && L - l >= 8 + 6 && MID8;
        if (nin == 1024)
            hipLaunchKernelGGL((k_tree_mid<1024>), dim3(grid), dim3(512), 0, s, t.tree, L, l, t.gst, gate, mx, mx_out, R);
        else if (eight)
            hipLaunchKernelGGL(k_tree_mid8, dim3(grid), dim3(256), 0, s, t.tree, L, l, t.gst, gate, mx, mx_out, R);
        else
            hipLaunchKernelGGL((k_tree_mid<256>), dim3(grid), dim3(128), 0, s, t.tree, L, l, t.gst, gate, mx, mx_out, R);
        if (commit) { mx = mx_out; mx_off += 3 * (size_t)grid; }
        G = grid;
        out_per_wg = eight ? 1u : nin / 16;
        l += eight ? 8u : 4u;
    }
    if (ev_before_top) hipStreamWaitEvent(s, ev_before_top, 0);
    if (commit) hipLaunchKernelGGL((k_tree_top<false, false, true>), dim3(1), dim3(512), 0, s, t, l, mx, G);
    else if (t.shard) hipLaunchKernelGGL((k_tree_top<false, false, false, true>), dim3(1), dim3(512), 0, s, t, l, nomx, G);
    else hipLaunchKernelGGL((k_tree_top<false, false, false>), dim3(1), dim3(512), 0, s, t, l, nomx, G);
}

void launch_tail(const LayerTask* ts, uint32_t n, hipStream_t s) {
    TailTask tt{};
    tt.n = n;
    for (uint32_t i = 0; i < n; i++) tt.t[i] = ts[i];
    tt.t[0] = with_gate(ts[0]);
    if (ts[0].prev) hipLaunchKernelGGL((k_tree_tail<true>), dim3(1), dim3(512), 0, s, tt);
    else hipLaunchKernelGGL((k_tree_tail<false>), dim3(1), dim3(512), 0, s, tt);
}

__global__ __launch_bounds__(256) void k_coef(LayerTask t) {
    if (gated_off(t)) return;
    __shared__ int32_t red[12];
    coef_task(t, blockIdx.x, gridDim.x, red);
}

void launch_coef(const LayerTask& tin, uint32_t G, hipStream_t s) {
    const LayerTask t = with_gate(tin);
    hipLaunchKernelGGL(k_coef, dim3(G), dim3(256), 0, s, t);
}

void launch_top(const LayerTask& tin, uint32_t l, const int32_t* mx, uint32_t G, hipStream_t s) {
    const LayerTask t = with_gate(tin);
    if (t.shard) hipLaunchKernelGGL((k_tree_top<false, false, true, true>), dim3(1), dim3(512), 0, s, t, l, mx, G);
    else hipLaunchKernelGGL((k_tree_top<false, false, true>), dim3(1), dim3(512), 0, s, t, l, mx, G);
}

}  // namespace fri
