// fri_internal.hpp — device state layout and kernel launchers shared by
// the kernel files (fri_kernels.hip, fri_layer.hip, ...) and the host code of
// the C ABI (fri_host.hpp and the files it lists).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <functional>
#include "field.hpp"

namespace fri {

constexpr int MAXR = 32;            // == FRI_MAX_ROUNDS
constexpr uint32_t TOP_LOG = 9;         // single-workgroup tree top: <= 512 inputs
#ifndef FRI_TAIL_LOG
#define FRI_TAIL_LOG 9
#endif
constexpr uint32_t TAIL_LOG = FRI_TAIL_LOG;   // layers of <= 2^TAIL_LOG elements run in the fused tail
constexpr uint32_t POW_LO_LOG = 12;     // two-level power tables s^j = lo[j&4095]*hi[j>>12]

// Device-resident commit state (one per context).  Every per-round kernel
// reads its gate (active[r]) and operands (beta, degrees) from here, so the
// whole commit is a static launch sequence that a hipGraph can replay and
// that needs no host round trip between Fiat-Shamir rounds.
struct DevState {
    uint32_t chan[8];            // channel state digest (src/channel/channel.rs:19)
    uint32_t chan_has;           // 0 => state == ""
    uint32_t chan_pending;       // 1 => true state = sha256_hex(hex(chan)) (receive's rehash deferred)
    uint32_t n_layers;
    uint32_t n_rounds;
    uint32_t final_value;
    int32_t  final_degree;
    uint32_t status;             // 0 ok, else FRI_E* raised on device
    uint32_t forced;             // FRI_FLAG_FORCE_BETAS
    int32_t  deg0max;            // max nonzero index of the input coefficients
    uint32_t active[MAXR + 1];   // active[r]: fold round r runs (deg_r >= 1)
    int32_t  deg[MAXR + 1];      // degree of poly_k (reference degree field)
    int32_t  newmax[MAXR];       // per round: max j with folded c'_j != 0
    int32_t  evenmax[MAXR];      //            max j with c_{2j}   != 0
    int32_t  oddmax[MAXR];       //            max j with c_{2j+1} != 0
    uint32_t beta[MAXR];
    uint32_t beta_mont[MAXR];
    uint32_t forced_beta[MAXR];
    uint32_t roots[MAXR + 1][8];
#ifdef FRI_STAMPS
    uint64_t stamps[MAXR + 1][64];   // diagnostic build only: s_memrealtime (100 MHz) per phase
#endif
};

// Tree layout: layer with 2^L leaves stores levels 0..L contiguously,
// level l at digest offset 2^(L+1) - 2^(L+1-l) (8 words per digest).
__host__ __device__ inline size_t level_offset(uint32_t L, uint32_t l) {
    return ((size_t)2 << L) - ((size_t)2 << (L - l));
}

// ---- launchers (fri_kernels.hip); all asynchronous on `s` ----------------
struct NttPlan {
    uint32_t log_n;              // transform size 2^log_n
    const uint32_t* tw;          // stage-packed Montgomery twiddles: tw[2^s + j] = w_{2^(s+1)}^j
    const uint32_t* pre_lo;      // optional input scale s^j (Montgomery, two-level)
    const uint32_t* pre_hi;
    const uint32_t* post_lo;     // optional output scale t^j (Montgomery, two-level)
    const uint32_t* post_hi;
    uint32_t* scratch;           // optional 2^log_n words the transform may use (2^24 coset LDE); else nullptr
};
// dst[k] = post(k) * sum_{j<d} src[j]*pre(j)*w^(jk); src may alias nothing in dst.
void launch_ntt(const NttPlan& p, const uint32_t* src, size_t d, uint32_t* dst, hipStream_t s);

// tw[2^s + j] = Montgomery(w_{2^(s+1)}^{+-j}), s < log_max, j < 2^s (2^log_max entries)
void launch_twiddles(uint32_t* tw, uint32_t log_max, bool inverse, hipStream_t s);
void launch_pow_table(uint32_t* lo, uint32_t* hi, uint32_t log_n, uint32_t base_std,
                      uint32_t scale_std, hipStream_t s);
void launch_batch_inverse(const uint32_t* in, uint32_t* out, size_t n, int out_mont,
                          hipStream_t s);
void launch_coset_points(uint32_t* out, size_t count, uint32_t offset, uint32_t log_n,
                         hipStream_t s);
void launch_square_mont(const uint32_t* in, uint32_t* out, size_t count, hipStream_t s);
// Arbitrary-point interpolation (fri_interpolate_points): prod_{i!=j}(x_j - x_i)
// into acc; c_j = y_j * w_j (w Montgomery) in place over w; f(w_N^k) for k < N.
// tmp: interp_tmp_words(n, log_N) words of segment partials.
size_t interp_tmp_words(size_t n, uint32_t log_N);
void launch_interp_weights(const uint32_t* xs, size_t n, uint32_t* acc, uint32_t* tmp, hipStream_t s);
void launch_interp_coeffs(const uint32_t* ys, uint32_t* w_to_c, size_t n, hipStream_t s);
void launch_interp_eval(const uint32_t* xs, const uint32_t* c, size_t n, uint32_t log_N, uint32_t* f, uint32_t* tmp,
                        hipStream_t s);
// Horner at arbitrary points; with few points and many coefficients (tmp of
// evaluate_tmp_words(d, count) > 0 words) the coefficients are split over lanes.
size_t evaluate_tmp_words(size_t d, size_t count);
void launch_evaluate(const uint32_t* coeffs, size_t d, const uint32_t* xs, size_t count, uint32_t* out,
                     uint32_t* tmp, hipStream_t s);
struct DecommitPlan {
    uint64_t index;
    uint32_t log_n, n_layers;
    uint64_t layer_off[MAXR + 1];
    uint64_t tree_off[MAXR + 1];
    uint32_t path_off[MAXR + 1];   // word offset of layer k's two paths (16 * L_j per earlier layer)
    // Sharded layers (fri_decommit_query_sharded): layer k with shard_lb1[k] =
    // log2(block size) + 1 (0: an ordinary whole layer) is held block-wise: this rank writes an opening
    // only when it owns the opened element's block (owned[k], bit b), taking
    // the path's lower log2(block) levels from its block-local tree and the
    // top log G levels from the layer's top tree (top + top_off[k]); openings
    // of blocks it does not hold are written as zeros (the ranks' outputs are
    // then combined by a max-reduction).  val_block[k]: the value slot holds
    // only this rank's block (index i mod B), else the whole layer (index i).
    uint32_t logG;
    uint8_t shard_lb1[MAXR + 1];    // log2(block size) + 1; 0: an ordinary (whole) layer
    uint8_t val_block[MAXR + 1];
    uint64_t owned[MAXR + 1];
    uint64_t top_off[MAXR + 1];
};
void launch_decommit_gather(const uint32_t* layers, const uint32_t* trees, const DecommitPlan& dp, uint32_t* out,
                            hipStream_t s, const uint32_t* top = nullptr);
void launch_fold_plain(const uint32_t* in, uint32_t* out, uint32_t log_m, const uint32_t* xinv_m,
                       uint32_t beta, hipStream_t s);

// Sharded layer k (run_commit_sharded), device-resident per layer: what
// the block top and the replicated top kernels of a coset-sharded layer read
// besides their LayerTask (k_tree_top<..., SHARD>, fri_layer.hip).
constexpr uint32_t REC_WORDS = 16;   // per-rank record: root (8), m0, m1, m2, first coefficient, 0 x 4
struct ShardTop {
    // block top (this rank): the record it writes
    uint32_t* rec_out;
    const int32_t* rec_mx;     // rec_R workgroup maxima triples of this rank's coefficient task
    const uint32_t* rec_c0;    // this rank's first coefficient of poly_k
    uint32_t rec_R;
    // replicated top: the G all-gathered records (rank order)
    uint32_t G;
    const uint32_t* recs_in;
    int32_t sched_deg;         // loopback rehearsal (sched_on): the recorded degree of this layer
    uint32_t sched_on;
    uint8_t rank_of_block[64]; // block b's root is in the record of rank rank_of_block[b]
};

// One FRI layer (fri_layer.hip): optional fold of the previous layer, leaf
// hashes, every tree level, and (commit mode, st != nullptr) the coefficient
// fold slice, degree resolution and Fiat-Shamir step of layer k.
struct LayerTask {
    const uint32_t* prev;      // layer k-1 values (fold) or nullptr
    const uint32_t* xinv;      // Montgomery (x_i)^-1 of layer k-1's domain, i < 2^L
    uint32_t* values;          // layer k values (written when folding)
    uint32_t* tree;            // layer k tree: levels 0..L (level_offset)
    uint32_t L;                // log2 |layer k|
    int k;                     // layer index (commit mode)
    uint32_t beta_m;           // Montgomery beta for a standalone fold (no state)
    const uint32_t* coef_in;   // k == 0: input coefficients; else poly_{k-1}
    uint32_t* coef_out;        // poly_k coefficients (k >= 1)
    size_t d0;                 // k == 0: input length
    int32_t* wgmax;            // [3 * workgroups] coefficient maxima
    DevState* st;              // nullptr: standalone Merkle tree (no degree / channel)
    const DevState* gst;       // gate for standalone trees inside a commit (sharded
    int gidx;                  //   layers): skip when !gst->active[gidx]
    // Sharded coefficient fold (run_commit_sharded, k_coef only): this rank
    // handles the coefficients j in [jlo, jhi) of poly_k (jhi == 0: all of
    // them); coef_in[0] holds global coefficient ibase of poly_{k-1} (of the
    // input at k == 0), coef_out[0] global coefficient obase of poly_k.
    size_t jlo, jhi, ibase, obase;
    const ShardTop* shard;     // sharded layer (device): nullptr otherwise
    // Sharded block tree with the pair fold fused in (run_commit_sharded):
    // the fold's second operand is prev2[i] (the partner's half-block)
    // instead of prev[i + 2^L]; beta is gst->beta_mont[gidx].  The leaf
    // kernel then runs as two launches, the half-block the next exchange
    // sends (send_half: 0 first half, 1 second half) first.
    const uint32_t* prev2;
    uint32_t send_half;
    uint32_t wg_base;          // (set per launch) first workgroup of a split launch
    uint32_t wg_total;         // (set per launch) workgroups of the whole layer
};
// after_leaf: called right after the leaf kernel is enqueued (and
// ev_leaf_end recorded), so the caller can start work on another stream
// behind it; ev_before_top: the stream waits for it before the top kernel
// (a sharded block top reads the coefficient maxima made on that stream).
// after_part1 (a fused sharded layer, t.prev2 set): called right after the
// leaf launch of the half-block the next exchange sends, so the caller can
// enqueue that exchange while the other half is hashed.
void launch_layer(const LayerTask& t, hipStream_t s, hipEvent_t ev_leaf_end = nullptr,
                  const std::function<void()>& after_leaf = {}, hipEvent_t ev_before_top = nullptr,
                  const std::function<void()>& after_part1 = {});
// Layers ts[0..n) (consecutive, 2^L <= 2^TAIL_LOG elements, commit mode) in
// one single-workgroup launch (k_tree_tail), n <= TAIL_LOG + 1.
void launch_tail(const LayerTask* ts, uint32_t n, hipStream_t s);
// Coefficient task of layer t.k alone (grid G): k == 0 scans the input for
// deg_0, k >= 1 folds poly_{k-1} -> poly_k; maxima into t.wgmax[3*G].
void launch_coef(const LayerTask& t, uint32_t G, hipStream_t s);
// fri_dist_kernels.hip
void launch_coset_coeffs(const uint32_t* a, size_t d, uint32_t* out, size_t M, uint32_t c_std, hipStream_t s);
void launch_decimate(const uint32_t* a, size_t d, uint32_t* ev, uint32_t* od, hipStream_t s);
void launch_radix2_block(const uint32_t* E, const uint32_t* O, const uint32_t* tlo, const uint32_t* thi,
                         uint32_t* out, size_t M, uint32_t negate, hipStream_t s);
void launch_cyclic_to_block(const uint32_t* recv, uint32_t* block, size_t B, uint32_t G, hipStream_t s);
// layer[block_of[r] * B ..] = gath[r * B ..] for r < G (B a multiple of 4).
void launch_place_blocks(const uint32_t* gath, uint32_t* layer, size_t B, uint32_t G, const uint32_t* block_of,
                         hipStream_t s);
// In-process peer transport: dst[p * words ..] = src[p][0 .. words) for p < n
// (n <= 64 sources, each another rank's buffer); vec4: every pointer 16-byte
// aligned and words % 4 == 0.
struct PeerPull {
    const uint32_t* src[64];
    uint32_t* dst;
    size_t words;
    uint32_t n;
    uint32_t vec4;
};
void launch_peer_pull(const PeerPull& pp, hipStream_t s);
// *out = position-sensitive 64-bit checksum of v[0..n) (FRI_FLAG_RANK_INPUTS).
void launch_checksum(const uint32_t* v, size_t n, uint64_t* out, hipStream_t s);
// Loopback rehearsal: dst = G copies of src (words each), one launch.
void launch_replicate(const uint32_t* src, uint32_t* dst, size_t words, uint32_t G, hipStream_t s);
// Tree top + degree + channel step for a layer whose level `l` (2^(L-l)
// nodes, <= 512) is already in t.tree; mx/G: coefficient maxima.
void launch_top(const LayerTask& t, uint32_t l, const int32_t* mx, uint32_t G, hipStream_t s);

// fri_prover.hip — STARK-101 FibonacciSq composition on the LDE coset.
constexpr uint32_t FIBSQ_MAX_B = 16;   // blowup <= 2^4
struct FibsqParams {
    uint32_t log_n;              // LDE size n = B * T
    uint32_t B;                  // blowup (power of two, 2..16): g = w_n^B
    uint32_t offset_m;           // Montgomery(offset)
    uint32_t w_m, winv_m;        // Montgomery(w_n^{+-1})
    uint32_t glast_m, gprev_m;   // Montgomery(g^{T-1}), Montgomery(g^{T-2})
    uint32_t a_last;             // canonical a_{T-1}
    uint32_t alpha_m[3];         // Montgomery(alpha_0..2)
    uint32_t zinv_m[FIBSQ_MAX_B];// Montgomery((offset^T w_B^j - 1)^-1), j < B
};
void launch_fibsq_cp(const uint32_t* f_lde, uint32_t* out, const FibsqParams& q, hipStream_t s);
// out[j] = lde[(index + j*stride) mod 2^L], then count paths of L big-endian digests
void launch_trace_gather(const uint32_t* lde, const uint32_t* tree, uint32_t L, uint64_t index, uint64_t stride,
                         uint32_t count, uint32_t* out, hipStream_t s);

}  // namespace fri
