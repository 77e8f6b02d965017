// fri_kernels.hip — gfx950 kernels of the FRI commit path.
//
//   NTT (coset LDE / interpolation)  replaces Horner evaluate at every domain
//                                     point (src/fri/fri_commit.rs:78,
//                                     src/polynomial/ops.rs:76-83) and Lagrange
//                                     interpolation (interpolation.rs:121-152)
//   Merkle subtree                    replaces MerkleTree::new (src/merkle/mod.rs:10-22)
//   fold (evaluation form)            replaces next_fri_layer (src/fri/fri_commit.rs:53-65)
//   coefficient fold                  next_fri_polynomial (fri_commit.rs:32-50), O(d),
//                                     kept for the exact degree / loop condition (:89)
//   channel step (single lane)        Channel::send / receive_random_field_element
//                                     (src/channel/channel.rs:35-55) on the device
//   batch inverse                     FieldElement::inverse (element.rs:54-57), 0 -> 0
//
// Data in HBM is canonical u32 (value < p); constants are Montgomery (field.hpp).
#include "fri_internal.hpp"
#include "sha256.hpp"

namespace fri {

// ============================================================== NTT ======
// Natural order in -> natural order out, DIT after a bit-reversal gather.
// Passes of NS <= 8 stages over 4096-element tiles (256 threads x 16
// elements in registers): the first min(4, NS) stages run in registers on 16
// consecutive tile elements, one LDS exchange, the remaining <= 4 stages run
// in registers on stride-2^A groups, one LDS exchange back for coalesced
// stores.  Pass 1 gathers input[bitrev(i)] (zero beyond d) scaled by pre(j)
// = s^j (coset shift of the LDE); the last pass applies post(i) (n^-1 and
// offset^-i for interpolation).  Later passes see the transform as columns
// of 2^NS points at stride 2^s0; a workgroup takes 4096/2^NS consecutive
// columns, so its loads/stores are contiguous runs across columns.
// Twiddles: stage-packed table tw[2^s + j] = w_{2^(s+1)}^j (Montgomery).

__device__ __forceinline__ uint32_t pow2lvl(const uint32_t* lo, const uint32_t* hi, size_t j, uint32_t v) {
    return mmul(mmul(v, hi[j >> POW_LO_LOG]), lo[j & ((1u << POW_LO_LOG) - 1)]);
}
// LDS word of tile element x.  One pad word per 16 keeps a thread's 16
// consecutive elements (phase A) and the stride-16 groups (phase B) on 64
// distinct banks; two more per 1024 spread the 32 columns of the load and
// store phases (column stride 256 + 16 = 16 mod 64 banks alone: 8-way
// conflicts, SQ_LDS_BANK_CONFLICT) over distinct banks.
#ifndef NTT_PAD10
#define NTT_PAD10 1
#endif
__device__ __forceinline__ uint32_t ntt_laddr(uint32_t x) { return x + (x >> 4) + (NTT_PAD10 ? (x >> 10) << 1 : 0u); }

#ifndef NTT_VEC
#define NTT_VEC 1            // 16-byte load/store phases where the tile allows (launch_pass)
#endif
#ifndef NTT_TWS
#define NTT_TWS 1            // small twiddle table staged in LDS (phase B reads it per lane)
#endif
#ifndef NTT_TPB
#define NTT_TPB 512          // threads per NTT tile (16 elements each; 512: 128-byte row runs)
#endif
#ifndef NTT_WIDE
#define NTT_WIDE 1           // first pass of 9..12 stages instead of a 1..4-stage pass (k_ntt_first_wide)
#endif
#ifndef NTT_LDE24
#define NTT_LDE24 0          // A/B: 2^24 LDE (d <= 2^21) as gather + two passes (k_lde24_*); measured slower
#endif
#ifndef NTT_WIDE24
#define NTT_WIDE24 0         // A/B: 2^24 in two 12-stage passes (k_ntt_later_wide12) instead of 8 + 8 + 8
#endif

// Z (FIRST only): the input has d <= n / 2^Z coefficients, so after the
// bit-reversal gather every row q with q mod 2^Z != 0 is zero and DIT stages
// 0..Z-1 only copy a row into its zero partners (u + w*0 = u - w*0 = u):
// they become register copies (an LDE of blowup 8 skips 3 of its log_n stages).
// VEC: full tiles of 32 contiguous columns (NS = 8, n >= TILE, 16-byte
// aligned buffers, s0 >= 2): the load and store phases move 4 consecutive
// words per lane as one 16-byte access, all four of a lane's accesses issued
// before the first LDS write (or HBM store), instead of 16 4-byte accesses
// issued four at a time.
// YSRC (the second pass of the 2^24 coset LDE, k_lde24_a): the source is the
// coset-major array y[c][row][q] that k_lde24_a writes, element (row, column
// lo) of this pass at y[lo mod 8][row][lo / 8]; tiles are dealt XCD-aware (the
// eight tiles reading 16-byte pieces of the same y lines on one L2).
template <int A, int B, bool FIRST, int TPB, int Z = 0, bool VEC = false, bool YSRC = false>
__global__ __launch_bounds__(TPB) void k_ntt_pass(const uint32_t* src, size_t d, uint32_t* dst,
                                                  uint32_t log_n, uint32_t s0, const uint32_t* __restrict__ tw,
                                                  const uint32_t* __restrict__ pre_lo, const uint32_t* __restrict__ pre_hi,
                                                  const uint32_t* __restrict__ post_lo,
                                                  const uint32_t* __restrict__ post_hi) {
    // tile: 16 elements per thread; C columns (C consecutive words per row)
    constexpr uint32_t NS = A + B, P = 1u << NS, TILE = 16u * TPB, C = TILE / P;
    __shared__ uint32_t lds[TILE + TILE / 16 + 2 * (TILE >> 10)];
    __shared__ uint32_t tws[NTT_TWS ? P : 1];   // the pass's small twiddle table tw[0 .. 2^NS), read per lane in phase B
    const uint32_t tid = threadIdx.x;
    if (NTT_TWS && tid < P) tws[tid] = tw[tid];
    const size_t ncols = ((size_t)1 << log_n) >> NS;
    static_assert(!YSRC || (VEC && !FIRST && NS == 8 && C == 32), "coset source: later 8-stage vector pass");
    const uint32_t nb = gridDim.x;
    const size_t col0 = (size_t)(YSRC && !(nb & 7u) ? (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3) : blockIdx.x) * C;
    const size_t lomask = ((size_t)1 << s0) - 1;
    // FIRST (bit-reversed input): tile column c is output column
    // bitrev(col0 + c) over the log_n - NS column bits, so its row q reads
    // input bitrev_NS(q) * 2^(log_n-NS) + col0 + c: contiguous across c.
    const uint32_t cbits = log_n - NS;
    auto gidx = [&](uint32_t c, uint32_t q) -> size_t {
        const size_t col = col0 + c;
        if (FIRST) return (size_t)(cbits ? (__brev((uint32_t)col) >> (32 - cbits)) : 0u) * P + q;
        return ((col >> s0) << (s0 + NS)) + ((size_t)q << s0) + (col & lomask);
    };
    // ---- load (contiguous runs across the tile's columns) -----------------
    if (VEC) {
        static_assert(!VEC || C % 4 == 0, "vector phases need whole 4-column groups");
        constexpr uint32_t VPR = C / 4;          // 16-byte vectors per tile row
        uint4 v4[4];
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t y = r * TPB + tid;
            const uint32_t c = (y % VPR) * 4, q = y / VPR;
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (FIRST) {
                const size_t si = ((size_t)(__brev(q) >> (32 - NS)) << cbits) + col0 + c;
                if (si + 3 < d) {
                    v = *reinterpret_cast<const uint4*>(src + si);
                } else if (si < d) {   // the vector straddling d: zeros beyond it
                    v.x = src[si];
                    if (si + 1 < d) v.y = src[si + 1];
                    if (si + 2 < d) v.z = src[si + 2];
                }
                if (pre_lo && si < d) {
                    v.x = pow2lvl(pre_lo, pre_hi, si, v.x);
                    v.y = pow2lvl(pre_lo, pre_hi, si + 1, v.y);
                    v.z = pow2lvl(pre_lo, pre_hi, si + 2, v.z);
                    v.w = pow2lvl(pre_lo, pre_hi, si + 3, v.w);
                }
            } else if (YSRC) {
                // lane: row q, coset cc; words lo = col0 + 8 i + cc, i < 4 (y[cc][q][col0/8 + i])
                const size_t m8 = ((size_t)1 << log_n) >> 3;
                const uint32_t cc = y & 7u, qq = y >> 3;
                v = *reinterpret_cast<const uint4*>(src + cc * m8 + ((size_t)qq << (log_n - 3 - NS)) + (col0 >> 3));
            } else {
                v = *reinterpret_cast<const uint4*>(src + gidx(c, q));
            }
            v4[r] = v;
        }
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t y = r * TPB + tid;
            if (YSRC) {
                const uint32_t cc = y & 7u, qq = y >> 3;
                lds[ntt_laddr(cc * P + qq)] = v4[r].x;
                lds[ntt_laddr((8 + cc) * P + qq)] = v4[r].y;
                lds[ntt_laddr((16 + cc) * P + qq)] = v4[r].z;
                lds[ntt_laddr((24 + cc) * P + qq)] = v4[r].w;
                continue;
            }
            const uint32_t c = (y % VPR) * 4, q = y / VPR;
            lds[ntt_laddr(c * P + q)] = v4[r].x;
            lds[ntt_laddr((c + 1) * P + q)] = v4[r].y;
            lds[ntt_laddr((c + 2) * P + q)] = v4[r].z;
            lds[ntt_laddr((c + 3) * P + q)] = v4[r].w;
        }
    } else
#pragma unroll 4
    for (uint32_t r = 0; r < 16; r++) {
        const uint32_t y = r * TPB + tid;
        const uint32_t c = y % C, q = y / C;
        uint32_t v = 0;
        if (col0 + c < ncols) {
            if (FIRST) {
                const size_t si = ((size_t)(__brev(q) >> (32 - NS)) << cbits) + col0 + c;
                if (si < d) {
                    v = src[si];
                    if (pre_lo) v = pow2lvl(pre_lo, pre_hi, si, v);
                }
            } else {
                v = src[gidx(c, q)];
            }
        }
        lds[ntt_laddr(c * P + q)] = v;
    }
    __syncthreads();
    uint32_t r[16];
    // Twiddles.  Stage s = s0 + t of element (column lo, row q) uses
    // w_{2^(s+1)}^((q mod 2^t) * 2^s0 + lo) = w_{2^(t+1)}^(q mod 2^t) * w_{2^(s+1)}^lo:
    // a small-table entry (< 2^NS, cached) times a per-column factor.  All 16
    // elements of a thread share one column in both phases, so the factors
    // cost one table load per pass (top stage) and squarings below it
    // (w_{2^s}^lo = (w_{2^(s+1)}^lo)^2) instead of a load of the 2^s-entry
    // stage table per butterfly.
    uint32_t wl[NS];
    if (!FIRST) {
        const size_t lo = (col0 + ((tid * 16) >> NS)) & lomask;
        wl[NS - 1] = tw[((size_t)1 << (s0 + NS - 1)) + lo];
#pragma unroll
        for (int t = (int)NS - 2; t >= 0; t--) wl[t] = mmul(wl[t + 1], wl[t + 1]);
    }
    auto twid = [&](int t, uint32_t q0) -> uint32_t {
        const uint32_t j = q0 & ((1u << t) - 1);
        const uint32_t w = NTT_TWS ? tws[(1u << t) + j] : tw[(1u << t) + j];
        return FIRST ? w : mmul(w, wl[t]);
    };
    // ---- phase A: stages 0..A-1 on 16 consecutive elements ----------------
    static_assert(Z == 0 || (FIRST && Z <= A), "trivial stages only in the first pass, inside phase A");
#pragma unroll
    for (int e = 0; e < 16; e++) r[e] = (e & ((1 << Z) - 1)) ? 0u : lds[ntt_laddr(tid * 16 + e)];
#pragma unroll
    for (int e = 0; e < 16; e++) r[e] = r[e & ~((1 << Z) - 1)];       // stages 0..Z-1
    {
        const uint32_t x0 = tid * 16;
#pragma unroll
        for (int t = Z; t < A; t++) {
#pragma unroll
            for (int e = 0; e < 16; e++) {
                if (e & (1 << t)) continue;
                const uint32_t q0 = (x0 + e) & (P - 1);
                // row q0 = x0 + e with x0 a multiple of 16, so the small-table
                // twiddle w_{2^(t+1)}^(e mod 2^t) is 1 at e mod 2^t == 0: no
                // multiply in the first pass, the column factor alone in later ones
                const bool j0 = (e & ((1 << t) - 1)) == 0;
                const uint32_t u = r[e];
                const uint32_t v = (FIRST && j0) ? r[e + (1 << t)]
                                                 : mmul(r[e + (1 << t)], (!FIRST && j0) ? wl[t < NS ? t : 0] : twid(t, q0));
                r[e] = add(u, v);
                r[e + (1 << t)] = sub(u, v);
            }
        }
    }
    if (B > 0) {
#pragma unroll
        for (int e = 0; e < 16; e++) lds[ntt_laddr(tid * 16 + e)] = r[e];
        __syncthreads();
        // ---- phase B: stages A..NS-1 on groups of 2^B at stride 2^A ---------
        constexpr uint32_t GPT = 16u >> B;        // groups per thread
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t G = tid * GPT + (e >> B), m = e & ((1u << B) - 1);
            const uint32_t c = G >> A, ql = G & ((1u << A) - 1);
            r[e] = lds[ntt_laddr(c * P + ql + (m << A))];
        }
#pragma unroll
        for (int t = A; t < (int)NS; t++) {
            const uint32_t tb = t - A;
#pragma unroll
            for (int e = 0; e < 16; e++) {
                if (e & (1 << tb)) continue;
                const uint32_t G = tid * GPT + (e >> B), m = e & ((1u << B) - 1);
                const uint32_t ql = G & ((1u << A) - 1);
                const uint32_t q0 = ql + (m << A);
                const uint32_t w = twid(t, q0);
                const uint32_t u = r[e], v = mmul(r[e + (1 << tb)], w);
                r[e] = add(u, v);
                r[e + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t G = tid * GPT + (e >> B), m = e & ((1u << B) - 1);
            const uint32_t c = G >> A, ql = G & ((1u << A) - 1);
            lds[ntt_laddr(c * P + ql + (m << A))] = r[e];
        }
    } else {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 16; e++) lds[ntt_laddr(tid * 16 + e)] = r[e];
    }
    __syncthreads();
    // ---- store (contiguous runs) ------------------------------------------
    if (VEC) {
#pragma unroll
        for (uint32_t rr = 0; rr < 4; rr++) {
            const uint32_t y = rr * TPB + tid;
            uint32_t c, q, w[4];     // first element of the vector: 4 rows (FIRST) or 4 columns
            if (FIRST) { c = y / (P / 4); q = (y % (P / 4)) * 4; } else { c = (y % (C / 4)) * 4; q = y / (C / 4); }
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) w[j] = lds[ntt_laddr(FIRST ? c * P + q + j : (c + j) * P + q)];
            const size_t g = gidx(c, q);
            if (post_lo) {
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) w[j] = pow2lvl(post_lo, post_hi, g + j, w[j]);
            }
            *reinterpret_cast<uint4*>(dst + g) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        return;
    }
#pragma unroll 4
    for (uint32_t rr = 0; rr < 16; rr++) {
        const uint32_t y = rr * TPB + tid;
        uint32_t c, q;
        if (FIRST) { c = y / P; q = y % P; } else { c = y % C; q = y / C; }
        if (col0 + c >= ncols) continue;
        const size_t g = gidx(c, q);
        uint32_t v = lds[ntt_laddr(c * P + q)];
        if (post_lo) v = pow2lvl(post_lo, post_hi, g, v);
        dst[g] = v;
    }
}

// First pass with NS = 9..12 stages (k_ntt_first_wide).  A transform of
// 2^log_n with log_n mod 8 in 1..4 would otherwise start with a 1..4-stage
// pass that reads and writes the whole codeword for a few stages (2^25: 1 of
// 4 passes, 2^28: 4): this pass takes those stages together with the next 8.
// Same tile as k_ntt_pass (512 threads x 16 elements), now P = 2^NS rows x
// C = 8192 / P columns, in three register phases of 4, 4 and NS - 8 stages
// with two LDS exchanges between them.  The loads are the bit-reversed input
// rows (C consecutive words each, only the rows that are nonzero for d <=
// n / 2^Z), the stores whole contiguous columns of P words (16-byte vectors).
template <int NS, int TPB, int Z>
__global__ __launch_bounds__(TPB) void k_ntt_first_wide(const uint32_t* src, size_t d, uint32_t* dst, uint32_t log_n,
                                                        const uint32_t* __restrict__ tw,
                                                        const uint32_t* __restrict__ pre_lo,
                                                        const uint32_t* __restrict__ pre_hi,
                                                        const uint32_t* __restrict__ post_lo,
                                                        const uint32_t* __restrict__ post_hi) {
    static_assert(NS >= 9 && NS <= 12 && Z <= 3, "wide first pass: 9..12 stages");
    constexpr uint32_t P = 1u << NS, TILE = 16u * TPB, C = TILE / P;
    constexpr uint32_t VW = C < 4 ? C : 4;         // words per input vector (C consecutive words per row)
    constexpr uint32_t VPR = C / VW;               // input vectors per row
    constexpr uint32_t B2 = NS - 8;                // stages of phase 2
    __shared__ uint32_t lds[TILE + TILE / 16 + 2 * (TILE >> 10)];
    __shared__ uint32_t tws[P];                    // tw[0 .. 2^NS): w_{2^(t+1)}^j at 2^t + j
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < P; i += TPB) tws[i] = tw[i];
    // Neighbouring tiles read neighbouring C-word pieces of the same input
    // lines (8..64 bytes of each 128-byte line).  Blocks are dealt round-robin
    // over the 8 XCDs (MI355X_MICROARCH.md "Workgroup dispatch"), each with its
    // own L2: consecutive tiles go to blocks b, b + 8, b + 16, ... so that the
    // tiles sharing a line run on one XCD, close in time, and the line is
    // fetched from HBM once instead of once per XCD.
    const uint32_t nb = gridDim.x;
    const uint32_t tile = (nb & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
    const size_t col0 = (size_t)tile * C;
    const uint32_t cbits = log_n - NS;
    // ---- load: rows q = q' 2^Z (the others are zero), VW words per lane ----
    constexpr uint32_t NV = (P >> Z) * VPR;
    for (uint32_t v = tid; v < NV; v += TPB) {
        const uint32_t c = (v % VPR) * VW, q = (v / VPR) << Z;
        const size_t si = ((size_t)(__brev(q) >> (32 - NS)) << cbits) + col0 + c;
        uint32_t w[VW];
#pragma unroll
        for (uint32_t i = 0; i < VW; i++) w[i] = 0u;
        if (si + VW <= d) {
            if (VW == 4) {
                const uint4 x = *reinterpret_cast<const uint4*>(src + si);
                w[0] = x.x; w[1 % VW] = x.y; w[2 % VW] = x.z; w[3 % VW] = x.w;
            } else if (VW == 2) {
                const uint2 x = *reinterpret_cast<const uint2*>(src + si);
                w[0] = x.x; w[1 % VW] = x.y;
            } else {
                w[0] = src[si];
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < VW; i++) w[i] = si + i < d ? src[si + i] : 0u;
        }
        if (pre_lo) {
#pragma unroll
            for (uint32_t i = 0; i < VW; i++)
                if (si + i < d) w[i] = pow2lvl(pre_lo, pre_hi, si + i, w[i]);
        }
#pragma unroll
        for (uint32_t i = 0; i < VW; i++) lds[ntt_laddr((c + i) * P + q)] = w[i];
    }
    __syncthreads();
    uint32_t r[16];
    auto twid = [&](int t, uint32_t q0) -> uint32_t { return tws[(1u << t) + (q0 & ((1u << t) - 1))]; };
    // ---- phase 0: stages 0..3 on 16 consecutive rows (0..Z-1 are copies) ----
#pragma unroll
    for (int e = 0; e < 16; e++) r[e] = (e & ((1 << Z) - 1)) ? 0u : lds[ntt_laddr(tid * 16 + e)];
#pragma unroll
    for (int e = 0; e < 16; e++) r[e] = r[e & ~((1 << Z) - 1)];
    {
        const uint32_t x0 = tid * 16;
#pragma unroll
        for (int t = Z; t < 4; t++) {
#pragma unroll
            for (int e = 0; e < 16; e++) {
                if (e & (1 << t)) continue;
                const uint32_t u = r[e];
                // x0 is a multiple of 16: the twiddle of e mod 2^t == 0 is 1
                const uint32_t v = (e & ((1 << t) - 1)) == 0 ? r[e + (1 << t)]
                                                              : mmul(r[e + (1 << t)], twid(t, (x0 + e) & (P - 1)));
                r[e] = add(u, v);
                r[e + (1 << t)] = sub(u, v);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 16; e++) lds[ntt_laddr(tid * 16 + e)] = r[e];
    __syncthreads();
    // ---- phase 1: stages 4..7, one group of 16 rows at stride 16 per thread --
    {
        const uint32_t ql = tid & 15, qh = (tid >> 4) & ((1u << (NS - 8)) - 1), c = tid >> (NS - 4);
        const uint32_t base = c * P + ql + qh * 256;
#pragma unroll
        for (int m = 0; m < 16; m++) r[m] = lds[ntt_laddr(base + m * 16)];
#pragma unroll
        for (int t = 4; t < 8; t++) {
            const int tb = t - 4;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m & (1 << tb)) continue;
                const uint32_t u = r[m], v = mmul(r[m + (1 << tb)], twid(t, ql + ((uint32_t)m << 4)));
                r[m] = add(u, v);
                r[m + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++) lds[ntt_laddr(base + m * 16)] = r[m];
    }
    __syncthreads();
    // ---- phase 2: stages 8..NS-1, groups of 2^B2 rows at stride 256; group
    // g * TPB + tid, so the lanes of a wave read consecutive rows ----------
    {
        constexpr uint32_t GPT = 16u >> B2;
#pragma unroll
        for (uint32_t g = 0; g < GPT; g++) {
            const uint32_t G = g * TPB + tid, c = G >> 8, ql = G & 255;
#pragma unroll
            for (uint32_t m = 0; m < (1u << B2); m++) r[g * (1u << B2) + m] = lds[ntt_laddr(c * P + ql + m * 256)];
        }
#pragma unroll
        for (int t = 8; t < NS; t++) {
            const int tb = t - 8;
#pragma unroll
            for (uint32_t g = 0; g < GPT; g++) {
                const uint32_t ql = (g * TPB + tid) & 255;
#pragma unroll
                for (int m = 0; m < (1 << B2); m++) {
                    if (m & (1 << tb)) continue;
                    const int e = (int)g * (1 << B2) + m;
                    const uint32_t u = r[e], v = mmul(r[e + (1 << tb)], twid(t, ql + ((uint32_t)m << 8)));
                    r[e] = add(u, v);
                    r[e + (1 << tb)] = sub(u, v);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t g = 0; g < GPT; g++) {
            const uint32_t G = g * TPB + tid, c = G >> 8, ql = G & 255;
#pragma unroll
            for (uint32_t m = 0; m < (1u << B2); m++) lds[ntt_laddr(c * P + ql + m * 256)] = r[g * (1u << B2) + m];
        }
    }
    __syncthreads();
    // ---- store: tile column c is output column bitrev(col0 + c), P contiguous words
#pragma unroll
    for (uint32_t rr = 0; rr < 4; rr++) {
        const uint32_t y = rr * TPB + tid;
        const uint32_t c = y / (P / 4), q = (y % (P / 4)) * 4;
        uint32_t w[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) w[j] = lds[ntt_laddr(c * P + q + j)];
        const size_t col = col0 + c;
        const size_t g = (size_t)(cbits ? (__brev((uint32_t)col) >> (32 - cbits)) : 0u) * P + q;
        if (post_lo) {
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) w[j] = pow2lvl(post_lo, post_hi, g + j, w[j]);
        }
        *reinterpret_cast<uint4*>(dst + g) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// A later pass of 12 stages (k_ntt_later_wide12): the same 4 + 4 + 4 register
// phases on a tile of 4096 rows x 2 columns, rows at stride 2^s0.  Each row
// piece is 8 bytes, so the tiles sharing a 128-byte line are dealt to one XCD
// (as in k_ntt_first_wide) and its L2 merges their reads and partial-line
// writes.  Twiddles: small-table entry times one per-column factor, as in
// k_ntt_pass; every element of a thread is in column tid / 256.
template <int TPB>
__global__ __launch_bounds__(TPB) void k_ntt_later_wide12(const uint32_t* src, uint32_t* dst, uint32_t log_n,
                                                          uint32_t s0, const uint32_t* __restrict__ tw,
                                                          const uint32_t* __restrict__ post_lo,
                                                          const uint32_t* __restrict__ post_hi) {
    constexpr uint32_t NS = 12, P = 1u << NS, TILE = 16u * TPB, C = TILE / P;
    static_assert(C == 2 && TPB == 512, "4096 rows x 2 columns");
    __shared__ uint32_t lds[TILE + TILE / 16 + 2 * (TILE >> 10)];
    __shared__ uint32_t tws[P];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < P; i += TPB) tws[i] = tw[i];
    const uint32_t nb = gridDim.x;
    const uint32_t tile = (nb & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
    const size_t col0 = (size_t)tile * C;
    const size_t lomask = ((size_t)1 << s0) - 1;
    auto gidx = [&](uint32_t q) -> size_t { return ((col0 >> s0) << (s0 + NS)) + ((size_t)q << s0) + (col0 & lomask); };
    // ---- load: one 8-byte row piece per lane and step --------------------
    uint2 v8[8];
#pragma unroll
    for (uint32_t r = 0; r < 8; r++) v8[r] = *reinterpret_cast<const uint2*>(src + gidx(r * TPB + tid));
#pragma unroll
    for (uint32_t r = 0; r < 8; r++) {
        const uint32_t q = r * TPB + tid;
        lds[ntt_laddr(q)] = v8[r].x;
        lds[ntt_laddr(P + q)] = v8[r].y;
    }
    // column factor w_{2^(s+1)}^lo of stage s = s0 + t, by squarings from the top
    uint32_t wl[NS];
    {
        const size_t lo = (col0 + (tid >> 8)) & lomask;
        wl[NS - 1] = tw[((size_t)1 << (s0 + NS - 1)) + lo];
#pragma unroll
        for (int t = (int)NS - 2; t >= 0; t--) wl[t] = mmul(wl[t + 1], wl[t + 1]);
    }
    __syncthreads();
    auto twid = [&](int t, uint32_t q0) -> uint32_t {
        const uint32_t j = q0 & ((1u << t) - 1);
        return j ? mmul(tws[(1u << t) + j], wl[t]) : wl[t];
    };
    uint32_t r[16];
    // ---- phase 0: stages 0..3 on 16 consecutive rows ----------------------
#pragma unroll
    for (int e = 0; e < 16; e++) r[e] = lds[ntt_laddr(tid * 16 + e)];
    {
        const uint32_t x0 = tid * 16;
#pragma unroll
        for (int t = 0; t < 4; t++) {
#pragma unroll
            for (int e = 0; e < 16; e++) {
                if (e & (1 << t)) continue;
                const uint32_t u = r[e], v = mmul(r[e + (1 << t)], twid(t, (x0 + e) & (P - 1)));
                r[e] = add(u, v);
                r[e + (1 << t)] = sub(u, v);
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 16; e++) lds[ntt_laddr(tid * 16 + e)] = r[e];
    __syncthreads();
    // ---- phase 1: stages 4..7 -----------------------------------------------
    {
        const uint32_t ql = tid & 15, qh = (tid >> 4) & 15, c = tid >> 8;
        const uint32_t base = c * P + ql + qh * 256;
#pragma unroll
        for (int m = 0; m < 16; m++) r[m] = lds[ntt_laddr(base + m * 16)];
#pragma unroll
        for (int t = 4; t < 8; t++) {
            const int tb = t - 4;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m & (1 << tb)) continue;
                const uint32_t u = r[m], v = mmul(r[m + (1 << tb)], twid(t, ql + ((uint32_t)m << 4)));
                r[m] = add(u, v);
                r[m + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++) lds[ntt_laddr(base + m * 16)] = r[m];
    }
    __syncthreads();
    // ---- phase 2: stages 8..11, 16 rows at stride 256 -----------------------
    {
        const uint32_t c = tid >> 8, ql = tid & 255;
#pragma unroll
        for (int m = 0; m < 16; m++) r[m] = lds[ntt_laddr(c * P + ql + m * 256)];
#pragma unroll
        for (int t = 8; t < 12; t++) {
            const int tb = t - 8;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m & (1 << tb)) continue;
                const uint32_t u = r[m], v = mmul(r[m + (1 << tb)], twid(t, ql + ((uint32_t)m << 8)));
                r[m] = add(u, v);
                r[m + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++) lds[ntt_laddr(c * P + ql + m * 256)] = r[m];
    }
    __syncthreads();
    // ---- store --------------------------------------------------------------
#pragma unroll
    for (uint32_t rr = 0; rr < 8; rr++) {
        const uint32_t q = rr * TPB + tid;
        uint32_t a = lds[ntt_laddr(q)], b = lds[ntt_laddr(P + q)];
        const size_t g = gidx(q);
        if (post_lo) {
            a = pow2lvl(post_lo, post_hi, g, a);
            b = pow2lvl(post_lo, post_hi, g + 1, b);
        }
        *reinterpret_cast<uint2*>(dst + g) = make_uint2(a, b);
    }
}

// ---- 2^24 coset LDE in two passes (NTT_LDE24) ----------------------------
// With d <= 2^21 = n/8 coefficients, the DIT's first three stages only copy
// (the bit-reversed input is nonzero only at positions p = 0 mod 8), and the
// positions p = 8q + c of one residue c never meet another residue's in a
// later butterfly: stages 3..15 of the transform split into 8 independent
// 13-stage transforms per 2^16-position column, one per coset class c
// (eval[i], i = c mod 8, is P on the coset offset*w_n^c*<w_n^8>).  Stage
// s = t + 3 of class c uses the twiddle w_{2^(t+4)}^(8 (q mod 2^t) + c) =
// tw[2^(t+3) + 8 (q mod 2^t) + c].  So:
//   k_lde24_gather  X[r][k] = coeff[256 r + k] * offset^(256 r + k), written
//                   transposed: a0[col][r] = X[r][bitrev8(col)] (8 MB);
//   k_lde24_a       one (column, class) per workgroup: the 2^13 values
//                   X[bitrev13(q)][bitrev8(col)], 13 stages in LDS, written
//                   contiguously to y[c][col][q] (32 KB per workgroup);
//   k_ntt_pass<YSRC> stages 16..23 from y into the natural-order output:
//                   rows of 32 consecutive words (128-byte lines).
// Both passes write whole lines; the three-pass form reads and writes the
// 64 MB codeword three times (8 + 8 + 8 stages).  Measured (kernel trace,
// profiles/r03_lde24_kt.txt): gather 21.9 + pass A 72.5 + pass B 45.8 us
// against 37.5 + 39.8 + 39.7 us for the three passes.  Both forms cost about
// 5.6 us per real stage (21 either way): the passes are bound by butterfly
// issue, not by their loads and stores, so the pass count is not the lever.
// Off by default (-DNTT_LDE24=1 builds it; parity green).
__global__ __launch_bounds__(256) void k_lde24_gather(const uint32_t* __restrict__ src, size_t d, uint32_t* __restrict__ a0,
                                                      const uint32_t* __restrict__ pre_lo,
                                                      const uint32_t* __restrict__ pre_hi) {
    __shared__ uint32_t t[32][257];
    const uint32_t tid = threadIdx.x;
    const uint32_t r0 = blockIdx.x * 32u;
#pragma unroll 4
    for (uint32_t i = 0; i < 32; i++) {                    // rows r0 + i: 1 KB each, coalesced
        const size_t j = (size_t)(r0 + i) * 256u + tid;
        uint32_t v = 0u;
        if (j < d) {
            v = src[j];
            if (pre_lo) v = pow2lvl(pre_lo, pre_hi, j, v);
        }
        t[i][tid] = v;
    }
    __syncthreads();
    // 256 output rows col of 32 words (r0 .. r0 + 31): 8 lanes x 16 bytes per row
#pragma unroll
    for (uint32_t it = 0; it < 8; it++) {
        const uint32_t col = it * 32u + (tid >> 3), part = tid & 7u;
        const uint32_t k = __brev(col) >> 24;
        const uint4 w = make_uint4(t[4 * part][k], t[4 * part + 1][k], t[4 * part + 2][k], t[4 * part + 3][k]);
        *reinterpret_cast<uint4*>(a0 + (size_t)col * 8192u + r0 + 4 * part) = w;
    }
}

__global__ __launch_bounds__(512) void k_lde24_a(const uint32_t* __restrict__ a0, uint32_t* __restrict__ y,
                                                 const uint32_t* __restrict__ tw) {
    constexpr uint32_t P = 8192, TPB = 512;
    __shared__ uint32_t lds[P + P / 16 + 2 * (P >> 10)];
    __shared__ uint32_t twc[P];                  // twc[2^t + j] = w_{2^(t+4)}^(8 j + c), t < 13
    const uint32_t tid = threadIdx.x;
    // the eight classes of a column share its input: on one XCD (block b on XCD b mod 8)
    const uint32_t col = blockIdx.x & 255u, c = blockIdx.x >> 8;
    // w_{2^(t+4)}^(8j + c) = w_{2^(t+1)}^j * w_{2^(t+4)}^c: the standard stage
    // table tw[0 .. 8192) (contiguous, L2-resident) times one factor per stage
    for (uint32_t i = tid; i < P; i += TPB) {
        const uint32_t t = 31u - __clz(i | 1u);
        twc[i] = i ? mmul(tw[i], tw[(1u << (t + 3)) + c]) : 0u;
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(a0 + (size_t)col * P);
        uint4 v[4];
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) v[r] = src[r * TPB + tid];
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) {
            const uint32_t x = 4u * (r * TPB + tid);
            lds[ntt_laddr(x)] = v[r].x;
            lds[ntt_laddr(x + 1)] = v[r].y;
            lds[ntt_laddr(x + 2)] = v[r].z;
            lds[ntt_laddr(x + 3)] = v[r].w;
        }
    }
    __syncthreads();
    uint32_t R[16];
    // ---- phase 0: stages 0..3 on positions q = 16 tid + e, read bit-reversed
#pragma unroll
    for (int e = 0; e < 16; e++) R[e] = lds[ntt_laddr(__brev(16u * tid + (uint32_t)e) >> 19)];
#pragma unroll
    for (int t = 0; t < 4; t++) {
#pragma unroll
        for (int e = 0; e < 16; e++) {
            if (e & (1 << t)) continue;
            const uint32_t u = R[e], v = mmul(R[e + (1 << t)], twc[(1u << t) + ((uint32_t)e & ((1u << t) - 1))]);
            R[e] = add(u, v);
            R[e + (1 << t)] = sub(u, v);
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 16; e++) lds[ntt_laddr(16u * tid + e)] = R[e];
    __syncthreads();
    // ---- phase 1: stages 4..7, 16 positions at stride 16 --------------------
    {
        const uint32_t ql = tid & 15u, base = ql + (tid >> 4) * 256u;
#pragma unroll
        for (int m = 0; m < 16; m++) R[m] = lds[ntt_laddr(base + 16u * m)];
#pragma unroll
        for (int t = 4; t < 8; t++) {
            const int tb = t - 4;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m & (1 << tb)) continue;
                const uint32_t q = ql + 16u * (uint32_t)m;
                const uint32_t u = R[m], v = mmul(R[m + (1 << tb)], twc[(1u << t) + (q & ((1u << t) - 1))]);
                R[m] = add(u, v);
                R[m + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++) lds[ntt_laddr(base + 16u * m)] = R[m];
    }
    __syncthreads();
    // ---- phase 2: stages 8..11, 16 positions at stride 256 ------------------
    {
        const uint32_t ql = tid & 255u, base = ql + (tid >> 8) * 4096u;
#pragma unroll
        for (int m = 0; m < 16; m++) R[m] = lds[ntt_laddr(base + 256u * m)];
#pragma unroll
        for (int t = 8; t < 12; t++) {
            const int tb = t - 8;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                if (m & (1 << tb)) continue;
                const uint32_t q = ql + 256u * (uint32_t)m;
                const uint32_t u = R[m], v = mmul(R[m + (1 << tb)], twc[(1u << t) + (q & ((1u << t) - 1))]);
                R[m] = add(u, v);
                R[m + (1 << tb)] = sub(u, v);
            }
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; m++) lds[ntt_laddr(base + 256u * m)] = R[m];
    }
    __syncthreads();
    // ---- stage 12 (pairs q, q + 4096) and the store: 8 consecutive q per lane
    uint32_t* out = y + (size_t)c * ((size_t)1 << 21) + (size_t)col * P;
    uint32_t lo[8], hi[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t q = 8u * tid + i;
        const uint32_t u = lds[ntt_laddr(q)], v = mmul(lds[ntt_laddr(q + 4096u)], twc[4096u + q]);
        lo[i] = add(u, v);
        hi[i] = sub(u, v);
    }
    uint4* o = reinterpret_cast<uint4*>(out + 8u * tid);
    o[0] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    o[1] = make_uint4(lo[4], lo[5], lo[6], lo[7]);
    uint4* oh = reinterpret_cast<uint4*>(out + 4096u + 8u * tid);
    oh[0] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    oh[1] = make_uint4(hi[4], hi[5], hi[6], hi[7]);
}

template <int NS>
static void launch_first_wide(const uint32_t* src, size_t d, uint32_t* dst, uint32_t log_n, const NttPlan& p,
                              bool last, uint32_t z, hipStream_t s) {
    constexpr int TPB = 512;
    const unsigned blocks = (unsigned)(((size_t)1 << log_n) / (16 * TPB));
    const uint32_t* qlo = last ? p.post_lo : nullptr;
    const uint32_t* qhi = last ? p.post_hi : nullptr;
    switch (z) {
#define WIDE_CASE(ZV)                                                                                        \
    case ZV:                                                                                                 \
        hipLaunchKernelGGL((k_ntt_first_wide<NS, TPB, ZV>), dim3(blocks), dim3(TPB), 0, s, src, d, dst, log_n, \
                           p.tw, p.pre_lo, p.pre_hi, qlo, qhi);                                              \
        break;
        WIDE_CASE(0) WIDE_CASE(1) WIDE_CASE(2) default: WIDE_CASE(3)
#undef WIDE_CASE
    }
}

__global__ void k_ntt_one(const uint32_t* src, size_t d, uint32_t* dst, const uint32_t* pre_lo,
                          const uint32_t* pre_hi, const uint32_t* post_lo, const uint32_t* post_hi) {
    if (threadIdx.x) return;
    uint32_t v = d ? src[0] : 0u;
    if (d && pre_lo) v = pow2lvl(pre_lo, pre_hi, 0, v);
    if (post_lo) v = pow2lvl(post_lo, post_hi, 0, v);
    dst[0] = v;
}

template <bool FIRST, int Z = 0>
static void launch_pass(uint32_t ns, const uint32_t* src, size_t d, uint32_t* dst, uint32_t log_n, uint32_t s0,
                        const NttPlan& p, bool last, hipStream_t s) {
    const size_t n = (size_t)1 << log_n;
    constexpr int TPB = NTT_TPB;
    const unsigned blocks = (unsigned)((n + 16 * TPB - 1) / (16 * TPB));
    const uint32_t* plo = FIRST ? p.pre_lo : nullptr;
    const uint32_t* phi = FIRST ? p.pre_hi : nullptr;
    const uint32_t* qlo = last ? p.post_lo : nullptr;
    const uint32_t* qhi = last ? p.post_hi : nullptr;
#define NTT_CASE(NSV, AV, BV)                                                                                   \
    case NSV:                                                                                                   \
        hipLaunchKernelGGL((k_ntt_pass<AV, BV, FIRST, TPB, (Z < AV ? Z : AV)>), dim3(blocks), dim3(TPB), 0, s, src, d, \
                           dst, log_n, s0, p.tw, plo, phi, qlo, qhi);                                           \
        break;
    // vector load/store phases: whole tiles of 32 contiguous columns, 16-byte aligned buffers
    const bool vec = NTT_VEC && ns == 8 && n >= 16u * TPB && (FIRST || s0 >= 2) &&
                     ((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0;
    if (vec) {
        hipLaunchKernelGGL((k_ntt_pass<4, 4, FIRST, TPB, (Z < 4 ? Z : 4), true>), dim3(blocks), dim3(TPB), 0, s, src,
                           d, dst, log_n, s0, p.tw, plo, phi, qlo, qhi);
        return;
    }
    switch (ns) {
        NTT_CASE(1, 1, 0) NTT_CASE(2, 2, 0) NTT_CASE(3, 3, 0) NTT_CASE(4, 4, 0)
        NTT_CASE(5, 4, 1) NTT_CASE(6, 4, 2) NTT_CASE(7, 4, 3) NTT_CASE(8, 4, 4)
        default: break;
    }
#undef NTT_CASE
}

// First pass with the zero rows of a padded input skipped: z trivial stages
// when d <= n / 2^z (z <= 3, and at most the pass's phase-A stages).
static void launch_first(uint32_t ns, const uint32_t* src, size_t d, uint32_t* dst, uint32_t log_n, const NttPlan& p,
                         bool last, hipStream_t s) {
    uint32_t z = 0;
    while (z < 3 && z < ns && ((size_t)d << (z + 1)) <= ((size_t)1 << log_n)) z++;
    switch (z) {
        case 0: launch_pass<true, 0>(ns, src, d, dst, log_n, 0, p, last, s); break;
        case 1: launch_pass<true, 1>(ns, src, d, dst, log_n, 0, p, last, s); break;
        case 2: launch_pass<true, 2>(ns, src, d, dst, log_n, 0, p, last, s); break;
        default: launch_pass<true, 3>(ns, src, d, dst, log_n, 0, p, last, s); break;
    }
}

void launch_ntt(const NttPlan& p, const uint32_t* src, size_t d, uint32_t* dst, hipStream_t s) {
    const uint32_t log_n = p.log_n;
    if (log_n == 0) {   // one point: dst[0] = post(0) * pre(0) * src[0]
        hipLaunchKernelGGL(k_ntt_one, dim3(1), dim3(64), 0, s, src, d, dst, p.pre_lo, p.pre_hi, p.post_lo, p.post_hi);
        return;
    }
    uint32_t first = log_n % 8;
    if (first == 0) first = 8;
#if NTT_LDE24
    // 2^24 from <= 2^21 coefficients (blowup >= 8): gather + two passes (k_lde24_*)
    if (log_n == 24 && p.scratch && !p.post_lo && d <= ((size_t)1 << 21) &&
        ((((uintptr_t)src) | ((uintptr_t)dst) | ((uintptr_t)p.scratch)) & 15u) == 0) {
        hipLaunchKernelGGL(k_lde24_gather, dim3(256), dim3(256), 0, s, src, d, dst, p.pre_lo, p.pre_hi);
        hipLaunchKernelGGL(k_lde24_a, dim3(2048), dim3(512), 0, s, dst, p.scratch, p.tw);
        hipLaunchKernelGGL((k_ntt_pass<4, 4, false, 512, 0, true, true>), dim3(2048), dim3(512), 0, s, p.scratch,
                           (size_t)0, dst, 24u, 16u, p.tw, nullptr, nullptr, nullptr, nullptr);
        return;
    }
#endif
#if NTT_WIDE24
    // 2^24: two passes of 12 stages (k_ntt_first_wide<12> + k_ntt_later_wide12)
    if (log_n == 24 && ((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0) {
        uint32_t z = 0;
        while (z < 3 && ((size_t)d << (z + 1)) <= ((size_t)1 << log_n)) z++;
        launch_first_wide<12>(src, d, dst, log_n, p, false, z, s);
        hipLaunchKernelGGL((k_ntt_later_wide12<512>), dim3((unsigned)(((size_t)1 << log_n) / 8192)), dim3(512), 0, s,
                           dst, dst, log_n, 12u, p.tw, p.post_lo, p.post_hi);
        return;
    }
#endif
#if NTT_WIDE
    // a short first pass (1..4 stages) merged with the next 8: one pass fewer
    if (first <= 4 && log_n >= 13 && log_n - first >= 8 &&
        ((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0) {
        first += 8;
        uint32_t z = 0;
        while (z < 3 && ((size_t)d << (z + 1)) <= ((size_t)1 << log_n)) z++;
        const bool last = first == log_n;
        switch (first) {
            case 9: launch_first_wide<9>(src, d, dst, log_n, p, last, z, s); break;
            case 10: launch_first_wide<10>(src, d, dst, log_n, p, last, z, s); break;
            case 11: launch_first_wide<11>(src, d, dst, log_n, p, last, z, s); break;
            default: launch_first_wide<12>(src, d, dst, log_n, p, last, z, s); break;
        }
        for (uint32_t s0 = first; s0 < log_n; s0 += 8)
            launch_pass<false>(8, dst, 0, dst, log_n, s0, p, s0 + 8 == log_n, s);
        return;
    }
#endif
    launch_first(first, src, d, dst, log_n, p, first == log_n, s);
    for (uint32_t s0 = first; s0 < log_n; s0 += 8)
        launch_pass<false>(8, dst, 0, dst, log_n, s0, p, s0 + 8 == log_n, s);
}

// Stage-packed twiddles: tw[2^s + j] = Montgomery(w_{2^(s+1)}^j), so every
// DIT stage s reads a contiguous run (independent of the transform size).
struct StageBases { uint32_t b[32]; };
__global__ void k_twiddles(uint32_t* tw, size_t count, StageBases sb) {
    size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    if (e == 0) { tw[0] = R_MOD_P; return; }
    uint32_t s = 63u - (uint32_t)__clzll((unsigned long long)e);
    tw[e] = mpow(sb.b[s], e - ((size_t)1 << s));
}
void launch_twiddles(uint32_t* tw, uint32_t log_max, bool inverse, hipStream_t s) {
    StageBases sb{};
    for (uint32_t st = 0; st < log_max && st < 31; st++) {
        uint32_t w = root_of_unity(st + 1);
        sb.b[st] = to_mont(inverse ? inv_std(w) : w);
    }
    size_t count = (size_t)1 << log_max;
    hipLaunchKernelGGL(k_twiddles, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, tw, count, sb);
}

// Two-level power table of base^j scaled by `scale`: lo[t] = base^t,
// hi[t] = scale * base^(4096 t)  (Montgomery).
__global__ void k_pow_table(uint32_t* lo, uint32_t* hi, uint32_t nhi, uint32_t base_m, uint32_t scale_m) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nlo = 1u << POW_LO_LOG;
    if (t < nlo) lo[t] = mpow(base_m, t);
    else if (t < nlo + nhi) {
        uint32_t q = t - nlo;
        hi[q] = mmul(scale_m, mpow(base_m, (uint64_t)q << POW_LO_LOG));
    }
}
void launch_pow_table(uint32_t* lo, uint32_t* hi, uint32_t log_n, uint32_t base_std, uint32_t scale_std,
                      hipStream_t s) {
    uint32_t nhi = log_n > POW_LO_LOG ? (1u << (log_n - POW_LO_LOG)) : 1u;
    uint32_t tot = (1u << POW_LO_LOG) + nhi;
    hipLaunchKernelGGL(k_pow_table, dim3((tot + 255) / 256), dim3(256), 0, s, lo, hi, nhi, to_mont(base_std),
                       to_mont(scale_std));
}

// ========================================================= batch inverse ==
// Montgomery's trick per thread over BI_K strided elements (coalesced), one
// Fermat inversion per thread; zeros are skipped and map to 0 exactly like
// FieldElement::inverse (0^(p-2) = 0).
constexpr uint32_t BI_K = 16;
__global__ __launch_bounds__(256) void k_batch_inverse(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       size_t n, size_t stride, int out_mont) {
    size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= stride) return;
    uint32_t a[BI_K], pre[BI_K];
    uint32_t acc = R_MOD_P;
#pragma unroll
    for (uint32_t k = 0; k < BI_K; k++) {
        size_t i = g + k * stride;
        uint32_t x = i < n ? in[i] : 0u;
        a[k] = x ? to_mont(x) : 0u;
        pre[k] = acc;
        if (x) acc = mmul(acc, a[k]);
    }
    uint32_t inv = mpow(acc, P - 2);
#pragma unroll
    for (int k = BI_K - 1; k >= 0; k--) {
        size_t i = g + (size_t)k * stride;
        uint32_t r = 0;
        if (a[k]) { r = mmul(inv, pre[k]); inv = mmul(inv, a[k]); }
        if (i < n) out[i] = out_mont ? r : from_mont(r);
    }
}
void launch_batch_inverse(const uint32_t* in, uint32_t* out, size_t n, int out_mont, hipStream_t s) {
    size_t stride = (n + BI_K - 1) / BI_K;
    if (!stride) return;
    hipLaunchKernelGGL(k_batch_inverse, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, s, in, out, n, stride,
                       out_mont);
}

// out[i] = offset * w_n^i (canonical)
__global__ void k_coset_points(uint32_t* out, size_t count, uint32_t off, uint32_t w_m) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = mmul(off, mpow(w_m, i));
}
void launch_coset_points(uint32_t* out, size_t count, uint32_t offset, uint32_t log_n, hipStream_t s) {
    hipLaunchKernelGGL(k_coset_points, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, out, count, offset,
                       to_mont(root_of_unity(log_n)));
}

__global__ void k_square_mont(const uint32_t* in, uint32_t* out, size_t count) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) { uint32_t x = in[i]; out[i] = mmul(x, x); }
}
void launch_square_mont(const uint32_t* in, uint32_t* out, size_t count, hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(k_square_mont, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, in, out, count);
}

// Horner at arbitrary points (ops.rs:76-83): one lane per point.
__global__ void k_evaluate(const uint32_t* __restrict__ c, size_t d, const uint32_t* __restrict__ xs, size_t count,
                           uint32_t* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t xm = to_mont(xs[i]), r = 0;
    for (size_t k = d; k-- > 0;) r = add(mmul(r, xm), c[k]);
    out[i] = r;
}
// Few points, many coefficients: lane l of the S lanes of a point takes the
// coefficients j = k S + l (coalesced across lanes) and evaluates
// H_l = sum_k c[kS + l] (x^S)^k by Horner in y = x^S; then
// p(x) = sum_l x^l H_l, summed per workgroup here and over the B workgroups
// of the point by k_evaluate_join.  Exact field arithmetic: the same value as
// Horner's rule in any order.
__global__ __launch_bounds__(256) void k_evaluate_strided(const uint32_t* __restrict__ c, size_t d,
                                                          const uint32_t* __restrict__ xs, uint32_t S,
                                                          uint32_t* __restrict__ part) {
    __shared__ uint32_t red[4];
    const uint32_t p = blockIdx.y, l = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t xm = to_mont(xs[p]);
    const uint32_t ym = mpow(xm, S);                               // x^S, Montgomery
    const size_t K = (d + S - 1) / S;
    uint32_t h = 0;
    for (size_t k = K; k-- > 0;) {
        const size_t j = k * S + l;
        h = add(mmul(h, ym), j < d ? c[j] : 0u);
    }
    uint32_t v = mmul(h, mpow(xm, l));                             // x^l H_l, canonical
    for (int o = 32; o >= 1; o >>= 1) v = add(v, (uint32_t)__shfl_xor((int)v, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) part[(size_t)p * gridDim.x + blockIdx.x] = add(add(red[0], red[1]), add(red[2], red[3]));
}
__global__ void k_evaluate_join(const uint32_t* __restrict__ part, uint32_t B, size_t count, uint32_t* __restrict__ out) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= count) return;
    uint32_t v = 0;
    for (uint32_t b = 0; b < B; b++) v = add(v, part[p * B + b]);
    out[p] = v;
}
size_t evaluate_tmp_words(size_t d, size_t count) {
    if (count >= ((size_t)1 << 16) || d < 4096) return 0;          // one lane per point is enough
    size_t S = 256;                                                // >= 2^18 lanes, >= 16 coefficients each
    while (S < 8192 && count * S < ((size_t)1 << 18) && d / (2 * S) >= 16) S *= 2;
    return count * (S / 256);
}
void launch_evaluate(const uint32_t* coeffs, size_t d, const uint32_t* xs, size_t count, uint32_t* out,
                     uint32_t* tmp, hipStream_t s) {
    if (!count) return;
    const size_t tw = evaluate_tmp_words(d, count);
    if (!tw) {
        hipLaunchKernelGGL(k_evaluate, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, coeffs, d, xs, count,
                           out);
        return;
    }
    const uint32_t B = (uint32_t)(tw / count), S = 256 * B;
    hipLaunchKernelGGL(k_evaluate_strided, dim3(B, (unsigned)count), dim3(256), 0, s, coeffs, d, xs, S, tmp);
    hipLaunchKernelGGL(k_evaluate_join, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, tmp, B, count, out);
}

// ============================================ arbitrary-point interpolate ==
// Polynomial::interpolate on points that are not a coset (interpolation.rs:
// 121-152): f = sum_j y_j w_j Z(x)/(x - x_j), w_j = 1/prod_{i!=j}(x_j - x_i).
// Products run in the "R^-1 per step" form: mmul(acc, t) = acc*t*R^-1 with
// both operands canonical, so a chain of m products carries R^-m, fixed by one
// product with R^(m+1) at the end.  x and c tiles are staged in LDS.  One
// lane per output point leaves a wave per SIMD at n = 2^16, so the point range
// is cut into S segments (blockIdx.y) whose partial results are combined by a
// second kernel.
constexpr uint32_t INTERP_TILE = 1024;

// segment s of prod_{i!=j}(x_j - x_i): part[s*n + j], exponent (segment
// length - [j in segment]) of R^-1
__global__ __launch_bounds__(256) void k_interp_weights(const uint32_t* __restrict__ xs, size_t n, size_t seg,
                                                        uint32_t* __restrict__ part) {
    __shared__ uint32_t xt[INTERP_TILE];
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = (size_t)blockIdx.y * seg, hi = lo + seg < n ? lo + seg : n;
    const uint32_t xj = j < n ? xs[j] : 0u;
    uint32_t a = 1u;
    for (size_t base = lo; base < hi; base += INTERP_TILE) {
        const uint32_t m = (uint32_t)(hi - base < INTERP_TILE ? hi - base : INTERP_TILE);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) xt[i] = xs[base + i];
        __syncthreads();
        const uint32_t self = (j >= base && j < base + m) ? (uint32_t)(j - base) : INTERP_TILE;
        for (uint32_t i = 0; i < m; i++) {
            const uint32_t t = i == self ? R_MOD_P : sub(xj, xt[i]);   // skip i == j: a Montgomery 1
            a = mmul(a, t);
        }
    }
    if (j < n) part[blockIdx.y * n + j] = a;
}
// prod over the S segments (S - 1 more R^-1), times the fix-up: the exact
// prod_{i!=j}(x_j - x_i), canonical
__global__ void k_interp_weights_join(const uint32_t* __restrict__ part, size_t n, uint32_t S, uint32_t fix,
                                      uint32_t* __restrict__ acc) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t a = part[j];
    for (uint32_t s = 1; s < S; s++) a = mmul(a, part[s * n + j]);
    acc[j] = mmul(a, fix);
}
static uint32_t interp_segments(size_t n, size_t lanes) {
    uint32_t S = 1;                          // >= 2^20 lanes in flight, segments of >= 256 points
    while (S < 64 && lanes * S < ((size_t)1 << 20) && n / (2 * S) >= 256) S *= 2;
    return S;
}
size_t interp_tmp_words(size_t n, uint32_t log_N) {
    const size_t N = (size_t)1 << log_N;
    const size_t a = interp_segments(n, n) * n, b = 2 * (size_t)interp_segments(n, N) * N;
    return a > b ? a : b;
}
void launch_interp_weights(const uint32_t* xs, size_t n, uint32_t* acc, uint32_t* tmp, hipStream_t s) {
    const uint32_t S = interp_segments(n, n);
    const size_t seg = (n + S - 1) / S;
    // n - 1 factors carry R^-1 (the skipped i == j does not), plus S - 1 joins
    const uint32_t fix = pow_std(R_MOD_P, (uint64_t)n + S - 1);
    hipLaunchKernelGGL(k_interp_weights, dim3((unsigned)((n + 255) / 256), S), dim3(256), 0, s, xs, n, seg, tmp);
    hipLaunchKernelGGL(k_interp_weights_join, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tmp, n, S, fix,
                       acc);
}

__global__ void k_interp_coeffs(const uint32_t* __restrict__ ys, uint32_t* __restrict__ w, size_t n) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) w[j] = mmul(ys[j], w[j]);        // w Montgomery -> c_j = y_j w_j canonical
}
void launch_interp_coeffs(const uint32_t* ys, uint32_t* w_to_c, size_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_interp_coeffs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ys, w_to_c, n);
}

// f(u), u = w_N^k: num/den = sum_j c_j/(u - x_j) as one running fraction over
// the segment's points, num <- num (u - x_j) + c_j den, den <- den (u - x_j).
// Over all n points den = Z(u) and num = Z(u) * sum_j c_j/(u - x_j) = f(u): a
// polynomial identity in u, so it holds at u = x_j too (no inverse, no
// special case).  Segments are fractions over disjoint point sets and join as
// num = num_a den_b + num_b den_a, den = den_a den_b.
__global__ __launch_bounds__(256) void k_interp_eval(const uint32_t* __restrict__ xs, const uint32_t* __restrict__ c,
                                                     size_t n, size_t seg, uint32_t w_m, size_t N,
                                                     uint32_t* __restrict__ part) {
    __shared__ uint2 tile[INTERP_TILE];
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t lo = (size_t)blockIdx.y * seg, hi = lo + seg < n ? lo + seg : n;
    const uint32_t u = from_mont(mpow(w_m, k));
    uint32_t num = 0u, den = 1u;
    for (size_t base = lo; base < hi; base += INTERP_TILE) {
        const uint32_t m = (uint32_t)(hi - base < INTERP_TILE ? hi - base : INTERP_TILE);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) tile[i] = make_uint2(xs[base + i], c[base + i]);
        __syncthreads();
#pragma unroll 4
        for (uint32_t i = 0; i < m; i++) {
            const uint2 xc = tile[i];
            const uint32_t t = sub(u, xc.x);
            num = add(mmul(num, t), mmul(xc.y, den));
            den = mmul(den, t);
        }
    }
    if (k < N) {
        part[(2 * (size_t)blockIdx.y) * N + k] = num;
        part[(2 * (size_t)blockIdx.y + 1) * N + k] = den;
    }
}
__global__ void k_interp_eval_join(const uint32_t* __restrict__ part, size_t N, uint32_t S, uint32_t fix,
                                   uint32_t* __restrict__ f) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    uint32_t num = part[k], den = part[N + k];
    for (uint32_t s = 1; s < S; s++) {
        const uint32_t nb = part[2 * s * N + k], db = part[(2 * s + 1) * N + k];
        num = add(mmul(num, db), mmul(nb, den));
        den = mmul(den, db);
    }
    f[k] = mmul(num, fix);
}
void launch_interp_eval(const uint32_t* xs, const uint32_t* c, size_t n, uint32_t log_N, uint32_t* f, uint32_t* tmp,
                        hipStream_t s) {
    const size_t N = (size_t)1 << log_N;
    const uint32_t S = interp_segments(n, N);
    const size_t seg = (n + S - 1) / S;
    // n steps and S - 1 joins of R^-1: mmul(num, R^(n+S)) = num R^(n+S-1)
    const uint32_t fix = pow_std(R_MOD_P, (uint64_t)n + S);
    hipLaunchKernelGGL(k_interp_eval, dim3((unsigned)((N + 255) / 256), S), dim3(256), 0, s, xs, c, n, seg,
                       to_mont(root_of_unity(log_N)), N, tmp);
    hipLaunchKernelGGL(k_interp_eval_join, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, tmp, N, S, fix, f);
}

// ================================================================== fold ==
// L'[i] = 2^-1 * ((a+b) + beta*(a-b)*x_i^-1),  a = L[i], b = L[i+m/2] = L(-x_i).
// xinv_m[i] = Montgomery(x_i^-1) for the layer's domain.
constexpr uint32_t INV2_M = 0x80000000u;   // Montgomery(2^-1) = 2^31 mod p (static_assert below)
static_assert(((unsigned __int128)INV2_M * 2) % P == R_MOD_P, "INV2_M");

__device__ __forceinline__ uint32_t fold_one(uint32_t a, uint32_t b, uint32_t xinv_m, uint32_t beta_m) {
    uint32_t s = add(a, b), t = sub(a, b);
    uint32_t v = mmul(mmul(t, xinv_m), beta_m);
    return mmul(add(s, v), INV2_M);
}

__global__ __launch_bounds__(256) void k_fold(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                              size_t half, const uint32_t* __restrict__ xinv_m, uint32_t beta_m,
                                              const DevState* __restrict__ st, int r) {
    if (st && !st->active[r]) return;
    if (st) beta_m = st->beta_mont[r];
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < half) out[i] = fold_one(in[i], in[i + half], xinv_m[i], beta_m);
}
void launch_fold_plain(const uint32_t* in, uint32_t* out, uint32_t log_m, const uint32_t* xinv_m, uint32_t beta,
                       hipStream_t s) {
    size_t half = ((size_t)1 << log_m) / 2;
    hipLaunchKernelGGL(k_fold, dim3((unsigned)((half + 255) / 256)), dim3(256), 0, s, in, out, half, xinv_m,
                       to_mont(beta), (const DevState*)nullptr, 0);
}

// Decommitment gather for one query (fri_commit.rs:137-163): block k reads
// layer k's value at idx = index % m_k and at its sibling (idx + m_k/2) % m_k,
// and the two authentication paths (sibling digest per level, leaf -> root),
// as raw big-endian bytes.  One launch + one copy per query.
__global__ void k_decommit_gather(const uint32_t* __restrict__ layers, const uint32_t* __restrict__ trees,
                                  const uint32_t* __restrict__ top, DecommitPlan dp, uint32_t* __restrict__ out) {
    const uint32_t k = blockIdx.x;
    const uint32_t L = dp.log_n - k;
    const uint64_t m = (uint64_t)1 << L;
    const uint64_t idx = dp.index % m;
    const uint64_t sib = (idx + m / 2) % m;
    const bool sharded = dp.shard_lb1[k] != 0;
    const uint32_t lb = sharded ? dp.shard_lb1[k] - 1u : 0u;
    const uint64_t bmask = sharded ? ((uint64_t)1 << lb) - 1 : ~(uint64_t)0;
    // a sharded layer: is the opened element in a block this rank holds?
    auto mine = [&](uint64_t i) -> bool { return !sharded || ((dp.owned[k] >> (i >> lb)) & 1u); };
    auto vidx = [&](uint64_t i) -> uint64_t { return (sharded && dp.val_block[k]) ? (i & bmask) : i; };
    if (threadIdx.x == 0) {
        out[2 * k] = mine(idx) ? layers[dp.layer_off[k] + vidx(idx)] : 0u;
        out[2 * k + 1] = mine(sib) ? layers[dp.layer_off[k] + vidx(sib)] : 0u;
    }
    const uint32_t l = threadIdx.x;
    if (l >= L) return;
    const uint32_t* tr = trees + dp.tree_off[k];
    uint32_t* paths = out + 2 * dp.n_layers + dp.path_off[k];
#pragma unroll
    for (int which = 0; which < 2; which++) {
        const uint64_t leaf = which ? sib : idx;
        uint32_t* o = paths + (size_t)which * 8 * L + 8 * l;
        if (!mine(leaf)) {
#pragma unroll
            for (int w = 0; w < 8; w++) o[w] = 0u;
            continue;
        }
        const uint32_t* d;
        if (!sharded) {
            d = tr + 8 * (level_offset(L, l) + ((leaf >> l) ^ 1u));
        } else if (l < lb) {                         // inside the block: the block-local tree
            d = tr + 8 * (level_offset(lb, l) + (((leaf & bmask) >> l) ^ 1u));
        } else {                                     // above it: the replicated top tree of block roots
            const uint32_t t = l - lb;
            d = top + dp.top_off[k] + 8 * (level_offset(dp.logG, t) + (((leaf >> lb) >> t) ^ 1u));
        }
#pragma unroll
        for (int w = 0; w < 8; w++) o[w] = __builtin_bswap32(d[w]);
    }
}
void launch_decommit_gather(const uint32_t* layers, const uint32_t* trees, const DecommitPlan& dp, uint32_t* out,
                            hipStream_t s, const uint32_t* top) {
    hipLaunchKernelGGL(k_decommit_gather, dim3(dp.n_layers), dim3(64), 0, s, layers, trees, top, dp, out);
}

}  // namespace fri
