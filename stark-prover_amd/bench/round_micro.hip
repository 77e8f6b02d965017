// Dev microbenchmark: issue order and lane layout of the lane-pair SHA-256
// round (sha256_quad.hpp) on a lone wave.
//
// A lone wave issues one VALU instruction per ~4 cycles and a dependent
// instruction waits ~8.  The product round (11 instructions,
// E lane = even lane of a quad_perm pair) ends in the chain
//     V = S + F + hk  ->  Z = me ? V : x3  ->  n = V + swap(Z)
// where the select Z sits between the round's value and the DPP add, and its
// two independent instructions (h + K + W, the lane mask) are left after Z.
//
// Mirror layout (mode 1): the two lanes of a pair are j and 7 - j of each
// group of eight (row_half_mirror is its own inverse), E lanes 0..3, A lanes
// 4..7 = DPP banks 1 and 3.  The round's new value is then written by two
// instructions that both read V directly:
//     n = V + dc                      (all lanes; right on E: dc = d)
//     n = V + mirror(V), banks 1, 3   (A lanes only: T2 + T1)
// with dc = mirror(x3) fetched at the start of the round (x3 is three rounds
// old) and the next round's h + K + W computed in the slots the chain leaves:
// 12 instructions, no select on the critical path, in one asm block so the
// order is the one written.
//
// One wave, NB dependent padding-block compressions (the constant-K+W block
// of every node), s_memtime around the chain; both modes must give the same
// digests (checked).
//   hipcc -O3 --offload-arch=gfx950 -I../csrc round_micro.hip -o round_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "sha256_quad.hpp"
using namespace fri;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int NB = 32;

// mirror-layout round: kwn = the next round's K + W (scalar)
#define MR_S(kwn)                                                                                   \
    {                                                                                               \
        uint32_t n_, t1_, t2_, t3_, sel_, dc_, hkn_;                                                \
        asm volatile("v_mov_b32_dpp %[dc], %[x3] row_half_mirror row_mask:0xf bank_mask:0xf\n\t"   \
                     "v_alignbit_b32 %[t1], %[x0], %[x0], %[r1]\n\t"                                \
                     "v_alignbit_b32 %[t2], %[x0], %[x0], %[r2]\n\t"                                \
                     "v_alignbit_b32 %[t3], %[x0], %[x0], %[r3]\n\t"                                \
                     "v_bitop3_b32 %[sel], %[x0], %[x1], %[m] bitop3:0x2d\n\t"                      \
                     "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                      \
                     "v_bitop3_b32 %[t2], %[sel], %[x2], %[x1] bitop3:0xca\n\t"                     \
                     "v_add_u32 %[hkn], %[kw], %[x2]\n\t"                                           \
                     "v_add3_u32 %[t1], %[t1], %[t2], %[hk]\n\t"                                    \
                     "v_and_b32 %[hkn], %[hkn], %[me]\n\t"                                          \
                     "v_add_u32 %[n], %[t1], %[dc]\n\t"                                             \
                     "v_add_u32_dpp %[n], %[t1], %[t1] row_half_mirror row_mask:0xf bank_mask:0xa"  \
                     : [n] "=&v"(n_), [t1] "=&v"(t1_), [t2] "=&v"(t2_), [t3] "=&v"(t3_), [sel] "=&v"(sel_), \
                       [dc] "=&v"(dc_), [hkn] "=&v"(hkn_)                                           \
                     : [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3), [hk] "v"(hk), [kw] "s"(kwn), \
                       [r1] "v"(R.r1), [r2] "v"(R.r2), [r3] "v"(R.r3), [m] "v"(R.m), [me] "v"(R.me));   \
        x3 = x2; x2 = x1; x1 = x0; x0 = n_; hk = hkn_;                                              \
    }

__device__ __forceinline__ void compress_kw_mirror(uint32_t st[4], const uint32_t* kw, const shaq::Role& R) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    uint32_t hk = (x3 + kw[0]) & R.me;
    asm volatile("s_nop 1" ::: "memory");         // x3 may have just been written: DPP read hazard
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
        // this group's next-round constants, loaded up front (scalar loads
        // are not moved across the asm statements)
        uint32_t k[16];
#pragma unroll
        for (int i = 0; i < 15; i++) k[i] = kw[16 * r + i + 1];
        k[15] = r < 3 ? kw[16 * r + 16] : 0u;
#pragma unroll
        for (int i = 0; i < 16; i++) MR_S(k[i]);
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}

// Four rounds per asm block (mode 2): the register names rotate back after
// four rounds, and the compiler's guard between asm blocks (an s_nop, for a
// DPP read it cannot see) is paid once per four rounds.
#define MR_ROUND(X0, X1, X2, X3, HK, HKN, KW) MR_ROUND_B(X0, X1, X2, X3, HK, HKN, KW, "0xa")
#define MR_ROUND_B(X0, X1, X2, X3, HK, HKN, KW, BM)                                     \
    "v_mov_b32_dpp %[dc], %[" #X3 "] row_half_mirror row_mask:0xf bank_mask:0xf\n\t"  \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                         \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                         \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                         \
    "v_bitop3_b32 %[sel], %[" #X0 "], %[" #X1 "], %[m] bitop3:0x2d\n\t"               \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                         \
    "v_bitop3_b32 %[t2], %[sel], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"              \
    "v_add_u32 %[" #HKN "], %[" #KW "], %[" #X2 "]\n\t"                               \
    "v_add3_u32 %[t1], %[t1], %[t2], %[" #HK "]\n\t"                                  \
    "v_and_b32 %[" #HKN "], %[" #HKN "], %[me]\n\t"                                   \
    "v_add_u32 %[" #X3 "], %[t1], %[dc]\n\t"                                          \
    "v_add_u32_dpp %[" #X3 "], %[t1], %[t1] row_half_mirror row_mask:0xf bank_mask:" BM "\n\t"
// product round (quad_perm pairs) in asm, the compiler's order, four per block
#define PQ_ROUND(X0, X1, X2, X3, HK, HKN, KW, DPPC)                                      \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                         \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                         \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                         \
    "v_bitop3_b32 %[sel], %[" #X0 "], %[" #X1 "], %[m] bitop3:0x2d\n\t"               \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                         \
    "v_bitop3_b32 %[t2], %[sel], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"              \
    "v_add3_u32 %[t1], %[t1], %[t2], %[" #HK "]\n\t"                                  \
    "v_bitop3_b32 %[dc], %[me], %[t1], %[" #X3 "] bitop3:0xca\n\t"                    \
    "v_add_u32 %[" #HKN "], %[" #KW "], %[" #X2 "]\n\t"                               \
    "v_and_b32 %[" #HKN "], %[" #HKN "], %[me]\n\t"                                   \
    "v_add_u32_dpp %[" #X3 "], %[dc], %[t1] " DPPC " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define PQ_OPT(X0, X1, X2, X3, HK, HKN, KW)                                              \
    "v_add_u32 %[" #HKN "], %[" #KW "], %[" #X2 "]\n\t"                               \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                         \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                         \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                         \
    "v_bitop3_b32 %[sel], %[" #X0 "], %[" #X1 "], %[m] bitop3:0x2d\n\t"               \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                         \
    "v_bitop3_b32 %[t2], %[sel], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"              \
    "v_and_b32 %[" #HKN "], %[" #HKN "], %[me]\n\t"                                   \
    "v_add3_u32 %[t1], %[t1], %[t2], %[" #HK "]\n\t"                                  \
    "v_bitop3_b32 %[dc], %[me], %[t1], %[" #X3 "] bitop3:0xca\n\t"                    \
    "s_nop 1\n\t"                                                                     \
    "v_add_u32_dpp %[" #X3 "], %[dc], %[t1] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
// m8: mirror round with the d fetch as a plain move (wrong digests: timing only)
#define MR_NODC(X0, X1, X2, X3, HK, HKN, KW)                                             \
    "v_mov_b32 %[dc], %[" #X3 "]\n\t"                                                 \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                         \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                         \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                         \
    "v_bitop3_b32 %[sel], %[" #X0 "], %[" #X1 "], %[m] bitop3:0x2d\n\t"               \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                         \
    "v_bitop3_b32 %[t2], %[sel], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"              \
    "v_add_u32 %[" #HKN "], %[" #KW "], %[" #X2 "]\n\t"                               \
    "v_add3_u32 %[t1], %[t1], %[t2], %[" #HK "]\n\t"                                  \
    "v_and_b32 %[" #HKN "], %[" #HKN "], %[me]\n\t"                                   \
    "v_add_u32 %[" #X3 "], %[t1], %[dc]\n\t"                                          \
    "v_add_u32_dpp %[" #X3 "], %[t1], %[t1] row_half_mirror row_mask:0xf bank_mask:0xa\n\t"
// m9-m11: the compiler's exact form of the product round (Z into x3's
// register, DPP add with dst = src0, lane mask by v_cndmask on an SGPR pair)
// and its two differences from m4 one at a time
#define PQ_GEN(X0, X1, X2, X3, HK, HKN, KW, ZREG, MASKOP)                                \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                         \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                         \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                         \
    "v_bitop3_b32 %[sel], %[" #X0 "], %[" #X1 "], %[m] bitop3:0x2d\n\t"               \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                         \
    "v_bitop3_b32 %[t2], %[sel], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"              \
    "v_add3_u32 %[t1], %[t1], %[t2], %[" #HK "]\n\t"                                  \
    "v_bitop3_b32 %[" ZREG "], %[me], %[t1], %[" #X3 "] bitop3:0xca\n\t"              \
    "v_add_u32 %[" #HKN "], %[" #KW "], %[" #X2 "]\n\t"                               \
    MASKOP(HKN)                                                                         \
    "v_add_u32_dpp %[" #X3 "], %[" ZREG "], %[t1] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define MASK_CND(HKN) "v_cndmask_b32_e64 %[" #HKN "], 0, %[" #HKN "], %[msk]\n\t"
#define MASK_AND(HKN) "v_and_b32 %[" #HKN "], %[" #HKN "], %[me]\n\t"
#define PQ_C9(X0, X1, X2, X3, HK, HKN, KW) PQ_GEN(X0, X1, X2, X3, HK, HKN, KW, #X3, MASK_CND)
#define PQ_C10(X0, X1, X2, X3, HK, HKN, KW) PQ_GEN(X0, X1, X2, X3, HK, HKN, KW, #X3, MASK_AND)
#define PQ_C11(X0, X1, X2, X3, HK, HKN, KW) PQ_GEN(X0, X1, X2, X3, HK, HKN, KW, "dc", MASK_CND)
#define MR_4(KA, KB, KC, KD) MR_4X(KA, KB, KC, KD, MR_ROUND)
#define MR_4X(KA, KB, KC, KD, RND)                                                                     \
    {                                                                                            \
        uint32_t hb_, t1_, t2_, t3_, sel_, dc_, dm_;                                             \
        asm volatile(RND(a, b, c, d, ha, hb, k0) RND(d, a, b, c, hb, ha, k1)                     \
                     RND(c, d, a, b, ha, hb, k2) RND(b, c, d, a, hb, ha, k3)                     \
                     : [a] "+v"(x0), [b] "+v"(x1), [c] "+v"(x2), [d] "+v"(x3), [ha] "+v"(hk),   \
                       [hb] "=&v"(hb_), [t1] "=&v"(t1_), [t2] "=&v"(t2_), [t3] "=&v"(t3_),       \
                       [sel] "=&v"(sel_), [dc] "=&v"(dc_), [dm] "=&v"(dm_)                       \
                     : [k0] "s"(KA), [k1] "s"(KB), [k2] "s"(KC), [k3] "s"(KD), [msk] "s"(msk64), [r1] "v"(R.r1),  \
                       [r2] "v"(R.r2), [r3] "v"(R.r3), [m] "v"(R.m), [me] "v"(R.me));           \
    }

#define MR_FULLW(X0, X1, X2, X3, HK, HKN, KW) MR_ROUND_B(X0, X1, X2, X3, HK, HKN, KW, "0xf")
#define PQ_QUAD(X0, X1, X2, X3, HK, HKN, KW) PQ_ROUND(X0, X1, X2, X3, HK, HKN, KW, "quad_perm:[1,0,3,2]")
#define PQ_XDPP(X0, X1, X2, X3, HK, HKN, KW) "v_mov_b32_dpp %[dm], %[" #X3 "] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t" PQ_QUAD(X0, X1, X2, X3, HK, HKN, KW)
#define PQ_MIRR(X0, X1, X2, X3, HK, HKN, KW) PQ_ROUND(X0, X1, X2, X3, HK, HKN, KW, "row_half_mirror")
template <int V>
__device__ __forceinline__ void compress_kw_asm4(uint32_t st[4], const uint32_t* kw, const shaq::Role& R) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    uint32_t hk = (x3 + kw[0]) & R.me;
    const uint64_t msk64 = __ballot(R.me != 0u);
    asm volatile("s_nop 1" ::: "memory");
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
        uint32_t k[16];
#pragma unroll
        for (int i = 0; i < 15; i++) k[i] = kw[16 * r + i + 1];
        k[15] = r < 3 ? kw[16 * r + 16] : 0u;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            if (V == 0) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], MR_FULLW);
            if (V == 1) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_QUAD);
            if (V == 2) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_MIRR);
            if (V == 3) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_XDPP);
            if (V == 4) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_OPT);
            if (V == 5) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], MR_NODC);
            if (V == 6) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_C9);
            if (V == 7) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_C10);
            if (V == 8) MR_4X(k[4 * g], k[4 * g + 1], k[4 * g + 2], k[4 * g + 3], PQ_C11);
        }
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}

__device__ __forceinline__ void compress_kw_mirror4(uint32_t st[4], const uint32_t* kw, const shaq::Role& R) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    uint32_t hk = (x3 + kw[0]) & R.me;
    const uint64_t msk64 = 0;
    asm volatile("s_nop 1" ::: "memory");         // x3 may have just been written: DPP read hazard
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
        uint32_t k[16];
#pragma unroll
        for (int i = 0; i < 15; i++) k[i] = kw[16 * r + i + 1];
        k[15] = r < 3 ? kw[16 * r + 16] : 0u;
        MR_4(k[0], k[1], k[2], k[3]);
        MR_4(k[4], k[5], k[6], k[7]);
        MR_4(k[8], k[9], k[10], k[11]);
        MR_4(k[12], k[13], k[14], k[15]);
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}

__device__ __forceinline__ uint32_t pair_of(uint32_t lane, int mode) {
    if (mode == 0 || mode == 4 || mode == 6 || mode == 7 || mode >= 9) return lane >> 1;
    const uint32_t j = lane & 7u;
    return 4u * (lane >> 3) + (j < 4 ? j : 7u - j);
}
__device__ __forceinline__ bool is_e(uint32_t lane, int mode) { return (mode == 0 || mode == 4 || mode == 6 || mode == 7 || mode >= 9) ? (lane & 1u) == 0 : (lane & 7u) < 4; }

__global__ __launch_bounds__(64) void k_round(const uint32_t* in, uint32_t* out, unsigned long long* clk, int mode) {
    const uint32_t lane = threadIdx.x;
    const uint32_t p = pair_of(lane, mode);
    const bool e = is_e(lane, mode);
    const shaq::Role R = shaq::role_of(e ? 0u : 1u);
    uint32_t st[4];
    for (int k = 0; k < 4; k++) st[k] = in[8 * p + (e ? 4 : 0) + k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int b = 0; b < NB; b++) {
        if (mode == 0) shaq::compress_kw(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 1) compress_kw_mirror(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 2) compress_kw_mirror4(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 3) compress_kw_asm4<0>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 4) compress_kw_asm4<1>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 5) compress_kw_asm4<2>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 6) compress_kw_asm4<3>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 7) compress_kw_asm4<4>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 8) compress_kw_asm4<5>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 9) compress_kw_asm4<6>(st, shaf::PAD_KW_C.kw, R);
        else if (mode == 10) compress_kw_asm4<7>(st, shaf::PAD_KW_C.kw, R);
        else compress_kw_asm4<8>(st, shaf::PAD_KW_C.kw, R);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < 4; k++) out[8 * p + (e ? 4 : 0) + k] = st[k];
    if (lane == 0) *clk = c1 - c0;
}

int main() {
    uint32_t h_in[32 * 8];
    for (int i = 0; i < 32 * 8; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 9);
    uint32_t *d_in, *d_out;
    unsigned long long* d_clk;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    CK(hipMalloc(&d_out, sizeof(h_in)));
    CK(hipMalloc(&d_clk, 8));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    uint32_t ref[32 * 8];
    const char* names[12] = {"product round (quad_perm pairs, compiler order)", "mirror pairs, asm order, no select",
                            "mirror pairs, four rounds per asm block",
                            "as 2, A-lane add writes all lanes (timing only)",
                            "product round in asm, four per block",
                            "product round in asm, row_half_mirror DPP (timing only)",
                            "product round in asm + one unused DPP mov per round",
                            "product round in asm, stall slots filled, s_nop 1",
                            "as 2, d fetched by a plain move (timing only)",
                            "compiler's exact round form in asm (Z in x3, cndmask)",
                            "as 9 with v_and for the lane mask",
                            "as 9 with Z in a separate register"};
    for (int mode = 0; mode < 12; mode++) {
        double best = 1e30, sum = 0;
        bool same = true;
        for (int rep = 0; rep < 10; rep++) {
            hipLaunchKernelGGL(k_round, dim3(1), dim3(64), 0, 0, d_in, d_out, d_clk, mode);
            CK(hipDeviceSynchronize());
            unsigned long long c;
            uint32_t o[32 * 8];
            CK(hipMemcpy(&c, d_clk, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost));
            if (mode == 0 && rep == 0) memcpy(ref, o, sizeof(o));
            same = same && memcmp(ref, o, sizeof(o)) == 0;
            const double per_round = (double)c / (NB * 64.0);
            if (rep > 0) { sum += per_round; best = per_round < best ? per_round : best; }
        }
        printf("mode %d: %-52s cycles/round mean %.2f best %.2f  digests equal to mode 0: %s\n", mode, names[mode],
               sum / 9, best, same ? "yes" : "NO");
    }
    return 0;
}
