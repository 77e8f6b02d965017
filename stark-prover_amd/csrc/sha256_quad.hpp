// sha256_quad.hpp — SHA-256 Merkle node for the latency-bound tree levels,
// one node per PAIR of lanes (gfx950, device only).
//
// A lone wave issues about one VALU instruction per 4-5 cycles while a
// dependent instruction waits ~8, so a node hash on the
// serial tree top is bound by its instruction COUNT.  A SHA-256 round has
// two halves: the e-path (Sigma1, Ch, T1, e' = d + T1) and the a-path
// (Sigma0, Maj, a' = T1 + T2).  Here the even lane of a pair runs the e-path
// and the odd lane the a-path with the SAME instructions (per-lane rotation
// amounts and masks).  One DPP quad_perm add per round swaps the halves'
// results:
//     E: V = Sigma1(e) + Ch(e,f,g) + h + K + W = T1      exports T1
//     A: V = Sigma0(a) + Maj(a,b,c)            = T2      exports d
//     E: e' = V + d (from A)      A: a' = V + T1 (from E)
// 11 instructions per round instead of 14.  The shift registers (e,f,g,h)
// and (a,b,c,d) never move between lanes, so the chaining value and the
// digest stay split: E holds words 4..7, A holds words 0..3.
//
// The message schedule is split the same way: E computes sigma1(W[t-2]),
// A computes sigma0(W[t-15]) (per-lane operand select, rotation and shift
// amounts) and the two halves meet through one more DPP add: 7 instructions
// per word instead of 10.  Both lanes keep the whole schedule.
//
// Measured (stark-prover_amd/bench/quad_micro.hip, one wave, dependent
// chain): 9.0 K cycles per node against 9.9 K for the compact per-lane node;
// used for the tree levels of <= 64 nodes in k_tree_top and k_tree_mid
// (5.19 -> 5.02 ms per 2^24 commit, tools/abn.sh).  The DPP add must carry
// bound_ctrl so the compiler fuses it (v_add_u32_dpp) instead of emitting a
// separate v_mov_b32_dpp.
#pragma once
#include <stdint.h>
#include "sha256_fast.hpp"

namespace fri {
namespace shaq {

// quad_perm [1,0,3,2]: lane 2k <-> lane 2k+1
constexpr int SWAP01 = 1 | (0 << 2) | (3 << 4) | (2 << 6);

__device__ __forceinline__ uint32_t swap01(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, SWAP01, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t rot(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
#define bop(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))

// Per-lane role constants of a pair.
struct Role {
    uint32_t r1, r2, r3;    // round rotations: E 6,11,25 (Sigma1)  A 2,13,22 (Sigma0)
    uint32_t m;             // sel mask:  E 0 (sel = ~e -> Ch)     A ~0 (sel = a^b -> Maj)
    uint32_t me;            // ~0 on E only
    uint32_t q1, q2, q3;    // schedule: E sigma1 (17,19,>>10), A sigma0 (7,18,>>3)
    uint32_t is_a;          // ~0 on A only (schedule operand select)
    uint32_t iv[4];         // initial chaining words of this lane's half
};

__device__ __forceinline__ Role role_of(uint32_t lane) {
    Role r{};
    const uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                            0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    if ((lane & 1u) == 0) {
        r.r1 = 6; r.r2 = 11; r.r3 = 25; r.m = 0u; r.me = ~0u;
        r.q1 = 17; r.q2 = 19; r.q3 = 10; r.is_a = 0u;
        for (int i = 0; i < 4; i++) r.iv[i] = IV[4 + i];
    } else {
        r.r1 = 2; r.r2 = 13; r.r3 = 22; r.m = ~0u; r.me = 0u;
        r.q1 = 7; r.q2 = 18; r.q3 = 3; r.is_a = ~0u;
        for (int i = 0; i < 4; i++) r.iv[i] = IV[i];
    }
    return r;
}

// One round on this lane's half (x0..x3 = e,f,g,h on E; a,b,c,d on A).
#define SHAQ_R(kw)                                                                   \
    {                                                                                \
        const uint32_t _S = bop(rot(x0, R.r1), rot(x0, R.r2), rot(x0, R.r3), 0x96);  \
        const uint32_t _sel = bop(x0, x1, R.m, 0x2D);   /* x0 ^ (x1 & m) ^ ~m */     \
        const uint32_t _F = bop(_sel, x2, x1, 0xCA);    /* sel ? x2 : x1 */          \
        const uint32_t _hk = (x3 + (kw)) & R.me;                                     \
        const uint32_t _V = _S + _F + _hk;                                           \
        const uint32_t _Z = bop(R.me, _V, x3, 0xCA);    /* E: T1, A: d */            \
        const uint32_t _n = _V + swap01(_Z);                                         \
        x3 = x2; x2 = x1; x1 = x0; x0 = _n;                                          \
    }

// Split schedule word: w[i] (= W[t-16]) <- W[t]
#define SHAQ_W(i)                                                                            \
    {                                                                                        \
        const uint32_t _x = bop(R.is_a, w[((i) + 1) & 15], w[((i) + 14) & 15], 0xCA);        \
        const uint32_t _s = bop(rot(_x, R.q1), rot(_x, R.q2), _x >> R.q3, 0x96);             \
        w[i] = w[i] + w[((i) + 9) & 15] + _s + swap01(_s);                                   \
    }

// Block on a register message w[16] (consumed), looped 16 rounds at a time.
__device__ __forceinline__ void compress(uint32_t st[4], uint32_t w[16], const Role& R) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
#pragma unroll
    for (int i = 0; i < 16; i++) SHAQ_R(w[i] + shaf::KTAB[i]);
#pragma unroll 1
    for (int r = 1; r < 4; r++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            SHAQ_W(i);
            SHAQ_R(w[i] + shaf::KTAB[16 * r + i]);
        }
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}
// Block with a constant K+W table (the padding block of a 64-byte message).
__device__ __forceinline__ void compress_kw(uint32_t st[4], const uint32_t* kw, const Role& R) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int i = 0; i < 16; i++) SHAQ_R(kw[16 * r + i]);
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}
// ---- schedule producer (stark-prover_amd/bench/sched_micro.hip)
// The first block's message schedule W16..W63 depends only on the message,
// not on the round state, so a second wave of the workgroup, on another
// SIMD, expands it (with the round constants: W[t] + K[t]) into LDS while the
// round wave runs rounds 0..15 on the message words; the round wave reads it
// 4 words at a time after one flag check per 16-word block.  The round wave
// issues 48 x 7 fewer instructions per node: 8.51 -> 7.51 K cycles per
// dependent node in the micro (profiles/r05_sched_micro.txt).  A producer on
// the round wave's own SIMD is slower than none (9.09 K): the two waves then
// share one issue port.
//
// Producer: the node's schedule into wk[0..47] (48 words, 16-byte aligned),
// flag = base + b + 1 once block b's 16 words are stored.  Both lanes of a
// pair run (the split schedule needs the pair); `store` on one lane of it.
__device__ __forceinline__ void produce(uint32_t w[16], uint32_t* wk, uint32_t* flag, uint32_t base, bool store,
                                        bool flag_lane, const Role& R) {
#pragma unroll 1
    for (int b = 0; b < 3; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) SHAQ_W(i);
        if (store) {
            uint4* o = reinterpret_cast<uint4*>(wk + 16 * b);
#pragma unroll
            for (int j = 0; j < 4; j++)
                o[j] = make_uint4(w[4 * j] + shaf::KTAB[16 * (b + 1) + 4 * j],
                                  w[4 * j + 1] + shaf::KTAB[16 * (b + 1) + 4 * j + 1],
                                  w[4 * j + 2] + shaf::KTAB[16 * (b + 1) + 4 * j + 2],
                                  w[4 * j + 3] + shaf::KTAB[16 * (b + 1) + 4 * j + 3]);
        }
        // (release: the wave's schedule stores are complete before the flag)
        if (flag_lane) __hip_atomic_store(flag, base + b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// Round wave: one block on a register message w[0..15] (rounds 0..15) whose
// rounds 16..63 are fed from wk (W + K, written by produce); st += result.
__device__ __forceinline__ void compress_ext(uint32_t st[4], const uint32_t w[16], const Role& R, const uint32_t* wk,
                                             const uint32_t* flag, uint32_t base) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
#pragma unroll
    for (int i = 0; i < 16; i++) SHAQ_R(w[i] + shaf::KTAB[i]);
#pragma unroll 1
    for (int b = 0; b < 3; b++) {
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < base + b + 1) {}
        const uint4* q = reinterpret_cast<const uint4*>(wk + 16 * b);
        const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        SHAQ_R(q0.x); SHAQ_R(q0.y); SHAQ_R(q0.z); SHAQ_R(q0.w);
        SHAQ_R(q1.x); SHAQ_R(q1.y); SHAQ_R(q1.z); SHAQ_R(q1.w);
        SHAQ_R(q2.x); SHAQ_R(q2.y); SHAQ_R(q2.z); SHAQ_R(q2.w);
        SHAQ_R(q3.x); SHAQ_R(q3.y); SHAQ_R(q3.z); SHAQ_R(q3.w);
    }
    st[0] += x0; st[1] += x1; st[2] += x2; st[3] += x3;
}

// Round wave: node SHA256(l || r) with the first block's rounds 16..63 fed
// from wk (W + K, written by produce), then the padding block.  Same digest
// halves as node().
__device__ __forceinline__ void node_ext(const uint32_t l[8], const uint32_t r[8], uint32_t out[4], const Role& R,
                                         const uint32_t* wk, const uint32_t* flag, uint32_t base) {
    uint32_t x0 = R.iv[0], x1 = R.iv[1], x2 = R.iv[2], x3 = R.iv[3];
#pragma unroll
    for (int i = 0; i < 8; i++) SHAQ_R(l[i] + shaf::KTAB[i]);
#pragma unroll
    for (int i = 0; i < 8; i++) SHAQ_R(r[i] + shaf::KTAB[8 + i]);
#pragma unroll 1
    for (int b = 0; b < 3; b++) {
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < base + b + 1) {}
        const uint4* q = reinterpret_cast<const uint4*>(wk + 16 * b);
        const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        SHAQ_R(q0.x); SHAQ_R(q0.y); SHAQ_R(q0.z); SHAQ_R(q0.w);
        SHAQ_R(q1.x); SHAQ_R(q1.y); SHAQ_R(q1.z); SHAQ_R(q1.w);
        SHAQ_R(q2.x); SHAQ_R(q2.y); SHAQ_R(q2.z); SHAQ_R(q2.w);
        SHAQ_R(q3.x); SHAQ_R(q3.y); SHAQ_R(q3.z); SHAQ_R(q3.w);
    }
    out[0] = R.iv[0] + x0; out[1] = R.iv[1] + x1; out[2] = R.iv[2] + x2; out[3] = R.iv[3] + x3;
    compress_kw(out, shaf::PAD_KW_C.kw, R);
}

#undef SHAQ_R
#undef SHAQ_W
#undef bop

// Node hash SHA256(l || r): both lanes of the pair pass the same 16
// message words; out = this lane's half of the digest (even lane: words
// 4..7, odd lane: words 0..3).
__device__ __forceinline__ void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[4], const Role& R) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
#pragma unroll
    for (int i = 0; i < 4; i++) out[i] = R.iv[i];
    compress(out, w, R);
    compress_kw(out, shaf::PAD_KW_C.kw, R);
}

}  // namespace shaq
}  // namespace fri
