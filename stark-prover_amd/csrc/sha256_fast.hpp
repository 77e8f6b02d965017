// sha256_fast.hpp — gfx950 SHA-256 rounds written for the v_bitop3_b32 /
// v_alignbit_b32 / v_add3_u32 instruction set (device only).
//
// Per round: Sigma1, Sigma0 = 3 alignbit + 1 bitop3(0x96 = xor3) each;
// Ch = bitop3(0xCA); Maj = bitop3(0xE8); T1 = add3(h + K + W, Sigma1, Ch);
// a' = add3(T1, Sigma0, Maj); e' = d + T1  ->  14 VALU ops.
// Message schedule per word: sigma0/sigma1 = 2 alignbit + shift + bitop3,
// w = add3(w16, s0, w7) + s1  ->  10 VALU ops.
// The padding block of a 64-byte message (internal Merkle node) has a
// constant schedule: K[t] + W[t] folds into one literal per round.
#pragma once
#include <stdint.h>
#include "sha256.hpp"

namespace fri {
namespace shaf {

// Constant operands (schedule words of the constant message parts) must
// still fold at compile time, so the builtin is used only on live values.
#define SHAF_CONST3(a, b, c) (__builtin_constant_p(a) && __builtin_constant_p(b) && __builtin_constant_p(c))
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    if (SHAF_CONST3(a, b, c)) return a ^ b ^ c;
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t chf(uint32_t e, uint32_t f, uint32_t g) {
    if (SHAF_CONST3(e, f, g)) return (e & f) ^ (~e & g);
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);      // e ? f : g
}
__device__ __forceinline__ uint32_t majf(uint32_t a, uint32_t b, uint32_t c) {
    if (SHAF_CONST3(a, b, c)) return (a & b) ^ (a & c) ^ (b & c);
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);      // majority
}
__device__ __forceinline__ uint32_t ror(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t S0(uint32_t a) { return xor3(ror(a, 2), ror(a, 13), ror(a, 22)); }
__device__ __forceinline__ uint32_t S1(uint32_t e) { return xor3(ror(e, 6), ror(e, 11), ror(e, 25)); }
__device__ __forceinline__ uint32_t s0(uint32_t x) { return xor3(ror(x, 7), ror(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t s1(uint32_t x) { return xor3(ror(x, 17), ror(x, 19), x >> 10); }

// Host/compile-time schedule of the constant padding block of a 64-byte
// message: W0 = 0x80000000, W15 = 512, others 0;  KWPAD[t] = K[t] + W[t].
struct PadKW {
    uint32_t kw[64];
    constexpr PadKW(uint32_t bits = 512u) : kw() {
        uint32_t w[64] = {};
        w[0] = 0x80000000u;
        w[15] = bits;
        for (int t = 16; t < 64; t++) {
            uint32_t x = w[t - 15], y = w[t - 2];
            uint32_t a = ((x >> 7) | (x << 25)) ^ ((x >> 18) | (x << 14)) ^ (x >> 3);
            uint32_t b = ((y >> 17) | (y << 15)) ^ ((y >> 19) | (y << 13)) ^ (y >> 10);
            w[t] = w[t - 16] + a + w[t - 7] + b;
        }
        constexpr uint32_t k[64] = {
            0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
            0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
            0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
            0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
            0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
            0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
            0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
            0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
        for (int t = 0; t < 64; t++) kw[t] = k[t] + w[t];
    }
};
constexpr PadKW PAD_KW{};
// Padding-only final blocks of 128- and 192-byte messages (channel sends).
// (plain __constant__, not constexpr: one symbol per table, read by scalar
// loads, so a scalar-cache touch at kernel start covers every later use)
__constant__ PadKW PAD_KW_1024{1024u};
__constant__ PadKW PAD_KW_1536{1536u};

// Rounds on a register-resident schedule w[16] (consumed).  Variables are
// rotated by renaming through the 8-way unrolled macro.
__device__ __forceinline__ void rounds_var(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int tt = t + u;
            uint32_t wt;
            if (tt < 16) {
                wt = w[tt];
            } else {
                wt = w[tt & 15] + s0(w[(tt - 15) & 15]) + w[(tt - 7) & 15] + s1(w[(tt - 2) & 15]);
                w[tt & 15] = wt;
            }
            const uint32_t kw = sha::K(tt) + wt;
            uint32_t t1 = h + kw + S1(e) + chf(e, f, g);
            uint32_t t2 = S0(a) + majf(a, b, c);
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Rounds on the constant padding block (64-byte message second block).
__device__ __forceinline__ void rounds_pad64(uint32_t st[8]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t t1 = h + PAD_KW.kw[t] + S1(e) + chf(e, f, g);
        uint32_t t2 = S0(a) + majf(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ---- compact forms for latency-bound code (executed once per launch, so
// I-cache footprint matters more than the last few percent of issue rate):
// 16 rounds unrolled, looped 4x; K and padding schedules via scalar loads.
__constant__ uint32_t KTAB[64] = {
    0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
    0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
    0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
    0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
    0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
    0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
    0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
    0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
__constant__ PadKW PAD_KW_C{};

#define SHAF_R(kwv)                                                            \
    {                                                                          \
        uint32_t _t1 = h + (kwv) + S1(e) + chf(e, f, g);                        \
        uint32_t _t2 = S0(a) + majf(a, b, c);                                  \
        h = g; g = f; f = e; e = d + _t1; d = c; c = b; b = a; a = _t1 + _t2;   \
    }

__device__ __forceinline__ void compress_loop(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 16; i++) SHAF_R(w[i] + KTAB[i]);
#pragma unroll 1
    for (int r = 1; r < 4; r++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w[i] = w[i] + s0(w[(i + 1) & 15]) + w[(i + 9) & 15] + s1(w[(i + 14) & 15]);
            SHAF_R(w[i] + KTAB[16 * r + i]);
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Rounds with a K+W table in constant memory, looped.
__device__ __forceinline__ void kwtab_loop(uint32_t st[8], const uint32_t* kw) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int i = 0; i < 16; i++) SHAF_R(kw[16 * r + i]);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
#undef SHAF_R

__device__ __forceinline__ void node_compact(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    sha::init(out);
    compress_loop(out, w);
    kwtab_loop(out, PAD_KW_C.kw);
}
__device__ __forceinline__ void leaf_compact(uint32_t v, uint32_t out[8]) {
    uint32_t w[16] = {0u, v, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 64u};
    sha::init(out);
    compress_loop(out, w);
}

// ---- rate-ordered rounds for the throughput-bound leaf kernels.
// A SIMD issues the half-rate ops (v_alignbit, v_add3) and the full-rate ones
// (v_bitop3, v_add) faster when each kind comes in a run than when the
// compiler interleaves them: one asm block per round issues the six
// rotations and the h+K+W sum first, then the four v_bitop3, then the adds
// (bench/order_micro.hip: +4-5% node hashes/s at the same instruction
// count).  Inside k_layer_leaf the dual-issued quad-cycles rise from 5.2% to
// 8.2% and busy cycles fall 2.5% (PMC), but the launch is only 0.5-1%
// shorter: the chip lowers its clock (2.09 GHz) as the issue stream packs
// closer (MI355X DVFS give-back).  It also needs 60 VGPRs instead of 92.
// The round variables still rotate by renaming: a round updates d (-> new
// e) and h (-> new a) in place.  K (+ a constant W) is an SGPR.
// Operand names are x*/y*/r* so the macro parameters a..h do not rename them.
#define SHAF_RND_W(a, b, c, d, e, f, g, h, W, K)                                                       \
    {                                                                                                  \
        uint32_t _r1, _r2, _r3, _r4, _r5, _r6;                                                         \
        asm volatile("v_alignbit_b32 %[r1], %[xe], %[xe], 6\n\t"                                       \
                     "v_alignbit_b32 %[r2], %[xe], %[xe], 11\n\t"                                      \
                     "v_alignbit_b32 %[r3], %[xe], %[xe], 25\n\t"                                      \
                     "v_alignbit_b32 %[r4], %[xa], %[xa], 2\n\t"                                       \
                     "v_alignbit_b32 %[r5], %[xa], %[xa], 13\n\t"                                      \
                     "v_alignbit_b32 %[r6], %[xa], %[xa], 22\n\t"                                      \
                     "v_add3_u32 %[xh], %[xh], %[xw], %[xk]\n\t"                                       \
                     "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                         \
                     "v_bitop3_b32 %[r4], %[r4], %[r5], %[r6] bitop3:0x96\n\t"                         \
                     "v_bitop3_b32 %[r2], %[xe], %[xf], %[xg] bitop3:0xca\n\t"                         \
                     "v_bitop3_b32 %[r5], %[xa], %[xb], %[xc] bitop3:0xe8\n\t"                         \
                     "v_add3_u32 %[xh], %[xh], %[r1], %[r2]\n\t"                                       \
                     "v_add_u32 %[xd], %[xd], %[xh]\n\t"                                               \
                     "v_add3_u32 %[xh], %[xh], %[r4], %[r5]"                                           \
                     : [xd] "+v"(d), [xh] "+v"(h), [r1] "=&v"(_r1), [r2] "=&v"(_r2), [r3] "=&v"(_r3),  \
                       [r4] "=&v"(_r4), [r5] "=&v"(_r5), [r6] "=&v"(_r6)                               \
                     : [xa] "v"(a), [xb] "v"(b), [xc] "v"(c), [xe] "v"(e), [xf] "v"(f), [xg] "v"(g),   \
                       [xw] "v"(W), [xk] "s"(K));                                                      \
    }
// Same with a constant message word folded into K (h + KW is a full-rate add
// issued with the v_bitop3 run).
#define SHAF_RND_K(a, b, c, d, e, f, g, h, K)                                                          \
    {                                                                                                  \
        uint32_t _r1, _r2, _r3, _r4, _r5, _r6;                                                         \
        asm volatile("v_alignbit_b32 %[r1], %[xe], %[xe], 6\n\t"                                       \
                     "v_alignbit_b32 %[r2], %[xe], %[xe], 11\n\t"                                      \
                     "v_alignbit_b32 %[r3], %[xe], %[xe], 25\n\t"                                      \
                     "v_alignbit_b32 %[r4], %[xa], %[xa], 2\n\t"                                       \
                     "v_alignbit_b32 %[r5], %[xa], %[xa], 13\n\t"                                      \
                     "v_alignbit_b32 %[r6], %[xa], %[xa], 22\n\t"                                      \
                     "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                         \
                     "v_bitop3_b32 %[r4], %[r4], %[r5], %[r6] bitop3:0x96\n\t"                         \
                     "v_bitop3_b32 %[r2], %[xe], %[xf], %[xg] bitop3:0xca\n\t"                         \
                     "v_bitop3_b32 %[r5], %[xa], %[xb], %[xc] bitop3:0xe8\n\t"                         \
                     "v_add_u32 %[xh], %[xk], %[xh]\n\t"                                               \
                     "v_add3_u32 %[xh], %[xh], %[r1], %[r2]\n\t"                                       \
                     "v_add_u32 %[xd], %[xd], %[xh]\n\t"                                               \
                     "v_add3_u32 %[xh], %[xh], %[r4], %[r5]"                                           \
                     : [xd] "+v"(d), [xh] "+v"(h), [r1] "=&v"(_r1), [r2] "=&v"(_r2), [r3] "=&v"(_r3),  \
                       [r4] "=&v"(_r4), [r5] "=&v"(_r5), [r6] "=&v"(_r6)                               \
                     : [xa] "v"(a), [xb] "v"(b), [xc] "v"(c), [xe] "v"(e), [xf] "v"(f), [xg] "v"(g),   \
                       [xk] "s"(K));                                                                   \
    }
// Plain C round in the same renaming convention (folds when the state is a
// compile-time constant, e.g. the first rounds after the IV).
#define SHAF_RND_C(a, b, c, d, e, f, g, h, KW)                                                         \
    {                                                                                                  \
        const uint32_t _t1 = h + (KW) + S1(e) + chf(e, f, g);                                          \
        d += _t1;                                                                                      \
        h = _t1 + S0(a) + majf(a, b, c);                                                               \
    }
// Round t of a block with the working variables renamed by t mod 8.
#define SHAF_ROUND8(MAC, u, ...)                                                                       \
    switch (u) {                                                                                       \
        case 0: MAC(a, b, c, d, e, f, g, h, __VA_ARGS__); break;                                       \
        case 1: MAC(h, a, b, c, d, e, f, g, __VA_ARGS__); break;                                       \
        case 2: MAC(g, h, a, b, c, d, e, f, __VA_ARGS__); break;                                       \
        case 3: MAC(f, g, h, a, b, c, d, e, __VA_ARGS__); break;                                       \
        case 4: MAC(e, f, g, h, a, b, c, d, __VA_ARGS__); break;                                       \
        case 5: MAC(d, e, f, g, h, a, b, c, __VA_ARGS__); break;                                       \
        case 6: MAC(c, d, e, f, g, h, a, b, __VA_ARGS__); break;                                       \
        case 7: MAC(b, c, d, e, f, g, h, a, __VA_ARGS__); break;                                       \
    }
// Schedule word w16 <- w16 + s0(w15) + w7 + s1(w2): rotations, then the
// shifts, w16 + w7 and the XORs (full rate), then the final add3.
#define SHAF_SCH(w16, w15, w7, w2)                                                                     \
    {                                                                                                  \
        uint32_t _x1, _x2, _x3, _y1, _y2, _y3;                                                         \
        asm volatile("v_alignbit_b32 %[x1], %[yp], %[yp], 7\n\t"                                       \
                     "v_alignbit_b32 %[x2], %[yp], %[yp], 18\n\t"                                      \
                     "v_alignbit_b32 %[y1], %[yq], %[yq], 17\n\t"                                      \
                     "v_alignbit_b32 %[y2], %[yq], %[yq], 19\n\t"                                      \
                     "v_lshrrev_b32 %[x3], 3, %[yp]\n\t"                                               \
                     "v_lshrrev_b32 %[y3], 10, %[yq]\n\t"                                              \
                     "v_add_u32 %[yw], %[yw], %[ys]\n\t"                                               \
                     "v_bitop3_b32 %[x1], %[x1], %[x2], %[x3] bitop3:0x96\n\t"                         \
                     "v_bitop3_b32 %[y1], %[y1], %[y2], %[y3] bitop3:0x96\n\t"                         \
                     "v_add3_u32 %[yw], %[yw], %[x1], %[y1]"                                           \
                     : [yw] "+v"(w16), [x1] "=&v"(_x1), [x2] "=&v"(_x2), [x3] "=&v"(_x3),              \
                       [y1] "=&v"(_y1), [y2] "=&v"(_y2), [y3] "=&v"(_y3)                               \
                     : [yp] "v"(w15), [yq] "v"(w2), [ys] "v"(w7));                                     \
    }

// Rate-ordered compression of a register-resident block w[16] (consumed).
// Rounds [0, c_rounds) stay in C so a constant state (IV) folds.
template <int c_rounds>
__device__ __forceinline__ void rounds_var_ord(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int tt = t + u;
            if (tt >= 16) SHAF_SCH(w[tt & 15], w[(tt - 15) & 15], w[(tt - 7) & 15], w[(tt - 2) & 15]);
            if (tt < c_rounds) {
                SHAF_ROUND8(SHAF_RND_C, u, sha::K(tt) + w[tt])
            } else {
                SHAF_ROUND8(SHAF_RND_W, u, w[tt & 15], sha::K(tt))
            }
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
__device__ __forceinline__ void rounds_pad64_ord(uint32_t st[8]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) SHAF_ROUND8(SHAF_RND_K, u, PAD_KW.kw[t + u])
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
// Leaf block (W0 = 0, W1 = v, W2 = 0x80000000, W15 = 64): rounds 0-1 fold
// in C; rounds 2-15 have constant words (K + W in one SGPR); the schedule
// stays in C so its v-independent parts (most of w16..w30) fold.
__device__ __forceinline__ void leaf_ord(uint32_t v, uint32_t out[8]) {
    uint32_t w[16] = {0u, v, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 64u};
    sha::init(out);
    uint32_t a = out[0], b = out[1], c = out[2], d = out[3], e = out[4], f = out[5], g = out[6], h = out[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int tt = t + u;
            if (tt < 2) {
                SHAF_ROUND8(SHAF_RND_C, u, sha::K(tt) + w[tt])
            } else if (tt < 16) {
                SHAF_ROUND8(SHAF_RND_K, u, sha::K(tt) + w[tt])
            } else {
                const uint32_t wt = w[tt & 15] + s0(w[(tt - 15) & 15]) + w[(tt - 7) & 15] + s1(w[(tt - 2) & 15]);
                w[tt & 15] = wt;
                SHAF_ROUND8(SHAF_RND_W, u, wt, sha::K(tt))
            }
        }
    }
    out[0] += a; out[1] += b; out[2] += c; out[3] += d; out[4] += e; out[5] += f; out[6] += g; out[7] += h;
}

#ifndef FRI_SHA_ORDERED
#define FRI_SHA_ORDERED 1
#endif

// Leaf: SHA256 of the 8-byte big-endian encoding of a u32 value.
// Message words: W0 = 0, W1 = v, W2 = 0x80000000, W3..14 = 0, W15 = 64.
// Round 0 (W0 = 0) is a compile-time constant after IV; the schedule words
// that do not depend on v fold into literals.
__device__ __forceinline__ void leaf(uint32_t v, uint32_t out[8]) {
#if FRI_SHA_ORDERED
    leaf_ord(v, out);
#else
    uint32_t w[16] = {0u, v, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 64u};
    sha::init(out);
    rounds_var(out, w);
#endif
}

// Internal node: SHA256(l || r) = two compressions, second on the constant pad.
__device__ __forceinline__ void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    sha::init(out);
#if FRI_SHA_ORDERED
    rounds_var_ord<1>(out, w);
    rounds_pad64_ord(out);
#else
    rounds_var(out, w);
    rounds_pad64(out);
#endif
}

}  // namespace shaf
}  // namespace fri
