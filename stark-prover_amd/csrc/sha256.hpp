// sha256.hpp — SHA-256 compression for gfx950 (and host), FIPS 180-4.
//
// Replaces the SHA-256 behind the reference's Merkle tree (rs_merkle 1.4.2 ->
// sha2 0.10.8, src/merkle/mod.rs:2,15,19) and channel (sha256 1.5.0,
// src/channel/channel.rs:39,76).  Digests are kept as the eight state words
// H0..H7 (native u32): the digest's byte string is their big-endian
// encoding, so a parent's message block is exactly left.H0..7 || right.H0..7
// and the tree never byte-swaps.
//
// Everything is fully unrolled: K[t] and every constant message word fold
// into literals, the round variables rename instead of moving, and the
// compiler lowers ROTR to v_alignbit_b32, Ch/Maj to v_bitop3_b32 and the
// 3-input sums to v_add3_u32 / v_xor3_b32 on gfx950.
#pragma once
#include <stdint.h>
#include "field.hpp"

namespace fri {
namespace sha {

struct Digest { uint32_t h[8]; };

FRI_HD uint32_t rotr(uint32_t x, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(x, x, n);
#else
    return (x >> n) | (x << (32 - n));
#endif
}
FRI_HD uint32_t bsig0(uint32_t x) { return rotr(x, 2) ^ rotr(x, 13) ^ rotr(x, 22); }
FRI_HD uint32_t bsig1(uint32_t x) { return rotr(x, 6) ^ rotr(x, 11) ^ rotr(x, 25); }
FRI_HD uint32_t ssig0(uint32_t x) { return rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3); }
FRI_HD uint32_t ssig1(uint32_t x) { return rotr(x, 17) ^ rotr(x, 19) ^ (x >> 10); }
FRI_HD uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return (e & f) ^ (~e & g); }
FRI_HD uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return (a & b) ^ (a & c) ^ (b & c); }

FRI_HD uint32_t K(int t) {
    constexpr uint32_t k[64] = {
        0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
        0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
        0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
        0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
        0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
        0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
        0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
        0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
    return k[t];
}

FRI_HD void init(uint32_t s[8]) {
    s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
    s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

// One compression of the 16-word block w (consumed) into state s.
FRI_HD void compress(uint32_t s[8], uint32_t w[16]) {
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = w[t & 15] + ssig0(w[(t - 15) & 15]) + w[(t - 7) & 15] + ssig1(w[(t - 2) & 15]);
            w[t & 15] = wt;
        }
        uint32_t t1 = h + bsig1(e) + ch(e, f, g) + K(t) + wt;
        uint32_t t2 = bsig0(a) + maj(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// Leaf: SHA256(u64 big-endian of a canonical u32) — src/merkle/mod.rs:14-15.
// One block: W0 = 0 (high word), W1 = v, W2 = 0x80000000, W15 = 64 bits.
FRI_HD void leaf(uint32_t v, uint32_t out[8]) {
    uint32_t w[16] = {0u, v, 0x80000000u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 64u};
    init(out);
    compress(out, w);
}

// Internal node: SHA256(left || right) (64-byte message, rs_merkle
// concat_and_hash).  Second block is the constant padding block.
FRI_HD void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    init(out);
    compress(out, w);
    uint32_t p[16] = {0x80000000u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 512u};
    compress(out, p);
}

// Generic SHA-256 of a short byte string (<= 247 bytes) — used only by the
// single-lane channel (src/channel/channel.rs) and by host helpers.
FRI_HD void bytes(const uint8_t* msg, uint32_t len, uint32_t out[8]) {
    init(out);
    uint32_t nblk = (len + 9 + 63) / 64;
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++) {
            uint32_t word = 0;
            for (int j = 0; j < 4; j++) {
                uint32_t idx = b * 64 + i * 4 + j;
                uint32_t byte;
                if (idx < len) byte = msg[idx];
                else if (idx == len) byte = 0x80u;
                else byte = 0u;
                word = (word << 8) | byte;
            }
            w[i] = word;
        }
        if (b == nblk - 1) { w[14] = (uint32_t)(((uint64_t)len * 8) >> 32); w[15] = (uint32_t)((uint64_t)len * 8); }
        compress(out, w);
    }
}

FRI_HD char hexc(uint32_t nib) { return (char)(nib < 10 ? '0' + nib : 'a' + nib - 10); }

// Lowercase hex of a digest's 32 bytes (rs_merkle root_hex, sha256::digest).
FRI_HD void digest_hex(const uint32_t d[8], char out[64]) {
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) out[8 * i + j] = hexc((d[i] >> (28 - 4 * j)) & 15u);
}

}  // namespace sha
}  // namespace fri
