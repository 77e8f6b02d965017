// Dev microbenchmark: latency of a dependent chain of Merkle node hashes in
// the lane-pair form (sha256_quad.hpp, 32 chains on one wave), alone vs with
// the first block's message schedule expanded by a helper wave on another
// SIMD.  The helper writes K+W for rounds 16..63 into LDS in two halves and
// publishes each with a workgroup-scope release; the main wave runs rounds
// 0..15 from registers and acquires each half before using it.
//   hipcc -O3 --offload-arch=gfx950 -I../csrc pair_helper_micro.hip -o pair_helper_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "sha256_quad.hpp"
using namespace fri;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#define bop(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))

using shaq::Role;
using shaq::rot;
using shaq::swap01;

#define PR(kw)                                                                       \
    {                                                                                \
        const uint32_t _S = bop(rot(x0, R.r1), rot(x0, R.r2), rot(x0, R.r3), 0x96);  \
        const uint32_t _sel = bop(x0, x1, R.m, 0x2D);                                \
        const uint32_t _F = bop(_sel, x2, x1, 0xCA);                                 \
        const uint32_t _hk = (x3 + (kw)) & R.me;                                     \
        const uint32_t _V = _S + _F + _hk;                                           \
        const uint32_t _Z = bop(R.me, _V, x3, 0xCA);                                 \
        const uint32_t _n = _V + swap01(_Z);                                         \
        x3 = x2; x2 = x1; x1 = x0; x0 = _n;                                          \
    }
#define PW(i)                                                                                \
    {                                                                                        \
        const uint32_t _x = bop(R.is_a, w[((i) + 1) & 15], w[((i) + 14) & 15], 0xCA);        \
        const uint32_t _s = bop(rot(_x, R.q1), rot(_x, R.q2), _x >> R.q3, 0x96);             \
        w[i] = w[i] + w[((i) + 9) & 15] + _s + swap01(_s);                                   \
    }

__device__ __forceinline__ uint32_t flag_acquire(uint32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void flag_release(uint32_t* f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// kw: [32][48] K+W of rounds 16..63, row q = pair q, published in three
// chunks (rounds 16-27, 28-43, 44-63) so the main wave never waits for the
// helper.  A chunk is read with ds_read_b128 issued right behind a relaxed
// read of the flag (LDS serves one wave's requests in order and the helper
// stores the words before the flag), so one wait covers both; the reads
// repeat only if the flag was short.
constexpr int CH0 = 16, CH1 = 28, CH2 = 44, CH3 = 64;
template <int T0, int T1>
__device__ __forceinline__ void kw_chunk(const uint32_t* kw, uint32_t q, uint32_t v[T1 - T0], uint32_t* flag,
                                         uint32_t want) {
    const uint4* src = reinterpret_cast<const uint4*>(kw + q * 48 + (T0 - 16));
    for (int spin = 0; spin < (1 << 20); spin++) {
        const uint32_t f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < (T1 - T0) / 4; j++) {
            const uint4 x = src[j];
            v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (f >= want) break;
        __builtin_amdgcn_s_sleep(0);
    }
}
__device__ __forceinline__ void main_node(const uint32_t l[8], const uint32_t r[8], uint32_t out[4], const Role& R,
                                          const uint32_t* kw, uint32_t q, uint32_t* flag, uint32_t gen) {
    uint32_t x0 = R.iv[0], x1 = R.iv[1], x2 = R.iv[2], x3 = R.iv[3];
#pragma unroll
    for (int i = 0; i < 8; i++) PR(l[i] + shaf::KTAB[i]);
#pragma unroll
    for (int i = 0; i < 8; i++) PR(r[i] + shaf::KTAB[8 + i]);
    {
        uint32_t v[CH1 - CH0];
        kw_chunk<CH0, CH1>(kw, q, v, flag, gen + 1);
#pragma unroll
        for (int t = 0; t < CH1 - CH0; t++) PR(v[t]);
    }
    {
        uint32_t v[CH2 - CH1];
        kw_chunk<CH1, CH2>(kw, q, v, flag, gen + 2);
#pragma unroll
        for (int t = 0; t < CH2 - CH1; t++) PR(v[t]);
    }
    {
        uint32_t v[CH3 - CH2];
        kw_chunk<CH2, CH3>(kw, q, v, flag, gen + 3);
#pragma unroll
        for (int t = 0; t < CH3 - CH2; t++) PR(v[t]);
    }
    out[0] = R.iv[0] + x0; out[1] = R.iv[1] + x1; out[2] = R.iv[2] + x2; out[3] = R.iv[3] + x3;
    x0 = out[0]; x1 = out[1]; x2 = out[2]; x3 = out[3];
#pragma unroll 1
    for (int rr = 0; rr < 4; rr++) {
#pragma unroll
        for (int i = 0; i < 16; i++) PR(shaf::PAD_KW_C.kw[16 * rr + i]);
    }
    out[0] += x0; out[1] += x1; out[2] += x2; out[3] += x3;
}

__device__ __forceinline__ void helper_sched(const uint32_t l[8], const uint32_t r[8], const Role& R, uint32_t* kw,
                                             uint32_t q, bool writer, uint32_t* flag, uint32_t gen) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
#pragma unroll
    for (int t = 16; t < 64; t++) {
        const int i = t & 15;
        PW(i);
        if (writer) kw[q * 48 + t - 16] = w[i] + shaf::KTAB[t];
        if (t + 1 == CH1 || t + 1 == CH2 || t + 1 == CH3) {
            if (threadIdx.x == 64) flag_release(flag, gen + (t + 1 == CH1 ? 1u : t + 1 == CH2 ? 2u : 3u));
        }
    }
}

// dig: 32 chains x 16 words (l || r)
__global__ void k_chain(const uint32_t* in, uint32_t* out, int reps, unsigned long long* t, int mode) {
    __shared__ uint32_t dig[32 * 16];
    __shared__ __attribute__((aligned(16))) uint32_t kw[48 * 32];
    __shared__ uint32_t flag;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 1, role = lane & 1;
    const Role R = shaq::role_of(lane);
    for (uint32_t i = threadIdx.x; i < 32 * 16; i += blockDim.x) dig[i] = in[i];
    if (threadIdx.x == 0) flag = 0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < reps; k++) {
        uint32_t l[8], r[8], o[4];
#pragma unroll
        for (int i = 0; i < 8; i++) { l[i] = dig[q * 16 + i]; r[i] = dig[q * 16 + 8 + i]; }
        if (mode == 0) {
            if (wave == 0) shaq::node(l, r, o, R);
        } else {
            if (wave == 0) main_node(l, r, o, R, kw, q, &flag, 3u * k);
            else helper_sched(l, r, R, kw, q, role == 0, &flag, 3u * k);
        }
        __syncthreads();
        if (wave == 0) {
            const int base = role == 0 ? 4 : 0;
#pragma unroll
            for (int i = 0; i < 4; i++) { dig[q * 16 + base + i] = o[i]; dig[q * 16 + 8 + base + i] = r[base + i] ^ o[i]; }
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = threadIdx.x; i < 32 * 16; i += blockDim.x) out[i] = dig[i];
    if (threadIdx.x == 0) { t[2 * mode] = t1 - t0; t[2 * mode + 1] = c1 - c0; }
}

int main() {
    const int reps = 64;
    uint32_t h_in[32 * 16];
    for (int i = 0; i < 32 * 16; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 7);
    uint32_t *d_in, *d_o0, *d_o1;
    unsigned long long* d_t;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    CK(hipMalloc(&d_o0, sizeof(h_in)));
    CK(hipMalloc(&d_o1, sizeof(h_in)));
    CK(hipMalloc(&d_t, 4 * 8));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    int bad = 0;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, d_in, d_o0, reps, d_t, 0);
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(128), 0, 0, d_in, d_o1, reps, d_t, 1);
        CK(hipDeviceSynchronize());
        unsigned long long t[4];
        uint32_t a[32 * 16], b[32 * 16];
        CK(hipMemcpy(t, d_t, sizeof(t), hipMemcpyDeviceToHost));
        CK(hipMemcpy(a, d_o0, sizeof(a), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b, d_o1, sizeof(b), hipMemcpyDeviceToHost));
        bad = memcmp(a, b, sizeof(a)) != 0;
        printf("pair node: %.2f us/node (%.0f cycles)   pair + helper schedule: %.2f us/node (%.0f cycles)   match=%d\n",
               t[0] / 100.0 / reps, (double)t[1] / reps, t[2] / 100.0 / reps, (double)t[3] / reps, (int)!bad);
    }
    return bad;
}
