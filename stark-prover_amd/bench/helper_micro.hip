// Dev microbenchmark: latency of a dependent chain of Merkle node hashes
// (one wave of 64 independent chains), compact SHA vs "schedule on a helper
// wave": wave 1 (another SIMD) expands the first block's message schedule
// into LDS while wave 0 runs the rounds (two barriers per node).
//   hipcc -O3 --offload-arch=gfx950 -I../csrc helper_micro.hip -o helper_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "sha256_fast.hpp"
using namespace fri;

// rounds 0..15 from registers, 16..63 from the LDS schedule (K+W), then pad block
__device__ __forceinline__ void main_node(const uint32_t l[8], const uint32_t r[8], const uint32_t* kw_lds,
                                          uint32_t out[8]) {
    uint32_t st[8];
    sha::init(st);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#define R(kwv)                                                                      \
    {                                                                               \
        uint32_t t1 = h + (kwv) + shaf::S1(e) + shaf::chf(e, f, g);                 \
        uint32_t t2 = shaf::S0(a) + shaf::majf(a, b, c);                            \
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;          \
    }
#pragma unroll
    for (int i = 0; i < 8; i++) R(l[i] + shaf::KTAB[i])
#pragma unroll
    for (int i = 0; i < 8; i++) R(r[i] + shaf::KTAB[8 + i])
    __syncthreads();                                      // W16..39 ready
#pragma unroll 1
    for (int i = 16; i < 40; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) R(kw_lds[(i + u) * 64])
    }
    __syncthreads();                                      // W40..63 ready
#pragma unroll 1
    for (int i = 40; i < 64; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) R(kw_lds[(i + u) * 64])
    }
#undef R
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    shaf::kwtab_loop(st, shaf::PAD_KW_C.kw);
    for (int i = 0; i < 8; i++) out[i] = st[i];
}
__device__ __forceinline__ void helper_sched(const uint32_t l[8], const uint32_t r[8], uint32_t* kw_lds) {
    uint32_t w[16];
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
#pragma unroll
    for (int t = 16; t < 40; t++) {
        const int i = t & 15;
        w[i] = w[i] + shaf::s0(w[(i + 1) & 15]) + w[(i + 9) & 15] + shaf::s1(w[(i + 14) & 15]);
        kw_lds[t * 64] = w[i] + shaf::KTAB[t];
    }
    __syncthreads();
#pragma unroll
    for (int t = 40; t < 64; t++) {
        const int i = t & 15;
        w[i] = w[i] + shaf::s0(w[(i + 1) & 15]) + w[(i + 9) & 15] + shaf::s1(w[(i + 14) & 15]);
        kw_lds[t * 64] = w[i] + shaf::KTAB[t];
    }
    __syncthreads();
}

__global__ void k_chain(const uint32_t* in, uint32_t* out, int reps, unsigned long long* t, int mode) {
    __shared__ uint32_t kw[64 * 64];
    __shared__ uint32_t dig[64 * 16];                     // l, r of each lane's chain
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave == 0) for (int i = 0; i < 16; i++) dig[lane * 16 + i] = in[lane * 16 + i];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < reps; k++) {
        uint32_t l[8], r[8], o[8];
        for (int i = 0; i < 8; i++) { l[i] = dig[lane * 16 + i]; r[i] = dig[lane * 16 + 8 + i]; }
        if (mode == 0) {
            if (wave == 0) shaf::node_compact(l, r, o);
        } else {
            if (wave == 0) main_node(l, r, kw + lane, o);
            else helper_sched(l, r, kw + lane);
        }
        if (wave == 0) for (int i = 0; i < 8; i++) { dig[lane * 16 + i] = o[i]; dig[lane * 16 + 8 + i] = r[i] ^ o[i]; }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (wave == 0) for (int i = 0; i < 16; i++) out[lane * 16 + i] = dig[lane * 16 + i];
    if (threadIdx.x == 0) *t = t1 - t0;
}

int main() {
    uint32_t *in, *o0, *o1; unsigned long long* t;
    hipMalloc(&in, 64 * 64); hipMalloc(&o0, 64 * 64); hipMalloc(&o1, 64 * 64); hipMalloc(&t, 8);
    uint32_t h[64 * 16];
    for (int i = 0; i < 64 * 16; i++) h[i] = (uint32_t)rand() * 2654435761u + i;
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 64;
    for (int mode = 0; mode < 2; mode++) {
        unsigned long long ht = 0;
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(k_chain, dim3(1), dim3(mode ? 128 : 64), 0, 0, in, mode ? o1 : o0, reps, t, mode);
            hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
        }
        printf("%s: %.3f us per dependent node\n", mode ? "main+helper schedule" : "node_compact", ht / 100.0 / reps);
    }
    uint32_t a[64 * 16], b[64 * 16];
    hipMemcpy(a, o0, sizeof a, hipMemcpyDeviceToHost); hipMemcpy(b, o1, sizeof b, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64 * 16; i++) bad += a[i] != b[i];
    printf("chain mismatches: %d\n", bad);
    return bad != 0;
}
