// Dev microbenchmark: latency of a dependent chain of Merkle node hashes on
// ONE wave (the tree-top regime): compact per-lane node (64 chains) vs the
// quad-lane node of sha256_quad.hpp (16 chains, 4 lanes each).  Checks that
// both give the same digests.
//   hipcc -O3 --offload-arch=gfx950 -I../csrc quad_micro.hip -o quad_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "sha256_quad.hpp"
using namespace fri;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_std(const uint32_t* in, uint32_t* out, int reps, unsigned long long* t) {
    __shared__ uint32_t dig[64 * 16];
    const int lane = threadIdx.x;
    for (int i = 0; i < 16; i++) dig[lane * 16 + i] = in[(lane & 15) * 16 + i];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < reps; k++) {
        uint32_t l[8], r[8], o[8];
        for (int i = 0; i < 8; i++) { l[i] = dig[lane * 16 + i]; r[i] = dig[lane * 16 + 8 + i]; }
        shaf::node_compact(l, r, o);
        for (int i = 0; i < 8; i++) { dig[lane * 16 + i] = o[i]; dig[lane * 16 + 8 + i] = r[i] ^ o[i]; }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 16; i++) out[lane * 16 + i] = dig[lane * 16 + i];
    if (lane == 0) { t[0] = t1 - t0; t[1] = c1 - c0; }
}

__global__ void k_quad(const uint32_t* in, uint32_t* out, int reps, unsigned long long* t) {
    __shared__ uint32_t dig[32 * 16];
    const int lane = threadIdx.x, q = lane >> 1, role = lane & 1;
    const shaq::Role R = shaq::role_of(lane);
    if (role == 0) for (int i = 0; i < 16; i++) dig[q * 16 + i] = in[(q & 15) * 16 + i];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < reps; k++) {
        uint32_t l[8], r[8], o[4];
        for (int i = 0; i < 8; i++) { l[i] = dig[q * 16 + i]; r[i] = dig[q * 16 + 8 + i]; }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        shaq::node(l, r, o, R);
        // E writes words 4..7 (and r ^ o), A writes words 0..3
        {
            const int base = role == 0 ? 4 : 0;
            for (int i = 0; i < 4; i++) { dig[q * 16 + base + i] = o[i]; dig[q * 16 + 8 + base + i] = r[base + i] ^ o[i]; }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
    if (role == 0) for (int i = 0; i < 16; i++) out[q * 16 + i] = dig[q * 16 + i];
    if (lane == 0) { t[2] = t1 - t0; t[3] = c1 - c0; }
}

int main() {
    const int reps = 64;
    uint32_t h_in[16 * 16];
    for (int i = 0; i < 256; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 7);
    uint32_t *d_in, *d_o1, *d_o2;
    unsigned long long* d_t;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    CK(hipMalloc(&d_o1, 64 * 16 * 4));
    CK(hipMalloc(&d_o2, 16 * 16 * 4));
    CK(hipMalloc(&d_t, 8 * 8));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_std, dim3(1), dim3(64), 0, 0, d_in, d_o1, reps, d_t);
        hipLaunchKernelGGL(k_quad, dim3(1), dim3(64), 0, 0, d_in, d_o2, reps, d_t);
        CK(hipDeviceSynchronize());
        unsigned long long t[4];
        uint32_t o1[64 * 16], o2[16 * 16];
        CK(hipMemcpy(t, d_t, sizeof(t), hipMemcpyDeviceToHost));
        CK(hipMemcpy(o1, d_o1, sizeof(o1), hipMemcpyDeviceToHost));
        CK(hipMemcpy(o2, d_o2, sizeof(o2), hipMemcpyDeviceToHost));
        bool ok = memcmp(o1, o2, sizeof(o2)) == 0;
        printf("compact node: %.2f us/node (%.0f cycles)   quad node: %.2f us/node (%.0f cycles)   match=%d\n",
               t[0] / 100.0 / reps, (double)t[1] / reps, t[2] / 100.0 / reps, (double)t[3] / reps, (int)ok);
    }
    return 0;
}
