// Dev probe: do the tree-top "plateaus" (some levels of a
// k_tree_top launch take 9-11.4 K cycles per lane-pair node instead of 8.6 K,
// in ~0.4 K steps, stable once they start) appear outside the FRI kernel?
// One 512-thread workgroup, 24 levels of 32 lane-pair nodes on wave 0 (each
// level hashes the previous level's digests), an LDS-only barrier per level
// for all eight waves, s_memtime around each level's node on lane 0.
//   mode 0: the other waves only pass the barriers
//   mode 1: + wave 7 runs one compression in each of the first 3 levels
//   mode 2: + every level's digests are also stored to HBM (as the tops do)
//   modes 3-5: as mode 2, but the timed region also covers the store and its
//   completion (s_waitcnt vmcnt(0)); level `it` writes at it * STRIDE[mode]
//   bytes, so 3 stays in one page and 4/5 touch a new 2 MB / 16 MB region
//   per level (the tops write each level at its own tree offset)
//   mode 6: as mode 0, but wave 7 runs ~10 KB of distinct straight-line code
//   per level, cycling through 6 variants (~60 KB: instruction-cache
//   pressure from a concurrent wave, as the channel wave of k_tree_top adds)
//   mode 7: as mode 6 with one variant every level (warm after level 0)
//   mode 8: as mode 0 with k_tree_top's LDS layout and addressing: 48 KB
//   array, B 32 KB above A, node q reads digests 2q and 2q+1 (pair_level)
//   hipcc -O3 --offload-arch=gfx950 -I../csrc plateau_micro.hip -o plateau_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "sha256_quad.hpp"
using namespace fri;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int LEVELS = 24;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V>
__device__ __attribute__((noinline)) uint32_t junk(uint32_t a, uint32_t b) {
#pragma unroll
    for (int i = 0; i < 256; i++) {
        a = __builtin_rotateleft32(a ^ (b + 0x9e3779b9u * (uint32_t)(i + 97 * V)), (i + V) % 31 + 1);
        b += a ^ (uint32_t)(7919 * V + 131 * i);
    }
    return a ^ b;
}

__device__ uint32_t junk_any(int v, uint32_t a, uint32_t b) {
    switch (v) {
        case 0: return junk<0>(a, b);
        case 1: return junk<1>(a, b);
        case 2: return junk<2>(a, b);
        case 3: return junk<3>(a, b);
        case 4: return junk<4>(a, b);
        default: return junk<5>(a, b);
    }
}

template <bool TOP_LDS, bool PRESSURE = false>
__global__ __launch_bounds__(512) void k_plateau(const uint32_t* in, uint32_t* hbm, unsigned long long* clk, int mode, size_t stride) {
    __shared__ uint4 lds[TOP_LDS ? 3 * 1024 : 4 * 64];
    uint4* A = lds;
    uint4* B = lds + (TOP_LDS ? 2 * 1024 : 2 * 64);
    const uint32_t tid = threadIdx.x;
    if (tid < 128) A[tid] = reinterpret_cast<const uint4*>(in)[tid];
    __syncthreads();
    const shaq::Role R = shaq::role_of(tid);
    uint32_t X[4] = {R.iv[0], R.iv[1], R.iv[2], R.iv[3]};
    uint4* a = A;
    uint4* b = B;
    constexpr int NP = PRESSURE ? 48 : 1;
    uint32_t pad[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) pad[i] = in[(tid + 7 * i) & 511];
    for (int it = 0; it < LEVELS; it++) {
        const uint32_t active = mode == 10 ? 64u >> (it % 6) : 64u;
        if (tid < active) {                              // 32 pairs: node q hashes digests q and q+32 (mod 64)
            const uint32_t q = tid >> 1, half = (tid & 1u) ^ 1u;
            uint32_t l[8], r[8], o[4];
            const uint32_t li = TOP_LDS ? 4 * q : 2 * q, ri = TOP_LDS ? 4 * q + 2 : 2 * ((q + 16) & 31);
            const uint4 l0 = a[li], l1 = a[li + 1], r0 = a[ri], r1 = a[ri + 1];
            l[0] = l0.x; l[1] = l0.y; l[2] = l0.z; l[3] = l0.w; l[4] = l1.x; l[5] = l1.y; l[6] = l1.z; l[7] = l1.w;
            r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w; r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const unsigned long long c0 = __builtin_amdgcn_s_memtime();
            shaq::node(l, r, o, R);
            unsigned long long c1 = __builtin_amdgcn_s_memtime();
            const uint4 v = make_uint4(o[0], o[1], o[2], o[3]);
            b[2 * q + half] = v;
            if (mode >= 2 && mode < 6) reinterpret_cast<uint4*>(hbm + it * stride + 8 * q)[half] = v;
            if (mode >= 3 && mode < 6) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                c1 = __builtin_amdgcn_s_memtime();
            }
            if (tid == 0) clk[it] = c1 - c0;
        }
        if (mode >= 6 && mode < 8 && tid >= 448) X[0] ^= junk_any(mode == 6 ? it % 6 : 0, X[1] + it, tid);
        if (mode >= 1 && mode < 6 && tid >= 448 && it < 3) {         // wave 7: one compression (channel pre-job)
            uint32_t w[16];
            for (int i = 0; i < 16; i++) w[i] = it * 16 + i;
            shaq::compress(X, w, R);
        }
        if (PRESSURE) {
#pragma unroll
            for (int i = 0; i < NP; i++) asm volatile("" : "+v"(pad[i]));
        }
        lds_barrier();
        uint4* t = a; a = b; b = t;
    }
    if (tid >= 448 && tid < 452) hbm[tid - 448] = X[tid & 3];
    if (tid == 0) {                                      // placement of this launch: XCC_ID, HW_ID
        clk[LEVELS] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        clk[LEVELS + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
    if (PRESSURE) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < NP; i++) acc += pad[i] * (i + 1);
        hbm[64 + tid] = acc;
    }
}

int main() {
    uint32_t h_in[512];
    for (int i = 0; i < 512; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 9);
    uint32_t *d_in, *d_hbm;
    unsigned long long* d_clk;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    const size_t STRIDE[11] = {512, 512, 512, 512, (2u << 20) / 4, (16u << 20) / 4, 512, 512, 512, 512, 512};   // u32 words
    CK(hipMalloc(&d_hbm, (size_t)LEVELS * STRIDE[5] * 4 + 4096));
    CK(hipMalloc(&d_clk, (LEVELS + 2) * 8));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    for (int mode = 0; mode < 11; mode++) {
        printf("mode %d\n", mode);
        for (int rep = 0; rep < 8; rep++) {
            if (mode == 9) hipLaunchKernelGGL((k_plateau<true, true>), dim3(1), dim3(512), 0, 0, d_in, d_hbm, d_clk, 0, STRIDE[mode]);
            else if (mode >= 8) hipLaunchKernelGGL(k_plateau<true>, dim3(1), dim3(512), 0, 0, d_in, d_hbm, d_clk, mode == 10 ? 10 : 0, STRIDE[mode]);
            else hipLaunchKernelGGL(k_plateau<false>, dim3(1), dim3(512), 0, 0, d_in, d_hbm, d_clk, mode, STRIDE[mode]);
            CK(hipDeviceSynchronize());
            unsigned long long c[LEVELS + 2];
            CK(hipMemcpy(c, d_clk, sizeof(c), hipMemcpyDeviceToHost));
            printf("  ");
            for (int i = 0; i < LEVELS; i++) printf("%.1f ", c[i] / 1000.0);
            printf(" xcc=%llu hw_id=0x%08llx\n", c[LEVELS], c[LEVELS + 1]);
        }
    }
    return 0;
}
