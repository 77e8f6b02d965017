// order_micro.hip — does the ORDER of a SHA-256 round's instructions change
// the chip-wide hash rate on gfx950?  The unrolled node hash (shaf::node) as
// the compiler schedules it, against the same instructions issued in fixed
// groups by one asm block per round: the six rotations and the h+K+W add3
// (half rate) first, then the four v_bitop3 (full rate), then the adds.
// Checks both against each other and prints node hashes/s (not part of the
// library).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../csrc/sha256.hpp"
#include "../csrc/sha256_fast.hpp"

using namespace fri;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// One round: d += T1 (new e), h = T1 + T2 (new a); K in an SGPR.
#define RND_ASM(a, b, c, d, e, f, g, h, W, K)                                                      \
    {                                                                                              \
        uint32_t r1, r2, r3, r4, r5, r6;                                                           \
        asm volatile("v_alignbit_b32 %[r1], %[xe], %[xe], 6\n\t"                                     \
                     "v_alignbit_b32 %[r2], %[xe], %[xe], 11\n\t"                                    \
                     "v_alignbit_b32 %[r3], %[xe], %[xe], 25\n\t"                                    \
                     "v_alignbit_b32 %[r4], %[xa], %[xa], 2\n\t"                                     \
                     "v_alignbit_b32 %[r5], %[xa], %[xa], 13\n\t"                                    \
                     "v_alignbit_b32 %[r6], %[xa], %[xa], 22\n\t"                                    \
                     "v_add3_u32 %[xh], %[xh], %[xw], %[xk]\n\t"                                       \
                     "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[r4], %[r4], %[r5], %[r6] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[r2], %[xe], %[xf], %[xg] bitop3:0xca\n\t"                        \
                     "v_bitop3_b32 %[r5], %[xa], %[xb], %[xc] bitop3:0xe8\n\t"                        \
                     "v_add3_u32 %[xh], %[xh], %[r1], %[r2]\n\t"                                     \
                     "v_add_u32 %[xd], %[xd], %[xh]\n\t"                                              \
                     "v_add3_u32 %[xh], %[xh], %[r4], %[r5]"                                         \
                     : [xd] "+v"(d), [xh] "+v"(h), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3),   \
                       [r4] "=&v"(r4), [r5] "=&v"(r5), [r6] "=&v"(r6)                               \
                     : [xa] "v"(a), [xb] "v"(b), [xc] "v"(c), [xe] "v"(e), [xf] "v"(f), [xg] "v"(g),      \
                       [xw] "v"(W), [xk] "s"(K));                                                    \
    }
// Schedule word w16 <- w16 + s0(w15) + w7 + s1(w2): rotations first, then
// the shifts and XORs, then the adds.
#define SCH_ASM(w16, w15, w7, w2)                                                                  \
    {                                                                                              \
        uint32_t x1, x2, x3, y1, y2, y3;                                                           \
        asm volatile("v_alignbit_b32 %[x1], %[yp], %[yp], 7\n\t"                                     \
                     "v_alignbit_b32 %[x2], %[yp], %[yp], 18\n\t"                                    \
                     "v_alignbit_b32 %[y1], %[yq], %[yq], 17\n\t"                                    \
                     "v_alignbit_b32 %[y2], %[yq], %[yq], 19\n\t"                                    \
                     "v_add3_u32 %[yw], %[yw], %[ys], 0\n\t"                                          \
                     "v_lshrrev_b32 %[x3], 3, %[yp]\n\t"                                            \
                     "v_lshrrev_b32 %[y3], 10, %[yq]\n\t"                                           \
                     "v_bitop3_b32 %[x1], %[x1], %[x2], %[x3] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[y1], %[y1], %[y2], %[y3] bitop3:0x96\n\t"                     \
                     "v_add3_u32 %[yw], %[yw], %[x1], %[y1]"                                         \
                     : [yw] "+v"(w16), [x1] "=&v"(x1), [x2] "=&v"(x2), [x3] "=&v"(x3), [y1] "=&v"(y1),\
                       [y2] "=&v"(y2), [y3] "=&v"(y3)                                               \
                     : [yp] "v"(w15), [yq] "v"(w2), [ys] "v"(w7));                                    \
    }

#define RND8(Wexpr, Kexpr)                                                                         \
    switch (u) {                                                                                   \
        case 0: RND_ASM(a, b, c, d, e, f, g, h, (Wexpr), (Kexpr)); break;                          \
        case 1: RND_ASM(h, a, b, c, d, e, f, g, (Wexpr), (Kexpr)); break;                          \
        case 2: RND_ASM(g, h, a, b, c, d, e, f, (Wexpr), (Kexpr)); break;                          \
        case 3: RND_ASM(f, g, h, a, b, c, d, e, (Wexpr), (Kexpr)); break;                          \
        case 4: RND_ASM(e, f, g, h, a, b, c, d, (Wexpr), (Kexpr)); break;                          \
        case 5: RND_ASM(d, e, f, g, h, a, b, c, (Wexpr), (Kexpr)); break;                          \
        case 6: RND_ASM(c, d, e, f, g, h, a, b, (Wexpr), (Kexpr)); break;                          \
        case 7: RND_ASM(b, c, d, e, f, g, h, a, (Wexpr), (Kexpr)); break;                          \
    }

__device__ __forceinline__ void compress_var_asm(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int tt = t + u;
            if (tt >= 16) SCH_ASM(w[tt & 15], w[(tt - 15) & 15], w[(tt - 7) & 15], w[(tt - 2) & 15]);
            const uint32_t wt = w[tt & 15];
            const uint32_t kk = sha::K(tt);
            RND8(wt, kk)
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
__device__ __forceinline__ void compress_pad_asm(uint32_t st[8]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    const uint32_t zero = 0u;
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t kk = shaf::PAD_KW.kw[t + u];
            RND8(zero, kk)
        }
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
__device__ __forceinline__ void compress_asm(uint32_t st[8], uint32_t w[16], const uint32_t* kw_pad) {
    if (kw_pad) compress_pad_asm(st); else compress_var_asm(st, w);
}

__device__ __forceinline__ void node_asm(const uint32_t* l, const uint32_t* r, uint32_t* o) {
    uint32_t w[16];
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    sha::init(o);
    compress_var_asm(o, w);
    compress_pad_asm(o);
}


__global__ void k_dbg(uint32_t* out) {
    if (threadIdx.x) return;
    uint32_t w0[16], w1[16], s0[8], s1[8];
    for (int i = 0; i < 16; i++) { w0[i] = w1[i] = 0x01234567u * (i + 1); }
    sha::init(s0); sha::init(s1);
    shaf::rounds_var(s0, w0);
    compress_asm(s1, w1, nullptr);
    for (int i = 0; i < 8; i++) { out[i] = s0[i]; out[8 + i] = s1[i]; }
    shaf::rounds_pad64(s0);
    compress_asm(s1, w1, shaf::PAD_KW.kw);
    for (int i = 0; i < 8; i++) { out[16 + i] = s0[i]; out[24 + i] = s1[i]; }
}

template <int V>
__global__ __launch_bounds__(256) void k_node(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
#pragma unroll 1
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = in[4 * i], b = in[4 * i + 1], c = in[4 * i + 2], d = in[4 * i + 3];
        uint32_t l[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t r[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
        uint32_t o[8];
        if (V == 0) shaf::node(l, r, o); else node_asm(l, r, o);
        out[2 * i] = make_uint4(o[0], o[1], o[2], o[3]);
        out[2 * i + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
}

// Two independent hashes per thread, one asm block per round for both:
// 12 rotations + 2 add3 (half rate), then 8 v_bitop3 (full rate), then the adds.
#define RND2_ASM(a, b, c, d, e, f, g, h, A, B, C, D, E, F, G, H, W0, W1, K)                        \
    {                                                                                              \
        uint32_t r1, r2, r3, r4, r5, r6, q1, q2, q3, q4, q5, q6;                                   \
        asm volatile("v_alignbit_b32 %[r1], %[xe], %[xe], 6\n\t"                                   \
                     "v_alignbit_b32 %[q1], %[ye], %[ye], 6\n\t"                                   \
                     "v_alignbit_b32 %[r2], %[xe], %[xe], 11\n\t"                                  \
                     "v_alignbit_b32 %[q2], %[ye], %[ye], 11\n\t"                                  \
                     "v_alignbit_b32 %[r3], %[xe], %[xe], 25\n\t"                                  \
                     "v_alignbit_b32 %[q3], %[ye], %[ye], 25\n\t"                                  \
                     "v_alignbit_b32 %[r4], %[xa], %[xa], 2\n\t"                                   \
                     "v_alignbit_b32 %[q4], %[ya], %[ya], 2\n\t"                                   \
                     "v_alignbit_b32 %[r5], %[xa], %[xa], 13\n\t"                                  \
                     "v_alignbit_b32 %[q5], %[ya], %[ya], 13\n\t"                                  \
                     "v_alignbit_b32 %[r6], %[xa], %[xa], 22\n\t"                                  \
                     "v_alignbit_b32 %[q6], %[ya], %[ya], 22\n\t"                                  \
                     "v_add3_u32 %[xh], %[xh], %[xw], %[xk]\n\t"                                   \
                     "v_add3_u32 %[yh], %[yh], %[yw], %[xk]\n\t"                                   \
                     "v_bitop3_b32 %[r1], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[q1], %[q1], %[q2], %[q3] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[r4], %[r4], %[r5], %[r6] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[q4], %[q4], %[q5], %[q6] bitop3:0x96\n\t"                     \
                     "v_bitop3_b32 %[r2], %[xe], %[xf], %[xg] bitop3:0xca\n\t"                     \
                     "v_bitop3_b32 %[q2], %[ye], %[yf], %[yg] bitop3:0xca\n\t"                     \
                     "v_bitop3_b32 %[r5], %[xa], %[xb], %[xc] bitop3:0xe8\n\t"                     \
                     "v_bitop3_b32 %[q5], %[ya], %[yb], %[yc] bitop3:0xe8\n\t"                     \
                     "v_add3_u32 %[xh], %[xh], %[r1], %[r2]\n\t"                                   \
                     "v_add3_u32 %[yh], %[yh], %[q1], %[q2]\n\t"                                   \
                     "v_add_u32 %[xd], %[xd], %[xh]\n\t"                                           \
                     "v_add_u32 %[yd], %[yd], %[yh]\n\t"                                           \
                     "v_add3_u32 %[xh], %[xh], %[r4], %[r5]\n\t"                                   \
                     "v_add3_u32 %[yh], %[yh], %[q4], %[q5]"                                       \
                     : [xd] "+v"(d), [xh] "+v"(h), [yd] "+v"(D), [yh] "+v"(H), [r1] "=&v"(r1),     \
                       [r2] "=&v"(r2), [r3] "=&v"(r3), [r4] "=&v"(r4), [r5] "=&v"(r5), [r6] "=&v"(r6),\
                       [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [q4] "=&v"(q4), [q5] "=&v"(q5), \
                       [q6] "=&v"(q6)                                                              \
                     : [xa] "v"(a), [xb] "v"(b), [xc] "v"(c), [xe] "v"(e), [xf] "v"(f), [xg] "v"(g),\
                       [ya] "v"(A), [yb] "v"(B), [yc] "v"(C), [ye] "v"(E), [yf] "v"(F), [yg] "v"(G),\
                       [xw] "v"(W0), [yw] "v"(W1), [xk] "s"(K));                                   \
    }
#define RND2X8(W0e, W1e, Ke)                                                                       \
    switch (u) {                                                                                   \
        case 0: RND2_ASM(a, b, c, d, e, f, g, h, A, B, C, D, E, F, G, H, (W0e), (W1e), (Ke)); break; \
        case 1: RND2_ASM(h, a, b, c, d, e, f, g, H, A, B, C, D, E, F, G, (W0e), (W1e), (Ke)); break; \
        case 2: RND2_ASM(g, h, a, b, c, d, e, f, G, H, A, B, C, D, E, F, (W0e), (W1e), (Ke)); break; \
        case 3: RND2_ASM(f, g, h, a, b, c, d, e, F, G, H, A, B, C, D, E, (W0e), (W1e), (Ke)); break; \
        case 4: RND2_ASM(e, f, g, h, a, b, c, d, E, F, G, H, A, B, C, D, (W0e), (W1e), (Ke)); break; \
        case 5: RND2_ASM(d, e, f, g, h, a, b, c, D, E, F, G, H, A, B, C, (W0e), (W1e), (Ke)); break; \
        case 6: RND2_ASM(c, d, e, f, g, h, a, b, C, D, E, F, G, H, A, B, (W0e), (W1e), (Ke)); break; \
        case 7: RND2_ASM(b, c, d, e, f, g, h, a, B, C, D, E, F, G, H, A, (W0e), (W1e), (Ke)); break; \
    }
__device__ __forceinline__ void node2_asm(const uint32_t* l0, const uint32_t* r0, uint32_t* o0,
                                          const uint32_t* l1, const uint32_t* r1, uint32_t* o1) {
    uint32_t w[16], v[16];
    for (int i = 0; i < 8; i++) { w[i] = l0[i]; w[8 + i] = r0[i]; v[i] = l1[i]; v[8 + i] = r1[i]; }
    sha::init(o0); sha::init(o1);
    uint32_t a = o0[0], b = o0[1], c = o0[2], d = o0[3], e = o0[4], f = o0[5], g = o0[6], h = o0[7];
    uint32_t A = o1[0], B = o1[1], C = o1[2], D = o1[3], E = o1[4], F = o1[5], G = o1[6], H = o1[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int tt = t + u;
            if (tt >= 16) {
                SCH_ASM(w[tt & 15], w[(tt - 15) & 15], w[(tt - 7) & 15], w[(tt - 2) & 15]);
                SCH_ASM(v[tt & 15], v[(tt - 15) & 15], v[(tt - 7) & 15], v[(tt - 2) & 15]);
            }
            const uint32_t kk = sha::K(tt);
            RND2X8(w[tt & 15], v[tt & 15], kk)
        }
    }
    o0[0] += a; o0[1] += b; o0[2] += c; o0[3] += d; o0[4] += e; o0[5] += f; o0[6] += g; o0[7] += h;
    o1[0] += A; o1[1] += B; o1[2] += C; o1[3] += D; o1[4] += E; o1[5] += F; o1[6] += G; o1[7] += H;
    a = o0[0]; b = o0[1]; c = o0[2]; d = o0[3]; e = o0[4]; f = o0[5]; g = o0[6]; h = o0[7];
    A = o1[0]; B = o1[1]; C = o1[2]; D = o1[3]; E = o1[4]; F = o1[5]; G = o1[6]; H = o1[7];
    const uint32_t zero = 0u;
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t kk = shaf::PAD_KW.kw[t + u];
            RND2X8(zero, zero, kk)
        }
    }
    o0[0] += a; o0[1] += b; o0[2] += c; o0[3] += d; o0[4] += e; o0[5] += f; o0[6] += g; o0[7] += h;
    o1[0] += A; o1[1] += B; o1[2] += C; o1[3] += D; o1[4] += E; o1[5] += F; o1[6] += G; o1[7] += H;
}
__global__ __launch_bounds__(256) void k_node_x2asm(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
    const size_t half = n / 2;
#pragma unroll 1
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < half; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t l0[8], r0[8], l1[8], r1[8], o0[8], o1[8];
        const uint32_t* p0 = reinterpret_cast<const uint32_t*>(in + 4 * i);
        const uint32_t* p1 = reinterpret_cast<const uint32_t*>(in + 4 * (i + half));
        for (int k = 0; k < 8; k++) { l0[k] = p0[k]; r0[k] = p0[8 + k]; l1[k] = p1[k]; r1[k] = p1[8 + k]; }
        node2_asm(l0, r0, o0, l1, r1, o1);
        out[2 * i] = make_uint4(o0[0], o0[1], o0[2], o0[3]);
        out[2 * i + 1] = make_uint4(o0[4], o0[5], o0[6], o0[7]);
        out[2 * (i + half)] = make_uint4(o1[0], o1[1], o1[2], o1[3]);
        out[2 * (i + half) + 1] = make_uint4(o1[4], o1[5], o1[6], o1[7]);
    }
}

int main() {
    const size_t n = 1u << 22;
    uint4 *nin, *out;
    CK(hipMalloc(&nin, n * 64)); CK(hipMalloc(&out, n * 32));
    uint32_t* h = (uint32_t*)malloc(n * 64);
    for (size_t i = 0; i < n * 16; i++) h[i] = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7);
    CK(hipMemcpy(nin, h, n * 64, hipMemcpyHostToDevice));
    uint32_t *o1 = (uint32_t*)malloc(n * 32), *o2 = (uint32_t*)malloc(n * 32);
    const int grid = (int)(n / 256);
    hipLaunchKernelGGL((k_node<0>), dim3(grid), dim3(256), 0, 0, nin, out, n);
    CK(hipMemcpy(o1, out, n * 32, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((k_node<1>), dim3(grid), dim3(256), 0, 0, nin, out, n);
    CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("asm node == compiler node: %d\n", memcmp(o1, o2, n * 32) == 0);
    hipLaunchKernelGGL(k_node_x2asm, dim3(grid / 2), dim3(256), 0, 0, nin, out, n);
    CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("asm x2 node == compiler node: %d\n", memcmp(o1, o2, n * 32) == 0);
    {
        uint32_t* d; uint32_t hd[32];
        CK(hipMalloc(&d, 128));
        hipLaunchKernelGGL(k_dbg, dim3(1), dim3(64), 0, 0, d);
        CK(hipMemcpy(hd, d, 128, hipMemcpyDeviceToHost));
        printf("var: "); for (int i = 0; i < 8; i++) printf("%08x/%08x ", hd[i], hd[8 + i]); printf("\n");
        printf("pad: "); for (int i = 0; i < 8; i++) printf("%08x/%08x ", hd[16 + i], hd[24 + i]); printf("\n");
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int rep = 0; rep < 6; rep++)
        for (int v = 0; v < 3; v++) {
            CK(hipEventRecord(a));
            for (int i = 0; i < 10; i++) {
                if (v == 0) hipLaunchKernelGGL((k_node<0>), dim3(grid), dim3(256), 0, 0, nin, out, n);
                else if (v == 1) hipLaunchKernelGGL((k_node<1>), dim3(grid), dim3(256), 0, 0, nin, out, n);
                else hipLaunchKernelGGL(k_node_x2asm, dim3(grid / 2), dim3(256), 0, 0, nin, out, n);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            ms /= 10;
            printf("%-34s %7.3f ms  %6.2f G nodes/s\n", v == 2 ? "asm x2, grouped by rate" : v ? "asm, grouped by rate" : "compiler-scheduled (shaf::node)",
                   ms, n / (ms * 1e-3) / 1e9);
        }
    return 0;
}
