// sha_micro.hip — SHA-256 throughput microbenchmark (leaf / node hash
// variants) on gfx950.  Not part of the library; used to pick the Merkle
// kernel's hash body.  Prints compressions/s and int32 ops/s per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../csrc/sha256.hpp"
#include "../csrc/sha256_fast.hpp"

using namespace fri;

template <int V>
__device__ __forceinline__ void do_node(const uint32_t* l, const uint32_t* r, uint32_t* o) {
    if (V == 1) sha::node(l, r, o); else if (V == 2) shaf::node(l, r, o); else if (V == 3) shaf::node_compact(l, r, o);
    else if (V == 4) { uint32_t w[16]; for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; } sha::init(o); shaf::compress_loop(o, w); }
    else if (V == 5) { for (int i = 0; i < 8; i++) o[i] = l[i]; shaf::kwtab_loop(o, shaf::PAD_KW_C.kw); }
    else if (V == 6) { for (int i = 0; i < 8; i++) o[i] = l[i]; shaf::rounds_pad64(o); }
    else if (V == 7) { uint32_t w[16]; for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; } sha::init(o); shaf::rounds_var(o, w); }
}
template <int V>
__device__ __forceinline__ void do_leaf(uint32_t v, uint32_t* o) {
    if (V == 1) sha::leaf(v, o); else shaf::leaf(v, o);
}

template <int V, int LB>
__global__ __launch_bounds__(256, LB) void k_leaf(const uint32_t* __restrict__ in, uint4* __restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t o[8];
        do_leaf<V>(in[i], o);
        out[2 * i] = make_uint4(o[0], o[1], o[2], o[3]);
        out[2 * i + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
}
template <int V, int LB>
__global__ __launch_bounds__(256, LB) void k_node(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = in[4 * i], b = in[4 * i + 1], c = in[4 * i + 2], d = in[4 * i + 3];
        uint32_t l[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t r[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
        uint32_t o[8];
        do_node<V>(l, r, o);
        out[2 * i] = make_uint4(o[0], o[1], o[2], o[3]);
        out[2 * i + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
}
// two independent node hashes per thread, interleaved by the compiler
template <int LB>
__global__ __launch_bounds__(256, LB) void k_node_x2(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
    size_t half = n / 2;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < half; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t w0[16], w1[16], s0[8], s1[8];
        const uint32_t* p0 = reinterpret_cast<const uint32_t*>(in + 4 * i);
        const uint32_t* p1 = reinterpret_cast<const uint32_t*>(in + 4 * (i + half));
        for (int k = 0; k < 16; k++) { w0[k] = p0[k]; w1[k] = p1[k]; }
        sha::init(s0); sha::init(s1);
        // interleave: schedule/rounds of both blocks in one unrolled loop
        uint32_t a0=s0[0],b0=s0[1],c0=s0[2],d0=s0[3],e0=s0[4],f0=s0[5],g0=s0[6],h0=s0[7];
        uint32_t a1=s1[0],b1=s1[1],c1=s1[2],d1=s1[3],e1=s1[4],f1=s1[5],g1=s1[6],h1=s1[7];
#pragma unroll
        for (int t = 0; t < 64; t++) {
            uint32_t x0, x1;
            if (t < 16) { x0 = w0[t]; x1 = w1[t]; }
            else {
                x0 = w0[t & 15] + shaf::s0(w0[(t - 15) & 15]) + w0[(t - 7) & 15] + shaf::s1(w0[(t - 2) & 15]); w0[t & 15] = x0;
                x1 = w1[t & 15] + shaf::s0(w1[(t - 15) & 15]) + w1[(t - 7) & 15] + shaf::s1(w1[(t - 2) & 15]); w1[t & 15] = x1;
            }
            uint32_t t10 = h0 + sha::K(t) + x0 + shaf::S1(e0) + shaf::chf(e0, f0, g0);
            uint32_t t11 = h1 + sha::K(t) + x1 + shaf::S1(e1) + shaf::chf(e1, f1, g1);
            uint32_t t20 = shaf::S0(a0) + shaf::majf(a0, b0, c0);
            uint32_t t21 = shaf::S0(a1) + shaf::majf(a1, b1, c1);
            h0=g0; g0=f0; f0=e0; e0=d0+t10; d0=c0; c0=b0; b0=a0; a0=t10+t20;
            h1=g1; g1=f1; f1=e1; e1=d1+t11; d1=c1; c1=b1; b1=a1; a1=t11+t21;
        }
        s0[0]+=a0;s0[1]+=b0;s0[2]+=c0;s0[3]+=d0;s0[4]+=e0;s0[5]+=f0;s0[6]+=g0;s0[7]+=h0;
        s1[0]+=a1;s1[1]+=b1;s1[2]+=c1;s1[3]+=d1;s1[4]+=e1;s1[5]+=f1;s1[6]+=g1;s1[7]+=h1;
        shaf::rounds_pad64(s0);
        shaf::rounds_pad64(s1);
        out[2 * i] = make_uint4(s0[0], s0[1], s0[2], s0[3]);
        out[2 * i + 1] = make_uint4(s0[4], s0[5], s0[6], s0[7]);
        out[2 * (i + half)] = make_uint4(s1[0], s1[1], s1[2], s1[3]);
        out[2 * (i + half) + 1] = make_uint4(s1[4], s1[5], s1[6], s1[7]);
    }
}

// ---- issue-mix probe: the unrolled node with every add as a separate
// full-rate v_add_u32 (inline asm, so the compiler cannot re-form v_add3):
// 17 instead of 14 instructions per round, but 11 of them full rate.
__device__ __forceinline__ uint32_t vadd(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t kadd(uint32_t k, uint32_t b) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "s"(k), "v"(b));
    return r;
}
__device__ __forceinline__ void rounds_noadd3(uint32_t st[8], uint32_t w[16], bool pad) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t kw;
        if (pad) {
            kw = kadd(shaf::PAD_KW.kw[t], 0u * h + h) ; // h + KW
        } else {
            uint32_t wt;
            if (t < 16) wt = w[t];
            else {
                wt = vadd(vadd(vadd(w[t & 15], shaf::s0(w[(t - 15) & 15])), w[(t - 7) & 15]), shaf::s1(w[(t - 2) & 15]));
                w[t & 15] = wt;
            }
            kw = vadd(kadd(sha::K(t), wt), h);
        }
        const uint32_t t1 = vadd(vadd(kw, shaf::S1(e)), shaf::chf(e, f, g));
        const uint32_t t2 = vadd(shaf::S0(a), shaf::majf(a, b, c));
        h = g; g = f; f = e; e = vadd(d, t1); d = c; c = b; b = a; a = vadd(t1, t2);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
__device__ __forceinline__ void node_noadd3(const uint32_t* l, const uint32_t* r, uint32_t* o) {
    uint32_t w[16];
    for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
    sha::init(o);
    rounds_noadd3(o, w, false);
    rounds_noadd3(o, w, true);
}
template <int LB>
__global__ __launch_bounds__(256, LB) void k_node_na3(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 a = in[4 * i], b = in[4 * i + 1], c = in[4 * i + 2], d = in[4 * i + 3];
        uint32_t l[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t r[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
        uint32_t o[8];
        node_noadd3(l, r, o);
        out[2 * i] = make_uint4(o[0], o[1], o[2], o[3]);
        out[2 * i + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
}


// ---- VALU calibration: 16 independent chains per lane, OP per iteration
template <int OP>
__global__ __launch_bounds__(256) void k_cal(uint32_t* out, int iters, uint32_t seed) {
    uint32_t r[16];
    for (int i = 0; i < 16; i++) r[i] = seed * (threadIdx.x + 1) + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t a = r[i], b = r[(i + 1) & 15], c = r[(i + 5) & 15];
            if (OP == 0) r[i] = a + b + c;                                  // v_add3_u32
            else if (OP == 1) r[i] = __builtin_amdgcn_alignbit(a, b, 7);     // v_alignbit_b32
            else if (OP == 2) r[i] = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
            else r[i] = a + b;                                              // v_add_u32
        }
    }
    uint32_t x = 0;
    for (int i = 0; i < 16; i++) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}


// ---- latency: one lane hashes a dependent chain of nodes
template <int V>
__global__ void k_chain(uint32_t* out, int n) {
    uint32_t s[8] = {1, 2, 3, 4, 5, 6, 7, (uint32_t)threadIdx.x};
    uint32_t r[8] = {9, 8, 7, 6, 5, 4, 3, 2};
    for (int i = 0; i < n; i++) {
        uint32_t o[8];
        do_node<V>(s, r, o);
        for (int j = 0; j < 8; j++) s[j] = o[j];
    }
    for (int j = 0; j < 8; j++) out[threadIdx.x * 8 + j] = s[j];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <typename F>
float timeit(F f, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main() {
    const size_t n = 1u << 22;
    uint32_t *in; uint4 *nin, *out;
    CK(hipMalloc(&in, n * 4)); CK(hipMalloc(&nin, n * 64)); CK(hipMalloc(&out, n * 32));
    uint32_t* h = (uint32_t*)malloc(n * 64);
    for (size_t i = 0; i < n * 16; i++) h[i] = (uint32_t)(i * 2654435761u) % 3221225473u;
    CK(hipMemcpy(in, h, n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(nin, h, n * 64, hipMemcpyHostToDevice));
    // correctness: v2 == v1
    uint32_t *o1 = (uint32_t*)malloc(n * 32), *o2 = (uint32_t*)malloc(n * 32);
    int grid = (int)(n / 256);
    hipLaunchKernelGGL((k_leaf<1, 1>), dim3(grid), dim3(256), 0, 0, in, out, n); CK(hipMemcpy(o1, out, n * 32, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((k_leaf<2, 1>), dim3(grid), dim3(256), 0, 0, in, out, n); CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("leaf v2==v1: %d\n", memcmp(o1, o2, n * 32) == 0);
    hipLaunchKernelGGL((k_node<1, 1>), dim3(grid), dim3(256), 0, 0, nin, out, n); CK(hipMemcpy(o1, out, n * 32, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((k_node<2, 1>), dim3(grid), dim3(256), 0, 0, nin, out, n); CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("node v2==v1: %d\n", memcmp(o1, o2, n * 32) == 0);
    hipLaunchKernelGGL((k_node_x2<1>), dim3(grid / 2), dim3(256), 0, 0, nin, out, n); CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("node x2==v1: %d\n", memcmp(o1, o2, n * 32) == 0);
    hipLaunchKernelGGL((k_node_na3<1>), dim3(grid), dim3(256), 0, 0, nin, out, n); CK(hipMemcpy(o2, out, n * 32, hipMemcpyDeviceToHost));
    printf("node no-add3==v1: %d\n", memcmp(o1, o2, n * 32) == 0);
    const double peak = 256.0 * 128 * 2.4e9;
    auto rep = [&](const char* name, float ms, double comps, double ops_per_comp) {
        double cps = comps / (ms * 1e-3);
        printf("%-28s %8.3f ms  %7.2f Gcompr/s  est %6.1f Tops (%.0f%% of 78.6)\n", name, ms, cps / 1e9,
               cps * ops_per_comp / 1e12, 100.0 * cps * ops_per_comp / peak);
    };
    int it = 20;
    rep("leaf v1 lb1", timeit([&] { hipLaunchKernelGGL((k_leaf<1, 1>), dim3(grid), dim3(256), 0, 0, in, out, n); }, it), n, 1450);
    rep("leaf v2 lb1", timeit([&] { hipLaunchKernelGGL((k_leaf<2, 1>), dim3(grid), dim3(256), 0, 0, in, out, n); }, it), n, 1450);
    rep("leaf v2 lb4", timeit([&] { hipLaunchKernelGGL((k_leaf<2, 4>), dim3(grid), dim3(256), 0, 0, in, out, n); }, it), n, 1450);
    rep("leaf v2 lb8", timeit([&] { hipLaunchKernelGGL((k_leaf<2, 8>), dim3(grid), dim3(256), 0, 0, in, out, n); }, it), n, 1450);
    rep("node v1 lb1", timeit([&] { hipLaunchKernelGGL((k_node<1, 1>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node v2 lb1", timeit([&] { hipLaunchKernelGGL((k_node<2, 1>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node v2 lb4", timeit([&] { hipLaunchKernelGGL((k_node<2, 4>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node v2 lb8", timeit([&] { hipLaunchKernelGGL((k_node<2, 8>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node no-add3 lb1", timeit([&] { hipLaunchKernelGGL((k_node_na3<1>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node no-add3 lb4", timeit([&] { hipLaunchKernelGGL((k_node_na3<4>), dim3(grid), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node x2 lb1", timeit([&] { hipLaunchKernelGGL((k_node_x2<1>), dim3(grid / 2), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node x2 lb4", timeit([&] { hipLaunchKernelGGL((k_node_x2<4>), dim3(grid / 2), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    rep("node v2 lb1 grid2048", timeit([&] { hipLaunchKernelGGL((k_node<2, 1>), dim3(2048), dim3(256), 0, 0, nin, out, n); }, it), 2.0 * n, 1450);
    {
        uint32_t* o; CK(hipMalloc(&o, 64 * 8 * 4));
        const char* nm[8] = {"", "node v1 (plain C)", "node v2 (bitop3, unrolled)", "node compact (looped)",
                             "compress_loop (var block)", "kwtab_loop (pad block)", "rounds_pad64 (unrolled)",
                             "rounds_var (unrolled var)"};
        for (int v = 1; v <= 7; v++) {
            int nch = 256;
            float ms = timeit([&] {
                switch (v) {
                    case 1: hipLaunchKernelGGL((k_chain<1>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 2: hipLaunchKernelGGL((k_chain<2>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 3: hipLaunchKernelGGL((k_chain<3>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 4: hipLaunchKernelGGL((k_chain<4>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 5: hipLaunchKernelGGL((k_chain<5>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 6: hipLaunchKernelGGL((k_chain<6>), dim3(1), dim3(64), 0, 0, o, nch); break;
                    case 7: hipLaunchKernelGGL((k_chain<7>), dim3(1), dim3(64), 0, 0, o, nch); break;
                } }, 3);
            printf("single-wave latency %-28s %.2f us\n", nm[v], ms * 1e3 / nch);
        }
    }
    {
        uint32_t* o; CK(hipMalloc(&o, 256 * 4096 * 4));
        const char* names[4] = {"v_add3_u32", "v_alignbit_b32", "v_bitop3_b32", "v_add_u32"};
        for (int op = 0; op < 4; op++) {
            int iters = 2048;
            float ms = timeit([&] {
                if (op == 0) hipLaunchKernelGGL((k_cal<0>), dim3(4096), dim3(256), 0, 0, o, iters, 3u);
                if (op == 1) hipLaunchKernelGGL((k_cal<1>), dim3(4096), dim3(256), 0, 0, o, iters, 3u);
                if (op == 2) hipLaunchKernelGGL((k_cal<2>), dim3(4096), dim3(256), 0, 0, o, iters, 3u);
                if (op == 3) hipLaunchKernelGGL((k_cal<3>), dim3(4096), dim3(256), 0, 0, o, iters, 3u);
            }, 5);
            double ops = 4096.0 * 256 * iters * 16;
            printf("calibrate %-16s %8.3f ms  %6.1f T lane-ops/s (%.0f%% of 78.6)\n", names[op], ms, ops / (ms * 1e-3) / 1e12,
                   100.0 * ops / (ms * 1e-3) / peak);
        }
    }
    return 0;
}
