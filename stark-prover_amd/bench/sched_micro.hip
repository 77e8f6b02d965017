// Dev microbenchmark: the lane-pair chain node of
// sha256_quad.hpp with its message schedule W16..W63 made by a second wave.
//
// A tree-top level's node is bound by its instruction count on a lone wave
// (DESIGN.md §6): 1744 instructions per node, 48 x 7 of them the message
// schedule of the first block.  The schedule depends only on the message,
// not on the round state, so a producer wave on another SIMD can expand it
// (plus the round constants: W[t] + K[t]) into LDS while the round wave runs
// rounds 0..15 on the message words themselves; the round wave then reads
// the schedule 4 words at a time (ds_read_b128), after one flag check per
// 16-word block (three per node).
//
// One 512-thread workgroup, LEVELS levels of 32 lane-pair nodes on wave 0
// (node q hashes digests q and (q + 16) mod 32 of the previous level), an
// LDS-only barrier per level for all eight waves, s_memtime around each
// level on wave 0 lane 0:
//   mode 0: shaq::node (the product node), the other waves only pass the barriers
//   mode 1: producer on wave 1 (SIMD 1), round wave reads the schedule from LDS
//   mode 2: producer on wave 4 (the round wave's own SIMD): issue contention
//   mode 3: as mode 1, but the round wave skips the flag checks (the
//           producer's lead measured without the waits; result unchecked)
//   mode 4: as mode 1, the round wave prefetching each block's flag and
//           words during the previous block's rounds (node_pre)
// Every mode's last level must give the same digests as mode 0 (printed).
//   hipcc -O3 --offload-arch=gfx950 -I../csrc sched_micro.hip -o sched_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "sha256_quad.hpp"
using namespace fri;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int LEVELS = 24;
constexpr int NODES = 32;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#define bop(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
// sha256_quad.hpp's round and schedule step (the header #undefs its own)
#define MQ_R(kw)                                                                      \
    {                                                                                 \
        const uint32_t _S = bop(shaq::rot(x0, R.r1), shaq::rot(x0, R.r2), shaq::rot(x0, R.r3), 0x96); \
        const uint32_t _sel = bop(x0, x1, R.m, 0x2D);                                 \
        const uint32_t _F = bop(_sel, x2, x1, 0xCA);                                  \
        const uint32_t _hk = (x3 + (kw)) & R.me;                                      \
        const uint32_t _V = _S + _F + _hk;                                            \
        const uint32_t _Z = bop(R.me, _V, x3, 0xCA);                                  \
        const uint32_t _n = _V + shaq::swap01(_Z);                                    \
        x3 = x2; x2 = x1; x1 = x0; x0 = _n;                                           \
    }
// produce / node_ext: the product code (sha256_quad.hpp); node_pre below is
// the prefetching variant that measured slower (mode 4).
using shaq::node_ext;
using shaq::produce;

// mode 3: the schedule read without any flag check (unsynchronised: timing only)
__device__ __forceinline__ void node_nowait(const uint32_t l[8], const uint32_t r[8], uint32_t out[4],
                                            const shaq::Role& R, const uint32_t* wk) {
    uint32_t x0 = R.iv[0], x1 = R.iv[1], x2 = R.iv[2], x3 = R.iv[3];
#pragma unroll
    for (int i = 0; i < 8; i++) MQ_R(l[i] + shaf::KTAB[i]);
#pragma unroll
    for (int i = 0; i < 8; i++) MQ_R(r[i] + shaf::KTAB[8 + i]);
#pragma unroll 1
    for (int b = 0; b < 3; b++) {
        const uint4* q = reinterpret_cast<const uint4*>(wk + 16 * b);
        const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        MQ_R(q0.x); MQ_R(q0.y); MQ_R(q0.z); MQ_R(q0.w);
        MQ_R(q1.x); MQ_R(q1.y); MQ_R(q1.z); MQ_R(q1.w);
        MQ_R(q2.x); MQ_R(q2.y); MQ_R(q2.z); MQ_R(q2.w);
        MQ_R(q3.x); MQ_R(q3.y); MQ_R(q3.z); MQ_R(q3.w);
    }
    out[0] = R.iv[0] + x0; out[1] = R.iv[1] + x1; out[2] = R.iv[2] + x2; out[3] = R.iv[3] + x3;
    shaq::compress_kw(out, shaf::PAD_KW_C.kw, R);
}

// Round wave, prefetching: block b+1's flag and schedule words are read while
// block b's rounds run (relaxed flag load, then the data loads in program
// order: LDS executes a wave's operations in order, so data read after a flag
// that shows the block complete is that block's).  Only if the flag was not
// set yet does the wave wait and read the block again.
__device__ __forceinline__ uint32_t flag_relaxed(const uint32_t* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void node_pre(const uint32_t l[8], const uint32_t r[8], uint32_t out[4], const shaq::Role& R,
                                         const uint32_t* wk, const uint32_t* flag, uint32_t base) {
    uint32_t x0 = R.iv[0], x1 = R.iv[1], x2 = R.iv[2], x3 = R.iv[3];
#pragma unroll
    for (int i = 0; i < 8; i++) MQ_R(l[i] + shaf::KTAB[i]);
    const uint4* q = reinterpret_cast<const uint4*>(wk);
    uint32_t f = flag_relaxed(flag);
    asm volatile("" ::: "memory");
    uint4 c0 = q[0], c1 = q[1], c2 = q[2], c3 = q[3];
#pragma unroll
    for (int i = 0; i < 8; i++) MQ_R(r[i] + shaf::KTAB[8 + i]);
#pragma unroll 1
    for (int b = 0; b < 3; b++) {
        if (f < base + b + 1) {                         // not ready when prefetched: wait, read again
            while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < base + b + 1) {}
            c0 = q[4 * b]; c1 = q[4 * b + 1]; c2 = q[4 * b + 2]; c3 = q[4 * b + 3];
        }
        uint4 n0 = c0, n1 = c1, n2 = c2, n3 = c3;
        if (b < 2) {
            f = flag_relaxed(flag);
            asm volatile("" ::: "memory");
            n0 = q[4 * b + 4]; n1 = q[4 * b + 5]; n2 = q[4 * b + 6]; n3 = q[4 * b + 7];
        }
        MQ_R(c0.x); MQ_R(c0.y); MQ_R(c0.z); MQ_R(c0.w);
        MQ_R(c1.x); MQ_R(c1.y); MQ_R(c1.z); MQ_R(c1.w);
        MQ_R(c2.x); MQ_R(c2.y); MQ_R(c2.z); MQ_R(c2.w);
        MQ_R(c3.x); MQ_R(c3.y); MQ_R(c3.z); MQ_R(c3.w);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = R.iv[0] + x0; out[1] = R.iv[1] + x1; out[2] = R.iv[2] + x2; out[3] = R.iv[3] + x3;
    shaq::compress_kw(out, shaf::PAD_KW_C.kw, R);
}

__global__ __launch_bounds__(512) void k_sched(const uint32_t* in, uint32_t* out, unsigned long long* clk, int mode) {
    __shared__ uint4 lds[2 * 2 * NODES];                 // A, B: 32 digests each (2 x uint4)
    __shared__ __attribute__((aligned(16))) uint32_t wk[NODES * 48];
    __shared__ uint32_t flag;
    uint4* A = lds;
    uint4* B = lds + 2 * NODES;
    const uint32_t tid = threadIdx.x;
    if (tid < 2 * NODES) A[tid] = reinterpret_cast<const uint4*>(in)[tid];
    if (tid == 0) flag = 0;
    __syncthreads();
    const shaq::Role R = shaq::role_of(tid);
    const uint32_t prod_wave = mode == 2 ? 4u : 1u;
    const bool round_wave = tid < 64;
    const bool prod = mode >= 1 && (tid >> 6) == prod_wave;
    uint4* a = A;
    uint4* b = B;
    for (int it = 0; it < LEVELS; it++) {
        const uint32_t base = 3u * (uint32_t)it;
        if (round_wave || prod) {
            const uint32_t lane = tid & 63, q = lane >> 1, half = (lane & 1u) ^ 1u;
            const uint32_t li = 2 * q, ri = 2 * ((q + 16) & 31);
            const uint4 l0 = a[li], l1 = a[li + 1], r0 = a[ri], r1 = a[ri + 1];
            uint32_t l[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
            uint32_t r[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
            if (prod) {
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 8; i++) { w[i] = l[i]; w[8 + i] = r[i]; }
                produce(w, wk + 48 * q, &flag, base, (lane & 1u) == 0, lane == 0, R);
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const unsigned long long c0 = __builtin_amdgcn_s_memtime();
                uint32_t o[4];
                if (mode == 0) shaq::node(l, r, o, R);
                else if (mode == 3) node_nowait(l, r, o, R, wk + 48 * q);
                else if (mode == 4) node_pre(l, r, o, R, wk + 48 * q, &flag, base);
                else node_ext(l, r, o, R, wk + 48 * q, &flag, base);
                const unsigned long long c1 = __builtin_amdgcn_s_memtime();
                b[2 * q + half] = make_uint4(o[0], o[1], o[2], o[3]);
                if (tid == 0) clk[it] = c1 - c0;
            }
        }
        lds_barrier();
        uint4* t = a; a = b; b = t;
    }
    if (tid < 2 * NODES) reinterpret_cast<uint4*>(out)[tid] = a[tid];
}

int main() {
    uint32_t h_in[NODES * 8];
    for (int i = 0; i < NODES * 8; i++) h_in[i] = 0x9e3779b9u * (i + 1) ^ (i << 9);
    uint32_t *d_in, *d_out;
    unsigned long long* d_clk;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    CK(hipMalloc(&d_out, sizeof(h_in)));
    CK(hipMalloc(&d_clk, LEVELS * 8));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    uint32_t ref[NODES * 8];
    const char* names[5] = {"product node (schedule in the round wave)", "producer wave 1 (SIMD 1)",
                            "producer wave 4 (same SIMD)", "producer wave 1, no flag waits",
                            "producer wave 1, round wave prefetches the next block"};
    for (int mode = 0; mode < 5; mode++) {
        double sum = 0;
        int n = 0;
        bool same = true;
        printf("mode %d: %s\n", mode, names[mode]);
        for (int rep = 0; rep < 8; rep++) {
            hipLaunchKernelGGL(k_sched, dim3(1), dim3(512), 0, 0, d_in, d_out, d_clk, mode);
            CK(hipDeviceSynchronize());
            unsigned long long c[LEVELS];
            uint32_t o[NODES * 8];
            CK(hipMemcpy(c, d_clk, sizeof(c), hipMemcpyDeviceToHost));
            CK(hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost));
            if (mode == 0 && rep == 0) memcpy(ref, o, sizeof(o));
            same = same && memcmp(ref, o, sizeof(o)) == 0;
            printf("  ");
            for (int i = 0; i < LEVELS; i++) printf("%.2f ", c[i] / 1000.0);
            printf("\n");
            if (rep > 0)
                for (int i = 2; i < LEVELS; i++) { sum += c[i]; n++; }
        }
        printf("  mean level (K cycles, reps 1-7, levels 2-23): %.3f   digests equal to mode 0: %s\n", sum / n / 1000.0,
               same ? "yes" : "NO");
    }
    return 0;
}
