// lone_wave.hip — issue cadence of ONE wave64 on gfx950 (the latency-bound
// regime of the Merkle tree tops): cycles per VALU instruction for dependent
// chains vs K interleaved independent chains, per instruction kind, measured
// with s_memtime around the chain.  Also 2 / 4 waves on one SIMD (waves of a
// 256-thread workgroup land on 4 SIMDs; a 512-thread one puts 2 per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

#define N_ITERS 256

// K independent chains, interleaved: instruction i writes chain (i % K).
template <int K, int KIND>
__global__ void k_chain(unsigned long long* out, unsigned* sink, unsigned seed) {
    unsigned r[8], c = seed ^ threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = seed * (i + 3) + threadIdx.x;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < N_ITERS; it++) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int i = j % K;
            if (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(c));
            if (KIND == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[i]));
            if (KIND == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(c), "v"(r[(i + 1) % 8]));
            if (KIND == 3) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(c), "v"(r[(i + 1) % 8]));
            if (KIND == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(c));
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= r[i];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (blockIdx.x == 0 && threadIdx.x == 0) { out[0] = t1 - t0; out[1] = rt1 - rt0; }
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) { out[2 + 2 * (threadIdx.x >> 6)] = rt0; out[3 + 2 * (threadIdx.x >> 6)] = rt1; }
}

template <int K, int KIND>
static void run(const char* name, int threads) {
    unsigned long long* d_out; unsigned* d_sink;
    CK(hipMalloc(&d_out, 64 * sizeof(unsigned long long)));
    CK(hipMalloc(&d_sink, 4096 * 1024 * sizeof(unsigned)));
    CK(hipMemset(d_out, 0, 64 * sizeof(unsigned long long)));
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL((k_chain<K, KIND>), dim3(1), dim3(threads), 0, 0, d_out, d_sink, 12345u);
    CK(hipDeviceSynchronize());
    unsigned long long h[64];
    CK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
    // s_memtime counts the shader clock (SCLK) on gfx9
    double cyc = (double)h[0] / (N_ITERS * 16.0);
    printf("%-10s K=%d threads=%4d  cycles/instr (wave 0) = %5.2f   ns/instr = %5.2f  (clk %.2f GHz)\n", name, K, threads, cyc, h[1] * 10.0 / (N_ITERS * 16.0), (double)h[0] / (h[1] * 10.0));
    unsigned long long lo = ~0ull, hi = 0;
    for (int w = 0; w < threads / 64; w++) { lo = h[2 + 2 * w] < lo ? h[2 + 2 * w] : lo; hi = h[3 + 2 * w] > hi ? h[3 + 2 * w] : hi; }
    printf("      waves span %.2f us vs wave0 %.2f us\n", (hi - lo) / 100.0, h[1] / 100.0);
    if (threads == 256) {   // full chip: 2048 workgroups
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        hipLaunchKernelGGL((k_chain<K, KIND>), dim3(2048), dim3(1024), 0, 0, d_out, d_sink, 7u);
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_chain<K, KIND>), dim3(2048), dim3(1024), 0, 0, d_out, d_sink, 7u);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        double lane_ops = 2048.0 * 1024 * N_ITERS * 16;
        printf("      full chip 2048x1024: %.3f ms = %.1f T lane-ops/s\n", ms, lane_ops / ms / 1e9);
    }
    CK(hipFree(d_out)); CK(hipFree(d_sink));
}

int main() {
    const char* names[] = {"add", "alignbit", "bitop3", "add3", "xor"};
#define ALLK(KIND, T) run<1, KIND>(names[KIND], T); run<2, KIND>(names[KIND], T); run<4, KIND>(names[KIND], T); run<8, KIND>(names[KIND], T);
    for (int t : {64, 256, 1024}) {
        ALLK(0, t) ALLK(1, t) ALLK(2, t) ALLK(3, t) ALLK(4, t)
    }
    return 0;
}
