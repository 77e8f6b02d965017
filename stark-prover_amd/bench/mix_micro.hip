// mix_micro.hip — how a SIMD issues a MIX of half-rate (v_alignbit_b32,
// v_add3_u32) and full-rate (v_bitop3_b32, v_add_u32) wave64 instructions
// (gfx950).  Each pattern is 16 instructions per iteration on independent
// register chains, in a fixed order (one asm block per iteration), run by the
// whole chip; prints wave-instructions per quad-cycle per SIMD at the clock
// measured from s_memtime (not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// H = half rate (alignbit), F = full rate (bitop3); 16 instructions, 8 H + 8 F
#define H(d, a) "v_alignbit_b32 " d ", " a ", " a ", 7\n\t"
#define F(d, a, b) "v_bitop3_b32 " d ", " a ", " b ", " d " bitop3:0x96\n\t"

__global__ __launch_bounds__(256) void k_alt(unsigned* out, int iters) {      // H F H F ...
    unsigned r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 + 1, r5 = r0 + 2, r6 = r0 + 3, r7 = r0 + 4;
    for (int it = 0; it < iters; it++) {
        asm volatile(H("%0", "%0") F("%4", "%5", "%6") H("%1", "%1") F("%5", "%6", "%7") H("%2", "%2") F("%6", "%7", "%4")
                     H("%3", "%3") F("%7", "%4", "%5") H("%0", "%0") F("%4", "%5", "%6") H("%1", "%1") F("%5", "%6", "%7")
                     H("%2", "%2") F("%6", "%7", "%4") H("%3", "%3") F("%7", "%4", "%5")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}
__global__ __launch_bounds__(256) void k_clu(unsigned* out, int iters) {      // HHHHHHHH FFFFFFFF
    unsigned r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 + 1, r5 = r0 + 2, r6 = r0 + 3, r7 = r0 + 4;
    for (int it = 0; it < iters; it++) {
        asm volatile(H("%0", "%0") H("%1", "%1") H("%2", "%2") H("%3", "%3") H("%0", "%0") H("%1", "%1") H("%2", "%2")
                     H("%3", "%3") F("%4", "%5", "%6") F("%5", "%6", "%7") F("%6", "%7", "%4") F("%7", "%4", "%5")
                     F("%4", "%5", "%6") F("%5", "%6", "%7") F("%6", "%7", "%4") F("%7", "%4", "%5")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}
__global__ __launch_bounds__(256) void k_pair(unsigned* out, int iters) {     // HH FF HH FF ...
    unsigned r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 + 1, r5 = r0 + 2, r6 = r0 + 3, r7 = r0 + 4;
    for (int it = 0; it < iters; it++) {
        asm volatile(H("%0", "%0") H("%1", "%1") F("%4", "%5", "%6") F("%5", "%6", "%7") H("%2", "%2") H("%3", "%3")
                     F("%6", "%7", "%4") F("%7", "%4", "%5") H("%0", "%0") H("%1", "%1") F("%4", "%5", "%6")
                     F("%5", "%6", "%7") H("%2", "%2") H("%3", "%3") F("%6", "%7", "%4") F("%7", "%4", "%5")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}
__global__ __launch_bounds__(256) void k_allh(unsigned* out, int iters) {     // 16 H
    unsigned r0 = threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7;
    for (int it = 0; it < iters; it++) {
        asm volatile(H("%0", "%0") H("%1", "%1") H("%2", "%2") H("%3", "%3") H("%0", "%0") H("%1", "%1") H("%2", "%2")
                     H("%3", "%3") H("%0", "%0") H("%1", "%1") H("%2", "%2") H("%3", "%3") H("%0", "%0") H("%1", "%1")
                     H("%2", "%2") H("%3", "%3")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3;
}
__global__ __launch_bounds__(256) void k_allf(unsigned* out, int iters) {     // 16 F
    unsigned r4 = threadIdx.x + 1, r5 = r4 * 3, r6 = r4 * 5, r7 = r4 * 7;
    for (int it = 0; it < iters; it++) {
        asm volatile(F("%0", "%1", "%2") F("%1", "%2", "%3") F("%2", "%3", "%0") F("%3", "%0", "%1") F("%0", "%1", "%2")
                     F("%1", "%2", "%3") F("%2", "%3", "%0") F("%3", "%0", "%1") F("%0", "%1", "%2") F("%1", "%2", "%3")
                     F("%2", "%3", "%0") F("%3", "%0", "%1") F("%0", "%1", "%2") F("%1", "%2", "%3") F("%2", "%3", "%0")
                     F("%3", "%0", "%1")
                     : "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r4 ^ r5 ^ r6 ^ r7;
}
__global__ void k_clock(unsigned long long* t) {
    unsigned long long a = __builtin_amdgcn_s_memtime(), b = __builtin_amdgcn_s_memrealtime();
    t[0] = a; t[1] = b;
}

int main() {
    unsigned* o;
    unsigned long long* tc;
    CK(hipMalloc(&o, 8192 * 256 * 4));
    CK(hipMalloc(&tc, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    struct K { const char* n; void (*f)(unsigned*, int); };
    K ks[] = {{"16 H (alignbit)", k_allh}, {"16 F (bitop3)", k_allf}, {"H F H F ... (alternating)", k_alt},
              {"HH FF HH FF ...", k_pair}, {"8 H then 8 F (clustered)", k_clu}};
    const int iters = 4096;
    for (int blocks : {1024, 2048, 4096, 8192}) {      // 1, 2, 4, 8 waves per SIMD
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, o, iters);
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k_clock, dim3(1), dim3(1), 0, 0, tc);
            unsigned long long h0[2], h1[2];
            CK(hipMemcpy(h0, tc, 16, hipMemcpyDeviceToHost));
            CK(hipEventRecord(a));
            for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, o, iters);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            hipLaunchKernelGGL(k_clock, dim3(1), dim3(1), 0, 0, tc);
            CK(hipMemcpy(h1, tc, 16, hipMemcpyDeviceToHost));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            ms /= 3;
            const double ghz = (double)(h1[0] - h0[0]) / ((double)(h1[1] - h0[1]) / 100e6) / 1e9;   // memrealtime: 100 MHz
            const double winstr = (double)blocks * 4 * iters * 16;                                // 4 waves per block
            const double per_simd = winstr / 1024;
            const double quads = ms * 1e-3 * ghz * 1e9 / 4;
            printf("%5d WG (%d waves/SIMD) %-28s %7.3f ms  clk %.2f GHz  %.2f wave-instr per quad-cycle per SIMD\n",
                   blocks, blocks / 1024, k.n, ms, ghz, per_simd / quads);
        }
    }
    return 0;
}
