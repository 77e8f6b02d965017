// Dev probe: does a lone wave slow down over time when the rest of the chip
// is idle (power management lowering the shader clock)?  One wave runs a
// fixed dependent VALU chain per iteration and records s_memrealtime
// (100 MHz, constant) and s_memtime per iteration.  Mode 1 runs the same
// probe while a second stream keeps 240 other workgroups busy.
//   hipcc -O3 --offload-arch=gfx950 clock_probe.hip -o clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int ITERS = 4000;

__global__ void k_probe(unsigned long long* rt, unsigned long long* mt, unsigned* sink) {
    unsigned x = threadIdx.x + 1, c = threadIdx.x * 3 + 7;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int j = 0; j < 256; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));
        if (threadIdx.x == 0) { rt[it] = __builtin_amdgcn_s_memrealtime(); mt[it] = __builtin_amdgcn_s_memtime(); }
    }
    sink[threadIdx.x] = x;
}

__global__ void k_busy(unsigned* sink, volatile unsigned* stop) {
    unsigned x = threadIdx.x + 1, c = blockIdx.x;
    for (int it = 0; it < 200000; it++) {
#pragma unroll
        for (int j = 0; j < 64; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));
        if ((it & 255) == 0 && *stop) break;
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    unsigned long long *rt, *mt;
    unsigned *sink, *stop;
    CK(hipMalloc(&rt, ITERS * 8));
    CK(hipMalloc(&mt, ITERS * 8));
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipHostMalloc(&stop, 4, hipHostMallocDefault));
    hipStream_t s1, s2;
    CK(hipStreamCreate(&s1));
    CK(hipStreamCreate(&s2));
    static unsigned long long hrt[ITERS], hmt[ITERS];
    for (int mode = 0; mode < 2; mode++) {
        *stop = 0;
        if (mode == 1) hipLaunchKernelGGL(k_busy, dim3(240), dim3(64), 0, s2, sink + 1024, stop);
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s1, rt, mt, sink);
        CK(hipStreamSynchronize(s1));
        *stop = 1;
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hrt, rt, sizeof(hrt), hipMemcpyDeviceToHost));
        CK(hipMemcpy(hmt, mt, sizeof(hmt), hipMemcpyDeviceToHost));
        printf("mode %d (%s)\n", mode, mode ? "240 busy workgroups beside" : "alone");
        for (int it = 1; it < ITERS; it += (it < 40 ? 4 : 250)) {
            double ns = (hrt[it] - hrt[it - 1]) * 10.0, cyc = (double)(hmt[it] - hmt[it - 1]);
            printf("  iter %5d  t=%8.1f us  %6.1f ns/iter  %6.0f memtime/iter  -> %.2f GHz (memtime/realtime)\n", it,
                   (hrt[it] - hrt[0]) / 100.0, ns, cyc, cyc / ns);
        }
    }
    return 0;
}
