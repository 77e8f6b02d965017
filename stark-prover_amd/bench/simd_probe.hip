// Dev probe: which SIMD each wave of a 512-thread workgroup lands on
// (HW_REG_HW_ID).  Measured on gfx950: waves 0-3 on four different SIMDs,
// wave 4+i on the SIMD of wave i.
//   hipcc -O3 --offload-arch=gfx950 simd_probe.hip -o simd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void k(unsigned* out) {
    unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = hw;
}
int main() {
    unsigned* d; (void)hipMalloc(&d, 64 * 8 * 4);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(rep == 2 ? 4 : 1), dim3(512), 0, 0, d);
        (void)hipDeviceSynchronize();
        unsigned h[32]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        int nb = rep == 2 ? 4 : 1;
        for (int b = 0; b < nb; b++) {
            printf("launch %d wg %d:", rep, b);
            for (int w = 0; w < 8; w++) printf("  w%d simd%u wave%u cu%u", w, (h[b*8+w] >> 4) & 3, h[b*8+w] & 15, (h[b*8+w] >> 8) & 15);
            printf("\n");
        }
    }
    return 0;
}
