// Dev probe: does s_barrier still release when some waves of the workgroup
// have already ended (s_endpgm)?  Waves 4..7 of a 512-thread workgroup return
// at once; waves 0..3 then pass 33 LDS barriers and write a checksum.  Run it
// under `timeout`: if ended waves still counted, the kernel would never end.
//   hipcc -O3 --offload-arch=gfx950 barrier_exit.hip -o barrier_exit
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(512) void k_exit(unsigned* out) {
    __shared__ unsigned buf[256];
    const unsigned t = threadIdx.x;
    if (t >= 256) return;                       // waves 4..7 end here
    buf[t] = t;
    for (int r = 0; r < 16; r++) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const unsigned v = buf[(t + 1) & 255];
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        buf[t] = v + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t == 0) {
        unsigned s = 0;
        for (int i = 0; i < 256; i++) s += buf[i];
        out[0] = s;
    }
}

int main() {
    unsigned* d;
    CK(hipMalloc(&d, 4));
    CK(hipMemset(d, 0, 4));
    hipLaunchKernelGGL(k_exit, dim3(1), dim3(512), 0, 0, d);
    CK(hipDeviceSynchronize());
    unsigned h = 0;
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    // each round rotates and adds 1: sum = 0+..+255 + 16*256
    const unsigned want = 255u * 256u / 2u + 16u * 256u;
    printf("barrier after early exit: sum %u (want %u) -> %s\n", h, want, h == want ? "ok" : "MISMATCH");
    return h == want ? 0 : 1;
}
