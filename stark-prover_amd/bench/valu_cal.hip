// valu_cal.hip — per-instruction VALU throughput on gfx950 (wave64), used to
// build the SHA-256 / field-arithmetic cost model (DESIGN.md "VALU costs").
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

#define BODY3(INS) asm volatile(INS " %0, %1, %2, %3" : "=v"(r[i]) : "v"(r[i]), "v"(r[(i + 1) & 15]), "v"(r[(i + 5) & 15]))
#define BODY2(INS) asm volatile(INS " %0, %1, %2" : "=v"(r[i]) : "v"(r[i]), "v"(r[(i + 1) & 15]))
#define BODY1(INS) asm volatile(INS " %0, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 15]))
#define BODYSH(INS) asm volatile(INS " %0, 7, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 15]))
#define BODYALIGN(INS) asm volatile(INS " %0, %1, %2, 7" : "=v"(r[i]) : "v"(r[i]), "v"(r[(i + 1) & 15]))
#define BODYLSHOR(INS) asm volatile(INS " %0, %1, 7, %2" : "=v"(r[i]) : "v"(r[i]), "v"(r[(i + 1) & 15]))
#define BODYBOP(INS) asm volatile(INS " %0, %1, %2, %3 bitop3:0x96" : "=v"(r[i]) : "v"(r[i]), "v"(r[(i + 1) & 15]), "v"(r[(i + 5) & 15]))

#define KERNEL(NAME, BODY, INS)                                                           \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, int iters) {               \
        unsigned r[16];                                                                   \
        for (int i = 0; i < 16; i++) r[i] = threadIdx.x * 7 + i;                          \
        for (int it = 0; it < iters; it++) {                                              \
            _Pragma("unroll") for (int i = 0; i < 16; i++) BODY(INS);                     \
        }                                                                                 \
        unsigned x = 0;                                                                   \
        for (int i = 0; i < 16; i++) x ^= r[i];                                           \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                   \
    }

KERNEL(k_add, BODY2, "v_add_u32")
KERNEL(k_xor, BODY2, "v_xor_b32")
KERNEL(k_lshr, BODYSH, "v_lshrrev_b32")
KERNEL(k_add3, BODY3, "v_add3_u32")
KERNEL(k_xor3, BODYBOP, "v_bitop3_b32")
KERNEL(k_alignbit, BODYALIGN, "v_alignbit_b32")
KERNEL(k_lshl_or, BODYLSHOR, "v_lshl_or_b32")
KERNEL(k_lshl_add, BODYLSHOR, "v_lshl_add_u32")
KERNEL(k_xad, BODY3, "v_xad_u32")
KERNEL(k_bfi, BODY3, "v_bfi_b32")
KERNEL(k_or3, BODY3, "v_or3_b32")
KERNEL(k_and_or, BODY3, "v_and_or_b32")
KERNEL(k_perm, BODY3, "v_perm_b32")
KERNEL(k_mul_lo, BODY2, "v_mul_lo_u32")
KERNEL(k_mul_hi, BODY2, "v_mul_hi_u32")
KERNEL(k_mad24, BODY3, "v_mad_u32_u24")
KERNEL(k_mov, BODY1, "v_mov_b32")
KERNEL(k_not, BODY1, "v_not_b32")

// 64-bit shift: pair (x,x) >> 7 gives rotr(x,7) in the low half
__global__ __launch_bounds__(256) void k_lshr64(unsigned* out, int iters) {
    unsigned long long r[8];
    for (int i = 0; i < 8; i++) r[i] = (unsigned long long)(threadIdx.x * 7 + i) * 0x100000001ull;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_lshrrev_b64 %0, 7, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 7]));
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= (unsigned)r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ __launch_bounds__(256) void k_mad64(unsigned* out, int iters) {
    unsigned long long r[8];
    unsigned s = threadIdx.x;
    for (int i = 0; i < 8; i++) r[i] = (unsigned long long)(threadIdx.x * 7 + i) * 0x100000001ull;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r[i]) : "v"((unsigned)r[(i + 1) & 7]), "v"(s), "v"(r[(i + 3) & 7]) : "vcc");
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= (unsigned)r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// Sigma-style rotations: 3 alignbit + xor3 vs (x,x) pair + 3 64-bit shifts + xor3
__global__ __launch_bounds__(256) void k_sig_align(unsigned* out, int iters) {
    unsigned r[8];
    for (int i = 0; i < 8; i++) r[i] = threadIdx.x * 7 + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            unsigned a, b, c, x = r[i];
            asm volatile("v_alignbit_b32 %0, %1, %1, 6" : "=v"(a) : "v"(x));
            asm volatile("v_alignbit_b32 %0, %1, %1, 11" : "=v"(b) : "v"(x));
            asm volatile("v_alignbit_b32 %0, %1, %1, 25" : "=v"(c) : "v"(x));
            asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r[i]) : "v"(a), "v"(b), "v"(c));
        }
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ __launch_bounds__(256) void k_sig_64(unsigned* out, int iters) {
    unsigned r[8];
    for (int i = 0; i < 8; i++) r[i] = threadIdx.x * 7 + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            unsigned long long p, a, b, c;
            asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[0,0]" : "=v"(p) : "v"((unsigned long long)r[i]));
            asm volatile("v_lshrrev_b64 %0, 6, %1" : "=v"(a) : "v"(p));
            asm volatile("v_lshrrev_b64 %0, 11, %1" : "=v"(b) : "v"(p));
            asm volatile("v_lshrrev_b64 %0, 25, %1" : "=v"(c) : "v"(p));
            asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r[i]) : "v"((unsigned)a), "v"((unsigned)b), "v"((unsigned)c));
        }
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ __launch_bounds__(256) void k_pkmov(unsigned* out, int iters) {
    unsigned long long r[8];
    for (int i = 0; i < 8; i++) r[i] = (unsigned long long)(threadIdx.x * 7 + i) * 0x100000001ull;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]" : "=v"(r[i]) : "v"(r[(i + 1) & 7]));
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= (unsigned)r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ __launch_bounds__(256) void k_lshladd64(unsigned* out, int iters) {
    unsigned long long r[8];
    for (int i = 0; i < 8; i++) r[i] = (unsigned long long)(threadIdx.x * 7 + i) * 0x100000001ull;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_lshl_add_u64 %0, %1, 3, %2" : "=v"(r[i]) : "v"(r[(i + 1) & 7]), "v"(r[(i + 3) & 7]));
    }
    unsigned x = 0;
    for (int i = 0; i < 8; i++) x ^= (unsigned)r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
KERNEL(k_pklshr16, BODYSH, "v_pk_lshrrev_b16")

int main() {
    unsigned* o;
    CK(hipMalloc(&o, 4096 * 256 * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    struct K { const char* n; void (*f)(unsigned*, int); int per; };
    K ks[] = {{"v_add_u32", k_add, 16}, {"v_xor_b32", k_xor, 16}, {"v_lshrrev_b32", k_lshr, 16},
              {"v_add3_u32", k_add3, 16}, {"v_bitop3_b32", k_xor3, 16}, {"v_alignbit_b32", k_alignbit, 16},
              {"v_lshl_or_b32", k_lshl_or, 16}, {"v_lshl_add_u32", k_lshl_add, 16}, {"v_xad_u32", k_xad, 16},
              {"v_bfi_b32", k_bfi, 16}, {"v_or3_b32", k_or3, 16}, {"v_and_or_b32", k_and_or, 16},
              {"v_perm_b32", k_perm, 16}, {"v_mul_lo_u32", k_mul_lo, 16}, {"v_mul_hi_u32", k_mul_hi, 16},
              {"v_mad_u32_u24", k_mad24, 16}, {"v_mov_b32", k_mov, 16}, {"v_not_b32", k_not, 16},
              {"v_lshrrev_b64", k_lshr64, 8}, {"v_mad_u64_u32", k_mad64, 8}, {"Sigma align x3+xor3 (4 ins)", k_sig_align, 8}, {"Sigma pkmov+lshr64x3+xor3 (5 ins)", k_sig_64, 8}, {"v_pk_mov_b32", k_pkmov, 8}, {"v_lshl_add_u64", k_lshladd64, 8}, {"v_pk_lshrrev_b16", k_pklshr16, 16}};
    const int iters = 2048;
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(4096), dim3(256), 0, 0, o, iters);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int rep = 0; rep < 5; rep++) hipLaunchKernelGGL(k.f, dim3(4096), dim3(256), 0, 0, o, iters);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
        double ops = 4096.0 * 256 * iters * k.per;
        double waveinstr_per_simd = ops / 64 / 1024;
        printf("%-16s %7.3f ms  %6.1f T lane-ops/s  %5.2f ns per wave-instr per SIMD\n", k.n, ms, ops / (ms * 1e-3) / 1e12,
               ms * 1e6 / waveinstr_per_simd);
    }
    return 0;
}
