// fri_prover.hip — prover slice around the FRI commit (SURVEY.md §8(f) rank 2,
// BASELINE configs[3]): the STARK-101 FibonacciSq composition polynomial in
// evaluation form on the LDE coset, and the trace-tree decommitment gather.
//
// The reference's src/prover, src/trace and src/composition are empty files;
// the constraint system is STARK-101's (the crate is `stark-101`,
// Cargo.toml:2), restated on the full trace subgroup G = <g>, |G| = T:
//     a_0 = 1,  a_{T-1} = A,  a_{i+2} = a_{i+1}^2 + a_i^2  (i <= T-3)
//     p0 = (f(x) - 1) / (x - 1)
//     p1 = (f(x) - A) / (x - g^{T-1})
//     p2 = (f(g^2 x) - f(g x)^2 - f(x)^2) * (x - g^{T-2})(x - g^{T-1}) / (x^T - 1)
//     CP = alpha0 p0 + alpha1 p1 + alpha2 p2            (deg CP <= T)
// On the LDE coset x_i = offset * w_n^i (n = B*T) the shifts are index shifts:
// g = w_n^B, so f(g x_i) = f[i + B], f(g^2 x_i) = f[i + 2B] (mod n), and
// x_i^T = offset^T * w_B^(i mod B) takes B values (host-inverted table).
// The two per-point divisions share one batch inversion (Montgomery's trick
// over CP_K consecutive points per lane, one Fermat inverse per lane).
#include "fri_internal.hpp"

namespace fri {

constexpr uint32_t CP_K = 16;     // points per lane

__global__ __launch_bounds__(256) void k_fibsq_cp(const uint32_t* __restrict__ f, uint32_t* __restrict__ out,
                                                  FibsqParams q) {
    const size_t n = (size_t)1 << q.log_n;
    const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * CP_K;
    if (i0 >= n) return;
    const size_t mask = n - 1;
    const uint32_t one_m = R_MOD_P;
    // x_{i0} = offset * w^{i0} (Montgomery), then x_{i+1} = x_i * w
    uint32_t x = mmul(q.offset_m, mpow(q.w_m, i0));
    uint32_t xa[CP_K], xb[CP_K], pre[CP_K];
    uint32_t acc = one_m;
#pragma unroll
    for (uint32_t k = 0; k < CP_K; k++) {
        xa[k] = sub(x, one_m);              // (x - 1)        Montgomery
        xb[k] = sub(x, q.glast_m);          // (x - g^{T-1})  Montgomery
        pre[k] = acc;
        acc = mmul(acc, mmul(xa[k], xb[k]));
        x = mmul(x, q.w_m);
    }
    // x_i != 1 and x_i != g^{T-1}: the coset is disjoint from G, so acc != 0
    uint32_t inv = mpow(acc, P - 2);
    x = mmul(q.offset_m, mpow(q.w_m, i0 + CP_K - 1));
#pragma unroll
    for (int k = CP_K - 1; k >= 0; k--) {
        const uint32_t dinv = mmul(inv, pre[k]);           // 1 / ((x-1)(x-g^{T-1}))
        inv = mmul(inv, mmul(xa[k], xb[k]));
        const size_t i = i0 + k;
        const uint32_t fi = f[i], f1 = f[(i + q.B) & mask], f2 = f[(i + 2 * q.B) & mask];
        const uint32_t p0 = mmul(sub(fi, 1u), mmul(dinv, xb[k]));        // (f-1)/(x-1)
        const uint32_t p1 = mmul(sub(fi, q.a_last), mmul(dinv, xa[k]));  // (f-A)/(x-g^{T-1})
        const uint32_t sq = add(mmul(f1, to_mont(f1)), mmul(fi, to_mont(fi)));
        const uint32_t num2 = sub(f2, sq);
        const uint32_t zf = mmul(mmul(sub(x, q.gprev_m), xb[k]), q.zinv_m[i & (q.B - 1)]);
        const uint32_t p2 = mmul(num2, zf);
        out[i] = add(add(mmul(p0, q.alpha_m[0]), mmul(p1, q.alpha_m[1])), mmul(p2, q.alpha_m[2]));
        x = mmul(x, q.winv_m);
    }
}

void launch_fibsq_cp(const uint32_t* f_lde, uint32_t* out, const FibsqParams& q, hipStream_t s) {
    const size_t lanes = (((size_t)1 << q.log_n) + CP_K - 1) / CP_K;
    hipLaunchKernelGGL(k_fibsq_cp, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, f_lde, out, q);
}

// Trace-tree decommitment (STARK-101 decommit_on_query): values at
// index + j*stride (j < count) and their authentication paths, sibling
// digests leaf -> root as big-endian bytes.  Block j, lane l = level l.
__global__ void k_trace_gather(const uint32_t* __restrict__ lde, const uint32_t* __restrict__ tree, uint32_t L,
                               uint64_t index, uint64_t stride, uint32_t* __restrict__ out, uint32_t count) {
    const uint32_t j = blockIdx.x;
    const uint64_t leaf = (index + j * stride) & (((uint64_t)1 << L) - 1);
    if (threadIdx.x == 0) out[j] = lde[leaf];
    const uint32_t l = threadIdx.x;
    if (l >= L) return;
    const uint32_t* d = tree + 8 * (level_offset(L, l) + ((leaf >> l) ^ 1u));
    uint32_t* o = out + count + (size_t)j * 8 * L + 8 * l;
#pragma unroll
    for (int w = 0; w < 8; w++) o[w] = __builtin_bswap32(d[w]);
}

void launch_trace_gather(const uint32_t* lde, const uint32_t* tree, uint32_t L, uint64_t index, uint64_t stride,
                         uint32_t count, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_trace_gather, dim3(count), dim3(64), 0, s, lde, tree, L, index, stride, out, count);
}

}  // namespace fri
