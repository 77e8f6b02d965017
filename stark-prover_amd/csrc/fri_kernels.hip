// fri_kernels.hip — gfx950 kernels of the FRI commit path.
//
//   NTT (coset LDE / interpolation)  replaces Horner evaluate at every domain
//                                     point (src/fri/fri_commit.rs:78,
//                                     src/polynomial/ops.rs:76-83) and Lagrange
//                                     interpolation (interpolation.rs:121-152)
//   Merkle subtree                    replaces MerkleTree::new (src/merkle/mod.rs:10-22)
//   fold (evaluation form)            replaces next_fri_layer (src/fri/fri_commit.rs:53-65)
//   coefficient fold                  next_fri_polynomial (fri_commit.rs:32-50), O(d),
//                                     kept for the exact degree / loop condition (:89)
//   channel step (single lane)        Channel::send / receive_random_field_element
//                                     (src/channel/channel.rs:35-55) on the device
//   batch inverse                     FieldElement::inverse (element.rs:54-57), 0 -> 0
//
// Data in HBM is canonical u32 (value < p); constants are Montgomery (field.hpp).
#include "fri_internal.hpp"
#include "sha256.hpp"

namespace fri {

// ============================================================== NTT ======
// Natural order in -> natural order out.  Pass 1 gathers the input in
// bit-reversed order (optionally scaled by pre(j) = s^j: the coset shift of
// the LDE) into a 4096-element LDS tile and runs the first <= 12 DIT stages;
// each further pass runs <= 10 stages on LDS tiles of 16 contiguous columns
// x 1024 strided rows (64-byte coalesced runs).  Twiddles come from one
// Montgomery table of the largest transform (index stride for smaller ones).

__device__ __forceinline__ uint32_t pow2lvl(const uint32_t* lo, const uint32_t* hi, size_t j, uint32_t v) {
    return mmul(mmul(v, hi[j >> POW_LO_LOG]), lo[j & ((1u << POW_LO_LOG) - 1)]);
}

__global__ __launch_bounds__(256) void k_ntt_first(const uint32_t* __restrict__ src, size_t d,
                                                   uint32_t* __restrict__ dst, uint32_t log_n, uint32_t tb,
                                                   const uint32_t* __restrict__ tw,
                                                   const uint32_t* __restrict__ pre_lo,
                                                   const uint32_t* __restrict__ pre_hi,
                                                   const uint32_t* __restrict__ post_lo,
                                                   const uint32_t* __restrict__ post_hi) {
    __shared__ uint32_t lds[1u << NTT_TILE_LOG];
    __shared__ uint32_t twl[1u << NTT_TILE_LOG];
    const uint32_t T = 1u << tb;
    const size_t base = (size_t)blockIdx.x << tb;
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) twl[i] = tw[i];
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) {
        uint32_t pos = (uint32_t)(base + i);
        uint32_t si = log_n ? (__brev(pos) >> (32 - log_n)) : 0u;
        uint32_t v = 0;
        if (si < d) {
            v = src[si];
            if (pre_lo) v = pow2lvl(pre_lo, pre_hi, si, v);
        }
        lds[i] = v;
    }
    __syncthreads();
    for (uint32_t s = 0; s < tb; s++) {
        const uint32_t h = 1u << s;
        for (uint32_t b = threadIdx.x; b < T / 2; b += blockDim.x) {
            uint32_t j = b & (h - 1);
            uint32_t i0 = ((b >> s) << (s + 1)) + j, i1 = i0 + h;
            uint32_t w = twl[h + j];
            uint32_t u = lds[i0], v = mmul(lds[i1], w);
            lds[i0] = add(u, v);
            lds[i1] = sub(u, v);
        }
        __syncthreads();
    }
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) {
        uint32_t v = lds[i];
        if (post_lo) v = pow2lvl(post_lo, post_hi, base + i, v);
        dst[base + i] = v;
    }
}

__global__ __launch_bounds__(256) void k_ntt_mid(uint32_t* __restrict__ data, uint32_t log_n, uint32_t s0,
                                                 uint32_t ns, const uint32_t* __restrict__ tw,
                                                 const uint32_t* __restrict__ post_lo,
                                                 const uint32_t* __restrict__ post_hi) {
    __shared__ uint32_t lds[NTT_MID_W << NTT_MID_LOG];
    const uint32_t W = NTT_MID_W, M = 1u << ns;
    const uint32_t nlo = (1u << s0) / W;
    const uint32_t lo0 = (blockIdx.x % nlo) * W;
    const size_t hib = ((size_t)(blockIdx.x / nlo)) << (s0 + ns);
    for (uint32_t e = threadIdx.x; e < W * M; e += blockDim.x) {
        uint32_t lo = e % W, mid = e / W;
        lds[e] = data[hib + ((size_t)mid << s0) + lo0 + lo];
    }
    __syncthreads();
    for (uint32_t t = 0; t < ns; t++) {
        const uint32_t s = s0 + t, hm = 1u << t;
        for (uint32_t b = threadIdx.x; b < W * M / 2; b += blockDim.x) {
            uint32_t lo = b % W, bm = b / W;
            uint32_t jm = bm & (hm - 1);
            uint32_t m0 = ((bm >> t) << (t + 1)) + jm, m1 = m0 + hm;
            uint32_t j = lo0 + lo + (jm << s0);
            uint32_t w = tw[((size_t)1 << s) + j];
            uint32_t u = lds[m0 * W + lo], v = mmul(lds[m1 * W + lo], w);
            lds[m0 * W + lo] = add(u, v);
            lds[m1 * W + lo] = sub(u, v);
        }
        __syncthreads();
    }
    for (uint32_t e = threadIdx.x; e < W * M; e += blockDim.x) {
        uint32_t lo = e % W, mid = e / W;
        size_t idx = hib + ((size_t)mid << s0) + lo0 + lo;
        uint32_t v = lds[e];
        if (post_lo) v = pow2lvl(post_lo, post_hi, idx, v);
        data[idx] = v;
    }
}

void launch_ntt(const NttPlan& p, const uint32_t* src, size_t d, uint32_t* dst, hipStream_t s) {
    const uint32_t log_n = p.log_n;
    const uint32_t tb = log_n < NTT_TILE_LOG ? log_n : NTT_TILE_LOG;
    const bool single = (tb == log_n);
    const uint32_t nblk = 1u << (log_n - tb);
    hipLaunchKernelGGL(k_ntt_first, dim3(nblk), dim3(256), 0, s, src, d, dst, log_n, tb, p.tw,
                       p.pre_lo, p.pre_hi, single ? p.post_lo : nullptr, single ? p.post_hi : nullptr);
    for (uint32_t s0 = tb; s0 < log_n;) {
        uint32_t ns = (log_n - s0) < NTT_MID_LOG ? (log_n - s0) : NTT_MID_LOG;
        bool last = (s0 + ns == log_n);
        uint32_t blocks = (uint32_t)(((size_t)1 << log_n) / ((size_t)NTT_MID_W << ns));
        hipLaunchKernelGGL(k_ntt_mid, dim3(blocks), dim3(256), 0, s, dst, log_n, s0, ns, p.tw,
                           last ? p.post_lo : nullptr, last ? p.post_hi : nullptr);
        s0 += ns;
    }
}

// Stage-packed twiddles: tw[2^s + j] = Montgomery(w_{2^(s+1)}^j), so every
// DIT stage s reads a contiguous run (independent of the transform size).
struct StageBases { uint32_t b[32]; };
__global__ void k_twiddles(uint32_t* tw, size_t count, StageBases sb) {
    size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    if (e == 0) { tw[0] = R_MOD_P; return; }
    uint32_t s = 63u - (uint32_t)__clzll((unsigned long long)e);
    tw[e] = mpow(sb.b[s], e - ((size_t)1 << s));
}
void launch_twiddles(uint32_t* tw, uint32_t log_max, bool inverse, hipStream_t s) {
    StageBases sb{};
    for (uint32_t st = 0; st < log_max && st < 31; st++) {
        uint32_t w = root_of_unity(st + 1);
        sb.b[st] = to_mont(inverse ? inv_std(w) : w);
    }
    size_t count = (size_t)1 << log_max;
    hipLaunchKernelGGL(k_twiddles, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, tw, count, sb);
}

// Two-level power table of base^j scaled by `scale`: lo[t] = base^t,
// hi[t] = scale * base^(4096 t)  (Montgomery).
__global__ void k_pow_table(uint32_t* lo, uint32_t* hi, uint32_t nhi, uint32_t base_m, uint32_t scale_m) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nlo = 1u << POW_LO_LOG;
    if (t < nlo) lo[t] = mpow(base_m, t);
    else if (t < nlo + nhi) {
        uint32_t q = t - nlo;
        hi[q] = mmul(scale_m, mpow(base_m, (uint64_t)q << POW_LO_LOG));
    }
}
void launch_pow_table(uint32_t* lo, uint32_t* hi, uint32_t log_n, uint32_t base_std, uint32_t scale_std,
                      hipStream_t s) {
    uint32_t nhi = log_n > POW_LO_LOG ? (1u << (log_n - POW_LO_LOG)) : 1u;
    uint32_t tot = (1u << POW_LO_LOG) + nhi;
    hipLaunchKernelGGL(k_pow_table, dim3((tot + 255) / 256), dim3(256), 0, s, lo, hi, nhi, to_mont(base_std),
                       to_mont(scale_std));
}

// ========================================================= batch inverse ==
// Montgomery's trick per thread over BI_K strided elements (coalesced), one
// Fermat inversion per thread; zeros are skipped and map to 0 exactly like
// FieldElement::inverse (0^(p-2) = 0).
constexpr uint32_t BI_K = 16;
__global__ __launch_bounds__(256) void k_batch_inverse(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       size_t n, size_t stride, int out_mont) {
    size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= stride) return;
    uint32_t a[BI_K], pre[BI_K];
    uint32_t acc = R_MOD_P;
#pragma unroll
    for (uint32_t k = 0; k < BI_K; k++) {
        size_t i = g + k * stride;
        uint32_t x = i < n ? in[i] : 0u;
        a[k] = x ? to_mont(x) : 0u;
        pre[k] = acc;
        if (x) acc = mmul(acc, a[k]);
    }
    uint32_t inv = mpow(acc, P - 2);
#pragma unroll
    for (int k = BI_K - 1; k >= 0; k--) {
        size_t i = g + (size_t)k * stride;
        uint32_t r = 0;
        if (a[k]) { r = mmul(inv, pre[k]); inv = mmul(inv, a[k]); }
        if (i < n) out[i] = out_mont ? r : from_mont(r);
    }
}
void launch_batch_inverse(const uint32_t* in, uint32_t* out, size_t n, int out_mont, hipStream_t s) {
    size_t stride = (n + BI_K - 1) / BI_K;
    if (!stride) return;
    hipLaunchKernelGGL(k_batch_inverse, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, s, in, out, n, stride,
                       out_mont);
}

// out[i] = offset * w_n^i (canonical)
__global__ void k_coset_points(uint32_t* out, size_t count, uint32_t off, uint32_t w_m) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = mmul(off, mpow(w_m, i));
}
void launch_coset_points(uint32_t* out, size_t count, uint32_t offset, uint32_t log_n, hipStream_t s) {
    hipLaunchKernelGGL(k_coset_points, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, out, count, offset,
                       to_mont(root_of_unity(log_n)));
}

__global__ void k_square_mont(const uint32_t* in, uint32_t* out, size_t count) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) { uint32_t x = in[i]; out[i] = mmul(x, x); }
}
void launch_square_mont(const uint32_t* in, uint32_t* out, size_t count, hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(k_square_mont, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, in, out, count);
}

// Horner at arbitrary points (ops.rs:76-83): one lane per point.
__global__ void k_evaluate(const uint32_t* __restrict__ c, size_t d, const uint32_t* __restrict__ xs, size_t count,
                           uint32_t* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    uint32_t xm = to_mont(xs[i]), r = 0;
    for (size_t k = d; k-- > 0;) r = add(mmul(r, xm), c[k]);
    out[i] = r;
}
void launch_evaluate(const uint32_t* coeffs, size_t d, const uint32_t* xs, size_t count, uint32_t* out,
                     hipStream_t s) {
    if (!count) return;
    hipLaunchKernelGGL(k_evaluate, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, coeffs, d, xs, count, out);
}

// ================================================================== fold ==
// L'[i] = 2^-1 * ((a+b) + beta*(a-b)*x_i^-1),  a = L[i], b = L[i+m/2] = L(-x_i).
// xinv_m[i] = Montgomery(x_i^-1) for the layer's domain.
constexpr uint32_t INV2_M = 0x80000000u;   // Montgomery(2^-1) = 2^31 mod p (static_assert below)
static_assert(((unsigned __int128)INV2_M * 2) % P == R_MOD_P, "INV2_M");

__device__ __forceinline__ uint32_t fold_one(uint32_t a, uint32_t b, uint32_t xinv_m, uint32_t beta_m) {
    uint32_t s = add(a, b), t = sub(a, b);
    uint32_t v = mmul(mmul(t, xinv_m), beta_m);
    return mmul(add(s, v), INV2_M);
}

__global__ __launch_bounds__(256) void k_fold(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                              size_t half, const uint32_t* __restrict__ xinv_m, uint32_t beta_m,
                                              const DevState* __restrict__ st, int r) {
    if (st && !st->active[r]) return;
    if (st) beta_m = st->beta_mont[r];
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < half) out[i] = fold_one(in[i], in[i + half], xinv_m[i], beta_m);
}
void launch_fold_plain(const uint32_t* in, uint32_t* out, uint32_t log_m, const uint32_t* xinv_m, uint32_t beta,
                       hipStream_t s) {
    size_t half = ((size_t)1 << log_m) / 2;
    hipLaunchKernelGGL(k_fold, dim3((unsigned)((half + 255) / 256)), dim3(256), 0, s, in, out, half, xinv_m,
                       to_mont(beta), (const DevState*)nullptr, 0);
}

}  // namespace fri
