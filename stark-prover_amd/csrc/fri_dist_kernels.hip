// fri_dist_kernels.hip — data-layout kernels of the coset-sharded commit
// (one process per GPU, G ranks).
//
//   coset coefficients : rank r evaluates P on the coset s*<w_M>, s = offset*w_n^r,
//                        M = n/G, via P mod (x^M - s^M) (chunk fold) and a size-M
//                        NTT with pre-scale s^j  ->  evals[r + G*m], m < M
//   cyclic -> block     : after the all-to-all, rank g holds chunk t of every
//                        rank's slice; block[G*t + r] = recv[r][t]
//   pair fold           : layer k -> k+1 from the local half-block and the
//                        partner's half-block (fri_commit.rs:53-65)
//   root permute        : all-gathered block roots, rank order -> block order
#include "fri_internal.hpp"

namespace fri {

constexpr uint32_t INV2_MD = 0x80000000u;   // Montgomery(2^-1)

// out[j] = sum_t a[j + t*M] * c^t for j < M  (c = s^M, Montgomery c_m).
__global__ void k_coset_coeffs(const uint32_t* __restrict__ a, size_t d, uint32_t* __restrict__ out, size_t M,
                               uint32_t c_m) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    const size_t chunks = (d + M - 1) / M;
    uint32_t acc = 0;
    for (size_t t = chunks; t-- > 0;) {
        const size_t i = j + t * M;
        acc = add(mmul(acc, c_m), i < d ? a[i] : 0u);
    }
    out[j] = acc;
}
void launch_coset_coeffs(const uint32_t* a, size_t d, uint32_t* out, size_t M, uint32_t c_std, hipStream_t s) {
    hipLaunchKernelGGL(k_coset_coeffs, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, a, d, out, M, to_mont(c_std));
}

// block[G*t + r] = recv[r * (B/G) + t]
// Thread j writes the G consecutive block words j*G .. j*G+G-1 as 16-byte
// stores, reading word j of each of the G received slices (each read stream
// coalesced across the wave).  G >= 4 (G = 2 takes the radix-2 path).
__global__ void k_cyclic_to_block(const uint32_t* __restrict__ recv, uint32_t* __restrict__ block, size_t per,
                                  uint32_t G) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= per) return;
    uint4* out = reinterpret_cast<uint4*>(block + j * G);
    for (uint32_t g = 0; g < G; g += 4)
        out[g >> 2] = make_uint4(recv[g * per + j], recv[(g + 1) * per + j], recv[(g + 2) * per + j],
                                 recv[(g + 3) * per + j]);
}
void launch_cyclic_to_block(const uint32_t* recv, uint32_t* block, size_t B, uint32_t G, hipStream_t s) {
    const size_t per = B / G;
    hipLaunchKernelGGL(k_cyclic_to_block, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, s, recv, block, per, G);
}

// out[j] = fold(first[j], second[j], xinv[j], beta_r), gated on active[r].
__global__ void k_pair_fold(const uint32_t* __restrict__ first, const uint32_t* __restrict__ second,
                            const uint32_t* __restrict__ xinv, uint32_t* __restrict__ out, size_t h,
                            const DevState* __restrict__ st, int r) {
    if (!st->active[r]) return;
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= h) return;
    const uint32_t a = first[j], b = second[j];
    const uint32_t s = add(a, b), t = sub(a, b);
    out[j] = mmul(add(s, mmul(mmul(t, xinv[j]), st->beta_mont[r])), INV2_MD);
}
void launch_pair_fold(const uint32_t* first, const uint32_t* second, const uint32_t* xinv, uint32_t* out, size_t h,
                      const DevState* st, int r, hipStream_t s) {
    hipLaunchKernelGGL(k_pair_fold, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, s, first, second, xinv, out, h,
                       st, r);
}

// G = 2, layer 0 without an all-to-all (radix-2 decimation): even/odd
// coefficients for two size-M NTTs ...
__global__ void k_decimate(const uint32_t* __restrict__ a, size_t d, uint32_t* __restrict__ ev,
                           uint32_t* __restrict__ od) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * k < d) ev[k] = a[2 * k];
    if (2 * k + 1 < d) od[k] = a[2 * k + 1];
}
void launch_decimate(const uint32_t* a, size_t d, uint32_t* ev, uint32_t* od, hipStream_t s) {
    const size_t h = (d + 1) / 2;
    if (h) hipLaunchKernelGGL(k_decimate, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, s, a, d, ev, od);
}
// ... and the block of rank b:  L0[j] = E[j] + (-1)^b * offset * w_n^j * O[j],
// tw = pow table of offset * w_n^j (Montgomery lo/hi split).
__global__ void k_radix2_block(const uint32_t* __restrict__ E, const uint32_t* __restrict__ O,
                               const uint32_t* __restrict__ tlo, const uint32_t* __restrict__ thi,
                               uint32_t* __restrict__ out, size_t M, uint32_t negate) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    const uint32_t t = mmul(mmul(O[j], thi[j >> POW_LO_LOG]), tlo[j & ((1u << POW_LO_LOG) - 1)]);
    out[j] = negate ? sub(E[j], t) : add(E[j], t);
}
void launch_radix2_block(const uint32_t* E, const uint32_t* O, const uint32_t* tlo, const uint32_t* thi,
                         uint32_t* out, size_t M, uint32_t negate, hipStream_t s) {
    hipLaunchKernelGGL(k_radix2_block, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, E, O, tlo, thi, out, M,
                       negate);
}

struct Perm64 { uint32_t p[64]; };
// dst digest block_of_rank[r] <- src digest r  (G <= 64)
__global__ void k_permute_digests(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t G, Perm64 pm) {
    const uint32_t i = threadIdx.x;        // G * 8 words
    if (i >= G * 8) return;
    const uint32_t r = i / 8, w = i % 8;
    dst[8 * pm.p[r] + w] = src[8 * r + w];
}
void launch_permute_digests(const uint32_t* src, uint32_t* dst, uint32_t G, const uint32_t* block_of_rank, hipStream_t s) {
    Perm64 pm{};
    for (uint32_t r = 0; r < G && r < 64; r++) pm.p[r] = block_of_rank[r];
    hipLaunchKernelGGL(k_permute_digests, dim3(1), dim3(512), 0, s, src, dst, G, pm);
}

// Per-layer record of one rank (REC_WORDS words, all-gathered): its block
// root, the maxima (m0, m1, m2) of its slice of the coefficient task
// (reduced from the R workgroup triples) and its poly_k coefficient obase
// (the final value when rank 0's chunk starts at 0 and deg_k == 0).
// One wave; gated like the layer it belongs to.
__global__ void k_shard_record(const uint32_t* __restrict__ root, const int32_t* __restrict__ wgmax, uint32_t R,
                               const uint32_t* __restrict__ c0, uint32_t* __restrict__ rec, const DevState* st,
                               int gate) {
    if (gate >= 0 && !st->active[gate]) return;
    const uint32_t t = threadIdx.x;
    int a = -1, b = -1, c = -1;
    for (uint32_t i = t; i < R; i += 64) {
        a = max(a, wgmax[3 * i]); b = max(b, wgmax[3 * i + 1]); c = max(c, wgmax[3 * i + 2]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a = max(a, __shfl_xor(a, off)); b = max(b, __shfl_xor(b, off)); c = max(c, __shfl_xor(c, off));
    }
    if (t < 8) rec[t] = root[t];
    if (t == 0) {
        rec[8] = (uint32_t)a; rec[9] = (uint32_t)b; rec[10] = (uint32_t)c;
        rec[11] = c0 ? c0[0] : 0u;
        rec[12] = rec[13] = rec[14] = rec[15] = 0u;
    }
}
void launch_shard_record(const uint32_t* root, const int32_t* wgmax, uint32_t R, const uint32_t* c0, uint32_t* rec,
                         const DevState* st, int gate, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_record, dim3(1), dim3(64), 0, s, root, wgmax, R, c0, rec, st, gate);
}

// The G all-gathered records (rank order) -> the top tree's level 0 in block
// order, the G maxima triples for k_tree_top (mx[3r..3r+2]) and the final
// value candidate from the rank holding coefficient 0 (c0out).  sched
// (loopback rehearsal only): the recorded degree of every layer replaces the
// maxima, so one rank's share runs every round of the real commit.
__global__ void k_shard_unpack(const uint32_t* __restrict__ recs, uint32_t G, Perm64 pm, uint32_t c0_rank,
                               uint32_t* __restrict__ top, int32_t* __restrict__ mx, uint32_t* __restrict__ c0out,
                               const int32_t* __restrict__ sched, int k, const DevState* st, int gate) {
    if (gate >= 0 && !st->active[gate]) return;
    const uint32_t i = threadIdx.x;
    if (i < G * 8) {
        const uint32_t r = i / 8, w = i % 8;
        top[8 * pm.p[r] + w] = recs[REC_WORDS * r + w];
    }
    if (i < G * 3) {
        const uint32_t r = i / 3, j = i % 3;
        int32_t v = (int32_t)recs[REC_WORDS * r + 8 + j];
        if (sched) v = j == 0 ? sched[k] : j == 1 ? (k == 0 ? -1 : 0) : -1;   // k = 0: deg = m0, canonical
        mx[i] = v;
    }
    if (i == 0) c0out[0] = recs[REC_WORDS * c0_rank + 11];
}
void launch_shard_unpack(const uint32_t* recs, uint32_t G, const uint32_t* block_of_rank, uint32_t c0_rank,
                         uint32_t* top, int32_t* mx, uint32_t* c0out, const int32_t* sched, int k, const DevState* st,
                         int gate, hipStream_t s) {
    Perm64 pm{};
    for (uint32_t r = 0; r < G && r < 64; r++) pm.p[r] = block_of_rank[r];
    hipLaunchKernelGGL(k_shard_unpack, dim3(1), dim3(512), 0, s, recs, G, pm, c0_rank, top, mx, c0out, sched, k, st,
                       gate);
}

}  // namespace fri
