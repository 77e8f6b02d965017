// fri_dist_kernels.hip — data-layout kernels of the coset-sharded commit
// (one process per GPU, G ranks).
//
//   coset coefficients : rank r evaluates P on the coset s*<w_M>, s = offset*w_n^r,
//                        M = n/G, via P mod (x^M - s^M) (chunk fold) and a size-M
//                        NTT with pre-scale s^j  ->  evals[r + G*m], m < M
//   cyclic -> block     : after the all-to-all, rank g holds chunk t of every
//                        rank's slice; block[G*t + r] = recv[r][t]
//   (the pair fold of layer k -> k+1 from the local and the partner's
//    half-blocks, fri_commit.rs:53-65, runs inside layer k+1's leaf kernel:
//    k_layer_leaf<..., PAIR>, fri_layer.hip)
//   (the per-layer records of block roots and coefficient maxima are written
//    and read by the sharded top kernels, k_tree_top<..., SHARD>, fri_layer.hip)
#include <algorithm>

#include "fri_internal.hpp"

namespace fri {


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

// Switch to the local tail: the G gathered blocks (rank order) into their
// places in the whole layer, block_of[r] * B, as one launch (16-byte copies).
struct Blocks64 { uint32_t b[64]; };
__global__ void k_place_blocks(const uint4* __restrict__ gath, uint4* __restrict__ layer, size_t B4, uint32_t G,
                               Blocks64 bo) {
    const size_t tot = B4 * G;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / B4, j = i - r * B4;
        layer[(size_t)bo.b[r] * B4 + j] = gath[i];
    }
}
void launch_place_blocks(const uint32_t* gath, uint32_t* layer, size_t B, uint32_t G, const uint32_t* block_of,
                         hipStream_t s) {
    Blocks64 bo{};
    for (uint32_t r = 0; r < G && r < 64; r++) bo.b[r] = block_of[r];
    const size_t tot = (B / 4) * G;
    const unsigned blocks = (unsigned)std::min<size_t>(4096, (tot + 255) / 256);
    hipLaunchKernelGGL(k_place_blocks, dim3(blocks ? blocks : 1), dim3(256), 0, s, reinterpret_cast<const uint4*>(gath),
                       reinterpret_cast<uint4*>(layer), B / 4, G, bo);
}

// Loopback rehearsal (fri_debug_attach_loopback): the all-gather of G
// copies of this rank's bytes as one launch instead of G copies.
__global__ void k_replicate(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, size_t words, uint32_t G) {
    const size_t tot = words * G;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i % words];
}
void launch_replicate(const uint32_t* src, uint32_t* dst, size_t words, uint32_t G, hipStream_t s) {
    const size_t tot = words * G;
    const unsigned blocks = (unsigned)std::min<size_t>(2048, (tot + 255) / 256);
    hipLaunchKernelGGL(k_replicate, dim3(blocks ? blocks : 1), dim3(256), 0, s, src, dst, words, G);
}

// In-process peer transport (fri_ctx_create_multi): rank r copies source p's
// bytes (another rank's send buffer, on this device or, with peer access
// enabled, read over xGMI from another one) to dst + p * words, for every
// source p in one launch (grid.y = source).  16-byte accesses when every
// pointer and the size allow them.
__global__ __launch_bounds__(256) void k_peer_pull(PeerPull pp) {
    const uint32_t p = blockIdx.y;
    const uint32_t* __restrict__ src = pp.src[p];
    uint32_t* __restrict__ dst = pp.dst + (size_t)p * pp.words;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (pp.vec4) {
        const size_t nv = pp.words >> 2;
        for (; i < nv; i += stride) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else {
        for (; i < pp.words; i += stride) dst[i] = src[i];
    }
}
void launch_peer_pull(const PeerPull& pp, hipStream_t s) {
    const size_t units = pp.vec4 ? pp.words >> 2 : pp.words;
    const size_t want = std::max<size_t>(1, (units + 1023) / 1024);          // ~4 units per thread
    const uint32_t gx = (uint32_t)std::min<size_t>(want, std::max<size_t>(1, 2048 / std::max(1u, pp.n)));
    hipLaunchKernelGGL(k_peer_pull, dim3(gx, pp.n), dim3(256), 0, s, pp);
}

// Input checksum (FRI_FLAG_RANK_INPUTS: every rank's resident input must be
// rank 0's buffer): the wrapping 64-bit sum over i of mix(i << 32 | v[i]),
// mix = the splitmix64 finaliser.  Order- and position-sensitive, so a
// rewritten, shifted or truncated input changes it with probability
// 1 - 2^-64 per change; one atomic per workgroup (a vector global atomic).
__device__ inline uint64_t csum_mix(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
__global__ __launch_bounds__(256) void k_checksum(const uint32_t* __restrict__ v, size_t n,
                                                  unsigned long long* out) {
    __shared__ uint64_t part[256];
    uint64_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += csum_mix(((uint64_t)i << 32) | v[i]);
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)part[0]);
}
void launch_checksum(const uint32_t* v, size_t n, uint64_t* out, hipStream_t s) {
    (void)hipMemsetAsync(out, 0, sizeof(uint64_t), s);
    const unsigned blocks = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, (n + 2047) / 2048));
    hipLaunchKernelGGL(k_checksum, dim3(blocks), dim3(256), 0, s, v, n, reinterpret_cast<unsigned long long*>(out));
}

}  // namespace fri
