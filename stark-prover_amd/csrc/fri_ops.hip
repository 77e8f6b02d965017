// fri_ops.hip — kernel-level entry points of include/fri_amd.h: batch
// inverse (element.rs:54-57), coset LDE (fri_commit.rs:78), interpolation on
// a coset and through arbitrary points (ops.rs:239-241 ->
// interpolation.rs:121-152), evaluation (ops.rs:76-83), one fold
// (fri_commit.rs:53-65) and the Merkle root of any n (merkle/mod.rs:10-26).
#include "fri_host.hpp"
#include "sha256.hpp"

// ------------------------------------------------------- kernel-level ----
extern "C" int fri_batch_inverse(fri_ctx* ctx, const uint32_t* in, uint32_t* out, size_t n) {
    if (!ctx || (!in && n) || (!out && n)) return fail(ctx, FRI_EINVAL, "null argument");
    if (!check_canonical(in, n)) return fail(ctx, FRI_EINVAL, "input not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    const size_t cap = (size_t)1 << ctx->log_n_max;
    for (size_t off = 0; off < n; off += cap) {
        size_t m = n - off < cap ? n - off : cap;
        FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, in + off, m * 4, hipMemcpyHostToDevice, ctx->stream));
        launch_batch_inverse(ctx->scratch_a, ctx->scratch_b, m, 0, ctx->stream);
        FRI_HIP(ctx, hipGetLastError());
        FRI_HIP(ctx, hipMemcpyAsync(out + off, ctx->scratch_b, m * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}


extern "C" int fri_lde(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n, uint32_t offset,
                       uint32_t* evals_out) {
    if (!ctx || !evals_out || (d && !coeffs)) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_n > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n exceeds context capacity");
    const size_t n = (size_t)1 << log_n;
    if (d > n) return fail(ctx, FRI_EINVAL, "more coefficients than domain points");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    if (!check_canonical(coeffs, d)) return fail(ctx, FRI_EINVAL, "coefficient not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if (d) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, coeffs, d * 4, hipMemcpyHostToDevice, ctx->stream));
    NttPlan p = lde_plan(ctx, log_n);
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_n, offset, 1u, ctx->stream);
    p.pre_lo = ctx->pow_lo;
    p.pre_hi = ctx->pow_hi;
    p.scratch = ctx->scratch_c;
    launch_ntt(p, ctx->scratch_a, d, ctx->scratch_b, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(evals_out, ctx->scratch_b, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

extern "C" int fri_interpolate(fri_ctx* ctx, const uint32_t* ys, uint32_t log_n, uint32_t offset,
                               uint32_t* coeffs_out, size_t* len_out) {
    if (!ctx || !ys || !coeffs_out || !len_out) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_n > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_n exceeds context capacity");
    if (offset == 0 || offset >= P) return fail(ctx, FRI_EINVAL, "offset must be a nonzero canonical element");
    const size_t n = (size_t)1 << log_n;
    if (!check_canonical(ys, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, ys, n * 4, hipMemcpyHostToDevice, ctx->stream));
    NttPlan p{};
    p.log_n = log_n;
    p.tw = ctx->tw_inv;
    // coeff_j = n^-1 * offset^-j * sum_i ys_i w^-ij
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_n, inv_std(offset), inv_std((uint32_t)(n % P)), ctx->stream);
    p.post_lo = ctx->pow_lo;
    p.post_hi = ctx->pow_hi;
    launch_ntt(p, ctx->scratch_a, n, ctx->scratch_b, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(coeffs_out, ctx->scratch_b, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    size_t len = n;
    while (len > 0 && coeffs_out[len - 1] == 0) len--;          // Polynomial::new trim (ops.rs:19-37)
    *len_out = len;
    return FRI_OK;
}

// Device scratch of at least `words` words for the interpolation / evaluation
// partials (grown on demand, freed with the context).
static int ensure_tmp(fri_ctx* ctx, size_t words) {
    if (words <= ctx->interp_cap) return FRI_OK;
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->interp_tmp) dfree(ctx, ctx->interp_tmp);
    ctx->interp_tmp = nullptr;
    ctx->interp_cap = 0;
    if (dalloc(ctx, &ctx->interp_tmp, words * 4) != hipSuccess) return fail(ctx, FRI_ENOMEM, "partials scratch");
    ctx->interp_cap = words;
    return FRI_OK;
}
// Scratch grown past TMP_KEEP_WORDS is released after the call that grew it,
// so one large fri_merkle_root (the tree of 2^28 values is 16 GiB) does not
// pin HBM for the life of the context and starve a later commit plan; smaller
// scratch is kept (no hipFree, which synchronises the device, per call).
constexpr size_t TMP_KEEP_WORDS = (size_t)1 << 26;   // 256 MiB
static void tmp_trim(fri_ctx* ctx) {
    if (ctx->interp_cap <= TMP_KEEP_WORDS) return;
    (void)hipStreamSynchronize(ctx->stream);
    dfree(ctx, ctx->interp_tmp);
    ctx->interp_tmp = nullptr;
    ctx->interp_cap = 0;
}

// interpolate_lagrange_polynomials (interpolation.rs:121-152) on arbitrary
// points: weights, c_j = y_j w_j, f on the 2^k-th roots of unity, iNTT
// (fri_kernels.hip "arbitrary-point interpolate").
extern "C" int fri_interpolate_points(fri_ctx* ctx, const uint32_t* xs, const uint32_t* ys, size_t n,
                                      uint32_t* coeffs_out, size_t* len_out) {
    if (!ctx || !len_out || (n && (!xs || !ys || !coeffs_out))) return fail(ctx, FRI_EINVAL, "null argument");
    uint32_t log_N = 0;
    while (((size_t)1 << log_N) < n) log_N++;
    if (log_N > 17 || log_N > ctx->log_n_max)
        return fail(ctx, FRI_EINVAL, "arbitrary-point interpolation is O(n^2): n <= 2^17 and <= 2^log_n_max");
    if (!check_canonical(xs, n) || !check_canonical(ys, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    *len_out = 0;
    if (n == 0) return FRI_OK;                                   // Polynomial::zero() (interpolation.rs:133-136)
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t N = (size_t)1 << log_N;
    int rc = ensure_tmp(ctx, interp_tmp_words(n, log_N));
    if (rc) return rc;
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, xs, n * 4, hipMemcpyHostToDevice, s));
    launch_interp_weights(ctx->scratch_a, n, ctx->scratch_b, ctx->interp_tmp, s);   // prod_{i!=j}(x_j - x_i)
    launch_batch_inverse(ctx->scratch_b, ctx->scratch_c, n, 1, s);          // w_j (Montgomery; 0 -> 0)
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_b, ys, n * 4, hipMemcpyHostToDevice, s));   // after the inverse (stream order)
    launch_interp_coeffs(ctx->scratch_b, ctx->scratch_c, n, s);             // c_j = y_j w_j
    launch_interp_eval(ctx->scratch_a, ctx->scratch_c, n, log_N, ctx->scratch_b, ctx->interp_tmp, s);   // f(w_N^k)
    NttPlan p{};
    p.log_n = log_N;
    p.tw = ctx->tw_inv;
    launch_pow_table(ctx->pow_lo, ctx->pow_hi, log_N, 1u, inv_std((uint32_t)(N % P)), s);   // N^-1
    p.post_lo = ctx->pow_lo;
    p.post_hi = ctx->pow_hi;
    launch_ntt(p, ctx->scratch_b, N, ctx->scratch_a, s);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(coeffs_out, ctx->scratch_a, n * 4, hipMemcpyDeviceToHost, s));   // deg f < n
    FRI_HIP(ctx, hipStreamSynchronize(s));
    tmp_trim(ctx);
    size_t len = n;
    while (len > 0 && coeffs_out[len - 1] == 0) len--;          // Polynomial::new trim (ops.rs:19-37)
    *len_out = len;
    return FRI_OK;
}

extern "C" int fri_evaluate(fri_ctx* ctx, const uint32_t* coeffs, size_t d, const uint32_t* xs, size_t count,
                            uint32_t* out) {
    if (!ctx || (d && !coeffs) || (count && (!xs || !out))) return fail(ctx, FRI_EINVAL, "null argument");
    const size_t cap = (size_t)1 << ctx->log_n_max;
    if (d > cap || count > cap) return fail(ctx, FRI_EINVAL, "size exceeds context capacity");
    if (!check_canonical(coeffs, d) || !check_canonical(xs, count))
        return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    if (d) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, coeffs, d * 4, hipMemcpyHostToDevice, ctx->stream));
    if (count) FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_b, xs, count * 4, hipMemcpyHostToDevice, ctx->stream));
    const size_t tw = evaluate_tmp_words(d, count);
    if (tw) {
        const int rc = ensure_tmp(ctx, tw);
        if (rc) return rc;
    }
    launch_evaluate(ctx->scratch_a, d, ctx->scratch_b, count, ctx->scratch_c, ctx->interp_tmp, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    if (count) FRI_HIP(ctx, hipMemcpyAsync(out, ctx->scratch_c, count * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    tmp_trim(ctx);
    return FRI_OK;
}

extern "C" int fri_fold(fri_ctx* ctx, const uint32_t* layer, uint32_t log_m, uint32_t layer_offset, uint32_t beta,
                        uint32_t* out) {
    if (!ctx || !layer || !out) return fail(ctx, FRI_EINVAL, "null argument");
    if (log_m < 1 || log_m > ctx->log_n_max) return fail(ctx, FRI_EINVAL, "log_m out of range");
    if (layer_offset == 0 || layer_offset >= P || beta >= P) return fail(ctx, FRI_EINVAL, "bad offset/beta");
    const size_t m = (size_t)1 << log_m;
    if (!check_canonical(layer, m)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, layer, m * 4, hipMemcpyHostToDevice, ctx->stream));
    launch_coset_points(ctx->scratch_b, m / 2, layer_offset, log_m, ctx->stream);
    launch_batch_inverse(ctx->scratch_b, ctx->scratch_c, m / 2, 1, ctx->stream);
    launch_fold_plain(ctx->scratch_a, ctx->scratch_b, log_m, ctx->scratch_c, beta, ctx->stream);
    FRI_HIP(ctx, hipGetLastError());
    FRI_HIP(ctx, hipMemcpyAsync(out, ctx->scratch_b, (m / 2) * 4, hipMemcpyDeviceToHost, ctx->stream));
    FRI_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return FRI_OK;
}

// Non-power-of-two trees (rs_merkle promotes a lone right-most node).
__global__ void k_leaf_generic(const uint32_t* v, uint32_t* out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sha::leaf(v[i], out + 8 * i);
}
__global__ void k_level_generic(const uint32_t* in, uint32_t* out, size_t cnt) {
    size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t pc = (cnt + 1) / 2;
    if (j >= pc) return;
    if (2 * j + 1 < cnt) sha::node(in + 16 * j, in + 16 * j + 8, out + 8 * j);
    else for (int i = 0; i < 8; i++) out[8 * j + i] = in[16 * j + i];
}

extern "C" int fri_merkle_root(fri_ctx* ctx, const uint32_t* values, size_t n, uint8_t root32[32]) {
    if (!ctx || !values || !root32) return fail(ctx, FRI_EINVAL, "null argument");
    if (n == 0) return fail(ctx, FRI_EINVAL, "empty tree has no root (merkle/mod.rs:25)");
    const size_t cap = (size_t)1 << ctx->log_n_max;
    if (n > cap) return fail(ctx, FRI_EINVAL, "size exceeds context capacity");
    if (!check_canonical(values, n)) return fail(ctx, FRI_EINVAL, "value not canonical (>= p)");
    FRI_HIP(ctx, hipSetDevice(ctx->device));
    FRI_HIP(ctx, hipMemcpyAsync(ctx->scratch_a, values, n * 4, hipMemcpyHostToDevice, ctx->stream));
    // the tree lives in the context's partials scratch (no hipMalloc / hipFree,
    // which synchronises the device, per MerkleTree::new)
    uint32_t* root_dev;
    uint32_t* tree = nullptr;
    bool pow2 = (n & (n - 1)) == 0;
    if (pow2) {
        uint32_t L = 0;
        while (((size_t)1 << L) < n) L++;
        const int rc = ensure_tmp(ctx, ((size_t)2 << L) * 8);
        if (rc) return rc;
        tree = ctx->interp_tmp;
        LayerTask t{};
        t.values = ctx->scratch_a;
        t.tree = tree;
        t.L = L;
        launch_layer(t, ctx->stream);
        root_dev = tree + 8 * level_offset(L, L);
    } else {
        size_t total = 0;
        for (size_t m = n;; m = (m + 1) / 2) { total += m; if (m == 1) break; }
        const int rc = ensure_tmp(ctx, total * 8);
        if (rc) return rc;
        tree = ctx->interp_tmp;
        uint32_t* cur = tree;
        hipLaunchKernelGGL(k_leaf_generic, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                           ctx->scratch_a, cur, n);
        size_t cnt = n;
        while (cnt > 1) {
            size_t pc = (cnt + 1) / 2;
            uint32_t* nxt = cur + 8 * cnt;
            hipLaunchKernelGGL(k_level_generic, dim3((unsigned)((pc + 255) / 256)), dim3(256), 0, ctx->stream, cur,
                               nxt, cnt);
            cur = nxt;
            cnt = pc;
        }
        root_dev = cur;
    }
    FRI_HIP(ctx, hipGetLastError());
    uint32_t w[8];
    hipError_t e1 = hipMemcpyAsync(w, root_dev, 32, hipMemcpyDeviceToHost, ctx->stream);
    hipError_t e2 = hipStreamSynchronize(ctx->stream);
    tmp_trim(ctx);
    FRI_HIP(ctx, e1);
    FRI_HIP(ctx, e2);
    digest_to_bytes(w, root32);
    return FRI_OK;
}
