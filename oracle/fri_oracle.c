/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  NOT PART OF THE PRODUCT PATH.
 *
 * CPU restatement of the reference (RazorClient/Stark-prover, crate `stark-101`)
 * FRI-commit path, used only by tests/, __graft_entry__.smoke() and bench.py's
 * `cpu_baseline` leg as the checker.  The shipped library (libfri_amd.so) never
 * links, loads or calls anything in this file.
 *
 * Two restatements live here:
 *   A. "faithful"  — the reference's own algorithms, function for function:
 *        field ops  (src/fields/element.rs), Horner evaluate / trim / mul /
 *        div_rem    (src/polynomial/ops.rs), Lagrange interpolation
 *        (src/polynomial/interpolation.rs), coefficient-form FRI fold + Horner
 *        re-evaluation (src/fri/fri_commit.rs), rs_merkle-1.4.2 SHA-256 tree
 *        (src/merkle/mod.rs), hex/SHA-256 Fiat-Shamir channel
 *        (src/channel/channel.rs).  Generic over the u64 modulus so the
 *        reference's own unit-test KATs (moduli 7 / 17 / 23) replay exactly.
 *   B. "fast"      — same results by different algorithms (coset NTT LDE,
 *        evaluation-form fold, batch inverse), OpenMP-parallel; the CPU
 *        baseline at sizes where (A) is O(n*d)-infeasible.
 *
 * Parity status: field / polynomial / interpolation are pinned by the
 * reference's 60 unit-test KATs.  SHA-256 is pinned by FIPS 180-4 vectors and
 * Python hashlib.  The rs_merkle 1.4.2 tree shape (pairing, odd-node
 * promotion) is pinned by rs_merkle's documented example root over the
 * SHA-256 leaves of "a".."f" (tests/test_oracle_kats.py, via the Python twin,
 * which this file matches for every tree size 1..40).  The channel string
 * encoding and U256 reduction are restated from the reference's channel.rs and
 * the pinned crates' published behaviour (sha256 1.5.0, alloy-primitives
 * 0.8.21) — not vendored, and the reference has no tests for them: PARITY
 * UNPINNED for channel/fri beyond this repo's frozen spec (SURVEY.md §8
 * "Frozen spec") and committed golden vectors.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ======================================================================
 * A.1  Field — src/fields/element.rs (generic u64 modulus M)
 * ====================================================================== */

/* element.rs:13-17  FieldElement::new: value % MODULUS */
uint64_t orc_fe_new(uint64_t v, uint64_t M) { return v % M; }

/* element.rs:72-78  Add: new(self.value + rhs.value) */
uint64_t orc_fe_add(uint64_t a, uint64_t b, uint64_t M) { return (a + b) % M; }

/* element.rs:86-93  Sub: new((MODULUS + a - b) % MODULUS) */
uint64_t orc_fe_sub(uint64_t a, uint64_t b, uint64_t M) { return ((M + a - b) % M) % M; }

/* element.rs:102-108  Mul: u128 product % MODULUS */
uint64_t orc_fe_mul(uint64_t a, uint64_t b, uint64_t M) { return (uint64_t)(((u128)a * b) % M); }

/* element.rs:38-51  pow: square-and-multiply with u64 (wrapping) products —
 * exact only for M < 2^32, restated with the same u64 semantics. */
uint64_t orc_fe_pow(uint64_t a, uint64_t e, uint64_t M) {
    uint64_t result = 1, base = a;
    while (e > 0) {
        if (e & 1) result = (result * base) % M;
        base = (base * base) % M;
        e >>= 1;
    }
    return result;
}

/* element.rs:54-57  inverse = a^(M-2); inverse(0) = 0 */
uint64_t orc_fe_inverse(uint64_t a, uint64_t M) { return orc_fe_pow(a, M - 2, M); }

/* element.rs:130-136  Neg: new(MODULUS - value) */
uint64_t orc_fe_neg(uint64_t a, uint64_t M) { return (M - a) % M; }

/* element.rs:116-122  Div: self * rhs.inverse() */
uint64_t orc_fe_div(uint64_t a, uint64_t b, uint64_t M) { return orc_fe_mul(a, orc_fe_inverse(b, M), M); }

/* element.rs:59-61  to_bytes: u64 big-endian */
void orc_fe_to_bytes(uint64_t v, uint8_t out[8]) {
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(v >> (56 - 8 * i));
}

/* ======================================================================
 * A.2  Polynomial — src/polynomial/ops.rs
 *      A polynomial is (coeffs[], len, degree).  `degree` is tracked
 *      separately because the reference's scalar_mul does not re-trim
 *      (ops.rs:194-198) and add_assign early-returns on a zero rhs
 *      (ops.rs:87-91) — both are visible in fri_commit's loop condition.
 * ====================================================================== */

/* ops.rs:19-37  Polynomial::new trims trailing zeros; returns new length */
size_t orc_poly_trim(const uint64_t* c, size_t len) {
    while (len > 0 && c[len - 1] == 0) len--;
    return len;
}

/* ops.rs:76-83  evaluate: Horner from the highest coefficient */
uint64_t orc_poly_evaluate(const uint64_t* c, size_t len, uint64_t x, uint64_t M) {
    uint64_t r = 0;
    for (size_t i = len; i-- > 0;) r = orc_fe_add(orc_fe_mul(r, x, M), c[i], M);
    return r;
}

/* Timing helper of bench.py's configs[0] leg (benches/poly_ops.rs:161-181
 * shape): `reps` evaluations at x, x+1, ... in one call, so the per-call cost
 * of the caller's FFI is not part of the figure; returns the sum of the
 * values so the work stays live. */
uint64_t orc_bench_evaluate(const uint64_t* c, size_t len, uint64_t x, uint64_t M, size_t reps) {
    uint64_t acc = 0;
    for (size_t k = 0; k < reps; k++) acc += orc_poly_evaluate(c, len, (x + k) % M, M);
    return acc;
}

/* ops.rs:114-138  mul_assign (naive), result trimmed (update_degree).
 * out must hold la+lb-1 entries.  Returns trimmed length. */
size_t orc_poly_mul(const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                    uint64_t* out, uint64_t M) {
    if (la == 0 || lb == 0) return 0;
    size_t nl = la + lb - 1;
    for (size_t i = 0; i < nl; i++) out[i] = 0;
    for (size_t i = 0; i < la; i++) {
        if (a[i] == 0) continue;
        for (size_t j = 0; j < lb; j++)
            out[i + j] = orc_fe_add(out[i + j], orc_fe_mul(a[i], b[j], M), M);
    }
    return orc_poly_trim(out, nl);
}

/* ops.rs:141-191  div_rem (naive long division, one inverse per step).
 * a, b trimmed.  q must hold la entries, r must hold la entries.
 * Returns 0 on success, -1 for division by the zero polynomial (the
 * reference panics, ops.rs:143). */
int orc_poly_div_rem(const uint64_t* a, size_t la, const uint64_t* b, size_t lb,
                     uint64_t* q, size_t* lq, uint64_t* r, size_t* lr, uint64_t M) {
    if (lb == 0) return -1;
    if (la == 0 || la < lb) {                       /* ops.rs:145-147 */
        *lq = 0;
        memcpy(r, a, la * sizeof(uint64_t));
        *lr = la;
        return 0;
    }
    memcpy(r, a, la * sizeof(uint64_t));
    int64_t rem_deg = (int64_t)la - 1;
    size_t q_len = la - lb + 1;
    for (size_t i = 0; i < q_len; i++) q[i] = 0;
    uint64_t den_lead = b[lb - 1];
    int64_t den_deg = (int64_t)lb - 1;
    size_t rlen = la;
    while (rem_deg >= den_deg && rem_deg != -1) {
        uint64_t lead = r[rem_deg];
        uint64_t ratio = orc_fe_mul(lead, orc_fe_inverse(den_lead, M), M);
        size_t shift = (size_t)(rem_deg - den_deg);
        q[shift] = orc_fe_add(q[shift], ratio, M);
        for (int64_t i = 0; i <= den_deg; i++)
            r[i + shift] = orc_fe_sub(r[i + shift], orc_fe_mul(ratio, b[i], M), M);
        rlen = orc_poly_trim(r, rlen);
        rem_deg = (int64_t)rlen - 1;
    }
    *lq = orc_poly_trim(q, q_len);
    *lr = rlen;
    return 0;
}

/* ======================================================================
 * A.3  Lagrange interpolation — src/polynomial/interpolation.rs
 * ====================================================================== */

/* interpolation.rs:9-23  Z(x) = prod (x - root); out holds n+1 entries. */
size_t orc_poly_from_roots(const uint64_t* roots, size_t n, uint64_t* out, uint64_t M) {
    if (n == 0) return 0;
    uint64_t* tmp = (uint64_t*)malloc((n + 2) * sizeof(uint64_t));
    size_t len = 1;
    out[0] = 1;                                     /* poly![1] */
    for (size_t k = 0; k < n; k++) {
        uint64_t lin[2] = {orc_fe_neg(roots[k], M), 1};  /* poly![-root, 1] (trimmed: len 2) */
        len = orc_poly_mul(out, len, lin, 2, tmp, M);
        memcpy(out, tmp, len * sizeof(uint64_t));
    }
    free(tmp);
    return len;
}

/* interpolation.rs:121-152 (+ :80-115 basis, :46-78)  f = sum y_i L_i.
 * out holds n entries.  Returns trimmed length, or (size_t)-1 where the
 * reference panics (non-divisible Z, i.e. duplicate xs: interpolation.rs:104-106). */
size_t orc_interpolate_lagrange(const uint64_t* xs, const uint64_t* ys, size_t n,
                                uint64_t* out, uint64_t M) {
    if (n == 0) return 0;
    uint64_t* Z = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    uint64_t* q = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    uint64_t* r = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    size_t lz = orc_poly_from_roots(xs, n, Z, M);
    size_t acc_len = 0;                              /* acc = Polynomial::zero() */
    int64_t acc_deg = -1;
    for (size_t i = 0; i < n; i++) out[i] = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t denom = 1;
        for (size_t j = 0; j < n; j++)
            if (i != j) denom = orc_fe_mul(denom, orc_fe_sub(xs[i], xs[j], M), M);
        uint64_t dinv = orc_fe_inverse(denom, M);
        uint64_t lin[2] = {orc_fe_neg(xs[i], M), 1};
        size_t llin = orc_poly_trim(lin, 2);
        size_t lq, lr;
        orc_poly_div_rem(Z, lz, lin, llin, q, &lq, r, &lr, M);
        if (lr != 0) { acc_len = (size_t)-1; break; }
        /* li.scalar_mul(denom_inv) (ops.rs:194-198, degree unchanged), then
         * term.scalar_mul(ys[i]); acc.add_assign(&term) (ops.rs:87-98). */
        int64_t term_deg = (int64_t)lq - 1;
        if (term_deg == -1) continue;                 /* add_assign: rhs zero -> return */
        size_t ml = acc_len > lq ? acc_len : lq;
        for (size_t k = 0; k < lq; k++)
            out[k] = orc_fe_add(out[k], orc_fe_mul(orc_fe_mul(q[k], dinv, M), ys[i], M), M);
        acc_len = orc_poly_trim(out, ml);
        acc_deg = (int64_t)acc_len - 1;
    }
    (void)acc_deg;
    free(Z); free(q); free(r);
    return acc_len;
}

/* ======================================================================
 * A.4  SHA-256 — FIPS 180-4 (third-party: sha2 0.10.8 via rs_merkle,
 *      sha256 1.5.0 for the channel).  Restated from the standard.
 * ====================================================================== */
static const uint32_t SHA_K[64] = {
    0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
    0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
    0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
    0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
    0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
    0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
    0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
    0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
static const uint32_t SHA_IV[8] = {0x6a09e667u,0xbb67ae85u,0x3c6ef372u,0xa54ff53au,
                                   0x510e527fu,0x9b05688cu,0x1f83d9abu,0x5be0cd19u};
#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha_compress_portable(uint32_t st[8], const uint8_t blk[64]) {
    uint32_t w[64];
    for (int t = 0; t < 16; t++)
        w[t] = ((uint32_t)blk[4*t] << 24) | ((uint32_t)blk[4*t+1] << 16) | ((uint32_t)blk[4*t+2] << 8) | blk[4*t+3];
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ROTR(w[t-15], 7) ^ ROTR(w[t-15], 18) ^ (w[t-15] >> 3);
        uint32_t s1 = ROTR(w[t-2], 17) ^ ROTR(w[t-2], 19) ^ (w[t-2] >> 10);
        w[t] = w[t-16] + s0 + w[t-7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; t++) {
        uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + SHA_K[t] + w[t];
        uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
/* The same compression with the x86 SHA extensions.  The reference's SHA-256
 * (sha2 0.10.8, also under sha256 1.5.0) selects its x86 SHA-NI backend at run
 * time (cpufeatures) on CPUs that have it, as the GPU box's EPYC does, so the
 * CPU baseline's port does the same; orc_sha_backend() reports which one runs
 * and ORC_NO_SHANI=1 forces the portable code (tests check that both agree).
 * State as the instructions want it: ABEF = {F,E,B,A}, CDGH = {H,G,D,C}. */
__attribute__((target("sha,sse4.1,ssse3")))
static void sha_compress_shani(uint32_t st[8], const uint8_t blk[64]) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bLL, 0x0405060700010203LL);
    const __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)st), 0xB1);
    const __m128i efgh = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)(st + 4)), 0x1B);
    __m128i abef = _mm_alignr_epi8(abcd, efgh, 8);
    __m128i cdgh = _mm_blend_epi16(efgh, abcd, 0xF0);
    const __m128i abef0 = abef, cdgh0 = cdgh;
    __m128i m[4];
    for (int j = 0; j < 4; j++) m[j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk + 16 * j)), bswap);
    for (int g = 0; g < 16; g++) {
        if (g >= 4) {   /* W[t] = s1(W[t-2]) + W[t-7] + s0(W[t-15]) + W[t-16] */
            __m128i x = _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]);
            x = _mm_add_epi32(x, _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
            m[g & 3] = _mm_sha256msg2_epu32(x, m[(g + 3) & 3]);
        }
        __m128i wk = _mm_add_epi32(m[g & 3], _mm_loadu_si128((const __m128i*)(SHA_K + 4 * g)));
        cdgh = _mm_sha256rnds2_epu32(cdgh, abef, wk);
        wk = _mm_shuffle_epi32(wk, 0x0E);
        abef = _mm_sha256rnds2_epu32(abef, cdgh, wk);
    }
    abef = _mm_add_epi32(abef, abef0);
    cdgh = _mm_add_epi32(cdgh, cdgh0);
    const __m128i feba = _mm_shuffle_epi32(abef, 0x1B);
    const __m128i dchg = _mm_shuffle_epi32(cdgh, 0xB1);
    _mm_storeu_si128((__m128i*)st, _mm_blend_epi16(feba, dchg, 0xF0));
    _mm_storeu_si128((__m128i*)(st + 4), _mm_alignr_epi8(dchg, feba, 8));
}
static int orc_shani_on(void) {
    static int on = -1;            /* set once; every thread computes the same value */
    if (on < 0) {
        unsigned a = 0, b = 0, c = 0, d = 0;
        const int has = __get_cpuid_count(7, 0, &a, &b, &c, &d) && ((b >> 29) & 1u);
        const char* e = getenv("ORC_NO_SHANI");
        on = has && !(e && e[0] && e[0] != '0');
    }
    return on;
}
#else
static int orc_shani_on(void) { return 0; }
#endif

/* 1: the SHA extensions, 0: the portable restatement of FIPS 180-4 */
int orc_sha_backend(void) { return orc_shani_on(); }

static void sha_compress(uint32_t st[8], const uint8_t blk[64]) {
#if defined(__x86_64__)
    if (orc_shani_on()) {
        sha_compress_shani(st, blk);
        return;
    }
#endif
    sha_compress_portable(st, blk);
}

void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    uint32_t st[8];
    memcpy(st, SHA_IV, sizeof st);
    size_t off = 0;
    for (; off + 64 <= len; off += 64) sha_compress(st, msg + off);
    uint8_t blk[128];
    size_t rem = len - off;
    memset(blk, 0, sizeof blk);
    memcpy(blk, msg + off, rem);
    blk[rem] = 0x80;
    size_t tot = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) blk[tot - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha_compress(st, blk);
    if (tot == 128) sha_compress(st, blk + 64);
    for (int i = 0; i < 8; i++) {
        out[4*i] = (uint8_t)(st[i] >> 24); out[4*i+1] = (uint8_t)(st[i] >> 16);
        out[4*i+2] = (uint8_t)(st[i] >> 8); out[4*i+3] = (uint8_t)st[i];
    }
}

static void hex_lower(const uint8_t* in, size_t n, char* out) {
    static const char* H = "0123456789abcdef";
    for (size_t i = 0; i < n; i++) { out[2*i] = H[in[i] >> 4]; out[2*i+1] = H[in[i] & 15]; }
}

/* ======================================================================
 * A.5  Merkle — src/merkle/mod.rs:10-26 over rs_merkle 1.4.2
 *      leaf_i = SHA256(u64_be(value_i))               (mod.rs:14-15)
 *      from_leaves: pairwise SHA256(left || right); a lone right-most node
 *      is promoted unchanged (rs_merkle Hasher::concat_and_hash(l, None) = l)
 *      root_hex = lowercase hex of the top node      (mod.rs:24-26)
 *      Output: every level, leaves first, root last; returns node count.
 *      n == 0 returns 0 (the reference panics in root(): mod.rs:25).
 * ====================================================================== */
size_t orc_merkle_nodes_count(size_t n) {
    if (n == 0) return 0;
    size_t tot = 0;
    for (size_t m = n;; m = (m + 1) / 2) { tot += m; if (m == 1) break; }
    return tot;
}

size_t orc_merkle_build(const uint64_t* values, size_t n, uint8_t* nodes /* 32*count */) {
    if (n == 0) return 0;
    #pragma omp parallel for schedule(static) if (n > 4096)
    for (long i = 0; i < (long)n; i++) {
        uint8_t be[8];
        orc_fe_to_bytes(values[i], be);
        orc_sha256(be, 8, nodes + 32 * (size_t)i);
    }
    size_t base = 0, m = n;
    while (m > 1) {
        size_t pm = (m + 1) / 2;
        uint8_t* lvl = nodes + 32 * base;
        uint8_t* par = nodes + 32 * (base + m);
        #pragma omp parallel for schedule(static) if (pm > 4096)
        for (long j = 0; j < (long)pm; j++) {
            if (2 * (size_t)j + 1 < m) orc_sha256(lvl + 64 * (size_t)j, 64, par + 32 * (size_t)j);
            else memcpy(par + 32 * (size_t)j, lvl + 64 * (size_t)j, 32);
        }
        base += m;
        m = pm;
    }
    return base + 1;
}

/* ======================================================================
 * A.6  Channel — src/channel/channel.rs (sha256 1.5.0 digest() = lowercase
 *      hex of SHA-256 over the string's UTF-8 bytes; alloy hex::encode =
 *      lowercase; U256::from_str_radix(state,16) % range).
 *      state: 0..64 hex chars, NUL-terminated; state_len 0 means "".
 * ====================================================================== */
typedef struct { char state[65]; uint32_t state_len; } orc_channel;

void orc_channel_init(orc_channel* ch) { memset(ch, 0, sizeof *ch); }      /* channel.rs:24-30 */

/* channel.rs:35-44  state = sha256_hex(state || hex(message)) */
void orc_channel_send(orc_channel* ch, const uint8_t* msg, size_t len) {
    size_t tl = ch->state_len + 2 * len;
    char* buf = (char*)malloc(tl + 1);
    memcpy(buf, ch->state, ch->state_len);
    hex_lower(msg, len, buf + ch->state_len);
    uint8_t dg[32];
    orc_sha256((const uint8_t*)buf, tl, dg);
    hex_lower(dg, 32, ch->state);
    ch->state[64] = 0;
    ch->state_len = 64;
    free(buf);
}

/* U256::from_str_radix(state, 16) % range, returned as limb 0.  The
 * reference's `+ U256::from(min)` is applied before the reduction
 * (channel.rs:69-72); for min < range this is ((s mod r) + min) mod r. */
static uint64_t u256_hex_mod(const char* hex, size_t hl, uint64_t add, uint64_t range) {
    u128 r = 0;
    for (size_t i = 0; i < hl; i++) {
        char c = hex[i];
        uint32_t v = (c >= '0' && c <= '9') ? (uint32_t)(c - '0') : (uint32_t)(c - 'a' + 10);
        r = ((r << 4) | v) % range;
    }
    return (uint64_t)((r + add % range) % range);
}

/* channel.rs:58-84  receive_random_int(min, max, show_in_proof) */
uint64_t orc_channel_receive_int(orc_channel* ch, uint64_t min, uint64_t max) {
    uint64_t range = (max - min) + 1;
    uint64_t num = u256_hex_mod(ch->state, ch->state_len, min, range);
    uint8_t dg[32];
    orc_sha256((const uint8_t*)ch->state, ch->state_len, dg);    /* state = sha256::digest(old_state) */
    hex_lower(dg, 32, ch->state);
    ch->state[64] = 0;
    ch->state_len = 64;
    return num;
}

/* channel.rs:47-55  receive_random_field_element: receive_random_int(0, M-1) */
uint64_t orc_channel_receive_fe(orc_channel* ch, uint64_t M) {
    return orc_fe_new(orc_channel_receive_int(ch, 0, M - 1), M);
}

/* ======================================================================
 * A.7  FRI commit, faithful — src/fri/fri_commit.rs:18-122 + coset_fri.rs:32-36
 *      domain[i] = offset * omega^i, omega = g^((M-1)/n)   (frozen spec)
 *      Layers evaluated by Horner on every domain point (fri_commit.rs:78,:60-63).
 * ====================================================================== */
typedef struct {
    uint32_t n_layers;
    uint32_t n_rounds;
    uint64_t final_value;
    int64_t  final_degree;
    uint8_t  roots[64][32];
    uint64_t betas[64];
} orc_fri_result;

static void send_root(orc_channel* ch, const uint8_t root[32]) {
    char hx[64];
    hex_lower(root, 32, hx);                        /* rs_merkle root_hex() */
    orc_channel_send(ch, (const uint8_t*)hx, 64);   /* send(root_hex.as_bytes()) — frozen spec */
}

/* fri_commit.rs:32-50  next_fri_polynomial: new(odd)*beta + new(even).
 * Tracks `degree` exactly as the reference does (see A.2 note).  Returns
 * new degree; coefficients written to out (length returned in *olen). */
static int64_t next_fri_polynomial(const uint64_t* c, size_t len, uint64_t beta, uint64_t M,
                                   uint64_t* out, size_t* olen) {
    size_t lo = len / 2, le = (len + 1) / 2;
    uint64_t* odd = (uint64_t*)malloc((lo + 1) * sizeof(uint64_t));
    uint64_t* even = (uint64_t*)malloc((le + 1) * sizeof(uint64_t));
    for (size_t j = 0; j < lo; j++) odd[j] = c[2 * j + 1];
    for (size_t j = 0; j < le; j++) even[j] = c[2 * j];
    size_t lodd = orc_poly_trim(odd, lo), leven = orc_poly_trim(even, le);
    int64_t odd_deg = (int64_t)lodd - 1;
    for (size_t j = 0; j < lodd; j++) odd[j] = orc_fe_mul(odd[j], beta, M);   /* scalar_mul: degree kept */
    int64_t deg;
    size_t L;
    if (leven == 0) {                                 /* add_assign: rhs zero -> self unchanged */
        L = lodd; memcpy(out, odd, L * sizeof(uint64_t)); deg = odd_deg;
    } else {
        L = lodd > leven ? lodd : leven;
        for (size_t j = 0; j < L; j++) {
            uint64_t a = j < lodd ? odd[j] : 0;
            out[j] = j < leven ? orc_fe_add(a, even[j], M) : a;
        }
        L = orc_poly_trim(out, L);
        deg = (int64_t)L - 1;
    }
    *olen = L;
    free(odd); free(even);
    return deg;
}

/* Faithful commit.  coeffs: d values (< M).  Optional outputs:
 *   layers (all layers concatenated, sizes n, n/2, ...), trees (all layer
 *   trees concatenated, each orc_merkle_nodes_count(n_k) nodes).
 * forced_betas (nullable): test hook replacing the channel's beta (the
 * channel still absorbs roots so the transcript continues).
 * Returns 0, or -1 on invalid input (d > n). */
int orc_fri_commit_faithful(const uint64_t* coeffs, size_t d, uint32_t log_n, uint64_t offset,
                            uint64_t gen, uint64_t M, orc_channel* ch,
                            const uint64_t* forced_betas, orc_fri_result* res,
                            uint64_t* layers_out, uint8_t* trees_out) {
    size_t n = (size_t)1 << log_n;
    if (d > n) return -1;
    uint64_t omega = orc_fe_pow(gen, (M - 1) / n, M);
    uint64_t* poly = (uint64_t*)malloc((d + 1) * sizeof(uint64_t));
    uint64_t* npoly = (uint64_t*)malloc((d + 1) * sizeof(uint64_t));
    memcpy(poly, coeffs, d * sizeof(uint64_t));
    size_t plen = orc_poly_trim(poly, d);
    int64_t pdeg = (int64_t)plen - 1;
    uint64_t* dom = (uint64_t*)malloc(n * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++) dom[i] = orc_fe_mul(offset, orc_fe_pow(omega, i, M), M);  /* coset_fri.rs:34 */
    uint64_t* ev = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint8_t* nodes = (uint8_t*)malloc(32 * orc_merkle_nodes_count(n));
    size_t m = n, lay_off = 0, tree_off = 0;
    memset(res, 0, sizeof *res);
    for (uint32_t k = 0;; k++) {
        #pragma omp parallel for schedule(dynamic, 64) if (m * plen > 65536)
        for (long i = 0; i < (long)m; i++) ev[i] = orc_poly_evaluate(poly, plen, dom[i], M);
        size_t cnt = orc_merkle_build(ev, m, nodes);
        memcpy(res->roots[k], nodes + 32 * (cnt - 1), 32);
        if (layers_out) memcpy(layers_out + lay_off, ev, m * sizeof(uint64_t));
        if (trees_out) memcpy(trees_out + 32 * tree_off, nodes, 32 * cnt);
        lay_off += m; tree_off += cnt;
        send_root(ch, res->roots[k]);                              /* fri_commit.rs:86 / :100 */
        res->n_layers = k + 1;
        if (pdeg < 1) break;                                        /* fri_commit.rs:89 */
        uint64_t beta = orc_channel_receive_fe(ch, M);              /* :91 */
        if (forced_betas) beta = forced_betas[k];
        res->betas[k] = beta;
        size_t nl;
        pdeg = next_fri_polynomial(poly, plen, beta, M, npoly, &nl);   /* :94 -> :32-50 */
        memcpy(poly, npoly, nl * sizeof(uint64_t));
        plen = nl;
        for (size_t i = 0; i < m / 2; i++) dom[i] = orc_fe_pow(dom[i], 2, M);   /* :18-24 */
        m /= 2;
        res->n_rounds = k + 1;
        if (m == 0) { free(poly); free(npoly); free(dom); free(ev); free(nodes); return -1; }
    }
    res->final_degree = pdeg;
    res->final_value = (pdeg == -1) ? 0 : poly[0];                 /* :109-113 */
    uint8_t fb[8];
    orc_fe_to_bytes(res->final_value, fb);
    orc_channel_send(ch, fb, 8);                                    /* :114 */
    free(poly); free(npoly); free(dom); free(ev); free(nodes);
    return 0;
}

/* ======================================================================
 * B.   Fast CPU path (same results, different algorithms)
 *      - coset LDE via radix-2 NTT (replaces Horner at fri_commit.rs:78)
 *      - evaluation-form fold  L'[i] = (a+b)/2 + beta (a-b)/(2 x_i)
 *        (bit-identical to the coefficient fold + re-evaluation,
 *        fri_commit.rs:53-65, since x_{i+m/2} = -x_i on the coset)
 *      - batch inverse (Montgomery trick; inverse(0) = 0 as element.rs:54-57)
 *      - the coefficient-form fold is still run (O(d)) for the exact
 *        degree / round count / final value of fri_commit.rs:89,109-113.
 * ====================================================================== */
static void bitrev_permute(uint64_t* a, size_t n) {
    for (size_t i = 1, j = 0; i < n; i++) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) { uint64_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
}

/* In-place natural-order NTT: a[k] <- sum_j a[j] w^(jk), w of order n. */
void orc_ntt(uint64_t* a, size_t n, uint64_t w, uint64_t M) {
    bitrev_permute(a, n);
    for (size_t len = 2; len <= n; len <<= 1) {
        uint64_t wl = orc_fe_pow(w, n / len, M);
        size_t h = len / 2;
        uint64_t* tw = (uint64_t*)malloc(h * sizeof(uint64_t));
        tw[0] = 1;
        for (size_t j = 1; j < h; j++) tw[j] = orc_fe_mul(tw[j - 1], wl, M);
        #pragma omp parallel for schedule(static) if (n >= 1 << 14)
        for (long i = 0; i < (long)n; i += (long)len)
            for (size_t j = 0; j < h; j++) {
                uint64_t u = a[i + j], v = orc_fe_mul(a[i + j + h], tw[j], M);
                a[i + j] = orc_fe_add(u, v, M);
                a[i + j + h] = orc_fe_sub(u, v, M);
            }
        free(tw);
    }
}

/* evals[i] = P(offset * omega_n^i), P given by d coefficients (d <= n). */
int orc_lde(const uint64_t* coeffs, size_t d, uint32_t log_n, uint64_t offset, uint64_t gen,
            uint64_t M, uint64_t* evals) {
    size_t n = (size_t)1 << log_n;
    if (d > n) return -1;
    uint64_t omega = orc_fe_pow(gen, (M - 1) / n, M);
    uint64_t s = 1;
    for (size_t j = 0; j < n; j++) {
        evals[j] = j < d ? orc_fe_mul(coeffs[j], s, M) : 0;
        s = orc_fe_mul(s, offset, M);
    }
    orc_ntt(evals, n, omega, M);
    return 0;
}

/* Interpolation on the coset offset*<omega_n>: coeffs (length n, untrimmed)
 * such that P(offset*omega^i) = ys[i].  Returns trimmed length — identical
 * to orc_interpolate_lagrange on the same points (unique interpolant). */
size_t orc_interpolate_coset(const uint64_t* ys, uint32_t log_n, uint64_t offset, uint64_t gen,
                             uint64_t M, uint64_t* coeffs) {
    size_t n = (size_t)1 << log_n;
    uint64_t omega = orc_fe_pow(gen, (M - 1) / n, M);
    memcpy(coeffs, ys, n * sizeof(uint64_t));
    orc_ntt(coeffs, n, orc_fe_inverse(omega, M), M);
    uint64_t ninv = orc_fe_inverse(n % M, M), oinv = orc_fe_inverse(offset, M), s = ninv;
    for (size_t j = 0; j < n; j++) { coeffs[j] = orc_fe_mul(coeffs[j], s, M); s = orc_fe_mul(s, oinv, M); }
    return orc_poly_trim(coeffs, n);
}

/* Batch inverse with inverse(0) = 0 (element.rs:54-57). */
void orc_batch_inverse(const uint64_t* in, uint64_t* out, size_t n, uint64_t M) {
    uint64_t acc = 1;
    for (size_t i = 0; i < n; i++) { out[i] = acc; if (in[i]) acc = orc_fe_mul(acc, in[i], M); }
    uint64_t inv = orc_fe_inverse(acc, M);
    for (size_t i = n; i-- > 0;) {
        if (in[i] == 0) { out[i] = 0; continue; }
        out[i] = orc_fe_mul(out[i], inv, M);
        inv = orc_fe_mul(inv, in[i], M);
    }
}

/* Evaluation-form fold of a layer of size m on domain x_i = off_k * w_m^i. */
void orc_fold_eval(const uint64_t* L, size_t m, uint64_t off_k, uint64_t w_m, uint64_t beta,
                   uint64_t M, uint64_t* out) {
    size_t h = m / 2;
    uint64_t inv2 = orc_fe_inverse(2, M);
    uint64_t* xs = (uint64_t*)malloc(h * sizeof(uint64_t));
    uint64_t* xi = (uint64_t*)malloc(h * sizeof(uint64_t));
    uint64_t x = off_k;
    for (size_t i = 0; i < h; i++) { xs[i] = x; x = orc_fe_mul(x, w_m, M); }
    orc_batch_inverse(xs, xi, h, M);
    #pragma omp parallel for schedule(static) if (h >= 1 << 14)
    for (long i = 0; i < (long)h; i++) {
        uint64_t a = L[i], b = L[i + h];
        uint64_t s = orc_fe_add(a, b, M), t = orc_fe_sub(a, b, M);
        uint64_t v = orc_fe_add(s, orc_fe_mul(beta, orc_fe_mul(t, xi[i], M), M), M);
        out[i] = orc_fe_mul(v, inv2, M);
    }
    free(xs); free(xi);
}

int orc_fri_commit_fast(const uint64_t* coeffs, size_t d, uint32_t log_n, uint64_t offset,
                        uint64_t gen, uint64_t M, orc_channel* ch,
                        const uint64_t* forced_betas, orc_fri_result* res,
                        uint64_t* layers_out, uint8_t* trees_out) {
    size_t n = (size_t)1 << log_n;
    if (d > n) return -1;
    memset(res, 0, sizeof *res);
    uint64_t* poly = (uint64_t*)malloc((d + 1) * sizeof(uint64_t));
    uint64_t* npoly = (uint64_t*)malloc((d + 1) * sizeof(uint64_t));
    memcpy(poly, coeffs, d * sizeof(uint64_t));
    size_t plen = orc_poly_trim(poly, d);
    int64_t pdeg = (int64_t)plen - 1;
    uint64_t* cur = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint64_t* nxt = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint8_t* nodes = (uint8_t*)malloc(32 * orc_merkle_nodes_count(n));
    orc_lde(coeffs, d, log_n, offset, gen, M, cur);
    size_t m = n, lay_off = 0, tree_off = 0;
    uint64_t off_k = offset, w = orc_fe_pow(gen, (M - 1) / n, M);
    for (uint32_t k = 0;; k++) {
        size_t cnt = orc_merkle_build(cur, m, nodes);
        memcpy(res->roots[k], nodes + 32 * (cnt - 1), 32);
        if (layers_out) memcpy(layers_out + lay_off, cur, m * sizeof(uint64_t));
        if (trees_out) memcpy(trees_out + 32 * tree_off, nodes, 32 * cnt);
        lay_off += m; tree_off += cnt;
        send_root(ch, res->roots[k]);
        res->n_layers = k + 1;
        if (pdeg < 1) break;
        uint64_t beta = orc_channel_receive_fe(ch, M);
        if (forced_betas) beta = forced_betas[k];
        res->betas[k] = beta;
        size_t nl;
        pdeg = next_fri_polynomial(poly, plen, beta, M, npoly, &nl);
        memcpy(poly, npoly, nl * sizeof(uint64_t));
        plen = nl;
        if (m < 2) { free(poly); free(npoly); free(cur); free(nxt); free(nodes); return -1; }
        orc_fold_eval(cur, m, off_k, w, beta, M, nxt);
        uint64_t* t = cur; cur = nxt; nxt = t;
        m /= 2;
        off_k = orc_fe_mul(off_k, off_k, M);
        w = orc_fe_mul(w, w, M);
        res->n_rounds = k + 1;
    }
    res->final_degree = pdeg;
    res->final_value = (pdeg == -1) ? 0 : poly[0];
    uint8_t fb[8];
    orc_fe_to_bytes(res->final_value, fb);
    orc_channel_send(ch, fb, 8);
    free(poly); free(npoly); free(cur); free(nxt); free(nodes);
    return 0;
}

/* ======================================================================
 * C.   Prover slice — STARK-101 FibonacciSq (BASELINE configs[3]).
 *      The reference's src/prover, src/trace, src/composition are EMPTY;
 *      restated from the STARK-101 tutorial on the full trace subgroup
 *      G = <g>, |G| = T (PARITY UNPINNED; the Python twin's
 *      fibsq_cp_faithful builds the same polynomial with the reference's
 *      div_rem / mul / compose, ops.rs:114-237).
 *      CP = a0 (f-1)/(x-1) + a1 (f-A)/(x-g^{T-1})
 *         + a2 (f(g^2x) - f(gx)^2 - f^2)(x-g^{T-2})(x-g^{T-1})/(x^T-1)
 * ====================================================================== */
void orc_fibsq_trace(uint64_t a1, size_t T, uint64_t M, uint64_t* out) {
    for (size_t i = 0; i < T; i++)
        out[i] = i == 0 ? 1 : i == 1 ? a1 % M
                 : orc_fe_add(orc_fe_mul(out[i - 1], out[i - 1], M), orc_fe_mul(out[i - 2], out[i - 2], M), M);
}

/* f: LDE of the trace polynomial on offset*<w_n>, n = 2^(log_t+log_b). */
int orc_fibsq_cp_evals(const uint64_t* f, uint32_t log_t, uint32_t log_b, uint64_t offset, uint64_t gen,
                       uint64_t M, uint64_t a_last, const uint64_t* alphas, uint64_t* out) {
    const uint32_t L = log_t + log_b;
    const size_t n = (size_t)1 << L, T = (size_t)1 << log_t, B = (size_t)1 << log_b;
    const uint64_t w = orc_fe_pow(gen, (M - 1) >> L, M), g = orc_fe_pow(gen, (M - 1) >> log_t, M);
    const uint64_t glast = orc_fe_pow(g, T - 1, M), gprev = orc_fe_pow(g, T - 2, M);
    uint64_t* x = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint64_t* den = (uint64_t*)malloc(2 * n * sizeof(uint64_t));
    uint64_t* dinv = (uint64_t*)malloc(2 * n * sizeof(uint64_t));
    if (!x || !den || !dinv) { free(x); free(den); free(dinv); return -1; }
    uint64_t xv = offset;
    for (size_t i = 0; i < n; i++) { x[i] = xv; xv = orc_fe_mul(xv, w, M); }
    for (size_t i = 0; i < n; i++) {
        den[i] = orc_fe_sub(x[i], 1, M);                                   /* x - 1        */
        den[n + i] = orc_fe_sub(x[i], glast, M);                           /* x - g^{T-1}  */
    }
    orc_batch_inverse(den, dinv, 2 * n, M);
    uint64_t zinv[64];                      /* x^T depends on i mod B only */
    for (size_t j = 0; j < B && j < 64; j++) zinv[j] = orc_fe_inverse(orc_fe_sub(orc_fe_pow(x[j], T, M), 1, M), M);
    #pragma omp parallel for schedule(static) if (n >= 1 << 14)
    for (long li = 0; li < (long)n; li++) {
        size_t i = (size_t)li;
        uint64_t f0 = f[i], f1 = f[(i + B) % n], f2 = f[(i + 2 * B) % n];
        uint64_t p0 = orc_fe_mul(orc_fe_sub(f0, 1, M), dinv[i], M);
        uint64_t p1 = orc_fe_mul(orc_fe_sub(f0, a_last, M), dinv[n + i], M);
        uint64_t num = orc_fe_sub(f2, orc_fe_add(orc_fe_mul(f1, f1, M), orc_fe_mul(f0, f0, M), M), M);
        uint64_t zf = orc_fe_mul(orc_fe_mul(orc_fe_sub(x[i], gprev, M), orc_fe_sub(x[i], glast, M), M),
                                 zinv[i % B], M);
        uint64_t p2 = orc_fe_mul(num, zf, M);
        out[i] = orc_fe_add(orc_fe_add(orc_fe_mul(p0, alphas[0], M), orc_fe_mul(p1, alphas[1], M), M),
                            orc_fe_mul(p2, alphas[2], M), M);
    }
    free(x); free(den); free(dinv);
    return 0;
}

/* Commit phase of the prover (no queries): trace -> interpolate on G ->
 * LDE -> Merkle -> send(root hex) -> alpha_0..2 -> CP evals -> coefficients
 * -> orc_fri_commit_fast.  Optional outputs as orc_fri_commit_fast, plus the
 * trace LDE (n values) and its tree (orc_merkle_build layout). */
int orc_fibsq_prove_commit(uint64_t a1, uint32_t log_t, uint32_t log_b, uint64_t offset, uint64_t gen, uint64_t M,
                           orc_channel* ch, uint8_t trace_root[32], uint64_t alphas[3], orc_fri_result* res,
                           uint64_t* f_eval_out, uint8_t* f_tree_out, uint64_t* layers_out, uint8_t* trees_out) {
    const uint32_t L = log_t + log_b;
    const size_t n = (size_t)1 << L, T = (size_t)1 << log_t;
    uint64_t* tr = (uint64_t*)malloc(T * sizeof(uint64_t));
    uint64_t* fc = (uint64_t*)malloc(T * sizeof(uint64_t));
    uint64_t* fe = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint64_t* cp = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint64_t* cc = (uint64_t*)malloc(n * sizeof(uint64_t));
    size_t cnt = orc_merkle_nodes_count(n);
    uint8_t* nodes = (uint8_t*)malloc(32 * cnt);
    int rc = -1;
    if (!tr || !fc || !fe || !cp || !cc || !nodes) goto out;
    orc_fibsq_trace(a1, T, M, tr);
    {
        size_t fl = orc_interpolate_coset(tr, log_t, 1, gen, M, fc);
        if (orc_lde(fc, fl, L, offset, gen, M, fe)) goto out;
    }
    orc_merkle_build(fe, n, nodes);
    memcpy(trace_root, nodes + 32 * (cnt - 1), 32);
    send_root(ch, trace_root);
    for (int j = 0; j < 3; j++) alphas[j] = orc_channel_receive_fe(ch, M);
    if (orc_fibsq_cp_evals(fe, log_t, log_b, offset, gen, M, tr[T - 1], alphas, cp)) goto out;
    {
        size_t cl = orc_interpolate_coset(cp, L, offset, gen, M, cc);
        rc = orc_fri_commit_fast(cc, cl, L, offset, gen, M, ch, NULL, res, layers_out, trees_out);
    }
    if (f_eval_out) memcpy(f_eval_out, fe, n * sizeof(uint64_t));
    if (f_tree_out) memcpy(f_tree_out, nodes, 32 * cnt);
out:
    free(tr); free(fc); free(fe); free(cp); free(cc); free(nodes);
    return rc;
}

void orc_set_num_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
