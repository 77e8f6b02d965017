// stark101.cpp — host side of the C++ mirror (see stark101.hpp).  Everything
// field-sized on the commit path goes through libfri_amd.so; this file holds
// the transcript (SHA-256 on the host, as the reference's Channel does it),
// argument checks that reproduce the reference's panics, and the glue that
// turns fri_commit_result into Channel messages and an FRIProof.
#include "stark101.hpp"

#include <functional>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

namespace stark101 {

// ------------------------------------------------------------------ SHA-256
namespace {
constexpr uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void compress_scalar(uint32_t h[8], const uint8_t* data, size_t nblocks) {
    for (; nblocks; nblocks--, data += 64) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)data[4 * i] << 24 | (uint32_t)data[4 * i + 1] << 16 | (uint32_t)data[4 * i + 2] << 8 |
                   data[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
        for (int i = 0; i < 64; i++) {
            uint32_t t1 = k + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
            uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
    }
}

#if defined(__x86_64__)
// x86 SHA extensions: the transcript hashes ~3000 blocks per STARK-101 proof
// (hex-encoded authentication paths), which dominates the host side of
// prove/verify.  State kept as the instructions want it: ABEF = {F,E,B,A},
// CDGH = {H,G,D,C} (dword 0 first).  Each 4-round group: W+K, two
// sha256rnds2 (rounds 4g, 4g+1 from dwords 0-1, 4g+2, 4g+3 from 2-3); the
// schedule W[t] = s1(W[t-2]) + W[t-7] + s0(W[t-15]) + W[t-16] is msg1 (adds
// s0) + the W[t-7] lane window + msg2 (adds s1 with its in-vector chain).
__attribute__((target("sha,sse4.1,ssse3"))) void compress_shani(uint32_t h[8], const uint8_t* data, size_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    const __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h)), 0xB1);      // B,A,D,C
    const __m128i efgh = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h + 4)), 0x1B);  // H,G,F,E
    __m128i abef = _mm_alignr_epi8(abcd, efgh, 8);     // F,E,B,A
    __m128i cdgh = _mm_blend_epi16(efgh, abcd, 0xF0);  // H,G,D,C
    for (; nblocks; nblocks--, data += 64) {
        const __m128i abef0 = abef, cdgh0 = cdgh;
        __m128i m[4];
        for (int j = 0; j < 4; j++)
            m[j] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16 * j)), bswap);
        for (int g = 0; g < 16; g++) {
            if (g >= 4) {
                __m128i x = _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]);
                x = _mm_add_epi32(x, _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4));
                m[g & 3] = _mm_sha256msg2_epu32(x, m[(g + 3) & 3]);
            }
            __m128i wk = _mm_add_epi32(m[g & 3], _mm_loadu_si128(reinterpret_cast<const __m128i*>(K256 + 4 * g)));
            cdgh = _mm_sha256rnds2_epu32(cdgh, abef, wk);            // -> new ABEF; old ABEF is the new CDGH
            wk = _mm_shuffle_epi32(wk, 0x0E);
            abef = _mm_sha256rnds2_epu32(abef, cdgh, wk);
        }
        abef = _mm_add_epi32(abef, abef0);
        cdgh = _mm_add_epi32(cdgh, cdgh0);
    }
    const __m128i feba = _mm_shuffle_epi32(abef, 0x1B);  // A,B,E,F
    const __m128i dchg = _mm_shuffle_epi32(cdgh, 0xB1);  // G,H,C,D
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h), _mm_blend_epi16(feba, dchg, 0xF0));      // A,B,C,D
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h + 4), _mm_alignr_epi8(dchg, feba, 8));     // E,F,G,H
}

bool cpu_has_sha() {
    unsigned a = 0, b = 0, c = 0, d = 0;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    return (b >> 29) & 1u;
}
#endif

void compress_blocks(uint32_t h[8], const uint8_t* data, size_t nblocks) {
#if defined(__x86_64__)
    static const bool ni = cpu_has_sha() && std::getenv("STARK101_NO_SHANI") == nullptr;
    if (ni) {
        compress_shani(h, data, nblocks);
        return;
    }
#endif
    compress_scalar(h, data, nblocks);
}
}  // namespace

namespace sha {
namespace {
std::array<uint8_t, 32> digest_with(void (*fn)(uint32_t*, const uint8_t*, size_t), const uint8_t* data, size_t len) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = len / 64;
    fn(h, data, full);
    uint8_t tail[128] = {0};
    size_t rem = len - 64 * full;
    if (rem) std::memcpy(tail, data + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tl = rem + 9 <= 64 ? 64 : 128;
    uint64_t bits = static_cast<uint64_t>(len) * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = static_cast<uint8_t>(bits >> (8 * i));
    fn(h, tail, tl / 64);
    std::array<uint8_t, 32> out{};
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = static_cast<uint8_t>(h[i] >> (24 - 8 * j));
    return out;
}
}  // namespace

std::array<uint8_t, 32> digest(const uint8_t* data, size_t len) { return digest_with(compress_blocks, data, len); }
std::array<uint8_t, 32> digest_portable(const uint8_t* data, size_t len) {
    return digest_with(compress_scalar, data, len);
}
bool accelerated() {
#if defined(__x86_64__)
    return cpu_has_sha() && std::getenv("STARK101_NO_SHANI") == nullptr;
#else
    return false;
#endif
}

std::string hex(const uint8_t* data, size_t len) {
    static const char* d = "0123456789abcdef";
    std::string s(2 * len, '0');
    for (size_t i = 0; i < len; i++) {
        s[2 * i] = d[data[i] >> 4];
        s[2 * i + 1] = d[data[i] & 15];
    }
    return s;
}

std::string digest_hex(const std::string& s) {
    auto dg = digest(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    return hex(dg.data(), dg.size());
}

std::vector<uint8_t> from_hex(const std::string& s) {
    if (s.size() % 2) throw Panic("odd-length hex string");
    auto nib = [](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        throw Panic("invalid hex digit");
    };
    std::vector<uint8_t> out(s.size() / 2);
    for (size_t i = 0; i < out.size(); i++) out[i] = static_cast<uint8_t>(nib(s[2 * i]) << 4 | nib(s[2 * i + 1]));
    return out;
}
}  // namespace sha

uint64_t os_random_u64() {
    static thread_local std::random_device rd;      // OsRng (element.rs:32-36)
    return (static_cast<uint64_t>(rd()) << 32) ^ rd();
}

FE omega(uint32_t log_n) {
    if (log_n > 30) throw Panic("no subgroup of order 2^" + std::to_string(log_n));
    return FE(FRI_GENERATOR).pow((P - 1) >> log_n);
}

// ---------------------------------------------------------------------- Gpu
Gpu::Gpu(int device, uint32_t log_n_max) : log_n_max_(log_n_max) {
    int rc = fri_ctx_create(device, log_n_max, &ctx_);
    if (rc != FRI_OK) {
        std::string msg = ctx_ ? fri_last_error(ctx_) : "";
        if (ctx_) fri_ctx_destroy(ctx_);
        ctx_ = nullptr;
        throw Panic("fri_ctx_create failed (code " + std::to_string(rc) + ")" + (msg.empty() ? "" : ": " + msg));
    }
}

Gpu::Gpu(const std::vector<int>& devices, uint32_t log_n_max, int transport)
    : log_n_max_(log_n_max), n_ranks_(static_cast<uint32_t>(devices.size())) {
    int rc = fri_ctx_create_multi(devices.data(), static_cast<uint32_t>(devices.size()), log_n_max, transport, &ctx_);
    if (rc != FRI_OK) {
        ctx_ = nullptr;
        throw Panic("fri_ctx_create_multi failed (code " + std::to_string(rc) + ")");
    }
}

Gpu::Gpu(Default, uint32_t log_n_max) : log_n_max_(log_n_max) {
    int rc = fri_ctx_create_default(log_n_max, &ctx_, &n_ranks_);
    if (rc != FRI_OK) {
        ctx_ = nullptr;
        throw Panic("fri_ctx_create_default failed (code " + std::to_string(rc) +
                    (rc == FRI_EINVAL ? ": malformed FRI_DEVICES / FRI_TRANSPORT)" : ")"));
    }
}

Gpu::~Gpu() {
    if (ctx_) fri_ctx_destroy(ctx_);
}

void Gpu::check(int rc, const char* what) const {
    if (rc != FRI_OK) throw Panic(std::string(what) + ": " + fri_last_error(ctx_) + " (code " + std::to_string(rc) + ")");
}

std::shared_ptr<Gpu> Gpu::thread_default(uint32_t log_n) {
    static thread_local std::shared_ptr<Gpu> g;
    const uint32_t want = log_n < 12 ? 12 : log_n;
    if (!g || g->log_n_max() < want) g = std::make_shared<Gpu>(Gpu::Default{}, want);
    return g;
}

namespace {
uint32_t ceil_log2(size_t n) {
    uint32_t l = 0;
    while ((size_t{1} << l) < n) l++;
    return l;
}

std::vector<uint32_t> to_u32(const std::vector<FE>& v) {
    std::vector<uint32_t> o(v.size());
    for (size_t i = 0; i < v.size(); i++) o[i] = static_cast<uint32_t>(v[i].value());
    return o;
}

std::vector<FE> to_fe(const uint32_t* v, size_t n) {
    std::vector<FE> o(n);
    for (size_t i = 0; i < n; i++) o[i] = FE(v[i]);
    return o;
}

// The device evaluates on offset*<omega_n>: accept exactly that domain.
// Checks the length, D[0] = offset != 0, D[1] = offset*omega_n and the last
// point; the remaining points are the caller's contract (coset_fri.rs:32-36),
// as materialising and comparing 2^24 points would cost more than the commit.
uint32_t coset_log_n(const std::vector<FE>& d, FE* offset) {
    const size_t n = d.size();
    if (n == 0 || (n & (n - 1))) throw Panic("domain size must be a power of two (got " + std::to_string(n) + ")");
    const uint32_t log_n = ceil_log2(n);
    const FE off = d[0], w = omega(log_n);
    if (off == FE::zero()) throw Panic("domain offset must be non-zero");
    if (n > 1 && (d[1] != off * w || d[n - 1] != off * w.pow(n - 1)))
        throw Panic("domain is not the coset offset*<omega_n> in natural order (coset_fri.rs:32-36)");
    *offset = off;
    return log_n;
}
}  // namespace

// --------------------------------------------------------------- MerkleTree
MerkleTree::MerkleTree(const std::vector<FE>& data) {
    if (data.empty()) throw Panic("MerkleTree of no leaves has no root (merkle/mod.rs:25)");
    gpu_ = Gpu::thread_default(ceil_log2(data.size()));
    auto v = to_u32(data);
    uint8_t root[32];
    gpu_->check(fri_merkle_root(gpu_->ctx(), v.data(), v.size(), root), "fri_merkle_root");
    root_hex_ = sha::hex(root, 32);
    gpu_.reset();                                     // standalone: root only
}

std::array<uint8_t, 32> MerkleTree::root_bytes() const {
    auto b = sha::from_hex(root_hex_);
    std::array<uint8_t, 32> r{};
    std::memcpy(r.data(), b.data(), 32);
    return r;
}

std::vector<uint8_t> MerkleTree::get_authentication_path(size_t index) const {
    if (!gpu_) throw Panic("authentication paths are served by the trees of an FRIProof (standalone trees keep only the root)");
    if (gpu_->generation() != gen_) throw Panic("FRIProof layers were replaced by a later commit on the same Gpu");
    uint32_t value = 0, depth = 0;
    std::vector<uint8_t> path(32 * 32);
    gpu_->check(fri_auth_path(gpu_->ctx(), layer_, index, &value, path.data(), &depth), "fri_auth_path");
    path.resize(32 * size_t{depth});
    return path;
}

// ----------------------------------------------------------------- FRIProof
bool FRIProof::resident() const { return gpu_ && gpu_->generation() == gen_; }

void FRIProof::require_resident() const {
    if (!resident()) throw Panic("FRIProof layers were replaced by a later commit on the same Gpu");
}

std::vector<FE> FRIProof::fri_layer(size_t k) const {
    require_resident();
    if (k >= n_layers()) throw Panic("no such FRI layer");
    const size_t m = size_t{1} << (log_n - k);
    std::vector<uint32_t> v(m);
    gpu_->check(fri_layer_copy(gpu_->ctx(), static_cast<uint32_t>(k), v.data(), m), "fri_layer_copy");
    return to_fe(v.data(), m);
}

std::vector<std::vector<FE>> FRIProof::fri_layers() const {
    std::vector<std::vector<FE>> out;
    for (size_t k = 0; k < n_layers(); k++) out.push_back(fri_layer(k));
    return out;
}

// --------------------------------------------------------------- fri_commit
FRIProof fri_commit_coset(const Poly& poly, uint32_t log_n, FE offset, FriChannel& channel,
                          const std::shared_ptr<Gpu>& gpu) {
    if (!gpu) throw Panic("fri_commit: no Gpu");
    if (log_n > gpu->log_n_max()) throw Panic("fri_commit: codeword 2^" + std::to_string(log_n) + " exceeds the context");
    std::vector<uint32_t> coeffs = to_u32(poly.coefficients);
    fri_channel_state cin{};
    const fri_channel_state* pin = nullptr;
    if (!channel.state.empty()) {
        auto st = sha::from_hex(channel.state);
        if (st.size() != 32) throw Panic("Channel state is not a SHA-256 digest");
        std::memcpy(cin.digest, st.data(), 32);
        cin.has_state = 1;
        pin = &cin;
    }
    fri_commit_result res{};
    gpu->bump();                                    // previous layers are overwritten from here on
    gpu->check(fri_commit(gpu->ctx(), coeffs.data(), coeffs.size(), log_n, static_cast<uint32_t>(offset.value()), pin,
                          0, nullptr, &res),
               "fri_commit");

    return FRIProof::mirror(res, log_n, gpu, channel);
}

std::vector<FRIProof> fri_commit_pipelined(const std::vector<Poly>& polys, uint32_t log_n, FE offset,
                                           std::vector<FriChannel>& channels, const std::shared_ptr<Gpu>& gpu) {
    if (!gpu) throw Panic("fri_commit: no Gpu");
    if (channels.size() != polys.size()) throw Panic("fri_commit_pipelined: one channel per polynomial");
    if (log_n > gpu->log_n_max()) throw Panic("fri_commit: codeword 2^" + std::to_string(log_n) + " exceeds the context");
    struct Pending { size_t i; uint64_t ticket, gen; };
    std::vector<FRIProof> out(polys.size());
    std::vector<Pending> pend;
    auto collect = [&](const Pending& p) {
        fri_commit_result res{};
        gpu->check(fri_commit_wait(gpu->ctx(), p.ticket, &res), "fri_commit_wait");
        out[p.i] = FRIProof::mirror(res, log_n, gpu, channels[p.i], p.gen);
    };
    try {
        for (size_t i = 0; i < polys.size(); i++) {
            if (pend.size() == FRI_DEFAULT_LANES) {   // one pending commit per commit lane
                const Pending p = pend.front();
                pend.erase(pend.begin());   // waited below even if collect throws
                collect(p);
            }
            std::vector<uint32_t> coeffs = to_u32(polys[i].coefficients);
            fri_channel_state cin{};
            const fri_channel_state* pin = nullptr;
            if (!channels[i].state.empty()) {
                auto st = sha::from_hex(channels[i].state);
                if (st.size() != 32) throw Panic("Channel state is not a SHA-256 digest");
                std::memcpy(cin.digest, st.data(), 32);
                cin.has_state = 1;
                pin = &cin;
            }
            uint64_t ticket = 0;
            const uint64_t gen = gpu->bump();          // this commit's layers replace the previous ones
            gpu->check(fri_commit_async(gpu->ctx(), coeffs.data(), coeffs.size(), log_n,
                                        static_cast<uint32_t>(offset.value()), pin, 0, nullptr, &ticket),
                       "fri_commit_async");
            pend.push_back({i, ticket, gen});
        }
        while (!pend.empty()) {
            const Pending p = pend.front();
            pend.erase(pend.begin());
            collect(p);
        }
    } catch (...) {
        // a failed commit (reported at its wait) must not leave the other
        // result slots of this per-thread Gpu pending: wait for them all,
        // discarding their results, then re-throw
        for (const Pending& p : pend) {
            fri_commit_result res{};
            (void)fri_commit_wait(gpu->ctx(), p.ticket, &res);
        }
        throw;
    }
    return out;
}

FRIProof FRIProof::mirror(const fri_commit_result& res, uint32_t log_n, const std::shared_ptr<Gpu>& gpu,
                          FriChannel& channel, uint64_t gen) {
    // The channel messages the reference's loop produced (fri_commit.rs:84-114):
    // root_hex bytes per layer, beta (8 B BE, proof only) per round, final value.
    FRIProof proof;
    proof.log_n = log_n;
    proof.gpu_ = gpu;
    proof.gen_ = gen ? gen : gpu->generation();
    for (uint32_t k = 0; k < res.n_layers; k++) {
        const std::string hex = sha::hex(res.roots[k], 32);
        std::vector<uint8_t> msg(hex.begin(), hex.end());
        channel.proof.push_back(msg);
        channel.compressed_proof.push_back(msg);
        if (k < res.n_rounds) {
            channel.proof.push_back(FriChannel::be64(res.betas[k]));
            proof.betas.push_back(FE(res.betas[k]));
        }
        MerkleTree t;
        t.root_hex_ = hex;
        t.gpu_ = gpu;
        t.gen_ = proof.gen_;
        t.layer_ = k;
        proof.fri_merkles.push_back(std::move(t));
    }
    auto fv = FriChannel::be64(res.final_value);
    channel.proof.push_back(fv);
    channel.compressed_proof.push_back(fv);
    channel.state = res.channel_out.has_state ? sha::hex(res.channel_out.digest, 32) : "";
    proof.final_poly = res.final_degree < 0 ? Poly::zero() : Poly({FE(res.final_value)});
    return proof;
}

FRIProof fri_commit(Poly poly, std::vector<FE> domain, FriChannel& channel) {
    FE offset;
    const uint32_t log_n = coset_log_n(domain, &offset);
    domain.clear();
    domain.shrink_to_fit();
    return fri_commit_coset(poly, log_n, offset, channel, Gpu::thread_default(log_n));
}

FRIProof fri_commit(const Poly& poly, const Coset& coset, FriChannel& channel) {
    const size_t n = coset.domain_size;
    if (n == 0 || (n & (n - 1))) throw Panic("domain size must be a power of two");
    const uint32_t log_n = ceil_log2(n);
    if (coset.omega != omega(log_n)) throw Panic("coset omega must be g^((p-1)/n) (frozen spec)");
    if (coset.offset == FE::zero()) throw Panic("domain offset must be non-zero");
    return fri_commit_coset(poly, log_n, coset.offset, channel, Gpu::thread_default(log_n));
}

// ------------------------------------------------------------------ decommit
namespace {
// One query (decommit_fri_layers, fri_commit.rs:137-163) through the gather
// kernel on the commit resident on `gpu`: per layer send value, path,
// sibling value, sibling path (a 1-element layer sends its value first).
// `layers` (optional): the caller's FRIProof.fri_layers, checked against the
// device's openings.
void decommit_query(const Gpu& gpu, uint32_t log_n, size_t n_layers, uint64_t index, FriChannel& channel,
                    const std::vector<std::vector<FE>>* layers) {
    size_t path_bytes = 0;
    for (size_t k = 0; k < n_layers; k++) path_bytes += 2 * 32 * (log_n - k);
    std::vector<uint32_t> values(2 * n_layers);
    std::vector<uint8_t> paths(path_bytes ? path_bytes : 1);
    size_t got = 0;
    gpu.check(fri_decommit_query(gpu.ctx(), index, values.data(), values.size(), paths.data(), paths.size(), &got),
              "fri_decommit_query");
    size_t off = 0;
    for (size_t k = 0; k < n_layers; k++) {
        const size_t depth = log_n - k, pb = 32 * depth, m = size_t{1} << depth;
        if (layers) {
            const std::vector<FE>& lk = (*layers)[k];
            const size_t i = index % m, sib = (i + m / 2) % m;
            if (lk.size() != m || lk[i].value() != values[2 * k] || lk[sib].value() != values[2 * k + 1])
                throw Panic("fri_layers do not belong to the commit of these fri_merkles (layer " + std::to_string(k) +
                            ")");
        }
        std::vector<uint8_t> path(paths.begin() + off, paths.begin() + off + pb);
        std::vector<uint8_t> spath(paths.begin() + off + pb, paths.begin() + off + 2 * pb);
        off += 2 * pb;
        auto v = FE(values[2 * k]).to_bytes(), sv = FE(values[2 * k + 1]).to_bytes();
        if (depth == 0) channel.send(v);             // fri_commit.rs:147-149: length == 1 sends it first
        channel.send(v);
        channel.send(path);
        channel.send(sv);
        channel.send(spath);
    }
}
}  // namespace

void decommit_fri_layers(size_t index, const FRIProof& proof, FriChannel& channel) {
    proof.require_resident();
    decommit_query(*proof.gpu_, proof.log_n, proof.n_layers(), index, channel, nullptr);
}

void decommit_fri(size_t num_queries, size_t max_index, const FRIProof& proof, FriChannel& channel) {
    for (size_t q = 0; q < num_queries; q++) {
        const uint64_t idx = channel.receive_random_int(0, max_index, true);
        decommit_fri_layers(idx, proof, channel);
    }
}

void decommit_fri(size_t num_queries, size_t max_index, const std::vector<std::vector<FE>>& fri_layers,
                  const std::vector<MerkleTree>& fri_merkles, FriChannel& channel) {
    if (fri_merkles.empty()) throw Panic("decommit_fri: no FRI layers");
    if (fri_layers.size() != fri_merkles.size()) throw Panic("decommit_fri: one Merkle tree per FRI layer");
    const MerkleTree& t0 = fri_merkles[0];
    if (!t0.gpu_) throw Panic("decommit_fri: the trees of an FRIProof are device-backed; a standalone tree keeps only its root");
    for (size_t k = 0; k < fri_merkles.size(); k++) {
        const MerkleTree& t = fri_merkles[k];
        if (t.gpu_ != t0.gpu_ || t.gen_ != t0.gen_ || t.layer_ != k)
            throw Panic("decommit_fri: the trees are not the layers of one commit");
    }
    const Gpu& gpu = *t0.gpu_;
    if (gpu.generation() != t0.gen_) throw Panic("FRIProof layers were replaced by a later commit on the same Gpu");
    uint64_t g = 0;
    uint32_t log_n = 0, n_layers = 0;
    gpu.check(fri_commit_info(gpu.ctx(), &g, &log_n, &n_layers), "fri_commit_info");
    if (n_layers != fri_merkles.size() || fri_layers[0].size() != (size_t{1} << log_n))
        throw Panic("decommit_fri: the resident commit is not the one these trees belong to");
    for (size_t q = 0; q < num_queries; q++) {
        const uint64_t idx = channel.receive_random_int(0, max_index, true);
        decommit_query(gpu, log_n, n_layers, idx, channel, &fri_layers);
    }
}

// -------------------------------------------------------------------- verify
namespace {
bool path_ok(uint64_t value, uint64_t index, const std::vector<uint8_t>& path, size_t depth,
             const std::array<uint8_t, 32>& root) {
    if (path.size() != 32 * depth) return false;
    const auto leaf = FE(value).to_bytes();                     // merkle/mod.rs:14-15
    auto h = sha::digest(leaf.data(), 8);
    uint8_t buf[64];
    for (size_t lvl = 0; lvl < depth; lvl++) {
        const uint8_t* sib = path.data() + 32 * lvl;
        if ((index >> lvl) & 1) {
            std::memcpy(buf, sib, 32);
            std::memcpy(buf + 32, h.data(), 32);
        } else {
            std::memcpy(buf, h.data(), 32);
            std::memcpy(buf + 32, sib, 32);
        }
        h = sha::digest(buf, 64);
    }
    return h == root;
}

uint64_t be_u64(const std::vector<uint8_t>& b) {
    uint64_t v = 0;
    for (uint8_t c : b) v = v << 8 | c;
    return v;
}
}  // namespace

namespace {
using Msgs = std::vector<std::vector<uint8_t>>;
using Take = std::function<const std::vector<uint8_t>&()>;
// verify_fri's replay with two hooks for a STARK around the FRI:
// pre_commit consumes the messages before the first FRI root; on_query those
// between a query index and its layer openings and returns the value layer 0
// must hold there (or -1).  A hook rejects by throwing Panic.
bool verify_transcript(const Msgs& msgs, uint32_t log_n, size_t n_layers, size_t num_queries, size_t max_index,
                       FE offset, const std::string& channel_state,
                       const std::function<void(const Take&, FriChannel&)>& pre_commit,
                       const std::function<int64_t(const Take&, FriChannel&, uint64_t)>& on_query) {
    if (n_layers == 0 || n_layers > log_n + 1u) return false;
    size_t pos = 0;
    Take take = [&]() -> const std::vector<uint8_t>& {
        if (pos >= msgs.size()) throw Panic("transcript ended early");
        return msgs[pos++];
    };
    try {
        FriChannel ch;
        ch.state = channel_state;
        if (pre_commit) pre_commit(take, ch);
        std::vector<std::array<uint8_t, 32>> roots;
        std::vector<FE> betas;
        for (size_t k = 0; k < n_layers; k++) {
            const auto& r = take();
            if (r.size() != 64) return false;
            auto rb = sha::from_hex(std::string(r.begin(), r.end()));
            std::array<uint8_t, 32> ra{};
            std::memcpy(ra.data(), rb.data(), 32);
            roots.push_back(ra);
            ch.send(r);
            if (k + 1 < n_layers) {
                FE beta = ch.receive_random_field_element();
                if (take() != FriChannel::be64(beta.value())) return false;
                betas.push_back(beta);
            }
        }
        const auto& fin = take();
        if (fin.size() != 8) return false;
        const uint64_t final_value = be_u64(fin);
        ch.send(fin);
        const FE inv2 = FE(2).inverse();
        for (size_t q = 0; q < num_queries; q++) {
            const uint64_t idx = ch.receive_random_int(0, max_index, true);
            if (take() != FriChannel::be64(idx)) return false;
            const int64_t want0 = on_query ? on_query(take, ch, idx) : -1;
            bool have_prev = false;
            uint64_t pa = 0, pb = 0, pj = 0, pm = 0;           // L[pj], L[pj + pm/2] of layer k-1
            for (size_t k = 0; k < n_layers; k++) {
                const size_t depth = log_n - k;
                const uint64_t m = uint64_t{1} << depth;
                const std::vector<uint8_t>* extra = nullptr;
                if (m == 1) {                                    // fri_commit.rs:147-149 sends layer[0] first
                    extra = &take();
                    ch.send(*extra);
                }
                const uint64_t i = idx % m, sib = (i + m / 2) % m;
                const auto& vb = take();
                if (extra && *extra != vb) return false;
                const auto& path = take();
                const auto& sb = take();
                const auto& spath = take();
                for (auto* msg : {&vb, &path, &sb, &spath}) ch.send(*msg);
                if (vb.size() != 8 || sb.size() != 8) return false;
                const uint64_t v = be_u64(vb), sv = be_u64(sb);
                if (v >= P || sv >= P) return false;
                if (!path_ok(v, i, path, depth, roots[k]) || !path_ok(sv, sib, spath, depth, roots[k])) return false;
                if (k == 0 && want0 >= 0 && v != static_cast<uint64_t>(want0)) return false;
                if (have_prev) {
                    // x = offset^(2^(k-1)) * omega_pm^pj; fold = (a+b)/2 + beta*(a-b)/(2x)  (fri_commit.rs:32-65)
                    const FE x = offset.pow(uint64_t{1} << (k - 1)) * omega(ceil_log2(pm)).pow(pj);
                    const FE a(pa), b(pb);
                    const FE fold = ((a + b) + betas[k - 1] * (a - b) * x.inverse()) * inv2;
                    if (fold.value() != v) return false;
                }
                const uint64_t j = m > 1 ? i % (m / 2) : 0;
                if (i < m / 2 || m == 1) { pa = v; pb = sv; } else { pa = sv; pb = v; }
                pj = j;
                pm = m;
                have_prev = true;
                if (k + 1 == n_layers && (v != final_value || sv != final_value)) return false;
            }
        }
        return pos == msgs.size();
    } catch (const Panic&) {
        return false;
    }
}
}  // namespace

bool verify_fri(const Msgs& msgs, uint32_t log_n, size_t n_layers, size_t num_queries, size_t max_index, FE offset,
                const std::string& channel_state) {
    return verify_transcript(msgs, log_n, n_layers, num_queries, max_index, offset, channel_state, nullptr, nullptr);
}

// ----------------------------------------------------------- prover slice
std::vector<FE> fibsq_trace(FE a1, uint32_t log_t) {
    std::vector<uint32_t> t(size_t{1} << log_t);
    if (fri_fibsq_trace(static_cast<uint32_t>(a1.value()), log_t, t.data()) != FRI_OK) throw Panic("fri_fibsq_trace");
    return to_fe(t.data(), t.size());
}

StarkProof prove_fibsq(FE a1, uint32_t log_t, uint32_t log_blowup, size_t num_queries, FriChannel& channel, FE offset,
                       std::shared_ptr<Gpu> gpu) {
    const uint32_t L = log_t + log_blowup;
    const uint64_t B = uint64_t{1} << log_blowup, n = uint64_t{1} << L;
    if (!gpu) gpu = Gpu::thread_default(L);
    if (L > gpu->log_n_max()) throw Panic("prove_fibsq: LDE 2^" + std::to_string(L) + " exceeds the context");
    std::vector<uint32_t> trace(size_t{1} << log_t);
    gpu->check(fri_fibsq_trace(static_cast<uint32_t>(a1.value()), log_t, trace.data()), "fri_fibsq_trace");
    StarkProof sp;
    sp.log_t = log_t;
    sp.log_blowup = log_blowup;
    sp.a_last = FE(trace.back());
    const uint32_t off = static_cast<uint32_t>(offset.value());
    gpu->check(fri_trace_commit(gpu->ctx(), trace.data(), log_t, log_blowup, off, sp.trace_root.data(), nullptr,
                                nullptr, nullptr),
               "fri_trace_commit");
    const std::string root_hex = sha::hex(sp.trace_root.data(), 32);
    channel.send(reinterpret_cast<const uint8_t*>(root_hex.data()), root_hex.size());
    for (auto& a : sp.alphas) a = channel.receive_random_field_element();
    fri_channel_state cin{};
    auto st = sha::from_hex(channel.state);
    std::memcpy(cin.digest, st.data(), 32);
    cin.has_state = 1;
    const uint32_t al[3] = {static_cast<uint32_t>(sp.alphas[0].value()), static_cast<uint32_t>(sp.alphas[1].value()),
                            static_cast<uint32_t>(sp.alphas[2].value())};
    fri_commit_result res{};
    gpu->bump();
    gpu->check(fri_fibsq_composition_commit(gpu->ctx(), log_t, log_blowup, off, trace.back(), al, &cin, 0, &res),
               "fri_fibsq_composition_commit");
    sp.fri = FRIProof::mirror(res, L, gpu, channel);
    std::vector<uint32_t> vals(3);
    std::vector<uint8_t> paths(3 * 32 * size_t{L});
    for (size_t q = 0; q < num_queries; q++) {
        const uint64_t idx = channel.receive_random_int(0, n - 2 * B - 1, true);
        sp.queries.push_back(idx);
        gpu->check(fri_trace_decommit(gpu->ctx(), idx, B, 3, vals.data(), paths.data(), paths.size()),
                   "fri_trace_decommit");
        for (size_t j = 0; j < 3; j++) {
            channel.send(FE(vals[j]).to_bytes());
            channel.send(paths.data() + 32 * L * j, 32 * size_t{L});
        }
        decommit_fri_layers(idx, sp.fri, channel);
    }
    return sp;
}

FE fibsq_composition_at(FE f0, FE f1, FE f2, FE x, const std::array<FE, 3>& alphas, FE a_last, uint32_t log_t) {
    const uint64_t T = uint64_t{1} << log_t;
    const FE g = omega(log_t), glast = g.pow(T - 1), gprev = g.pow(T - 2);
    const FE p0 = (f0 - FE(1)) * (x - FE(1)).inverse();
    const FE p1 = (f0 - a_last) * (x - glast).inverse();
    const FE p2 = (f2 - f1 * f1 - f0 * f0) * (x - gprev) * (x - glast) * (x.pow(T) - FE(1)).inverse();
    return alphas[0] * p0 + alphas[1] * p1 + alphas[2] * p2;
}

bool verify_fibsq(const Msgs& msgs, FE a_last, uint32_t log_t, uint32_t log_blowup, size_t num_queries,
                  size_t n_layers, FE offset, const std::string& channel_state) {
    const uint32_t L = log_t + log_blowup;
    const uint64_t B = uint64_t{1} << log_blowup, n = uint64_t{1} << L;
    std::array<uint8_t, 32> root{};
    std::array<FE, 3> alphas{};
    auto pre = [&](const Take& take, FriChannel& ch) {
        const auto& r = take();
        if (r.size() != 64) throw Panic("trace root");
        auto rb = sha::from_hex(std::string(r.begin(), r.end()));
        std::memcpy(root.data(), rb.data(), 32);
        ch.send(r);
        for (auto& a : alphas) {
            a = ch.receive_random_field_element();
            if (take() != FriChannel::be64(a.value())) throw Panic("alpha");
        }
    };
    auto on_query = [&](const Take& take, FriChannel& ch, uint64_t idx) -> int64_t {
        FE f[3];
        for (int j = 0; j < 3; j++) {
            const auto& vb = take();
            const auto& path = take();
            ch.send(vb);
            ch.send(path);
            if (vb.size() != 8) throw Panic("trace value");
            const uint64_t v = be_u64(vb);
            if (v >= P || !path_ok(v, idx + j * B, path, L, root)) throw Panic("trace path");
            f[j] = FE(v);
        }
        const FE x = offset * omega(L).pow(idx);
        return static_cast<int64_t>(fibsq_composition_at(f[0], f[1], f[2], x, alphas, a_last, log_t).value());
    };
    return verify_transcript(msgs, L, n_layers, num_queries, n - 2 * B - 1, offset, channel_state, pre, on_query);
}


// ------------------------------------------------------- polynomial layer
std::vector<FE> evaluate_on_coset(const Poly& poly, const Coset& coset) {
    const size_t n = coset.domain_size;
    if (n == 0 || (n & (n - 1))) throw Panic("domain size must be a power of two");
    const uint32_t log_n = ceil_log2(n);
    if (coset.omega != omega(log_n)) throw Panic("coset omega must be g^((p-1)/n) (frozen spec)");
    auto gpu = Gpu::thread_default(log_n);
    auto c = to_u32(poly.coefficients);
    std::vector<uint32_t> out(n);
    gpu->check(fri_lde(gpu->ctx(), c.data(), c.size(), log_n, static_cast<uint32_t>(coset.offset.value()), out.data()),
               "fri_lde");
    return to_fe(out.data(), n);
}

namespace {
// xs == offset * w_n^i for every i (natural order, n a power of two)?
bool is_coset(const std::vector<FE>& xs, FE* offset, uint32_t* log_n) {
    const size_t n = xs.size();
    if (n == 0 || (n & (n - 1)) || xs[0] == FE::zero()) return false;
    *log_n = ceil_log2(n);
    *offset = xs[0];
    const FE w = omega(*log_n);
    FE x = xs[0];
    for (size_t i = 1; i < n; i++) {
        x = x * w;
        if (xs[i] != x) return false;
    }
    return true;
}
}  // namespace

Poly interpolate(const std::vector<FE>& xs, const std::vector<FE>& ys) {
    if (xs.size() != ys.size()) throw Panic("xs and ys must have the same length (interpolation.rs:127)");
    if (xs.empty()) return Poly();                              // Polynomial::zero() (interpolation.rs:133-136)
    FE offset;
    uint32_t log_n = 0;
    auto y = to_u32(ys);
    std::vector<uint32_t> c(xs.size());
    size_t len = 0;
    if (is_coset(xs, &offset, &log_n)) {                        // iNTT on the coset
        auto gpu = Gpu::thread_default(log_n);
        gpu->check(fri_interpolate(gpu->ctx(), y.data(), log_n, static_cast<uint32_t>(offset.value()), c.data(), &len),
                   "fri_interpolate");
    } else {                                                    // any other point set: O(n^2) on the device
        auto gpu = Gpu::thread_default(ceil_log2(xs.size()));
        auto x = to_u32(xs);
        gpu->check(fri_interpolate_points(gpu->ctx(), x.data(), y.data(), x.size(), c.data(), &len),
                   "fri_interpolate_points");
    }
    return Poly(to_fe(c.data(), len));
}

std::vector<FE> batch_inverse(const std::vector<FE>& xs) {
    if (xs.empty()) return {};
    auto gpu = Gpu::thread_default(ceil_log2(xs.size()));
    auto v = to_u32(xs);
    std::vector<uint32_t> out(v.size());
    gpu->check(fri_batch_inverse(gpu->ctx(), v.data(), out.data(), v.size()), "fri_batch_inverse");
    return to_fe(out.data(), out.size());
}

}  // namespace stark101
