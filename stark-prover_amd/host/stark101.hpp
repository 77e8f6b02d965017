// stark101.hpp — C++ host mirror of the reference crate `stark-101`'s FRI
// commit surface (RazorClient/Stark-prover), layered over libfri_amd.so.
//
// The reference is Rust and no Rust toolchain exists in this image, so this
// is the compiled host side above the C ABI (include/fri_amd.h).  It keeps
// the reference's names, argument meaning and panic behaviour:
//
//   FieldElement<M>   src/fields/element.rs:7-147   (host scalar arithmetic)
//   Polynomial<M>     src/polynomial/ops.rs:10-83   (new/trim, degree, Horner)
//   CosetFri<M>       src/fri/coset_fri.rs:9-36
//   Channel<M>        src/channel/channel.rs:14-96  (authoritative transcript)
//   MerkleTree        src/merkle/mod.rs:5-27        (built on the GPU)
//   FRIProof          src/fri/fri_commit.rs:9-13    (layers stay in HBM)
//   fri_commit        src/fri/fri_commit.rs:72-122
//   decommit_fri*     src/fri/fri_commit.rs:137-179
//   verify_fri        src/fri/fri_verify.rs:12-177  (completed; see below)
//
// Where the reference panics, these throw stark101::Panic.  The hot path
// runs on the device through the C ABI; there is no CPU fallback: the
// library links libfri_amd.so, and creating a context without a gfx950
// device throws.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "fri_amd.h"

namespace stark101 {

// A Rust panic!() in the reference.
struct Panic : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- SHA-256
// Host SHA-256 (FIPS 180-4) for the transcript: the reference's `sha256`
// 1.5.0 digest() (lowercase hex of the UTF-8 input) and rs_merkle's Sha256.
namespace sha {
std::array<uint8_t, 32> digest(const uint8_t* data, size_t len);
std::string hex(const uint8_t* data, size_t len);            // lowercase
std::string digest_hex(const std::string& s);                  // sha256::digest(s)
std::vector<uint8_t> from_hex(const std::string& s);           // throws Panic on bad hex
// digest() uses the x86 SHA extensions when the CPU has them (runtime check;
// STARK101_NO_SHANI=1 disables them); digest_portable() is always the plain
// C++ compression (the tests cross-check the two).
std::array<uint8_t, 32> digest_portable(const uint8_t* data, size_t len);
bool accelerated();
}  // namespace sha

// -------------------------------------------------------------- FieldElement
// element.rs:7-147.  value < MODULUS always.  Products go through 128 bits,
// which is what element.rs:106 does for mul; pow (element.rs:38-51) uses u64
// products, identical for every modulus below 2^32 (the frozen p included).
template <uint64_t MODULUS>
class FieldElement {
  public:
    constexpr FieldElement() : value_(0) {}
    constexpr explicit FieldElement(uint64_t v) : value_(v % MODULUS) {}
    static constexpr FieldElement new_(uint64_t v) { return FieldElement(v); }
    static constexpr FieldElement zero() { return FieldElement(0); }
    static constexpr FieldElement one() { return FieldElement(1); }
    constexpr uint64_t value() const { return value_; }
    static FieldElement random();                                // element.rs:32-36

    constexpr FieldElement pow(uint64_t e) const {
        unsigned __int128 r = 1, b = value_;
        while (e > 0) {
            if (e & 1) r = r * b % MODULUS;
            b = b * b % MODULUS;
            e >>= 1;
        }
        return FieldElement(static_cast<uint64_t>(r));
    }
    FieldElement inverse() const {                               // element.rs:54-57
        if (!(MODULUS > 2)) throw Panic("Modulus must be > 2 for inverse calculation");
        return pow(MODULUS - 2);
    }
    std::array<uint8_t, 8> to_bytes() const {                   // element.rs:59-61, big endian
        std::array<uint8_t, 8> b{};
        for (int i = 0; i < 8; i++) b[i] = static_cast<uint8_t>(value_ >> (56 - 8 * i));
        return b;
    }
    constexpr FieldElement square() const { return *this * *this; }

    friend constexpr FieldElement operator+(FieldElement a, FieldElement b) { return FieldElement(a.value_ + b.value_); }
    friend constexpr FieldElement operator-(FieldElement a, FieldElement b) {
        return FieldElement((MODULUS + a.value_ - b.value_) % MODULUS);
    }
    friend constexpr FieldElement operator*(FieldElement a, FieldElement b) {
        return FieldElement(static_cast<uint64_t>(static_cast<unsigned __int128>(a.value_) * b.value_ % MODULUS));
    }
    friend FieldElement operator/(FieldElement a, FieldElement b) { return a * b.inverse(); }
    constexpr FieldElement operator-() const { return FieldElement(MODULUS - value_); }
    FieldElement& operator+=(FieldElement b) { return *this = *this + b; }
    FieldElement& operator-=(FieldElement b) { return *this = *this - b; }
    FieldElement& operator*=(FieldElement b) { return *this = *this * b; }
    FieldElement& operator/=(FieldElement b) { return *this = *this / b; }
    friend constexpr bool operator==(FieldElement a, FieldElement b) { return a.value_ == b.value_; }
    friend constexpr bool operator!=(FieldElement a, FieldElement b) { return a.value_ != b.value_; }

    // From<i128> (element.rs:139-147)
    static constexpr FieldElement from_i128(__int128 v) {
        __int128 m = static_cast<__int128>(MODULUS), r = v % m;
        if (r < 0) r += m;
        return FieldElement(static_cast<uint64_t>(r));
    }

  private:
    uint64_t value_;
};

uint64_t os_random_u64();

template <uint64_t M>
FieldElement<M> FieldElement<M>::random() {
    return FieldElement(os_random_u64() % M);
}

// ---------------------------------------------------------------- Polynomial
// ops.rs:10-83: coefficients[i] multiplies x^i, trailing zeros trimmed,
// degree = len - 1 or -1 for the zero polynomial.
template <uint64_t MODULUS>
class Polynomial {
  public:
    using FE = FieldElement<MODULUS>;
    std::vector<FE> coefficients;
    int64_t degree = -1;

    Polynomial() = default;
    explicit Polynomial(std::vector<FE> coeffs) : coefficients(std::move(coeffs)) { update_degree(); }
    static Polynomial new_(std::vector<FE> coeffs) { return Polynomial(std::move(coeffs)); }
    static Polynomial zero() { return Polynomial(); }
    bool is_zero() const { return degree == -1; }
    std::optional<FE> leading_coefficient() const {
        if (is_zero()) return std::nullopt;
        return coefficients[static_cast<size_t>(degree)];
    }
    FE evaluate(FE x) const {                                    // ops.rs:76-83, Horner
        FE r = FE::zero();
        for (auto it = coefficients.rbegin(); it != coefficients.rend(); ++it) r = r * x + *it;
        return r;
    }
    friend bool operator==(const Polynomial& a, const Polynomial& b) { return a.coefficients == b.coefficients; }
    friend bool operator!=(const Polynomial& a, const Polynomial& b) { return !(a == b); }

  private:
    void update_degree() {
        while (!coefficients.empty() && coefficients.back() == FE::zero()) coefficients.pop_back();
        degree = coefficients.empty() ? -1 : static_cast<int64_t>(coefficients.size()) - 1;
    }
};

// ------------------------------------------------------------------ CosetFri
// coset_fri.rs:9-36: D = { offset * omega^i : i < domain_size }.
template <uint64_t M>
struct CosetFri {
    FieldElement<M> offset, omega;
    size_t domain_size = 0;
    CosetFri(FieldElement<M> off, FieldElement<M> om, size_t n) : offset(off), omega(om), domain_size(n) {}
    std::vector<FieldElement<M>> generate_coset_domain() const {
        std::vector<FieldElement<M>> d(domain_size);
        FieldElement<M> x = offset;
        for (size_t i = 0; i < domain_size; i++, x = x * omega) d[i] = x;
        return d;
    }
};

// ------------------------------------------------------------------- Channel
// channel.rs:14-96.  state is "" or the 64-char lowercase hex of a digest.
template <uint64_t MODULUS>
class Channel {
  public:
    std::vector<std::vector<uint8_t>> proof;
    std::vector<std::vector<uint8_t>> compressed_proof;
    std::string state;

    Channel() = default;
    static Channel new_() { return Channel(); }

    // channel.rs:35-44: state = sha256_hex(state || hex(message)).
    void send(const uint8_t* msg, size_t len) {
        state = sha::digest_hex(state + sha::hex(msg, len));
        proof.emplace_back(msg, msg + len);
        compressed_proof.emplace_back(msg, msg + len);
    }
    void send(const std::vector<uint8_t>& m) { send(m.data(), m.size()); }
    template <size_t N>
    void send(const std::array<uint8_t, N>& m) { send(m.data(), N); }

    // channel.rs:58-84: num = (U256(state) + min) % (max - min + 1), then
    // state = sha256_hex(state).  An empty state is not valid hex (:65).
    uint64_t receive_random_int(uint64_t min, uint64_t max, bool show_in_proof) {
        if (max < min) throw Panic("receive_random_int: max < min");
        const unsigned __int128 range = static_cast<unsigned __int128>(max - min) + 1;
        uint64_t num = static_cast<uint64_t>((state_mod(range) + min % range) % range);
        state = sha::digest_hex(state);
        if (show_in_proof) proof.push_back(be64(num));
        return num;
    }
    // channel.rs:47-55: the number is recorded in `proof` only.
    FieldElement<MODULUS> receive_random_field_element() {
        uint64_t num = receive_random_int(0, MODULUS - 1, false);
        proof.push_back(be64(num));
        return FieldElement<MODULUS>(num);
    }
    size_t proof_size() const { return total(proof); }                       // channel.rs:88-90
    size_t compressed_proof_size() const { return total(compressed_proof); } // channel.rs:93-95

    static std::vector<uint8_t> be64(uint64_t v) {
        std::vector<uint8_t> b(8);
        for (int i = 0; i < 8; i++) b[i] = static_cast<uint8_t>(v >> (56 - 8 * i));
        return b;
    }

  private:
    unsigned __int128 state_mod(unsigned __int128 range) const {
        if (state.empty() || state.size() > 64) throw Panic("Channel state is not valid hex");
        unsigned __int128 r = 0;
        for (char c : state) {
            int v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                  : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
            if (v < 0) throw Panic("Channel state is not valid hex");
            r = (r * 16 + static_cast<unsigned>(v)) % range;     // range <= 2^64: no overflow
        }
        return r;
    }
    static size_t total(const std::vector<std::vector<uint8_t>>& v) {
        size_t s = 0;
        for (auto& m : v) s += m.size();
        return s;
    }
};

// ======================================================= device-backed part
// Only the frozen field (p = 3*2^30+1, generator 5) has a
// device path.
constexpr uint64_t P = FRI_P;
using FE = FieldElement<P>;
using Poly = Polynomial<P>;
using FriChannel = Channel<P>;
using Coset = CosetFri<P>;

// omega_n = g^((p-1)/n) (frozen spec), n a power of two <= 2^30.
FE omega(uint32_t log_n);

// One fri_ctx (a device, its stream, graphs and HBM scratch).  Commits
// invalidate the layers of the previous commit on the same Gpu; FRIProof
// notices through the generation counter.
class Gpu {
  public:
    Gpu(int device, uint32_t log_n_max);
    // A team over several GPUs driven from this thread (fri_ctx_create_multi;
    // a device may repeat; transport FRI_TRANSPORT_NONE = the peer
    // transport, FRI_TRANSPORT_RCCL opt-in).  Every call below takes it
    // unchanged: a codeword >= 2^20 is committed coset-sharded over the
    // devices by ONE fri_commit, and the proof's layers and trees serve as on
    // one GPU.
    Gpu(const std::vector<int>& devices, uint32_t log_n_max, int transport = FRI_TRANSPORT_NONE);
    // The default devices (fri_ctx_create_default): FRI_DEVICES, else every
    // visible GPU (the largest power-of-two count); one device is an
    // ordinary context, several a team.
    struct Default {};
    Gpu(Default, uint32_t log_n_max);
    ~Gpu();
    Gpu(const Gpu&) = delete;
    Gpu& operator=(const Gpu&) = delete;
    fri_ctx* ctx() const { return ctx_; }
    uint32_t log_n_max() const { return log_n_max_; }
    uint64_t generation() const { return gen_; }
    uint32_t n_ranks() const { return n_ranks_; }
    uint64_t bump() { return ++gen_; }
    // Throws Panic("<what>: <fri_last_error>") when rc != FRI_OK.
    void check(int rc, const char* what) const;
    // The context behind the reference-signature calls (fri_commit(poly,
    // domain, channel), MerkleTree, interpolate, ...): per thread (a context
    // is not re-entrant), over the default devices (Gpu(Default, ...)), at
    // least 2^log_n (grown by replacing it; FRIProofs keep the old one alive).
    static std::shared_ptr<Gpu> thread_default(uint32_t log_n);

  private:
    fri_ctx* ctx_ = nullptr;
    uint32_t log_n_max_ = 0;
    uint64_t gen_ = 0;
    uint32_t n_ranks_ = 1;
};

class FRIProof;
struct StarkProof;

// merkle/mod.rs:5-27.  A standalone tree keeps only its root; the trees of
// an FRIProof stay in HBM and also serve authentication paths.
class MerkleTree {
  public:
    explicit MerkleTree(const std::vector<FE>& data);              // mod.rs:10-22
    std::string root() const { return root_hex_; }                  // mod.rs:24-26
    std::array<uint8_t, 32> root_bytes() const;
    // rs_merkle single-leaf proof: sibling digests leaf -> root, 32 bytes each.
    std::vector<uint8_t> get_authentication_path(size_t index) const;

  private:
    friend class FRIProof;
    friend void decommit_fri(size_t, size_t, const std::vector<std::vector<FE>>&, const std::vector<MerkleTree>&,
                             FriChannel&);
    friend FRIProof fri_commit_coset(const Poly&, uint32_t, FE, FriChannel&, const std::shared_ptr<Gpu>&);
    friend std::vector<FRIProof> fri_commit_pipelined(const std::vector<Poly>&, uint32_t, FE, std::vector<FriChannel>&,
                                                      const std::shared_ptr<Gpu>&);
    MerkleTree() = default;
    std::string root_hex_;
    std::shared_ptr<Gpu> gpu_;
    uint64_t gen_ = 0;
    uint32_t layer_ = 0;
};

// fri_commit.rs:9-13.  fri_layers are read back from HBM on demand.
class FRIProof {
  public:
    std::vector<MerkleTree> fri_merkles;
    Poly final_poly;
    std::vector<FE> betas;
    uint32_t log_n = 0;

    size_t n_layers() const { return fri_merkles.size(); }
    std::vector<FE> fri_layer(size_t k) const;
    std::vector<std::vector<FE>> fri_layers() const;
    // true while the Gpu has not committed anything since (layers resident)
    bool resident() const;

  private:
    friend FRIProof fri_commit_coset(const Poly&, uint32_t, FE, FriChannel&, const std::shared_ptr<Gpu>&);
    friend std::vector<FRIProof> fri_commit_pipelined(const std::vector<Poly>&, uint32_t, FE, std::vector<FriChannel>&,
                                                      const std::shared_ptr<Gpu>&);
    friend void decommit_fri_layers(size_t, const FRIProof&, FriChannel&);
    friend StarkProof prove_fibsq(FE, uint32_t, uint32_t, size_t, FriChannel&, FE, std::shared_ptr<Gpu>);
    // The proof of a device commit: appends the messages the device sent
    // (root hex per layer, beta per round, final value) to `channel` and
    // takes over its state (fri_commit.rs:84-114).
    // gen: the Gpu generation of that commit (default: the current one).
    static FRIProof mirror(const fri_commit_result& res, uint32_t log_n, const std::shared_ptr<Gpu>& gpu,
                           FriChannel& channel, uint64_t gen = 0);
    std::shared_ptr<Gpu> gpu_;
    uint64_t gen_ = 0;
    void require_resident() const;
};

// fri_commit.rs:72-122.  `domain` must be the coset offset*<omega_n> in
// natural order (coset_fri.rs:32-36) with n a power of two; the device
// evaluates on that coset, so an arbitrary domain is a Panic, not a
// silent recomputation.  Updates `channel` exactly as the reference does.
FRIProof fri_commit(Poly poly, std::vector<FE> domain, FriChannel& channel);
// Same, without materialising the domain.
FRIProof fri_commit(const Poly& poly, const Coset& coset, FriChannel& channel);
// Explicit context (log_n <= gpu->log_n_max()).
FRIProof fri_commit_coset(const Poly& poly, uint32_t log_n, FE offset, FriChannel& channel,
                          const std::shared_ptr<Gpu>& gpu);

// fri_commit (fri_commit.rs:72-122) of many polynomials in a row, each with
// its own channel, pipelined on one Gpu (fri_commit_async / fri_commit_wait,
// two in flight: the next upload overlaps the running commit).  Proof i equals
// fri_commit_coset(polys[i], ..., channels[i]); only the last proof's layers
// and trees stay resident (the earlier ones report resident() == false).
std::vector<FRIProof> fri_commit_pipelined(const std::vector<Poly>& polys, uint32_t log_n, FE offset,
                                           std::vector<FriChannel>& channels, const std::shared_ptr<Gpu>& gpu);

// fri_commit.rs:137-179 over the device-resident layers and trees.
void decommit_fri_layers(size_t index, const FRIProof& proof, FriChannel& channel);
void decommit_fri(size_t num_queries, size_t max_index, const FRIProof& proof, FriChannel& channel);
// The reference's own signature, decommit_fri(num_queries, max_index,
// &fri_layers, &fri_merkles, &mut channel) (fri_commit.rs:168-174): the
// commit is found through the device-backed trees (their Gpu and
// generation; a stale or standalone tree panics), the openings are gathered
// on the device and checked against `fri_layers` (a mismatch panics: the
// layers belong to another commit).
void decommit_fri(size_t num_queries, size_t max_index, const std::vector<std::vector<FE>>& fri_layers,
                  const std::vector<MerkleTree>& fri_merkles, FriChannel& channel);

// Checks a transcript (the messages fri_commit then decommit_fri appended to
// Channel::proof).  The reference's fri_verify.rs:12-177 is a sketch (it
// re-reads proof.last() and leaves the fold check as a placeholder); this
// is the check it outlines, completed: replay the channel from
// `channel_state`, every root/beta/index must match the replay, every
// authentication path must reach its layer root, every layer-k value must
// be the fold of its parents, the last layer must hold the final constant.
// Host-only (SHA-256 on the CPU); returns false on any mismatch.
bool verify_fri(const std::vector<std::vector<uint8_t>>& messages, uint32_t log_n, size_t n_layers,
                size_t num_queries, size_t max_index, FE offset = FE(FRI_GENERATOR),
                const std::string& channel_state = "");

// ------------------------------------------------ prover slice (configs[3])
// src/prover, src/trace and src/composition are empty in the reference; the
// constraint system is STARK-101's FibonacciSq on the full trace subgroup
// (include/fri_amd.h, fri_fibsq_composition_commit):
//   a_0 = 1, a_1 = a1, a_{i+2} = a_{i+1}^2 + a_i^2;  public output a_{T-1}.
// prove_fibsq: trace -> LDE + Merkle (GPU) -> send(root hex) -> alpha_0..2
// -> composition polynomial + its FRI commit (GPU) -> per query
// idx = receive_random_int(0, n - 2B - 1, true): f(x), path, f(gx), path,
// f(g^2x), path, then decommit_fri_layers (fri_commit.rs:137-163).
struct StarkProof {
    std::array<uint8_t, 32> trace_root{};
    std::array<FE, 3> alphas{};
    FE a_last;
    FRIProof fri;
    uint32_t log_t = 0, log_blowup = 0;
    std::vector<uint64_t> queries;
};
std::vector<FE> fibsq_trace(FE a1, uint32_t log_t);
StarkProof prove_fibsq(FE a1, uint32_t log_t, uint32_t log_blowup, size_t num_queries, FriChannel& channel,
                       FE offset = FE(FRI_GENERATOR), std::shared_ptr<Gpu> gpu = nullptr);
// CP(x) from f(x), f(gx), f(g^2 x): what layer 0 must hold at a query.
FE fibsq_composition_at(FE f0, FE f1, FE f2, FE x, const std::array<FE, 3>& alphas, FE a_last, uint32_t log_t);
// Verifier of prove_fibsq's transcript: replays the channel, checks the
// trace paths against the trace root, layer 0 against the composition at
// every query, then every check of verify_fri.  Host-only.
bool verify_fibsq(const std::vector<std::vector<uint8_t>>& messages, FE a_last, uint32_t log_t, uint32_t log_blowup,
                  size_t num_queries, size_t n_layers, FE offset = FE(FRI_GENERATOR),
                  const std::string& channel_state = "");

// ---------------------------------------------------- polynomial layer (GPU)
// evaluate() at every coset point (fri_commit.rs:78): the LDE.
std::vector<FE> evaluate_on_coset(const Poly& poly, const Coset& coset);
// Polynomial::interpolate (ops.rs:239-241): the iNTT when xs is a coset
// offset*<omega_n> in natural order, fri_interpolate_points otherwise.
Poly interpolate(const std::vector<FE>& xs, const std::vector<FE>& ys);
// Element-wise inverse with inverse(0) = 0 (element.rs:54-57).
std::vector<FE> batch_inverse(const std::vector<FE>& xs);

}  // namespace stark101
