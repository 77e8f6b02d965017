/*
 * fri_amd.h — C ABI of the MI355X-native FRI commit path (libfri_amd.so).
 *
 * Drop-in boundary for the reference crate `stark-101`
 * (RazorClient/Stark-prover).  Each entry point names the reference function
 * it replaces (path:line in the reference tree).  Plain pointers and sizes
 * only; no torch / HIP types in any signature.
 *
 * Field: p = 3*2^30 + 1 = 3221225473, generator g = 5 (frozen spec,
 * SURVEY.md §8).  Field elements cross the boundary as canonical uint32_t
 * (value < p) — the reference's FieldElement<M>{value: u64} is not repr(C),
 * so the Rust shim copies `.value() as u32`.
 *
 * Host buffers are caller-owned and only borrowed for the duration of a call.
 * Device memory, streams and graphs are owned by the fri_ctx.  A context is
 * not re-entrant: use one per host thread.  Every call returns FRI_OK (0) or
 * a FRI_E* code; fri_last_error() describes the last failure on the context.
 * The reference panics where these return an error (ops.rs:143,
 * interpolation.rs:127, merkle/mod.rs:25, channel.rs:65); the Rust shim maps
 * non-zero codes back to panic!().
 */
#ifndef FRI_AMD_H
#define FRI_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRI_P          3221225473u   /* 3*2^30 + 1 */
#define FRI_GENERATOR  5u
#define FRI_MAX_ROUNDS 32
#define FRI_MAX_LAYERS (FRI_MAX_ROUNDS + 1)

enum {
    FRI_OK      = 0,
    FRI_EINVAL  = 1,   /* bad argument (sizes, d > n, value >= p, ...)      */
    FRI_ENOMEM  = 2,   /* device or host allocation failed                  */
    FRI_EHIP    = 3,   /* HIP runtime error                                 */
    FRI_ENODEV  = 4,   /* no usable gfx950 device                           */
    FRI_ERCCL   = 5,   /* collective failure (multi-GPU)                    */
    FRI_ESTATE  = 6,   /* call out of order (e.g. no committed layers)      */
    FRI_EDEGREE = 7    /* polynomial degree too large for the domain: the
                          reference would exhaust the domain and panic in
                          MerkleTree::root() (merkle/mod.rs:25)             */
};

/* Fiat-Shamir transcript state — src/channel/channel.rs:14-20.
 * The reference keeps `state: String` = "" or the 64-char lowercase hex of
 * a SHA-256 digest; here it is the 32 raw digest bytes + has_state flag. */
typedef struct {
    uint8_t  digest[32];
    uint32_t has_state;   /* 0 => state == "" (Channel::new, channel.rs:24-30) */
} fri_channel_state;

/* Result of fri_commit — the transcript-visible part of FRIProof
 * (src/fri/fri_commit.rs:9-13) plus the channel messages it produced.
 * Layer evaluations and Merkle levels stay on the device and are read back
 * on demand with fri_layer_copy / fri_tree_level_copy. */
typedef struct {
    uint32_t n_layers;                       /* R+1 committed layers          */
    uint32_t n_rounds;                       /* R folds (= betas drawn)       */
    uint32_t log_n;                          /* layer k has 2^(log_n-k) elems */
    uint32_t final_value;                    /* fri_commit.rs:109-113         */
    int32_t  final_degree;                   /* 0, or -1 for the zero poly    */
    uint32_t reserved;
    uint8_t  roots[FRI_MAX_LAYERS][32];      /* Merkle root bytes per layer   */
    uint32_t betas[FRI_MAX_ROUNDS];          /* beta_k, canonical             */
    fri_channel_state channel_out;           /* channel state after the final send */
} fri_commit_result;

typedef struct fri_ctx fri_ctx;

/* flags for fri_commit* */
#define FRI_FLAG_FORCE_BETAS 1u   /* test hook: use forced_betas[k] instead of the
                                     channel's draw (transcript still absorbs roots) */
#define FRI_FLAG_NO_GRAPH    2u   /* run eagerly instead of replaying a hipGraph   */
#define FRI_FLAG_RANK_INPUTS 4u   /* multi-GPU context, fri_commit_device with
                                     fri_ctx_input_buffer(): ranks 1..n-1 commit the
                                     copy of rank 0's buffer their plan staged at the
                                     last team commit of this shape instead of
                                     copying it again over xGMI.  Verified, not
                                     trusted: every rank hashes the input it would
                                     commit (a position-sensitive 64-bit checksum)
                                     and the call returns FRI_ESTATE, committing
                                     nothing, when a rank's copy differs from rank
                                     0's buffer (rewritten since it was staged) or
                                     no copy of this shape was staged yet */

/* ---------------------------------------------------------------- context */
/* Opens `device` (HIP ordinal) and sizes scratch for codewords up to
 * 2^log_n_max.  Returns FRI_ENODEV when no gfx950 device is present. */
int         fri_ctx_create(int device, uint32_t log_n_max, fri_ctx** out);
int         fri_ctx_destroy(fri_ctx* ctx);
const char* fri_last_error(const fri_ctx* ctx);    /* never NULL; "" if none */
const char* fri_version(void);

/* ------------------------------------------------------- field / batch ops */
/* Batch inverse with inverse(0) = 0 — same results as element-wise
 * FieldElement::inverse (src/fields/element.rs:54-57, Fermat a^(p-2)). */
int fri_batch_inverse(fri_ctx* ctx, const uint32_t* in, uint32_t* out, size_t n);

/* ------------------------------------------------------ polynomial layer */
/* Low-degree extension: evals[i] = P(offset * w_n^i), i < n = 2^log_n,
 * P given by d <= n coefficients (coefficient j = x^j).  Replaces
 * `domain.map(|x| poly.evaluate(x))` (src/fri/fri_commit.rs:78,
 * src/polynomial/ops.rs:76-83) on the coset domain of
 * src/fri/coset_fri.rs:32-36.  offset = 1 gives the plain subgroup. */
int fri_lde(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n,
            uint32_t offset, uint32_t* evals_out);

/* Interpolation on the same coset: the unique P, deg P < n, with
 * P(offset*w_n^i) = ys[i].  Replaces Polynomial::interpolate
 * (src/polynomial/ops.rs:239-241 -> interpolation.rs:121-152) for coset
 * domains.  coeffs_out holds n entries; *len_out = trimmed length
 * (Polynomial::new semantics, ops.rs:19-37). */
int fri_interpolate(fri_ctx* ctx, const uint32_t* ys, uint32_t log_n, uint32_t offset,
                    uint32_t* coeffs_out, size_t* len_out);

/* Interpolation through n arbitrary points: Polynomial::interpolate(xs, ys)
 * (src/polynomial/ops.rs:239-241 -> interpolate_lagrange_polynomials,
 * interpolation.rs:121-152) for point sets that are not a coset.  Same
 * result as the reference's Lagrange sum, duplicates included (their basis
 * polynomials vanish through inverse(0) = 0, element.rs:54-57).  O(n^2) on
 * the device: weights w_j = 1/prod_{i!=j}(x_j - x_i), then f at the 2^k-th
 * roots of unity (2^k >= n) as the polynomial sum_j y_j w_j prod_{i!=j}(x - x_i)
 * without any division, then an iNTT.  n <= 2^17 and n <= 2^log_n_max.
 * coeffs_out holds n entries; *len_out = trimmed length. */
int fri_interpolate_points(fri_ctx* ctx, const uint32_t* xs, const uint32_t* ys, size_t n,
                           uint32_t* coeffs_out, size_t* len_out);

/* Evaluation of P (d coefficients) at `count` arbitrary points
 * (src/polynomial/ops.rs:76-83, Horner semantics). */
int fri_evaluate(fri_ctx* ctx, const uint32_t* coeffs, size_t d, const uint32_t* xs,
                 size_t count, uint32_t* out);

/* ---------------------------------------------------------------- FRI ops */
/* One FRI fold of a layer of size m = 2^log_m living on the coset
 * layer_offset * <w_m> (natural order): out[i] = P'(x_i^2), i < m/2, with
 * P' = even(P) + beta*odd(P).  Bit-identical to next_fri_layer's
 * coefficient fold + re-evaluation (src/fri/fri_commit.rs:53-65). */
int fri_fold(fri_ctx* ctx, const uint32_t* layer, uint32_t log_m, uint32_t layer_offset,
             uint32_t beta, uint32_t* out);

/* Merkle root of n field elements: MerkleTree::new(values).root()
 * (src/merkle/mod.rs:10-26 over rs_merkle 1.4.2, SHA-256, leaf =
 * SHA256(u64 big-endian)).  root32 = raw digest bytes; the reference's
 * `root() -> String` is their lowercase hex.  n must be >= 1. */
int fri_merkle_root(fri_ctx* ctx, const uint32_t* values, size_t n, uint8_t root32[32]);

/* Trace side of the prover (the reference's src/trace and src/prover are
 * empty): interpolate 2^log_t trace values on the subgroup
 * <w_{2^log_t}> (Polynomial::interpolate, src/polynomial/ops.rs:239-241),
 * evaluate the polynomial on the coset offset*<w_n>, n = 2^(log_t+log_blowup)
 * (the low-degree extension), and Merkle-commit the LDE (merkle/mod.rs:10-26).
 * root32 = LDE tree root.  Optional: coeffs_out (2^log_t entries, *coeff_len
 * = trimmed length), lde_out (n entries).  The tree stays on the device. */
int fri_trace_commit(fri_ctx* ctx, const uint32_t* trace, uint32_t log_t, uint32_t log_blowup,
                     uint32_t offset, uint8_t root32[32], uint32_t* coeffs_out, size_t* coeff_len,
                     uint32_t* lde_out);

/* Prover slice (BASELINE configs[3]; src/prover, src/composition are empty in
 * the reference, so the constraint system is STARK-101's FibonacciSq — the
 * crate is `stark-101`, Cargo.toml:2 — on the full trace subgroup G = <g>,
 * |G| = T = 2^log_t):  a_0 = 1, a_{T-1} = a_last, a_{i+2} = a_{i+1}^2 + a_i^2.
 * From the trace LDE kept by the last fri_trace_commit (same log_t,
 * log_blowup, offset) computes, on the coset offset*<w_n>,
 *   CP = alphas[0] (f-1)/(x-1) + alphas[1] (f-a_last)/(x-g^{T-1})
 *      + alphas[2] (f(g^2 x) - f(g x)^2 - f^2) (x-g^{T-2})(x-g^{T-1}) / (x^T-1)
 * (two divisions per point through one batch inversion), interpolates it and
 * runs fri_commit on it: the FRI of fri_commit.rs:72-122 over the composition
 * polynomial, channel continued from chan_in (after the trace root and the
 * three alphas were drawn).  FRI_EDEGREE if deg CP > T (trace violates the
 * constraints).  log_blowup 1..4.  Layers stay resident for fri_decommit_query. */
int fri_fibsq_composition_commit(fri_ctx* ctx, uint32_t log_t, uint32_t log_blowup, uint32_t offset,
                                 uint32_t a_last, const uint32_t alphas[3],
                                 const fri_channel_state* chan_in, uint32_t flags,
                                 fri_commit_result* out);

/* The FibonacciSq trace itself: out[0] = 1, out[1] = a1,
 * out[i+2] = out[i+1]^2 + out[i]^2 mod p, 2^log_t rows.  Host-side (a serial
 * recurrence); needs no context or device.  a1 must be canonical. */
int fri_fibsq_trace(uint32_t a1, uint32_t log_t, uint32_t* out);

/* Trace-tree decommitment (STARK-101 decommit_on_query: f(x), f(gx), f(g^2x)
 * with their paths): values[j] = LDE[(index + j*stride) mod n], j < count
 * (1..8); paths = count authentication paths of log2(n) sibling digests
 * (leaf -> root, 32 bytes each), as fri_auth_path formats them. */
int fri_trace_decommit(fri_ctx* ctx, uint64_t index, uint64_t stride, uint32_t count, uint32_t* values,
                       uint8_t* paths, size_t paths_cap);

/* ---------------------------------------------------------- FRI commit */
/* Full FRI commit — fri_commit(poly, domain, &mut channel)
 * (src/fri/fri_commit.rs:72-122): LDE of `coeffs` on offset*<w_n>,
 * n = 2^log_n; per layer SHA-256 Merkle tree, channel.send(root_hex),
 * beta = channel.receive_random_field_element(), fold; loop while the
 * folded polynomial's degree >= 1; channel.send(final.to_bytes()).
 * chan_in may be NULL (fresh Channel::new()).  Layers and trees stay on the
 * device until the next commit on this context.  A coefficient >= p gives
 * FRI_EINVAL: the device checks the coefficients in layer 0's coefficient
 * scan, so the call returns only after the commit has run, with nothing
 * served.  There is no host pass over the input. */
int fri_commit(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n,
               uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
               const uint32_t* forced_betas, fri_commit_result* out);

/* Same, with the coefficients already resident in device memory
 * (d_coeffs: a device pointer; may be fri_ctx_input_buffer()). */
int fri_commit_device(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                      uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                      const uint32_t* forced_betas, fri_commit_result* out);

/* The context's input buffer: a device buffer of >= d words (on rank 0's
 * device for a multi-GPU context) that fri_commit_device and
 * fri_commit_device_async read in place, on any commit lane, without a copy.
 * It belongs to the caller, as `poly` does in fri_commit(poly, domain,
 * &mut channel) (src/fri/fri_commit.rs:72-76): no commit ever writes it, so a
 * commit from it commits exactly what the caller last wrote there (with its
 * own kernels or copies, or fri_ctx_input_upload), whatever was committed
 * before or on which lane.  Commits from any other pointer stage their
 * coefficients in the plan's private buffer instead.  Created on first call;
 * valid until a call with a larger d moves it (contents kept) or
 * fri_ctx_destroy.  d <= 2^log_n_max. */
int fri_ctx_input_buffer(fri_ctx* ctx, size_t d, uint32_t** d_ptr);
/* Fills the input buffer (grown to >= d words as fri_ctx_input_buffer does)
 * with d host coefficients, after the pending pipelined commits that read it
 * have finished; returns when the copy is complete. */
int fri_ctx_input_upload(fri_ctx* ctx, const uint32_t* coeffs, size_t d);

/* Pipelined commits: a prover that commits many codewords in a row calls
 * fri_commit (src/fri/fri_commit.rs:72-122) in a loop; here it enqueues them.
 * fri_commit_device_async validates the arguments, enqueues the whole commit
 * of fri_commit_device on the context stream and returns at once with a
 * ticket; fri_commit_wait(ticket) waits for that commit and returns its
 * result, with the same errors fri_commit_device would have returned.  Up to
 * FRI_MAX_INFLIGHT commits may be pending (FRI_ESTATE beyond that).  They run
 * on separate lanes (fri_ctx_set_lanes): concurrently, with no host round
 * trip between one commit's kernels and the next one's.  A commit with another
 * (d, log_n, offset) first waits for the pending ones.  The read-backs
 * (fri_commit_info .. fri_decommit_query) serve the most recently enqueued
 * commit and wait for it.  Not while profiling (FRI_ESTATE).
 * d_coeffs is read when the commit runs on the device, not when the call
 * returns: it must stay unchanged until fri_commit_wait(ticket) has returned.
 * fri_ctx_input_buffer() is one buffer, read in place by every pending commit
 * handed it: refill it only through fri_ctx_input_upload (which waits for
 * them), give each pending commit its own device buffer, or use
 * fri_commit_async, which copies host coefficients into the ticket's own
 * pinned buffer before returning. */
#define FRI_MAX_INFLIGHT 4
int fri_commit_device_async(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                            uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                            const uint32_t* forced_betas, uint64_t* ticket);
/* Same, from host coefficients: copied into a pinned buffer of the result
 * slot before the call returns (the caller may reuse `coeffs` at once), then
 * to the device as an asynchronous copy on the context stream. */
int fri_commit_async(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n,
                     uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                     const uint32_t* forced_betas, uint64_t* ticket);
int fri_commit_wait(fri_ctx* ctx, uint64_t ticket, fri_commit_result* out);

/* Commit lanes of pipelined commits.  Each lane is a stream with its own
 * commit plan (input and coefficient buffers, layers, trees, x^-1 tables,
 * graphs, device state), created on first use.  A pipelined commit goes to
 * the lane with the fewest pending (un-waited) commits, ties to the lane
 * dealt a commit longest ago (an unused lane first, lower index first); a
 * lane that gets no HBM for its plan is dropped from the rotation until the
 * next fri_ctx_set_lanes or plan change (the commit runs on another lane;
 * FRI_ENOMEM only when lane 0 itself cannot get one).  Commits on different lanes run
 * concurrently, so one commit's serial tree tops (the Fiat-Shamir chain,
 * one workgroup) overlap the next commit's leaf hashing on the otherwise
 * idle chip.  Default FRI_DEFAULT_LANES (3) lanes: a caller keeping k <= 3
 * commits pending uses k lanes and k plans of HBM (about 2.3 GB per 2^24
 * plan, 38 GB per 2^28 plan); max_lanes = 1 runs them one after another on
 * one stream.  Three, because HIP spreads a process's streams over its
 * hardware queues (GPU_MAX_HW_QUEUES, 4 by default) in creation order: a
 * fourth lane shared a queue with another and ran serialised with it
 * (2^24: 3.41-3.45 ms per commit with 3 lanes and 3 pending, 3.75-3.86 with
 * 4 and 4; profiles/r04_lanes_queues.txt).  Lanes already created keep their
 * memory until the next plan change or fri_ctx_destroy.  FRI_ESTATE while
 * commits are pending. */
#define FRI_DEFAULT_LANES 3
int fri_ctx_set_lanes(fri_ctx* ctx, uint32_t max_lanes);
/* Diagnostic: the lane a pending pipelined commit was dealt to (0-based);
 * FRI_EINVAL for a ticket that is not pending. */
int fri_debug_ticket_lane(fri_ctx* ctx, uint64_t ticket, int* lane);

/* Which commit the read-backs below serve: `generation` grows with every
 * commit call on the context (successful or not), log_n / n_layers describe
 * the resident commit (n_layers = 0 when the last commit failed).  A binding
 * that hands out FRIProof objects records the generation at commit time and
 * refuses read-backs once it has moved on (the reference's FRIProof owns its
 * layers, src/fri/fri_commit.rs:9-13; here they live in the context). */
int fri_commit_info(fri_ctx* ctx, uint64_t* generation, uint32_t* log_n, uint32_t* n_layers);

/* Read-back of the last commit (FRIProof::fri_layers / fri_merkles). */
int fri_layer_copy(fri_ctx* ctx, uint32_t layer, uint32_t* out, size_t cap);
/* Merkle level `level` (0 = leaf hashes) of layer `layer`, as 32-byte digests. */
int fri_tree_level_copy(fri_ctx* ctx, uint32_t layer, uint32_t level, uint8_t* out, size_t cap);

/* Decommitment helper (src/fri/fri_commit.rs:137-165): value and the
 * rs_merkle authentication path (sibling hashes leaf->root) of `index` in
 * committed layer `layer`.  path must hold 32*depth bytes; *depth_out set. */
int fri_auth_path(fri_ctx* ctx, uint32_t layer, uint64_t index, uint32_t* value_out,
                  uint8_t* path, uint32_t* depth_out);

/* Decommitment of one FRI query (decommit_fri_layers, src/fri/fri_commit.rs:
 * 137-163) from the layers and trees of the last fri_commit, still in HBM.
 * For every committed layer k (m_k = 2^(log_n-k) elements): idx = index % m_k,
 * sib = (idx + m_k/2) % m_k; values[2k] = layer_k[idx], values[2k+1] =
 * layer_k[sib]; paths = for each k, the authentication path of idx then of
 * sib (rs_merkle single-leaf proof: sibling digests leaf -> root, 32 bytes
 * each, (log_n-k) per path) — the byte strings the reference sends.
 * *paths_len = total path bytes (also set when paths_cap is too small). */
int fri_decommit_query(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap,
                       uint8_t* paths, size_t paths_cap, size_t* paths_len);

/* ------------------------------------------- single-process multi-GPU team */
/* One context over n_devices GPUs, driven by ONE call from ONE host thread:
 * the reference's fri_commit(poly, domain, &mut channel)
 * (src/fri/fri_commit.rs:72-76) spread over 1-8 GPUs ("the library drives
 * 1-8 GPUs from one host thread").  devices: the HIP
 * ordinals of ranks 0..n-1 (NULL: 0..n-1); an ordinal may repeat (several
 * ranks on one GPU; peer transport only).  n_devices: a power of two <= 64;
 * 1 gives an ordinary context.  log_n_max: the largest codeword; every
 * rank's context is shard-sized (2^(log_n_max - log2 n), and at least
 * 2^min(log_n_max, 19) for the commits rank 0 runs alone).  transport:
 *   FRI_TRANSPORT_PEER  device copies between the ranks' buffers: one pull
 *                       kernel per collective reading the other ranks'
 *                       memory over xGMI peer access (hipMemcpyPeerAsync per
 *                       source where peer access is unavailable), ordered by
 *                       events;
 *   FRI_TRANSPORT_NONE  the default: the peer transport;
 *   FRI_TRANSPORT_RCCL  opt-in: communicators from ncclCommInitAll (xGMI),
 *                       distinct devices only (FRI_EINVAL otherwise).  A rank
 *                       that fails aborts its communicators at once and the
 *                       others theirs when they see it (FRI_ERCCL); the
 *                       team's later sharded calls then return FRI_ESTATE.
 * Inside, rank 0 runs on the calling thread and ranks 1..n-1 on worker
 * threads of the context (one per rank), each issuing the sharded protocol
 * of fri_commit_sharded on its device.  The returned context is rank 0's:
 *   fri_commit / fri_commit_device / fri_commit_sharded*: a codeword of
 *     >= 2^20 elements (and >= 2^(12 + log2 n)) is committed coset-sharded
 *     over the ranks in this one call, with the same result and transcript
 *     as a 1-GPU commit; smaller codewords run on rank 0 alone.
 *     fri_commit_device reads a buffer on rank 0's device (the other ranks
 *     copy it over xGMI);
 *   fri_layer_copy / fri_tree_level_copy / fri_auth_path / fri_decommit_query
 *     (and _sharded) serve every layer: the sharded ones are assembled from
 *     the ranks' blocks and the replicated top trees;
 *   fri_ctx_device_bytes: the sum over the ranks;
 *   the kernel-level calls (fri_lde, fri_merkle_root, ...) run on rank 0;
 *   fri_commit_*async and fri_dist_attach_* / fri_dist_detach: FRI_EINVAL.
 * Not re-entrant (one host thread at a time), like every context.
 * fri_ctx_destroy(ctx) releases every rank. */
int fri_ctx_create_multi(const int* devices, uint32_t n_devices, uint32_t log_n_max, int transport, fri_ctx** out);
/* The context a caller gets without naming devices -- what a binding that
 * keeps the reference's signatures (fri_commit(poly, domain, &mut channel),
 * decommit_fri(num_queries, max_index, &layers, &merkles, &mut channel);
 * src/fri/fri_commit.rs:72-76,168-174) opens behind them: the devices are
 *   FRI_DEVICES  (environment) comma-separated HIP ordinals, a power-of-two
 *                count <= 64, ordinals may repeat (e.g. "0,0,0,0": four
 *                ranks on one GPU);
 *   otherwise    0..k-1, k the largest power of two <= the visible devices;
 * one device gives fri_ctx_create, several fri_ctx_create_multi with the
 * transport FRI_TRANSPORT (environment: "peer", the default, or "rccl").
 * *n_ranks (may be NULL) = the number of ranks.  FRI_EINVAL for a malformed
 * FRI_DEVICES or FRI_TRANSPORT. */
int fri_ctx_create_default(uint32_t log_n_max, fri_ctx** out, uint32_t* n_ranks);
/* Diagnostic: rank `rank`'s context of a team (rank 0: ctx itself), e.g. for
 * its fri_debug_transport_log; owned by the team, never destroyed by the
 * caller (FRI_EINVAL). */
int fri_debug_team_rank(fri_ctx* ctx, uint32_t rank, fri_ctx** out);
/* Test hook (peer transport): the next team call makes rank `rank` fail
 * with FRI_ERCCL at its op_index-th collective (0-based), as a rank whose
 * transfer broke would; the other ranks must return instead of waiting for
 * it.  Applies to the next team call only (cleared at its end, fired or
 * not); op_index < 0 clears it. */
int fri_debug_team_inject_failure(fri_ctx* ctx, uint32_t rank, int64_t op_index);
/* Test hook (peer transport): enable != 0 makes every collective copy with
 * hipMemcpyPeerAsync per source, the path a team takes when peer access is
 * unavailable, instead of the pull kernel; 0 restores the pull kernel where
 * peer access allows it. */
int fri_debug_team_force_copy(fri_ctx* ctx, int enable);

/* -------------------------------------------------------------- multi-GPU */
/* One process per GPU.  A codeword of 2^log_n is committed by G ranks
 * (G a power of two): rank r computes the coset slice evals[r + G*m] of the
 * LDE (size n/G NTT), an all-to-all turns it into the contiguous block
 * [r*n/G, (r+1)*n/G), every layer is hashed block-locally, the G block roots
 * are all-gathered and the tree top + Fiat-Shamir step run redundantly on
 * every rank (identical transcript everywhere), and each fold pairs rank
 * blocks b and b + G/2 (one half-block exchange per layer).  Layers below
 * 2^20 elements are gathered and finished on every rank. */
typedef struct {
    void* user;
    /* host-staged collectives; buffers are host memory; return 0 on success */
    int (*allgather)(void* user, const void* send, void* recv, size_t bytes_per_rank);
    int (*alltoall)(void* user, const void* send, void* recv, size_t bytes_per_peer);
    int (*sendrecv)(void* user, const void* send, void* recv, size_t bytes, int peer);
} fri_collectives;

/* RCCL transport (xGMI): rank 0 creates the id, the caller distributes it.
 * A rendezvous that does not complete within FRI_RCCL_TIMEOUT_S seconds
 * (environment, default 120) returns FRI_ERCCL instead of blocking; a sharded
 * commit whose collectives make no progress for that long aborts the
 * communicators and returns FRI_ERCCL (the context then needs a new attach). */
int fri_dist_unique_id(uint8_t uid[128]);
int fri_dist_attach_rccl(fri_ctx* ctx, int rank, int world, const uint8_t uid[128]);
/* Host-callback transport (e.g. torch.distributed gloo; used by tests). */
int fri_dist_attach_host(fri_ctx* ctx, int rank, int world, const fri_collectives* ops);
int fri_dist_detach(fri_ctx* ctx);
/* The attached transport: FRI_TRANSPORT_NONE / _RCCL / _HOST, and for RCCL
 * the rank and world size the communicator itself reports
 * (ncclCommUserRank / ncclCommCount). */
#define FRI_TRANSPORT_NONE 0
#define FRI_TRANSPORT_RCCL 1
#define FRI_TRANSPORT_HOST 2
#define FRI_TRANSPORT_LOOPBACK 3   /* fri_debug_attach_loopback (timing rehearsal only) */
#define FRI_TRANSPORT_PEER     4   /* in-process team (fri_ctx_create_multi): device copies between ranks */
int fri_dist_info(fri_ctx* ctx, int* rank, int* world, int* transport);
/* Diagnostic: run the transport's all-to-all, all-gather and pair exchange
 * (both streams) on a known pattern and check the result; FRI_ERCCL with a
 * message on mismatch.  Collective: every rank must call it.  world == 1
 * exercises the same calls as self-communication. */
int fri_dist_selftest(fri_ctx* ctx, size_t words_per_peer);

/* Sharded fri_commit: every rank passes the same full coefficient vector and
 * channel state and gets the same result.  world == 1 is fri_commit.
 * Each rank's plan is shard-sized: it allocates only its block of every
 * sharded layer and tree and the x^-1 slices its folds read (plus the full
 * coefficient vector, which the coset LDE reads, and the < 2^20 local tail),
 * so a context created with log_n_max = log_n - log2(world) suffices (2^28
 * over 8 ranks: ~6 GiB each).  The coefficient fold that tracks the degree
 * (next_fri_polynomial, fri_commit.rs:32-50,89) is sharded too: rank r folds
 * coefficients [r*S_k, (r+1)*S_k) of poly_k, and the maxima that give the
 * degree travel with the block roots in the per-layer all-gather.
 * Afterwards fri_layer_copy / fri_tree_level_copy / fri_auth_path serve the
 * layers finished on every rank (the < 2^20 tail); the sharded layers return
 * FRI_ESTATE (each rank holds only its block). */
int fri_commit_sharded(fri_ctx* ctx, const uint32_t* coeffs, size_t d, uint32_t log_n,
                       uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                       const uint32_t* forced_betas, fri_commit_result* out);
int fri_commit_sharded_device(fri_ctx* ctx, const uint32_t* d_coeffs, size_t d, uint32_t log_n,
                              uint32_t offset, const fri_channel_state* chan_in, uint32_t flags,
                              const uint32_t* forced_betas, fri_commit_result* out);

/* Decommitment of one query after fri_commit_sharded (decommit_fri_layers,
 * src/fri/fri_commit.rs:137-163), same layout and bytes as fri_decommit_query
 * on a 1-GPU commit of the same codeword.  Collective: every rank calls it
 * with the same index (the reference draws it from the transcript, identical
 * on every rank) and receives the whole decommitment; each rank contributes
 * the openings that lie in the blocks it holds. */
int fri_decommit_query_sharded(fri_ctx* ctx, uint64_t index, uint32_t* values, size_t values_cap,
                               uint8_t* paths, size_t paths_cap, size_t* paths_len);

/* ------------------------------------------------------------ diagnostics */
/* Per-span device time (ms) accumulated while profiling is enabled (hipEvents
 * recorded on the context's stream; profiling commits run eagerly, no graph).
 * Classes: "lde" (LDE NTT), "merkle_layer0_leaf" (layer-0 leaf kernel: leaves
 * + levels 1-4, with its algorithmic bytes), "layer0" (all of layer 0's tree +
 * channel step), "layers" (layers >= 1), and for sharded commits "alltoall"
 * and "gather".  bytes = algorithmic bytes of the span where defined. */
int fri_set_profiling(fri_ctx* ctx, int enabled);
int fri_get_profile(fri_ctx* ctx, const char* kernel_class, double* total_ms, uint64_t* launches,
                    uint64_t* bytes);
int fri_reset_profile(fri_ctx* ctx);
/* Device memory (HBM) the context holds now and at most so far, in bytes:
 * twiddles, scratch, the commit plan (layers, trees, x^-1 tables), multi-GPU
 * buffers and any grown scratch.  (Diagnostic; no reference counterpart.) */
int fri_ctx_device_bytes(fri_ctx* ctx, uint64_t* current, uint64_t* peak);
/* Test hook: the context's device allocations fail (FRI_ENOMEM paths) once
 * they would take it past cap_bytes of HBM (0: no cap). */
int fri_debug_set_device_cap(fri_ctx* ctx, uint64_t cap_bytes);
/* Diagnostic build only (-DFRI_STAMPS): top-kernel phase timestamps of the
 * last commit, (FRI_MAX_LAYERS x 24) u64 ticks of the 100 MHz clock.
 * Returns FRI_ESTATE in the product build. */
int fri_debug_stamps(fri_ctx* ctx, uint64_t* out, size_t cap);
/* Host-only diagnostic (no context, no device): the commit plan's layout for
 * rank `rank` of `world` (world 1: the 1-GPU plan) of a codeword 2^log_n with
 * d coefficients.  out[0] = rounds bound R, out[1] = last sharded layer k_sw
 * (-1 for world 1), out[2] = bytes of layers + trees + x^-1 tables, out[3] =
 * log2 of the coefficient chunk S_0 a rank folds (world > 1; rank r holds
 * coefficients [r*S_k, (r+1)*S_k) of poly_k, S_k = S_0 / 2^k); then per
 * layer k <= R five words: layer-slot words, tree-slot words, x^-1 entries of
 * fold k, the domain index of the first of them, the block held of sharded
 * layer k.  cap >= 4 + 5 * FRI_MAX_LAYERS. */
int fri_debug_plan_layout(size_t d, uint32_t log_n, uint32_t world, uint32_t rank, uint64_t* out, size_t cap);
/* Test hook for the collective deadline (fri_dist_attach_rccl): with enable
 * != 0 the next RCCL all-to-all on the context is replaced by a kernel that
 * waits like a collective whose peer never arrives, until the deadline's
 * abort releases it.  The call then returns FRI_ERCCL and later sharded calls
 * FRI_ESTATE, exactly as for a real stall. */
int fri_debug_inject_stall(fri_ctx* ctx, int enable);

/* Timing rehearsal of one rank of a sharded commit on one device: attaches a
 * transport whose collectives return this rank's own bytes, as device-to-
 * device copies on the streams RCCL would use.  Every kernel of the rank runs
 * on data of the right shape with no host round trip, but the transcript is
 * not the real one (tools/shard_projection.py). */
int fri_debug_attach_loopback(fri_ctx* ctx, int rank, int world);
/* The degree schedule of the loopback rehearsal: deg[k] for every layer k of
 * a 1-GPU commit of the same polynomial (fri_commit_degrees).  The sharded
 * coefficient fold gives each rank only its slice of the degree maxima, and
 * the loopback all-gather returns this rank's own slice G times, so without
 * the recorded schedule the rehearsal would run fewer rounds than the real
 * commit.  deg = NULL or n = 0 clears it. */
int fri_debug_loopback_degrees(fri_ctx* ctx, const int32_t* deg, uint32_t n);

/* Degree of poly_k for every layer k of the resident commit (the
 * reference's Polynomial degree field, src/polynomial/ops.rs:47-60, as the
 * loop of fri_commit.rs:89 sees it): out[k], k < *n_out = n_layers. */
int fri_commit_degrees(fri_ctx* ctx, int32_t* out, size_t cap, uint32_t* n_out);

/* Transport schedule of the last sharded call on the context
 * (fri_commit_sharded*, fri_decommit_query_sharded, fri_dist_selftest): one
 * entry per collective in issue order.  chan 0 = the main communicator on the
 * context stream, 1 = the exchange communicator on the exchange stream (the
 * logical channel; the host transport runs both on the context stream).  An
 * RCCL run is deadlock-free when, per channel, every rank issues the same
 * sequence of (op, bytes) and each SENDRECV at position i with peer q is
 * matched by q's SENDRECV at position i with peer = this rank;
 * the multi-rank tests check exactly that on every rank's log. */
#define FRI_OP_ALLGATHER 1
#define FRI_OP_ALLTOALL  2
#define FRI_OP_SENDRECV  3
typedef struct {
    uint32_t chan;      /* 0: main, 1: exchange                                   */
    uint32_t op;        /* FRI_OP_*                                                */
    int32_t  peer;      /* SENDRECV partner; -1 for collectives                    */
    uint32_t reserved;
    uint64_t bytes;     /* ALLGATHER: per rank; ALLTOALL: per peer; SENDRECV: each way */
} fri_transport_op;
int fri_debug_transport_log(fri_ctx* ctx, fri_transport_op* out, size_t cap, size_t* count);

#ifdef __cplusplus
}
#endif
#endif /* FRI_AMD_H */
