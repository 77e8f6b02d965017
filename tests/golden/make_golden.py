"""Generate tests/golden/fri_golden.json from the pure-Python oracle twin
(oracle/fri_oracle.py, hashlib SHA-256).  Run from the repo root:

    python tests/golden/make_golden.py

The reference (Rust, nightly, crates not vendored) cannot be built or run in
this image, so these vectors are this repo's frozen-spec
restatement, cross-checked against the independent C oracle by
tests/test_oracle_crosscheck.py.  Layers are stored as SHA-256 of their little-endian
u32 bytes plus the first 8 values.  "fibsq" holds prover-slice transcripts (fo.fibsq_prove).  "decommit_q3" continues each case's
channel with decommit_fri(3, n - 1, ...) (fri_commit.rs:137-179): the state
after it, and the SHA-256 of the proof messages it appended.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import fri_oracle as fo  # noqa: E402


def layer_digest(vals):
    return hashlib.sha256(b"".join(int(v).to_bytes(4, "little") for v in vals)).hexdigest()


def case(name, coeffs, log_n, state="", forced=None, offset=fo.GEN):
    ch = fo.Channel(state=state)
    r = fo.fri_commit(coeffs, log_n, ch, offset=offset, forced_betas=forced)
    commit_state, commit_proof_size, n_msgs = ch.state, ch.proof_size(), len(ch.proof)
    fo.decommit_fri(3, (1 << log_n) - 1, r.layers, r.trees, ch)
    decommit = {"state": ch.state, "messages": len(ch.proof) - n_msgs,
                "proof_sha256": hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m
                                                        for m in ch.proof[n_msgs:])).hexdigest()}
    return {
        "name": name,
        "log_n": log_n,
        "offset": offset,
        "coeffs": [int(c) for c in coeffs],
        "channel_in": state,
        "forced_betas": forced,
        "roots": [x.hex() for x in r.roots],
        "betas": r.betas,
        "final_value": r.final_value,
        "final_degree": r.final_degree,
        "channel_out": commit_state,
        "proof_size": commit_proof_size,
        "decommit_q3": decommit,
        "layer_sha256": [layer_digest(l) for l in r.layers],
        "layer_head": [[int(v) for v in l[:8]] for l in r.layers],
        "leaf0_head": [h.hex() for h in r.trees[0][0][:4]],
    }


def proof_sha(msgs):
    return hashlib.sha256(b"".join(len(m).to_bytes(4, "little") + m for m in msgs)).hexdigest()


def fibsq_case(name, a1, log_t, log_b, queries, state=""):
    """Prover slice (STARK-101 FibonacciSq, fo.fibsq_prove): the whole
    transcript of trace commit, alphas, FRI commit of the composition
    polynomial and `queries` decommitments."""
    ch = fo.Channel(state=state)
    pr = fo.fibsq_prove(a1, log_t, log_b, queries, ch)
    return {
        "name": name, "a1": a1, "log_t": log_t, "log_blowup": log_b, "queries": queries, "channel_in": state,
        "trace_root": pr.trace_root.hex(), "alphas": pr.alphas, "a_last": fo.fibsq_trace(a1, 1 << log_t)[-1],
        "roots": [x.hex() for x in pr.fri.roots], "betas": pr.fri.betas, "final_value": pr.fri.final_value,
        "final_degree": pr.fri.final_degree, "n_layers": len(pr.fri.roots), "query_indices": pr.queries,
        "channel_out": ch.state, "messages": len(ch.proof), "proof_sha256": proof_sha(ch.proof),
    }


def main():
    fibsq = [fibsq_case("stark101_t8_b8", 3141592, 3, 3, 3), fibsq_case("stark101_t32_b8", 3141592, 5, 3, 3),
             fibsq_case("stark101_t64_b8", 3141592, 6, 3, 4), fibsq_case("a1_7_t16_b2", 7, 4, 1, 2),
             fibsq_case("a1_big_t32_b4", fo.P - 2, 5, 2, 3),
             fibsq_case("prefilled_t16_b16", 12345, 4, 4, 2, state=hashlib.sha256(b"public-input").hexdigest())]
    cases = []
    for log_n in range(3, 12):
        for seed in (42, 43, 44):
            d = max(1, (1 << log_n) // 8)
            cases.append(case(f"rand_n{log_n}_s{seed}", fo.splitmix64_field(seed, d), log_n))
    # edge cases (SURVEY.md §8 frozen spec; reference loop semantics fri_commit.rs:89-113)
    cases.append(case("zero_poly", [0, 0, 0, 0], 5))
    cases.append(case("empty_poly", [], 4))
    cases.append(case("constant", [7], 4))
    cases.append(case("trailing_zeros", fo.splitmix64_field(5, 3) + [0] * 13, 7))
    cases.append(case("blowup1", fo.splitmix64_field(6, 32), 5))
    cases.append(case("blowup2", fo.splitmix64_field(7, 64), 7))
    cases.append(case("d_not_pow2", fo.splitmix64_field(8, 37), 9))
    cases.append(case("channel_prefilled", fo.splitmix64_field(9, 16), 7,
                      state=hashlib.sha256(b"trace-root").hexdigest()))
    cases.append(case("offset_3", fo.splitmix64_field(10, 16), 7, offset=3))
    cases.append(case("max_values", [fo.P - 1] * 32, 8))
    # beta = 0 with an all-zero even part: the reference keeps the odd part's
    # degree (scalar_mul does not trim), so the loop runs one extra round.
    odd_only = []
    for v in fo.splitmix64_field(11, 8):
        odd_only += [0, v]
    cases.append(case("forced_beta0_even_zero", odd_only, 7, forced=[0] * 32))
    cases.append(case("forced_betas", fo.splitmix64_field(12, 16), 7, forced=list(range(1, 33))))
    out = os.path.join(HERE, "fri_golden.json")
    with open(out, "w") as f:
        json.dump({"p": fo.P, "generator": fo.GEN, "cases": cases, "fibsq": fibsq}, f, indent=1)
    print(f"wrote {len(cases)} cases to {out}")


if __name__ == "__main__":
    main()
