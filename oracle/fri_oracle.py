"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product path).

Pure-Python twin of ``oracle/fri_oracle.c``: a restatement of the reference
(RazorClient/Stark-prover, crate ``stark-101``) FRI-commit path for SMALL
cases, plus a ctypes loader for the C oracle.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it.

SHA-256 comes from Python's ``hashlib`` (an implementation independent of the
C oracle's), so C-oracle == Python-twin checks pin the C SHA-256, the Merkle
tree shape and the channel encoding against a second implementation.

Parity status (see DESIGN.md "Oracle"): field / polynomial / interpolation
semantics are pinned by the reference's unit-test KATs; the rs_merkle tree
shape (pairing and odd-node promotion) by rs_merkle's documented example root;
channel hex/U256 encoding and the FRI transcript are restated from the frozen
spec — PARITY UNPINNED beyond this repo's golden vectors.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

P = 3 * 2**30 + 1          # frozen spec: STARK-101 prime
GEN = 5                    # full-group generator; coset offset = GEN

# --------------------------------------------------------------------------
# Field — src/fields/element.rs (generic modulus M)
# --------------------------------------------------------------------------

def fe_new(v: int, M: int) -> int:            # element.rs:13-17
    return v % M


def fe_add(a: int, b: int, M: int) -> int:    # element.rs:72-78
    return (a + b) % M


def fe_sub(a: int, b: int, M: int) -> int:    # element.rs:86-93
    return ((M + a - b) % M) % M


def fe_mul(a: int, b: int, M: int) -> int:    # element.rs:102-108
    return (a * b) % M


def fe_pow(a: int, e: int, M: int) -> int:    # element.rs:38-51 (u64 wrapping products)
    mask = (1 << 64) - 1
    result, base = 1, a
    while e > 0:
        if e & 1:
            result = ((result * base) & mask) % M
        base = ((base * base) & mask) % M
        e >>= 1
    return result


def fe_inverse(a: int, M: int) -> int:        # element.rs:54-57 (inverse(0) == 0)
    assert M > 2
    return fe_pow(a, M - 2, M)


def fe_neg(a: int, M: int) -> int:            # element.rs:130-136
    return (M - a) % M


def fe_div(a: int, b: int, M: int) -> int:    # element.rs:116-122
    return fe_mul(a, fe_inverse(b, M), M)


def fe_to_bytes(v: int) -> bytes:             # element.rs:59-61
    return int(v).to_bytes(8, "big")


# --------------------------------------------------------------------------
# Polynomial — src/polynomial/ops.rs   (lists of ints, coefficient i = x^i)
# --------------------------------------------------------------------------

def poly_trim(c: Sequence[int]) -> List[int]:          # ops.rs:19-37
    c = list(c)
    while c and c[-1] == 0:
        c.pop()
    return c


def poly_degree(c: Sequence[int]) -> int:              # ops.rs:27-31 (trimmed)
    return len(poly_trim(c)) - 1


def poly_evaluate(c: Sequence[int], x: int, M: int) -> int:   # ops.rs:76-83
    r = 0
    for coef in reversed(c):
        r = fe_add(fe_mul(r, x, M), coef, M)
    return r


def poly_add(a, b, M):                                  # ops.rs:87-98 (both nonzero)
    n = max(len(a), len(b))
    out = [0] * n
    for i in range(n):
        out[i] = fe_add(a[i] if i < len(a) else 0, b[i] if i < len(b) else 0, M)
    return poly_trim(out)


def poly_sub(a, b, M):                                  # ops.rs:101-112
    if not b:
        return list(a)
    n = max(len(a), len(b))
    out = [0] * n
    for i in range(n):
        out[i] = fe_sub(a[i] if i < len(a) else 0, b[i] if i < len(b) else 0, M)
    return poly_trim(out)


def poly_mul(a, b, M):                                  # ops.rs:114-138
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x == 0:
            continue
        for j, y in enumerate(b):
            out[i + j] = fe_add(out[i + j], fe_mul(x, y, M), M)
    return poly_trim(out)


def poly_scalar_mul(a, s, M):                           # ops.rs:194-198
    return [fe_mul(x, s, M) for x in a]


def poly_div_rem(a, b, M):                              # ops.rs:141-191
    a, b = poly_trim(a), poly_trim(b)
    if not b:
        raise ZeroDivisionError("Division by zero polynomial")   # ops.rs:143
    if not a or len(a) < len(b):
        return [], list(a)
    rem = list(a)
    q = [0] * (len(a) - len(b) + 1)
    den_lead, den_deg = b[-1], len(b) - 1
    rem_deg = len(rem) - 1
    while rem_deg >= den_deg and rem_deg != -1:
        ratio = fe_mul(rem[rem_deg], fe_inverse(den_lead, M), M)
        shift = rem_deg - den_deg
        q[shift] = fe_add(q[shift], ratio, M)
        for i in range(den_deg + 1):
            rem[i + shift] = fe_sub(rem[i + shift], fe_mul(ratio, b[i], M), M)
        rem = poly_trim(rem)
        rem_deg = len(rem) - 1
    return poly_trim(q), rem


def poly_compose(p, q, M):                              # ops.rs:214-237 (KAT replay only)
    result: List[int] = []
    for coeff in reversed(p):
        if result:
            result = poly_mul(result, q, M)
            result = poly_add(result, poly_trim([coeff]), M) if poly_trim([coeff]) else result
        else:
            result = poly_trim([coeff])
    return result


# --------------------------------------------------------------------------
# Interpolation — src/polynomial/interpolation.rs
# --------------------------------------------------------------------------

def gen_polynomial_from_roots(roots, M):                # interpolation.rs:9-23
    if not roots:
        return []
    p = [1]
    for r in roots:
        p = poly_mul(p, poly_trim([fe_neg(r, M), 1]), M)
    return p


def gen_lagrange_polynomials(xs, M):                    # interpolation.rs:46-78 (== :80-115)
    n = len(xs)
    if n == 0:
        return []
    Z = gen_polynomial_from_roots(xs, M)
    out = []
    for i in range(n):
        denom = 1
        for j in range(n):
            if i != j:
                denom = fe_mul(denom, fe_sub(xs[i], xs[j], M), M)
        q, r = poly_div_rem(Z, gen_polynomial_from_roots([xs[i]], M), M)
        if r:
            raise ValueError("Z(x) should be divisible by (x - x_i)")
        out.append(poly_scalar_mul(q, fe_inverse(denom, M), M))
    return out


def interpolate_lagrange_polynomials(xs, ys, M):        # interpolation.rs:121-152
    if len(xs) != len(ys):
        raise ValueError("Mismatched x and y lengths")
    if not xs:
        return []
    acc: List[int] = []
    for li, y in zip(gen_lagrange_polynomials(xs, M), ys):
        term = poly_scalar_mul(li, y, M)
        if len(li) == 0:          # add_assign: rhs.is_zero() (degree field) -> unchanged
            continue
        acc = poly_add(acc, term, M) if acc else poly_trim(term)
    return acc


# --------------------------------------------------------------------------
# Merkle — src/merkle/mod.rs over rs_merkle 1.4.2 (hashlib SHA-256)
# --------------------------------------------------------------------------

def merkle_levels(values: Sequence[int]) -> List[List[bytes]]:
    """All levels, leaves first (mod.rs:10-22): leaf = SHA256(u64 BE);
    parent = SHA256(l || r); a lone right-most node is promoted."""
    if not values:
        raise ValueError("empty tree has no root")      # mod.rs:25 unwrap panics
    return merkle_levels_from_leaves([hashlib.sha256(fe_to_bytes(v)).digest() for v in values])


def merkle_levels_from_leaves(lvl: List[bytes]) -> List[List[bytes]]:
    """rs_merkle 1.4.2 ``MerkleTree::<Sha256>::from_leaves`` over leaf digests
    (mod.rs:15-19): parent = SHA256(l || r), a lone right-most node promoted
    unchanged.  Pinned by rs_merkle's own documented example (the root of the
    SHA-256 leaves of "a".."f", tests/test_oracle_kats.py)."""
    levels = [lvl]
    while len(lvl) > 1:
        nxt = []
        for j in range(0, len(lvl), 2):
            nxt.append(hashlib.sha256(lvl[j] + lvl[j + 1]).digest() if j + 1 < len(lvl) else lvl[j])
        levels.append(nxt)
        lvl = nxt
    return levels


def merkle_root_hex(values: Sequence[int]) -> str:     # mod.rs:24-26
    return merkle_levels(values)[-1][0].hex()


def merkle_proof(levels: List[List[bytes]], idx: int) -> bytes:
    """Authentication path of leaf `idx` as the bytes the decommitment sends
    (fri_commit.rs:155,159 `get_authentication_path`): the
    rs_merkle 1.4.2 single-leaf proof, sibling hashes leaf -> root, a level
    whose node has no sibling (odd promotion) contributing nothing.
    Parity unpinned: the wrapper in src/merkle/mod.rs has no such method."""
    out = b""
    for lvl in levels[:-1]:
        sib = idx ^ 1
        if sib < len(lvl):
            out += lvl[sib]
        idx >>= 1
    return out


# --------------------------------------------------------------------------
# Channel — src/channel/channel.rs
# --------------------------------------------------------------------------

@dataclass
class Channel:
    state: str = ""                                    # channel.rs:24-30
    proof: List[bytes] = field(default_factory=list)
    compressed_proof: List[bytes] = field(default_factory=list)

    def send(self, message: bytes) -> None:            # channel.rs:35-44
        self.state = hashlib.sha256((self.state + message.hex()).encode()).hexdigest()
        self.proof.append(bytes(message))
        self.compressed_proof.append(bytes(message))

    def receive_random_int(self, lo: int, hi: int, show_in_proof: bool) -> int:  # channel.rs:58-84
        num = (int(self.state, 16) + lo) % ((hi - lo) + 1)
        self.state = hashlib.sha256(self.state.encode()).hexdigest()
        if show_in_proof:
            self.proof.append((num & ((1 << 64) - 1)).to_bytes(8, "big"))
        return num & ((1 << 64) - 1)

    def receive_random_field_element(self, M: int = P) -> int:   # channel.rs:47-55
        num = self.receive_random_int(0, M - 1, False)
        self.proof.append(num.to_bytes(8, "big"))
        return fe_new(num, M)

    def proof_size(self) -> int:                       # channel.rs:88-90
        return sum(len(b) for b in self.proof)


# --------------------------------------------------------------------------
# FRI commit — src/fri/fri_commit.rs:18-122 (faithful; small n only)
# --------------------------------------------------------------------------

def next_fri_polynomial(c: List[int], deg: int, beta: int, M: int):
    """fri_commit.rs:32-50 with the reference's degree bookkeeping:
    returns (coeffs, degree)."""
    odd = poly_trim(c[1::2])
    even = poly_trim(c[0::2])
    odd_deg = len(odd) - 1
    odd = poly_scalar_mul(odd, beta, M)          # scalar_mul keeps the degree field
    if not even:                                 # add_assign: rhs zero -> unchanged
        return odd, odd_deg
    out = poly_add(odd, even, M) if odd else list(even)
    return out, len(out) - 1


@dataclass
class FriResult:
    roots: List[bytes]
    betas: List[int]
    final_value: int
    final_degree: int
    layers: List[List[int]]
    trees: List[List[List[bytes]]]


def coset_domain(log_n: int, offset: int = GEN, gen: int = GEN, M: int = P) -> List[int]:
    """coset_fri.rs:32-36 — D[i] = offset * omega^i, omega = gen^((M-1)/n)."""
    n = 1 << log_n
    w = fe_pow(gen, (M - 1) // n, M)
    return [fe_mul(offset, fe_pow(w, i, M), M) for i in range(n)]


def fri_commit(coeffs: Sequence[int], log_n: int, channel: Channel, offset: int = GEN,
               gen: int = GEN, M: int = P, forced_betas: Optional[Sequence[int]] = None,
               keep: bool = True) -> FriResult:
    """fri_commit.rs:72-122 (faithful Horner evaluation on every domain point)."""
    n = 1 << log_n
    if len(coeffs) > n:
        raise ValueError("degree bound exceeds domain")
    poly = poly_trim(coeffs)
    deg = len(poly) - 1
    domain = coset_domain(log_n, offset, gen, M)
    roots, betas, layers, trees = [], [], [], []
    k = 0
    while True:
        evals = [poly_evaluate(poly, x, M) for x in domain]          # :78 / :60-63
        levels = merkle_levels(evals)
        root = levels[-1][0]
        roots.append(root)
        if keep:
            layers.append(evals)
            trees.append(levels)
        channel.send(root.hex().encode())                            # :86 / :100
        if deg < 1:                                                  # :89
            break
        beta = channel.receive_random_field_element(M)               # :91
        if forced_betas is not None:
            beta = forced_betas[k]
        betas.append(beta)
        poly, deg = next_fri_polynomial(poly, deg, beta, M)          # :94
        domain = [fe_pow(x, 2, M) for x in domain[: len(domain) // 2]]   # :18-24
        if not domain:
            raise ValueError("domain exhausted before degree 0")
        k += 1
    final = 0 if deg == -1 else poly[0]                              # :109-113
    channel.send(fe_to_bytes(final))                                 # :114
    return FriResult(roots, betas, final, deg, layers, trees)


def decommit_fri_layers(index: int, layers, trees, channel: Channel) -> None:
    """fri_commit.rs:137-163, including its quirk: a 1-element layer sends
    its value and then still sends value/path/sibling/path (idx = sib = 0)."""
    for evals, levels in zip(layers, trees):
        length = len(evals)
        if length == 1:
            channel.send(fe_to_bytes(evals[0]))
        idx = index % length
        sib = (idx + length // 2) % length
        channel.send(fe_to_bytes(evals[idx]))
        channel.send(merkle_proof(levels, idx))
        channel.send(fe_to_bytes(evals[sib]))
        channel.send(merkle_proof(levels, sib))


def decommit_fri(num_queries: int, max_index: int, layers, trees, channel: Channel) -> None:
    """fri_commit.rs:168-179: each query index is drawn from the transcript."""
    for _ in range(num_queries):
        idx = channel.receive_random_int(0, max_index, True)
        decommit_fri_layers(idx, layers, trees, channel)


# --------------------------------------------------------------------------
# Prover slice — STARK-101 FibonacciSq (BASELINE configs[3]).  The
# reference's src/prover, src/trace, src/composition are EMPTY files, so this
# restates the STARK-101 tutorial's prover (the crate is `stark-101`,
# Cargo.toml:2) on the full trace subgroup G = <g>, |G| = T, with the
# reference's own polynomial operations (ops.rs add/sub/mul/div_rem/compose,
# interpolation.rs Lagrange, Horner evaluate) — PARITY UNPINNED (no reference
# prover exists to compare with).
# --------------------------------------------------------------------------

def fibsq_trace(a1: int, T: int, M: int = P) -> List[int]:
    """a_0 = 1, a_1 = a1, a_{i+2} = a_{i+1}^2 + a_i^2."""
    a = [1, a1 % M]
    while len(a) < T:
        a.append(fe_add(fe_mul(a[-1], a[-1], M), fe_mul(a[-2], a[-2], M), M))
    return a[:T]


def fibsq_cp_faithful(f: List[int], log_t: int, a_last: int, alphas: Sequence[int], M: int = P) -> List[int]:
    """Composition polynomial in coefficient form, STARK-101 part 2, with the
    reference's polynomial arithmetic:
      p0 = (f - 1) / (x - 1),  p1 = (f - A) / (x - g^{T-1}),
      p2 = (f(g^2 x) - f(g x)^2 - f^2) / ((x^T - 1) / ((x - g^{T-2})(x - g^{T-1}))),
      CP = a0 p0 + a1 p1 + a2 p2.   Every division must be exact."""
    T = 1 << log_t
    g = fe_pow(GEN, (M - 1) >> log_t, M)
    glast, gprev = fe_pow(g, T - 1, M), fe_pow(g, T - 2, M)
    x_minus = lambda c: poly_trim([fe_neg(c, M), 1])             # noqa: E731
    p0, r0 = poly_div_rem(poly_sub(f, [1], M), x_minus(1), M)
    p1, r1 = poly_div_rem(poly_sub(f, poly_trim([a_last]), M), x_minus(glast), M)
    f1 = poly_compose(f, [0, g], M)                              # f(g x)     (ops.rs:214-237)
    f2 = poly_compose(f, [0, fe_mul(g, g, M)], M)                # f(g^2 x)
    num = poly_sub(poly_sub(f2, poly_mul(f1, f1, M), M), poly_mul(f, f, M), M)
    xT1 = [fe_neg(1, M)] + [0] * (T - 1) + [1]
    z, rz = poly_div_rem(xT1, poly_mul(x_minus(gprev), x_minus(glast), M), M)
    p2, r2 = poly_div_rem(num, z, M)
    if r0 or r1 or rz or r2:
        raise ValueError("trace violates the constraints (non-exact division)")
    cp: List[int] = []
    for a, pk in zip(alphas, (p0, p1, p2)):
        term = poly_trim(poly_scalar_mul(pk, a, M))
        if term:
            cp = poly_add(cp, term, M) if cp else term
    return cp


@dataclass
class FibsqProof:
    trace_root: bytes
    alphas: List[int]
    fri: FriResult
    queries: List[int]


def fibsq_prove(a1: int, log_t: int, log_blowup: int, num_queries: int, channel: Channel,
                offset: int = GEN, M: int = P) -> FibsqProof:
    """STARK-101 prover, faithful algorithms (small T only: O(T^2)):
    Lagrange interpolation of the trace on G, Horner LDE on offset*<w_n>,
    rs_merkle tree, send(root), alpha_0..2, composition polynomial,
    fri_commit (fri_commit.rs:72-122), then per query
    idx = receive_random_int(0, n - 2B - 1, true): f(x), path, f(gx), path,
    f(g^2 x), path (STARK-101 decommit_on_query) and decommit_fri_layers."""
    T, B = 1 << log_t, 1 << log_blowup
    L = log_t + log_blowup
    n = 1 << L
    trace = fibsq_trace(a1, T, M)
    f = interpolate_lagrange_polynomials(coset_domain(log_t, offset=1, M=M), trace, M)
    f_eval = [poly_evaluate(f, x, M) for x in coset_domain(L, offset, M=M)]
    f_levels = merkle_levels(f_eval)
    channel.send(f_levels[-1][0].hex().encode())
    alphas = [channel.receive_random_field_element(M) for _ in range(3)]
    cp = fibsq_cp_faithful(f, log_t, trace[-1], alphas, M)
    fri = fri_commit(cp, L, channel, offset, M=M)
    queries = []
    for _ in range(num_queries):
        idx = channel.receive_random_int(0, n - 2 * B - 1, True)
        queries.append(idx)
        for j in range(3):
            channel.send(fe_to_bytes(f_eval[idx + j * B]))
            channel.send(merkle_proof(f_levels, idx + j * B))
        decommit_fri_layers(idx, fri.layers, fri.trees, channel)
    return FibsqProof(f_levels[-1][0], alphas, fri, queries)


def fibsq_cp_evals_np(f_eval, log_t: int, log_blowup: int, offset: int, a_last: int, alphas: Sequence[int]):
    """Composition polynomial on the LDE coset, evaluation form, numpy uint64
    (p < 2^32: products fit in 64 bits).  Same values as evaluating
    fibsq_cp_faithful's polynomial on offset*<w_n> (checked by tests)."""
    import numpy as np
    T, B = 1 << log_t, 1 << log_blowup
    L = log_t + log_blowup
    n = 1 << L
    Pu = np.uint64(P)
    f = np.asarray(f_eval, dtype=np.uint64) % Pu
    w = pow(GEN, (P - 1) >> L, P)
    g = pow(GEN, (P - 1) >> log_t, P)
    # x_i = offset * w^i via two-level tables
    lo = np.array([pow(w, j, P) for j in range(1024)], dtype=np.uint64)
    hi = np.array([pow(w, 1024 * j, P) * offset % P for j in range((n + 1023) // 1024)], dtype=np.uint64)
    idx = np.arange(n, dtype=np.uint64)
    x = lo[idx % 1024] * hi[idx // 1024] % Pu

    def mul(a, b):
        return a * b % Pu

    def inv(a):
        r = np.ones_like(a)
        e, base = P - 2, a.copy()
        while e:
            if e & 1:
                r = mul(r, base)
            base = mul(base, base)
            e >>= 1
        return r

    def sub(a, b):
        return (a + Pu - (b % Pu)) % Pu

    glast, gprev = np.uint64(pow(g, T - 1, P)), np.uint64(pow(g, T - 2, P))
    f1 = np.roll(f, -B)
    f2 = np.roll(f, -2 * B)
    p0 = mul(sub(f, np.uint64(1)), inv(sub(x, np.uint64(1))))
    p1 = mul(sub(f, np.uint64(a_last)), inv(sub(x, glast)))
    num = sub(f2, (mul(f1, f1) + mul(f, f)) % Pu)
    xT = x.copy()
    for _ in range(log_t):
        xT = mul(xT, xT)
    p2 = mul(mul(num, mul(sub(x, gprev), sub(x, glast))), inv(sub(xT, np.uint64(1))))
    a0, a1, a2 = (np.uint64(a) for a in alphas)
    return (mul(p0, a0) + mul(p1, a1) + mul(p2, a2)) % Pu


def splitmix64_field(seed: int, count: int, M: int = P) -> List[int]:
    """Synthetic coefficients: splitmix64(seed) % M."""
    mask = (1 << 64) - 1
    x = seed & mask
    out = []
    for _ in range(count):
        x = (x + 0x9E3779B97F4A7C15) & mask
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & mask
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & mask
        z ^= z >> 31
        out.append(z % M)
    return out


def splitmix64_np(seed: int, count: int, M: int = P):
    """splitmix64_field as a numpy uint64 array (the same stream, vectorised;
    tests check the two agree) for the large configs, 2^25 coefficients."""
    import numpy as np
    idx = np.arange(1, count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & ((1 << 64) - 1)) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z % np.uint64(M)


# --------------------------------------------------------------------------
# ctypes loader for the C oracle (oracle/fri_oracle.c -> oracle/_build/liboracle.so)
# --------------------------------------------------------------------------
_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(_HERE, "_build", "liboracle.so")


class OrcChannel(ctypes.Structure):
    _fields_ = [("state", ctypes.c_char * 65), ("state_len", ctypes.c_uint32)]


class OrcFriResult(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_uint32), ("n_rounds", ctypes.c_uint32),
                ("final_value", ctypes.c_uint64), ("final_degree", ctypes.c_int64),
                ("roots", (ctypes.c_uint8 * 32) * 64), ("betas", ctypes.c_uint64 * 64)]


def build_c_oracle() -> str:
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return ORACLE_SO


def load_c_oracle() -> ctypes.CDLL:
    # FRI_ORACLE_SO: another build of the same C oracle (tests/test_sanitizers.py
    # loads the ASan/UBSan one, oracle/Makefile `asan`)
    path = os.environ.get("FRI_ORACLE_SO", ORACLE_SO)
    if path == ORACLE_SO and not os.path.exists(ORACLE_SO):
        build_c_oracle()
    lib = ctypes.CDLL(path)
    u64, sz, p64 = ctypes.c_uint64, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)
    for name in ("orc_fe_add", "orc_fe_sub", "orc_fe_mul", "orc_fe_pow", "orc_fe_div"):
        getattr(lib, name).restype = u64
        getattr(lib, name).argtypes = [u64, u64, u64]
    for name in ("orc_fe_new", "orc_fe_inverse", "orc_fe_neg"):
        getattr(lib, name).restype = u64
        getattr(lib, name).argtypes = [u64, u64]
    lib.orc_poly_trim.restype = sz
    lib.orc_poly_trim.argtypes = [p64, sz]
    lib.orc_poly_evaluate.restype = u64
    lib.orc_poly_evaluate.argtypes = [p64, sz, u64, u64]
    lib.orc_bench_evaluate.restype = u64
    lib.orc_bench_evaluate.argtypes = [p64, sz, u64, u64, sz]
    lib.orc_poly_mul.restype = sz
    lib.orc_poly_mul.argtypes = [p64, sz, p64, sz, p64, u64]
    lib.orc_poly_div_rem.restype = ctypes.c_int
    lib.orc_poly_div_rem.argtypes = [p64, sz, p64, sz, p64, ctypes.POINTER(sz), p64,
                                     ctypes.POINTER(sz), u64]
    lib.orc_interpolate_lagrange.restype = sz
    lib.orc_interpolate_lagrange.argtypes = [p64, p64, sz, p64, u64]
    lib.orc_sha256.restype = None
    lib.orc_sha256.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p]
    lib.orc_merkle_nodes_count.restype = sz
    lib.orc_merkle_nodes_count.argtypes = [sz]
    lib.orc_merkle_build.restype = sz
    lib.orc_merkle_build.argtypes = [p64, sz, ctypes.c_char_p]
    lib.orc_channel_init.argtypes = [ctypes.POINTER(OrcChannel)]
    lib.orc_channel_send.argtypes = [ctypes.POINTER(OrcChannel), ctypes.c_char_p, sz]
    lib.orc_channel_receive_int.restype = u64
    lib.orc_channel_receive_int.argtypes = [ctypes.POINTER(OrcChannel), u64, u64]
    lib.orc_channel_receive_fe.restype = u64
    lib.orc_channel_receive_fe.argtypes = [ctypes.POINTER(OrcChannel), u64]
    for name in ("orc_fri_commit_faithful", "orc_fri_commit_fast"):
        fn = getattr(lib, name)
        fn.restype = ctypes.c_int
        fn.argtypes = [p64, sz, ctypes.c_uint32, u64, u64, u64, ctypes.POINTER(OrcChannel),
                       p64, ctypes.POINTER(OrcFriResult), p64, ctypes.c_char_p]
    lib.orc_lde.restype = ctypes.c_int
    lib.orc_lde.argtypes = [p64, sz, ctypes.c_uint32, u64, u64, u64, p64]
    lib.orc_interpolate_coset.restype = sz
    lib.orc_interpolate_coset.argtypes = [p64, ctypes.c_uint32, u64, u64, u64, p64]
    lib.orc_batch_inverse.restype = None
    lib.orc_batch_inverse.argtypes = [p64, p64, sz, u64]
    lib.orc_fold_eval.restype = None
    lib.orc_fold_eval.argtypes = [p64, sz, u64, u64, u64, u64, p64]
    lib.orc_fibsq_trace.restype = None
    lib.orc_fibsq_trace.argtypes = [u64, sz, u64, p64]
    lib.orc_fibsq_cp_evals.restype = ctypes.c_int
    lib.orc_fibsq_cp_evals.argtypes = [p64, ctypes.c_uint32, ctypes.c_uint32, u64, u64, u64, u64, p64, p64]
    lib.orc_fibsq_prove_commit.restype = ctypes.c_int
    lib.orc_fibsq_prove_commit.argtypes = [u64, ctypes.c_uint32, ctypes.c_uint32, u64, u64, u64,
                                           ctypes.POINTER(OrcChannel), ctypes.c_char_p, p64,
                                           ctypes.POINTER(OrcFriResult), p64, ctypes.c_char_p, p64, ctypes.c_char_p]
    lib.orc_num_threads.restype = ctypes.c_int
    lib.orc_set_num_threads.argtypes = [ctypes.c_int]
    lib.orc_set_num_threads.restype = None
    return lib
