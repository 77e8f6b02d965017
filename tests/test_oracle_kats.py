"""Pin the oracle: the reference's own unit-test known answers replayed on
both restatements (Python twin and C oracle), generic over the modulus.

Sources (reference tree, read as text only):
  src/fields/element.rs:149-290        (18 field tests, mod 7)
  src/polynomial/ops.rs:551-1089       (36 polynomial tests, mod 7)
  src/polynomial/interpolation.rs:154-374 (6 interpolation tests, mod 7)
  src/fields/README.md:56-90, src/polynomial/README.md:381-383,417,487,511-524
                                       (worked examples, mod 7 / 17 / 23)
Tests that use OsRng (element.rs:214-220, ops.rs:691-694,1044-1067) are
replayed with a seeded RNG and assert the same properties.
"""
import ctypes
import random

import pytest


def c_arr(vals):
    a = (ctypes.c_uint64 * max(1, len(vals)))(*vals)
    return a


@pytest.fixture(params=["py", "c"])
def F(request, oracle, corc):
    """Field/poly API over either restatement."""
    if request.param == "py":
        o = oracle

        class Py:
            add, sub, mul, pow = o.fe_add, o.fe_sub, o.fe_mul, o.fe_pow
            inv, neg, div, new = o.fe_inverse, o.fe_neg, o.fe_div, o.fe_new

            @staticmethod
            def poly_mul(a, b, M):
                return o.poly_mul(o.poly_trim(a), o.poly_trim(b), M)

            @staticmethod
            def div_rem(a, b, M):
                return o.poly_div_rem(a, b, M)

            @staticmethod
            def evaluate(c, x, M):
                return o.poly_evaluate(o.poly_trim(c), x, M)

            @staticmethod
            def interpolate(xs, ys, M):
                return o.interpolate_lagrange_polynomials(xs, ys, M)

            @staticmethod
            def trim(c):
                return o.poly_trim(c)

        return Py
    lib = corc

    class C:
        add = staticmethod(lambda a, b, M: lib.orc_fe_add(a, b, M))
        sub = staticmethod(lambda a, b, M: lib.orc_fe_sub(a, b, M))
        mul = staticmethod(lambda a, b, M: lib.orc_fe_mul(a, b, M))
        pow = staticmethod(lambda a, e, M: lib.orc_fe_pow(a, e, M))
        div = staticmethod(lambda a, b, M: lib.orc_fe_div(a, b, M))
        inv = staticmethod(lambda a, M: lib.orc_fe_inverse(a, M))
        neg = staticmethod(lambda a, M: lib.orc_fe_neg(a, M))
        new = staticmethod(lambda a, M: lib.orc_fe_new(a, M))

        @staticmethod
        def trim(c):
            return list(c[: lib.orc_poly_trim(c_arr(c), len(c))])

        @staticmethod
        def poly_mul(a, b, M):
            a, b = C.trim(a), C.trim(b)
            out = (ctypes.c_uint64 * (len(a) + len(b) + 1))()
            n = lib.orc_poly_mul(c_arr(a), len(a), c_arr(b), len(b), out, M)
            return list(out[:n])

        @staticmethod
        def div_rem(a, b, M):
            a, b = C.trim(a), C.trim(b)
            q = (ctypes.c_uint64 * (len(a) + 1))()
            r = (ctypes.c_uint64 * (len(a) + 1))()
            lq, lr = ctypes.c_size_t(), ctypes.c_size_t()
            rc = lib.orc_poly_div_rem(c_arr(a), len(a), c_arr(b), len(b), q, ctypes.byref(lq), r,
                                      ctypes.byref(lr), M)
            if rc != 0:
                raise ZeroDivisionError("Division by zero polynomial")
            return list(q[: lq.value]), list(r[: lr.value])

        @staticmethod
        def evaluate(c, x, M):
            c = C.trim(c)
            return lib.orc_poly_evaluate(c_arr(c), len(c), x, M)

        @staticmethod
        def interpolate(xs, ys, M):
            out = (ctypes.c_uint64 * len(xs))()
            n = lib.orc_interpolate_lagrange(c_arr(xs), c_arr(ys), len(xs), out, M)
            return list(out[:n])

    return C


# ------------------------------------------------ src/fields/element.rs:149-290
def test_field_add(F):            assert F.add(1, 2, 7) == 3                 # :154-159
def test_field_sub(F):            assert F.sub(1, 2, 7) == 6                 # :162-167
def test_field_mul(F):            assert F.mul(3, 4, 7) == 5                 # :170-175
def test_field_div(F):            assert F.div(1, 3, 7) == 5                 # :178-183
def test_field_inverse(F):        assert F.inv(3, 7) == 5                    # :186-190
def test_field_pow(F):            assert F.pow(3, 3, 7) == 6                 # :193-197
def test_negation(F):             assert F.neg(3, 7) == 4                    # :208-212
def test_modular_wraparound(F):   assert F.add(F.new(10, 7), F.new(12, 7), 7) == 1   # :223-228
def test_equality(F):             assert F.new(3, 7) == F.new(10, 7)         # :231-235
def test_field_add_assign(F):     assert F.add(3, 5, 7) == 1                 # :238-243
def test_field_sub_assign(F):     assert F.sub(3, 5, 7) == 5                 # :246-251
def test_field_mul_assign(F):     assert F.mul(3, 5, 7) == 1                 # :254-259
def test_field_div_assign(F):     assert F.div(3, 5, 7) == 2                 # :262-267
def test_pow_zero(F):             assert F.pow(3, 0, 7) == 1                 # :271-275
def test_pow_one(F):              assert F.pow(3, 1, 7) == 3                 # :278-282
def test_inverse_multiplication(F): assert F.mul(3, F.inv(3, 7), 7) == 1     # :285-289


def test_zero_and_one(F):                                                    # :200-205
    assert F.new(0, 7) == 0 and F.new(1, 7) == 1


def test_random_generation(F):                                               # :214-220
    rng = random.Random(7)
    for _ in range(100):
        assert F.new(rng.getrandbits(64), 7) < 7


def test_inverse_of_zero_is_zero(F):                                         # element.rs:54-57 (0^(p-2))
    assert F.inv(0, 7) == 0 and F.inv(0, 3221225473) == 0


def test_field_readme_examples(F):                                           # src/fields/README.md:56-90
    a, b = 2, 5
    assert F.add(a, b, 7) == 0 and F.sub(b, a, 7) == 3 and F.mul(a, b, 7) == 3 and F.div(b, a, 7) == 6
    assert F.inv(3, 7) == 5 and F.pow(2, 3, 7) == 1


def test_stark101_prime_inverse(F):
    p = 3221225473
    for x in (1, 2, 5, 12345, p - 1):
        assert F.mul(x, F.inv(x, p), p) == 1


# --------------------------------------------- src/polynomial/ops.rs:551-1089
def test_zero_polynomial(F):                                                 # :572-576
    assert F.trim([]) == [] and len(F.trim([])) - 1 == -1


def test_evaluate_zero_polynomial(F):       assert F.evaluate([], 0, 7) == 0      # :579-584
def test_evaluate_constant_polynomial(F):   assert F.evaluate([5], 0, 7) == 5     # :587-593


def test_poly_addition(oracle):                                              # :596-604
    assert oracle.poly_add([2, 3], [4, 1], 7) == [6, 4]


def test_poly_subtraction(oracle):                                           # :607-616
    assert oracle.poly_sub([6, 5], [4, 3], 7) == [2, 2]


def test_poly_multiplication(F):            assert F.poly_mul([1, 2], [3, 4], 7) == [3, 3, 1]   # :619-632


def test_poly_scalar_multiplication(oracle):                                 # :636-647
    assert oracle.poly_scalar_mul([2, 3], 4, 7) == [1, 5]


def test_poly_division(F):                                                   # :650-672
    q, r = F.div_rem([1, 3, 2], [1, 1], 7)
    assert q == [1, 2] and r == []


def test_poly_composition(oracle):                                           # :676-687
    assert oracle.poly_compose([1, 1], [2, 3], 7) == [3, 3]


def test_poly_random_generation(F):                                          # :690-694
    rng = random.Random(1)
    c = [rng.randrange(7) for _ in range(5)] + [rng.randrange(1, 7)]
    assert len(F.trim(c)) - 1 == 5


def test_create_with_trailing_zeros(F):     assert F.trim([1, 2, 0, 0]) == [1, 2]     # :708-721
def test_is_zero(F):                        assert F.trim([0, 1]) != []               # :724-730


def test_leading_coefficient(F):                                             # :733-747
    assert F.trim([2, 5])[-1] == 5 and F.trim([]) == []


def test_add_zero_polynomial(oracle):       assert oracle.poly_add([3, 4], [], 7) == [3, 4]   # :750-756
def test_sub_zero_polynomial(oracle):       assert oracle.poly_sub([3, 4], [], 7) == [3, 4]   # :759-766
def test_add_assign(oracle):                assert oracle.poly_add([1, 2], [2, 3], 7) == [3, 5]  # :769-777
def test_sub_assign(oracle):                assert oracle.poly_sub([3, 5], [2, 3], 7) == [1, 2]  # :780-788
def test_mul_by_zero_polynomial(F):         assert F.poly_mul([1, 2], [], 7) == []        # :791-798
def test_mul_assign_polynomial(F):          assert F.poly_mul([1, 2], [2, 1], 7) == [2, 5, 2]  # :801-813


def test_poly_scalar_division(oracle):                                       # :816-826
    assert oracle.poly_scalar_mul([2, 4], oracle.fe_inverse(2, 7), 7) == [1, 2]


def test_poly_div_rem_no_remainder(F):                                       # :837-858
    q, r = F.div_rem([1, 3, 2], [1, 1], 7)
    assert q[0] == 1 and q[1] == 2 and r == []


def test_poly_rem_operator(F):                                               # :861-880
    q, r = F.div_rem([2, 5, 3], [1, 1], 7)
    assert r == F.div_rem([2, 5, 3], [1, 1], 7)[1]


def test_poly_rem_assign(F):                                                 # :883-905
    _, r = F.div_rem([1, 1, 1], [1, 1], 7)
    assert r == [1]


def test_poly_div_rem_nontrivial(F, oracle):                                 # :908-924
    q, r = F.div_rem([2, 5, 3], [1, 1], 7)
    rebuilt = oracle.poly_mul([1, 1], q, 7)
    if r:
        rebuilt = oracle.poly_add(rebuilt, r, 7)
    assert rebuilt == [2, 5, 3]


def test_poly_div_by_zero_polynomial(F):                                     # :927-933 (should_panic)
    with pytest.raises(ZeroDivisionError):
        F.div_rem([1, 2], [], 7)


def test_poly_div_assign_scalar(oracle):                                     # :935-941
    assert oracle.poly_scalar_mul([2, 4], oracle.fe_inverse(2, 7), 7) == [1, 2]


def test_neg(oracle):                                                        # :946-957
    p = [1, 2]
    assert oracle.poly_add(p, [oracle.fe_neg(c, 7) for c in p], 7) == []


def test_partial_eq_diff_length(F):         assert F.trim([1, 2]) != F.trim([1, 2, 3])   # :960-973
def test_partial_eq_diff_coeff(F):          assert F.trim([1, 2]) != F.trim([1, 3])      # :976-989


def test_compose_with_zero(oracle):         assert oracle.poly_compose([1, 1], [], 7) == [1]     # :993-1003
def test_compose_with_constant(oracle):     assert oracle.poly_compose([2, 1], [5], 7) == []     # :1006-1019
def test_compose_additional(oracle):        assert oracle.poly_compose([1, 1], [2, 3], 7) == [3, 3]  # :1021-1039


def test_div_rem_random_polys(F, oracle):                                    # :1041-1067
    rng = random.Random(5)
    for _ in range(20):
        a = [rng.randrange(7) for _ in range(rng.randrange(0, 5))] + [rng.randrange(1, 7)]
        b = [rng.randrange(7) for _ in range(rng.randrange(0, 5))] + [rng.randrange(1, 7)]
        q, r = F.div_rem(a, b, 7)
        if r:
            assert len(r) - 1 < len(oracle.poly_trim(b)) - 1
        rebuilt = oracle.poly_mul(oracle.poly_trim(b), q, 7) if q else []
        rebuilt = oracle.poly_add(rebuilt, r, 7) if r else rebuilt
        assert rebuilt == oracle.poly_trim(a)


def test_from_iter(F):                      assert F.trim([1, 2, 0]) == [1, 2]           # :1070-1089


def test_poly_readme_examples(F, oracle):                                    # src/polynomial/README.md
    assert F.evaluate([3, 2, 5], 4, 17) == 6                                 # :381-383
    p, q = [1, 2, 3], [4, 5]
    assert oracle.poly_add(p, q, 17) == [5, 7, 3]
    assert oracle.poly_sub(p, q, 17) == [14, 14, 3]
    assert F.poly_mul(p, q, 17) == [4, 13, 22 % 17, 15]
    assert F.evaluate(p, 2, 17) == 0                                         # :487
    assert oracle.poly_compose(p, q, 17) == [6, 11, 7]
    assert oracle.poly_compose([2, 3, 1], [1, 4], 23) == [6, 20, 16]        # :511-524


# -------------------------------------- src/polynomial/interpolation.rs:154-374
def test_gen_polynomial_from_roots(oracle, corc):                            # :170-184
    assert oracle.gen_polynomial_from_roots([1, 2, 3], 7) == [1, 4, 1, 1]
    out = (ctypes.c_uint64 * 4)()
    n = corc.orc_poly_from_roots(c_arr([1, 2, 3]), 3, out, 7)
    assert list(out[:n]) == [1, 4, 1, 1]


@pytest.mark.parametrize("xs", [[2, 3, 5], [2, 3, 5, 6], [1, 2, 3, 4, 6]])   # :187-221, :259-282, :307-372
def test_gen_lagrange_poly(F, oracle, xs):
    basis = oracle.gen_lagrange_polynomials(xs, 7)
    assert len(basis) == len(xs)
    for i, li in enumerate(basis):
        for j, xj in enumerate(xs):
            assert F.evaluate(li, xj, 7) == (1 if i == j else 0)


def test_interpolate_lagrange_polynomials(F):                               # :285-304
    assert F.interpolate([2, 3, 5], [1, 2, 3], 7) == [5, 3, 1]


def test_interpolation_roundtrip_random(F, oracle):                         # :223-256 (commented out upstream)
    rng = random.Random(11)
    p = 3221225473
    for deg in (0, 1, 5, 17):
        coeffs = [rng.randrange(p) for _ in range(deg)] + [rng.randrange(1, p)]
        xs = rng.sample(range(1, 10**6), deg + 1)
        ys = [F.evaluate(coeffs, x, p) for x in xs]
        assert F.interpolate(xs, ys, p) == coeffs


# ------------------------------------- third party: rs_merkle 1.4.2 (Cargo.lock:3456-3462)
def test_rs_merkle_documented_root(oracle):
    """rs_merkle's own documented example (crate README / `MerkleTree` docs):
    `MerkleTree::<Sha256>::from_leaves` over the SHA-256 digests of the
    strings "a".."f" has root_hex 1f7379...4da2.  Six leaves take the odd-node
    path on level 1 (three nodes, the last promoted unchanged), so this pins
    both the pairing and the promotion that src/merkle/mod.rs:15-25 inherits."""
    import hashlib
    leaves = [hashlib.sha256(s.encode()).digest() for s in "abcdef"]
    levels = oracle.merkle_levels_from_leaves(leaves)
    assert [len(lv) for lv in levels] == [6, 3, 2, 1]
    assert levels[1][2] == hashlib.sha256(leaves[4] + leaves[5]).digest()
    assert levels[2][1] == levels[1][2]                       # promoted, not re-hashed
    assert levels[-1][0].hex() == "1f7379539707bcaea00564168d1d4d626b09b73f8a2a365234c62d763f854da2"


def test_rs_merkle_shape_c_oracle_matches_twin(oracle, corc):
    """The C oracle's tree (orc_merkle_build over field values) has the twin's
    shape for every size 1..40, so the documented root above pins it too."""
    import ctypes as ct
    for n in range(1, 41):
        vals = [(7919 * i + 3) % 3221225473 for i in range(n)]
        cnt = corc.orc_merkle_nodes_count(n)
        nodes = ct.create_string_buffer(32 * cnt)
        corc.orc_merkle_build(c_arr(vals), n, nodes)
        assert nodes.raw[32 * (cnt - 1): 32 * cnt].hex() == oracle.merkle_root_hex(vals)


# ------------------- third party: sha256 1.5.0 and const-hex 1.14.0 (channel.rs:35-84)
def test_channel_sha256_crate_documented_digest(oracle):
    """sha256 1.5.0's documented example: digest("hello") is the lowercase hex
    2cf24d…9824.  Channel::send sets state = sha256::digest(state ‖ hex(msg))
    (channel.rs:35-40), so a state of "hello" and an empty message must give
    exactly that string."""
    ch = oracle.Channel(state="hello")
    ch.send(b"")
    assert ch.state == "2cf24dba5fb0a30e26e83b2ac5b9e29e1b161e5c1fa7425e73043362938b9824"


def test_channel_hex_crate_documented_encoding(oracle):
    """hex::encode (const-hex, the hex-crate API alloy re-exports; channel.rs:6,38)
    is documented as hex::encode("Hello world!") == "48656c6c6f20776f726c6421":
    lowercase, no prefix.  send hashes exactly that text after the old state."""
    import hashlib
    ch = oracle.Channel()
    ch.send(b"Hello world!")
    assert ch.state == hashlib.sha256(b"48656c6c6f20776f726c6421").hexdigest()
    beta = oracle.Channel(state=ch.state).receive_random_field_element()
    assert beta == int(ch.state, 16) % 3221225473           # U256::from_str_radix(state, 16) % p, min = 0
