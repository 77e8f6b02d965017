// field.hpp — arithmetic in F_p, p = 3*2^30 + 1, for host and gfx950 device.
//
// Replaces src/fields/element.rs (FieldElement<M>{value: u64}, u128 `%` per
// mul, Fermat inverse).  Data stays CANONICAL (standard form, value < p) in
// HBM and in registers; only constants (twiddles, 2^-1, beta, domain
// inverses) are kept in Montgomery form a*R mod p, R = 2^32, so one REDC of
// (canonical x Montgomery) yields a canonical product:
//     redc(a * (b*R)) = a*b mod p.
// REDC uses the subtractive form hi(t) - hi(m*p), valid for p < 2^32 without
// a 64-bit overflow (p > 2^31 forbids the additive t + m*p form).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define FRI_HD __host__ __device__ __forceinline__
#else
#define FRI_HD inline
#endif

namespace fri {

constexpr uint32_t P = 3221225473u;          // 0xC0000001
constexpr uint32_t GEN = 5u;
constexpr uint32_t PINV = 0x40000001u;       // p^-1 mod 2^32 ((1+a)(1-a) = 1 - a^2, a = 3*2^30)
constexpr uint32_t R_MOD_P = 0x3FFFFFFFu;    // 2^32 mod p
constexpr uint32_t R2_MOD_P = (uint32_t)(((unsigned __int128)1 << 64) % P);   // 2^64 mod p
static_assert((uint32_t)(P * PINV) == 1u, "PINV");

// Montgomery reduction of t < p * 2^32: returns t * 2^-32 mod p, canonical.
// m = tlo * PINV is tlo + (tlo << 30) (PINV = 2^30 + 1: one v_lshl_add).
// The borrow of hi(t) - hi(m*p) comes straight from v_sub_co_u32 (VCC):
// written as __builtin_usub_overflow the compiler no longer widens the
// compare to 64 bits (3 half-rate + 3 full-rate VALU per product).
FRI_HD uint32_t redc(uint64_t t) {
    uint32_t tlo = (uint32_t)t, thi = (uint32_t)(t >> 32);
    uint32_t m = tlo * PINV;
    uint32_t u = (uint32_t)(((uint64_t)m * P) >> 32);
    uint32_t r;
    const bool borrow = __builtin_usub_overflow(thi, u, &r);
    return borrow ? r + P : r;
}

// a (canonical or Montgomery) x b (Montgomery) -> a*b*R^-1*R ... i.e.
//   mmul(std, mont) = std product;  mmul(mont, mont) = mont product.
FRI_HD uint32_t mmul(uint32_t a, uint32_t b) { return redc((uint64_t)a * b); }

// a - b for a < p, b <= p: one borrow-producing subtract, +p on borrow.
FRI_HD uint32_t sub(uint32_t a, uint32_t b) {
    uint32_t d;
    const bool borrow = __builtin_usub_overflow(a, b, &d);
    return borrow ? d + P : d;
}
// a + b = a - (p - b): p > 2^31, so a + b can carry out of 32 bits; the
// subtract form needs no carry test and no 64-bit compare.
FRI_HD uint32_t add(uint32_t a, uint32_t b) { return sub(a, P - b); }
FRI_HD uint32_t neg(uint32_t a) { return a ? P - a : 0u; }

FRI_HD uint32_t to_mont(uint32_t a) { return mmul(a, R2_MOD_P); }
FRI_HD uint32_t from_mont(uint32_t a) { return redc((uint64_t)a); }

// Montgomery-domain power: base_m in Montgomery form, result Montgomery form.
FRI_HD uint32_t mpow(uint32_t base_m, uint64_t e) {
    uint32_t r = R_MOD_P;   // 1 in Montgomery form
    while (e) {
        if (e & 1) r = mmul(r, base_m);
        base_m = mmul(base_m, base_m);
        e >>= 1;
    }
    return r;
}

// Canonical helpers (host-side setup and small device uses).
FRI_HD uint32_t mul_std(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % P); }
FRI_HD uint32_t pow_std(uint32_t a, uint64_t e) {
    uint64_t r = 1, b = a;
    while (e) { if (e & 1) r = r * b % P; b = b * b % P; e >>= 1; }
    return (uint32_t)r;
}
// element.rs:54-57 semantics: inverse(0) = 0^(p-2) = 0.
FRI_HD uint32_t inv_std(uint32_t a) { return pow_std(a, P - 2); }

// Generator of the order-2^k subgroup: g^((p-1)/2^k), k <= 30.
FRI_HD uint32_t root_of_unity(uint32_t log_n) { return pow_std(GEN, (uint64_t)(P - 1) >> log_n); }

}  // namespace fri
