// Host check of stark-prover_amd/csrc/field.hpp (the arithmetic every kernel
// uses; FRI_HD makes it host-callable): add / sub / redc / mmul / to_mont /
// from_mont against __int128 arithmetic on edge values and random operands.
// Semantics follow src/fields/element.rs:72-122 (canonical value % p).
#include <stdio.h>
#include <stdint.h>
#include "../../stark-prover_amd/csrc/field.hpp"

using namespace fri;

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t next64() {      // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    const uint32_t edges[] = {0u, 1u, 2u, 3u, 5u, 0x7FFFFFFFu, 0x80000000u, 0x80000001u, 0xBFFFFFFFu,
                              0xC0000000u, P - 3, P - 2, P - 1, (P - 1) / 2, (P + 1) / 2, R_MOD_P, R2_MOD_P};
    const int ne = sizeof(edges) / sizeof(edges[0]);
    long fails = 0, checks = 0;
    auto check = [&](const char* what, uint32_t a, uint32_t b, uint32_t got, uint64_t want) {
        checks++;
        if (got != want || got >= P) {
            if (fails++ < 10) printf("FAIL %s(%u, %u) = %u, want %llu\n", what, a, b, got, (unsigned long long)want);
        }
    };
    const unsigned __int128 RINV = [] {     // 2^-32 mod p by Fermat
        unsigned __int128 r = 1, b = ((unsigned __int128)1 << 32) % P;
        uint64_t e = P - 2;
        while (e) { if (e & 1) r = r * b % P; b = b * b % P; e >>= 1; }
        return r;
    }();
    auto pair = [&](uint32_t a, uint32_t b) {
        check("add", a, b, add(a, b), ((uint64_t)a + b) % P);
        check("sub", a, b, sub(a, b), ((uint64_t)a + P - b) % P);
        check("mmul", a, b, mmul(a, b), (uint64_t)((unsigned __int128)a * b % P * RINV % P));
        check("mul_std", a, b, mmul(a, to_mont(b)), (uint64_t)((unsigned __int128)a * b % P));
    };
    for (int i = 0; i < ne; i++)
        for (int j = 0; j < ne; j++) pair(edges[i], edges[j]);
    for (int k = 0; k < 2000000; k++) {
        const uint32_t a = (uint32_t)(next64() % P), b = (uint32_t)(next64() % P);
        pair(a, b);
        // redc over its whole input range t < p * 2^32 (hi word up to p - 1)
        const uint64_t t = ((next64() % P) << 32) | (uint32_t)next64();
        check("redc", (uint32_t)(t >> 32), (uint32_t)t, redc(t), (uint64_t)((unsigned __int128)t % P * RINV % P));
    }
    for (int i = 0; i < ne; i++) {
        check("mont_roundtrip", edges[i], 0, from_mont(to_mont(edges[i])), edges[i]);
        check("neg", edges[i], 0, neg(edges[i]), (P - edges[i]) % P);
    }
    printf("%ld checks, %ld failures\n", checks, fails);
    return fails ? 1 : 0;
}
