// Host check of csrc/gpow2.h against the process's real pow(x, 2) (glibc's
// __pow_fma on this image). Built and run by tests/test_lib_cpu.py
// (g++ -O2 -ffp-contract=off -fopenmp). Every case compares bits.
//   pow2_check <millions of random samples per set>
// Sets: uniform 64-bit patterns (every exponent, subnormals, inf, nan),
// [0.5, 4) dense, squares within 2^-8 ulp of a midpoint (the discriminating
// ones: ~20 % of them differ from x*x; and 2^-8 .. 2^-4 ulp away, across the
// 2^-6 window of gp_sq), 27-bit mantissas (exact ties), and
// exact squares across every exponent (<= 26-bit mantissas), and sweeps
// across the special ranges (subnormal / overflowing squares,
// |2 ln x| < 2^-54, the exp specialcase range 2^+-369, the gp_sq filter edges).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../crypto-recommendation_amd/csrc/gpow2.h"

static double (*volatile real_pow)(double, double) = pow;

static inline uint64_t mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static double gen(int set, uint64_t i) {
    const uint64_t a = mix(i * 4 + 1), b = mix(i * 4 + 2);
    switch (set) {
    case 0: return gp_dbl(a);                                            // any bit pattern
    case 1: return gp_dbl(0x3fe0000000000000ull + (a % (3ull << 52)));   // [0.5, 4)
    case 2: {                                                            // 27-bit mantissa: exact ties possible
        uint64_t m = (a & ((1ull << 26) - 1)) << 26;
        int e = (int)(b % 200) - 100;
        return ldexp(gp_dbl(0x3ff0000000000000ull | m), e) * ((b >> 40) & 1 ? -1.0 : 1.0);
    }
    case 3: {                                                            // special ranges
        static const double c[] = {0x1p-537, 0x1p-511, 0x1p-500, 0x1p-369, 0x1p369, 0x1p511, 0x1p512,
                                   0x1p-40, 0x1p40, 1.0, 0x1p-1022, 0x1p-1074, 0x1p1023, 0x1.6a09e667f3bcdp0};
        const double base = c[b % (sizeof c / sizeof c[0])];
        const double f = 1.0 + ldexp((double)(int64_t)(a >> 11) - 0x1p52, -60 + (int)((b >> 8) % 58));
        return base * f;
    }
    case 6: {                                                            // <= 26-bit mantissas, any exponent:
        uint64_t m = (a & ((1ull << 25) - 1)) << 27;                     // exact squares down to the subnormal range
        int e = (int)(b % 2140) - 1100;
        return ldexp(gp_dbl(0x3ff0000000000000ull | m), e);
    }
    default: {                                                           // random exponent, uniform mantissa
        int e = (int)(b % 2100) - 1080;
        return ldexp(gp_dbl(0x3ff0000000000000ull | (a >> 12)), e);
    }
    }
}

int main(int argc, char** argv) {
    const long n = (argc > 1 ? atol(argv[1]) : 10) * 1000000L;
    long bad = 0, nearmid = 0, differ = 0;
    for (int set = 0; set < 8; set++) {
        long sbad = 0, sdiff = 0, snear = 0;
#pragma omp parallel for reduction(+ : sbad, sdiff, snear) schedule(static)
        for (long i = 0; i < n; i++) {
            double x;
            if (set == 5 || set == 7) {      // near midpoints (5: within 2^-8 ulp; 7: 2^-8 .. 2^-4
                                             // ulp away, across gp_sq's 2^-6 window edge)
                uint64_t j = (uint64_t)i * 64 + (set == 7 ? (1ull << 50) : 0);
                const double lo = set == 5 ? 0.0 : 0x1p-8, hi = set == 5 ? 0x1p-8 : 0x1p-4;
                for (;; j++) {
                    x = gen(j & 1 ? 1 : 4, j + 0x51ed);
                    const double p = x * x, e = fma(x, x, -p);
                    if (!(fabs(x) >= 0x1p-500 && fabs(x) <= 0x1p500)) continue;
                    const double u = gp_dbl(gp_bits(p) & 0x7ff0000000000000ull) * 0x1p-52;
                    const double dm = fabs(fabs(e) - 0.5 * u);
                    if (dm >= lo * u && dm <= hi * u) break;
                }
                snear++;
            } else {
                x = gen(set, (uint64_t)i + ((uint64_t)set << 40));
            }
            const double ref = real_pow(x, 2.0);
            const double em = gp_pow2_emul(x), sq = gp_sq(x);
            const uint64_t rb = gp_bits(ref);
            if (ref != x * x && !(ref != ref)) sdiff++;
            if (gp_bits(em) != rb || gp_bits(sq) != rb) {
                sbad++;
                if (sbad <= 5)
#pragma omp critical
                    printf("MISMATCH set %d x=%a pow=%a emul=%a sq=%a\n", set, x, ref, em, sq);
            }
        }
        printf("set %d: %ld samples, pow != x*x on %ld, mismatches %ld\n", set, n, sdiff, sbad);
        bad += sbad;
        differ += sdiff;
        nearmid += snear;
    }
    printf("total mismatches %ld (pow != x*x on %ld samples; %ld near-midpoint samples)\n", bad, differ, nearmid);
    return bad != 0;
}
