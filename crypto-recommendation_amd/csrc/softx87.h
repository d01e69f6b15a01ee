// softx87.h — exact emulation of the x87 80-bit `long double` operations the
// reference hot path performs, in 64-bit integer arithmetic, usable in gfx950
// kernels and in host code (the CPU tests check it against real long double).
//
// Why: the reference accumulates every inner product in long double
// (cust_vector.hpp:105-121) and floors (acc + t) / w in long double
// (euclidean_h_gen.hpp:73-76). The GPU has no 80-bit type. The fast path
// computes in fp64 with a rigorous error bound; a value whose floor or sign
// the bound cannot certify is recomputed here, bit-exactly, on the GPU.
//
// Model: x87 default precision control on x86-64 Linux = 64-bit significand,
// round-to-nearest-even, exponent range wide enough that no input we see
// (finite doubles/floats, |values| < 2^1000) over- or underflows it.
// A value is (-1)^s * m * 2^e with m normalised (bit 63 set) or m == 0.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SX_HD __host__ __device__ inline
#define SX_MD __host__ __device__ inline
#else
#define SX_HD static inline
#define SX_MD inline
#endif

struct sx80 {
    uint64_t m;
    int32_t e;
    int32_t s;
};

SX_HD int sx_clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return x ? __clzll((long long)x) : 64;
#else
    return x ? __builtin_clzll(x) : 64;
#endif
}

SX_HD sx80 sx_zero() { sx80 r; r.m = 0; r.e = 0; r.s = 0; return r; }

SX_HD sx80 sx_from_double(double v) {
    union { double d; uint64_t u; } c; c.d = v;
    sx80 r; r.s = (int32_t)(c.u >> 63);
    int be = (int)((c.u >> 52) & 0x7FF);
    uint64_t frac = c.u & 0xFFFFFFFFFFFFFull;
    if (be == 0) {                       // zero or subnormal
        if (frac == 0) { r.m = 0; r.e = 0; return r; }
        int lz = sx_clz64(frac);
        r.m = frac << lz;
        r.e = -1074 - lz;                // frac * 2^-1074
        return r;
    }
    r.m = (frac | (1ull << 52)) << 11;   // 53-bit significand -> bit 63
    r.e = be - 1075 - 11;
    return r;
}

SX_HD sx80 sx_from_float(float v) { return sx_from_double((double)v); }

// Round a non-negative 128-bit integer (hi:lo) * 2^e to 64 bits, nearest-even.
// sticky != 0 means "the true value is slightly above hi:lo" (bits below lo).
SX_HD sx80 sx_round128(uint64_t hi, uint64_t lo, int32_t e, int s, int sticky) {
    sx80 r; r.s = s;
    if (hi == 0 && lo == 0) { r.m = 0; r.e = 0; r.s = sticky ? s : 0; return r; }
    int p;   // index of the top set bit in 0..127
    if (hi) p = 127 - sx_clz64(hi); else p = 63 - sx_clz64(lo);
    if (p <= 63) {                       // fits in 64 bits exactly (modulo sticky, below bit 0)
        uint64_t v = hi ? 0 : lo;
        int sh = 63 - p;
        r.m = v << sh; r.e = e - sh;
        // sticky bits sit below bit 0 and therefore below half an ulp only if sh == 0;
        // with sh > 0 the value v<<sh is exact and the sticky part < 2^-sh ulp: rounds down.
        return r;
    }
    int drop = p - 63;                   // bits below the kept 64
    uint64_t keep, rem_hi_bit, rem_rest;
    if (drop < 64) {
        keep = (hi << (64 - drop)) | (lo >> drop);
        if (drop == 0) keep = lo;        // unreachable (p > 63), kept for clarity
        uint64_t rem = lo & ((drop == 64) ? ~0ull : ((1ull << drop) - 1));
        rem_hi_bit = (rem >> (drop - 1)) & 1;
        rem_rest = rem & ((1ull << (drop - 1)) - 1);
    } else {                             // drop == 64: keep = hi
        keep = hi;
        rem_hi_bit = lo >> 63;
        rem_rest = lo & 0x7FFFFFFFFFFFFFFFull;
    }
    int round_up = rem_hi_bit && (rem_rest || sticky || (keep & 1));
    int32_t ne = e + drop;
    if (round_up) {
        keep += 1;
        if (keep == 0) { keep = 1ull << 63; ne += 1; }
    }
    r.m = keep; r.e = ne;
    return r;
}

// a + b rounded to 64-bit significand, nearest-even (x87 FADD).
SX_HD sx80 sx_add(sx80 a, sx80 b) {
    if (b.m == 0) { if (a.m == 0) { sx80 z = sx_zero(); z.s = a.s & b.s; return z; } return a; }
    if (a.m == 0) return b;
    if (a.e < b.e || (a.e == b.e && a.m < b.m)) { sx80 t = a; a = b; b = t; }   // |a| >= |b|
    // place a.m at bits [63..126]: value = A * 2^(a.e - 63)
    uint64_t ahi = a.m >> 1, alo = a.m << 63;
    int64_t diff = (int64_t)a.e - (int64_t)b.e;   // >= 0
    uint64_t bhi, blo; int sticky = 0;
    if (diff > 126) { bhi = 0; blo = 0; sticky = 1; }
    else {
        // b.m << 63 >> diff
        uint64_t h = b.m >> 1, l = b.m << 63;
        if (diff >= 64) {
            int d2 = (int)(diff - 64);
            uint64_t lost = (d2 == 0) ? l : (l | (h & ((d2 >= 64) ? ~0ull : ((1ull << d2) - 1))));
            sticky = lost != 0;
            blo = (d2 >= 64) ? 0 : (h >> d2); bhi = 0;
        } else if (diff > 0) {
            int d = (int)diff;
            sticky = (l & ((1ull << d) - 1)) != 0;
            blo = (l >> d) | (h << (64 - d));
            bhi = h >> d;
        } else { bhi = h; blo = l; }
    }
    uint64_t rhi, rlo;
    if (a.s == b.s) {
        rlo = alo + blo; rhi = ahi + bhi + (rlo < alo ? 1 : 0);
        return sx_round128(rhi, rlo, a.e - 63, a.s, sticky);
    }
    // subtract: |a| >= |b|; a sticky b-part lowers the value slightly -> subtract 1 ulp of 2^0 and keep sticky set
    rlo = alo - blo; rhi = ahi - bhi - (alo < blo ? 1 : 0);
    if (sticky) {
        // true value = (rhi:rlo) - tiny: represent as (rhi:rlo) - 1 with sticky (the tiny remainder is in (0,1))
        uint64_t nlo = rlo - 1; rhi = rhi - (rlo == 0 ? 1 : 0); rlo = nlo;
    }
    if (rhi == 0 && rlo == 0 && !sticky) { return sx_zero(); }   // exact cancellation -> +0
    return sx_round128(rhi, rlo, a.e - 63, a.s, sticky);
}

SX_HD sx80 sx_add_double(sx80 a, double d) { return sx_add(a, sx_from_double(d)); }

// a / b rounded to 64 bits nearest-even (x87 FDIV). b != 0.
SX_HD sx80 sx_div(sx80 a, sx80 b) {
    sx80 r; r.s = a.s ^ b.s;
    if (a.m == 0) { r.m = 0; r.e = 0; return r; }
    // Q = floor(a.m * 2^64 / b.m) in [2^63, 2^65), remainder rem.
    uint64_t rem = a.m, q = 0; uint64_t qtop = 0;
    if (rem >= b.m) { qtop = 1; rem -= b.m; }
    for (int i = 0; i < 64; i++) {
        uint64_t carry = rem >> 63;
        rem <<= 1; q <<= 1;
        if (carry || rem >= b.m) { rem -= b.m; q |= 1; }
    }
    int32_t e = a.e - b.e - 64;
    if (qtop) {
        // 65-bit quotient: keep top 64, round bit = q & 1, sticky = rem != 0
        uint64_t keep = (1ull << 63) | (q >> 1);
        int rb = (int)(q & 1);
        int up = rb && (rem != 0 || (keep & 1));
        e += 1;
        if (up) { keep += 1; if (keep == 0) { keep = 1ull << 63; e += 1; } }
        r.m = keep; r.e = e; return r;
    }
    // 64-bit quotient (top bit set): next bit from 2*rem vs b.m
    uint64_t keep = q;
    int up;
    uint64_t carry = rem >> 63, r2 = rem << 1;
    if (carry || r2 > b.m) up = 1;
    else if (r2 == b.m) up = (int)(keep & 1);
    else up = 0;
    if (up) { keep += 1; if (keep == 0) { keep = 1ull << 63; e += 1; } }
    r.m = keep; r.e = e; return r;
}

// floorl(v) converted to int (values are in int range on the hash path).
SX_HD int64_t sx_floor_i64(sx80 v) {
    if (v.m == 0) return 0;
    if (v.e >= 0) {
        uint64_t mag = (v.e >= 63) ? ~0ull : (v.m << v.e);   // out of range: saturate
        return v.s ? -(int64_t)(mag >> 1) : (int64_t)(mag >> 1);  // (never taken on the hash path)
    }
    if (v.e <= -64) return v.s ? -1 : 0;                      // 0 < |v| < 1
    int sh = -v.e;
    uint64_t ip = v.m >> sh;
    uint64_t fr = v.m & ((1ull << sh) - 1);
    if (!v.s) return (int64_t)ip;
    return -(int64_t)ip - (fr ? 1 : 0);
}

SX_HD int sx_ge_zero(sx80 v) { return v.m == 0 || v.s == 0; }

// int(floorl(v)) as g++ -O0 compiles it (FISTP with truncation after floorl):
// a value outside the int range stores the x87 "integer indefinite" INT_MIN.
SX_HD int32_t sx_floor_int32(sx80 v) {
    if (v.m != 0 && v.e >= 0) return (int32_t)0x80000000;    // |v| >= 2^63
    const int64_t f = sx_floor_i64(v);
    return (f < -2147483648ll || f > 2147483647ll) ? (int32_t)0x80000000 : (int32_t)f;
}

// The reference's inner product (cust_vector.hpp:105-121): a long double
// chain over double products, which may be inf or NaN for fp64 inputs (SSE
// products overflow; the x87 sum of finite doubles never does). Finite products
// go through the soft FADD; special ones are tracked as IEEE addition would
// combine them (any NaN, or +inf with -inf, gives NaN).
struct SxSum {
    sx80 s;
    int pinf, ninf, nan;
    SX_MD void init() { s = sx_zero(); pinf = ninf = nan = 0; }
    SX_MD void add(double p) {
        union { double d; uint64_t u; } c; c.d = p;
        if (((c.u >> 52) & 0x7FF) != 0x7FF) { s = sx_add_double(s, p); return; }
        if (c.u & 0xFFFFFFFFFFFFFull) nan = 1;
        else if (c.u >> 63) ninf = 1;
        else pinf = 1;
    }
    // 0 finite (s holds it), 1 +inf, -1 -inf, 2 NaN
    SX_MD int special() const { return (nan || (pinf && ninf)) ? 2 : pinf ? 1 : ninf ? -1 : 0; }
};

// EuclideanHGen::generate (euclidean_h_gen.hpp:79-82): int(floorl((ip + t) / w)).
SX_HD int32_t sx_hash_floor(const SxSum& ip, double t, float w) {
    if (ip.special()) return (int32_t)0x80000000;             // floorl(inf / nan) -> indefinite
    return sx_floor_int32(sx_div(sx_add_double(ip.s, t), sx_from_float(w)));
}

// CosineHGen::generate (cosine_h_gen.hpp:71-76): ip >= 0 (false for NaN).
SX_HD int sx_hash_sign(const SxSum& ip) {
    const int sp = ip.special();
    return sp == 0 ? sx_ge_zero(ip.s) : sp == 1 ? 1 : 0;
}

// Round to double, nearest-even (x87 FST m64 / the long double -> double cast).
// The x87 running sum of doubles (FADD of a double operand, 64-bit
// significand, nearest-even) carried EXACTLY as a double-double: S = h + l
// (a 64-bit value fits in 106 bits). add(p): S <- RN64(S + p) in ~30 fp64
// operations instead of a soft FADD: with (s, e1) = TwoSum(h, p) and (t, dl) =
// TwoSum(l, e1), S + p = s + t + dl exactly; s lies on the 64-bit grid of the
// result's binade E (|t + dl| << |s|), so RN64(S + p) = s + RN_grid(t + dl),
// the grid rounding done by the magic constant 1.5 * 2^(E - 11) (whose ulp is
// the grid spacing 2^(E - 63); ties go to even multiples, and s is an even
// multiple, so that is the x87 tie rule), corrected when t sits exactly on a
// midpoint and dl decides. E is the binade of fl(s + t) unless that is a power
// of two, where the sign of S + p - 2^m decides between m and m - 1. Returns
// false (state unspecified; the caller takes the soft form) for a zero-sum
// with a nonzero residue or a magnitude outside [2^-899, 2^900] (incl.
// inf / NaN products).
struct X87dd {
    double h, l;
    SX_MD void init() { h = 0.0; l = 0.0; }
    static SX_MD uint64_t bits(double v) { union { double d; uint64_t u; } c; c.d = v; return c.u; }
    static SX_MD double from_bits(uint64_t u) { union { double d; uint64_t u; } c; c.u = u; return c.d; }
    SX_MD bool add(double p) {
        const double s = h + p, bb = s - h;
        const double e1 = (h - (s - bb)) + (p - bb);
        const double t = l + e1, b2 = t - l;
        const double dl = (l - (t - b2)) + (e1 - b2);
        const double u = s + t;
        const uint64_t ub = bits(u);
        int be = (int)((ub >> 52) & 0x7FF);
        if (u == 0.0) {
            if (dl != 0.0) return false;
            h = 0.0; l = 0.0;                             // exact cancellation: +0
            return true;
        }
        if (be < 124 || be > 1923) return false;
        if ((ub & 0xFFFFFFFFFFFFFull) == 0) {            // u = +-2^m: is |S + p| below 2^m?
            double w = (s - u) + t;                       // s - u exact (Sterbenz)
            if (w == 0.0) w = dl;
            if ((w < 0.0) != (u < 0.0) && w != 0.0) be -= 1;
        }
        const double ulp64 = from_bits((uint64_t)(be - 63) << 52);
        const double C = from_bits(((uint64_t)(be - 11) << 52) | (1ull << 51));   // 1.5 * 2^(E - 11)
        double r = (t + C) - C;
        const double diff = t - r;
        if (dl != 0.0 && (diff == 0.5 * ulp64 || diff == -0.5 * ulp64) && ((dl > 0.0) == (diff > 0.0)))
            r += diff > 0.0 ? ulp64 : -ulp64;
        const double nh = s + r, b3 = nh - s;
        l = (s - (nh - b3)) + (r - b3);
        h = nh;
        return true;
    }
    // the 64-bit value as sx80 (h + l is exact in 64 bits: one exact FADD)
    SX_MD sx80 value() const;
};

SX_MD sx80 X87dd::value() const { return sx_add_double(sx_from_double(h), l); }

// The x87 chain for any double terms: X87dd while it decides (add leaves the
// state untouched when it returns false), the soft FADD from that exact state
// on. A drop-in for `sx80 ip = sx_zero(); ip = sx_add_double(ip, p);`.
struct X87acc {
    X87dd dd;
    sx80 sx;
    bool soft;
    SX_MD void init() { dd.init(); sx = sx_zero(); soft = false; }
    SX_MD void add(double p) {
        if (!soft) {
            if (dd.add(p)) return;
            sx = dd.value();
            soft = true;
        }
        sx = sx_add_double(sx, p);
    }
    SX_MD sx80 value() const { return soft ? sx : dd.value(); }
};

SX_HD double sx_to_double(sx80 v) {
    if (v.m == 0) return v.s ? -0.0 : 0.0;
    uint64_t keep = v.m >> 11, rem = v.m & 0x7FF;
    int32_t e = v.e + 11;
    if (rem > 0x400 || (rem == 0x400 && (keep & 1))) {
        keep += 1;
        if (keep == (1ull << 53)) { keep >>= 1; e += 1; }
    }
    // value = keep * 2^e, keep in [2^52, 2^53)
    int be = e + 1075;
    union { double d; uint64_t u; } c;
    if (be <= 0 || be >= 0x7FF) {        // outside the normal range: not reached on our paths
        double x = (double)keep;
        for (int i = 0; i < (e > 0 ? e : -e); i++) x = e > 0 ? x * 2.0 : x * 0.5;
        return v.s ? -x : x;
    }
    c.u = ((uint64_t)v.s << 63) | ((uint64_t)be << 52) | (keep & 0xFFFFFFFFFFFFFull);
    return c.d;
}
