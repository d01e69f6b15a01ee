// pow2.hip — the reference's pow(x, 2) as an entry point (lshkm_pow2, the
// device restatement of glibc's pow, gpow2.h) and its host-side self-check
// against the running process's own pow (lshkm_pow_selfcheck).
//   cust_vector.hpp:132, :149-150, :168-169 (every square the reference takes)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <mutex>
#include <string>

#include "../../include/lshkm.h"
#include "common.h"
#include "gpow2.h"
#include "index.h"

namespace lshkm {

__global__ __launch_bounds__(256) void pow2_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) out[i] = gp_sq(x[i]);
}

static uint64_t sc_mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

}  // namespace lshkm

using namespace lshkm;

// the process's pow, called for real (never folded to x*x)
static double (*volatile g_libm_pow)(double, double) = pow;

// Test build only (LSHKM_POW_HOST=rn): stand in for a host whose libm squares
// correctly rounded (another glibc variant, musl, ...), to exercise the
// refusal path of lshkm_ctx_create.
static double pow_rn(double x, double y) { return y == 2.0 ? x * x : pow(x, y); }

namespace lshkm {
// The pow contract, checked once per process (lshkm_ctx_create): 0 when the
// restatement matches this process's pow on the self-check's inputs.
int pow_contract_check() {
    static std::once_flag once;
    static int64_t bad = -1, tested = 0;
    std::call_once(once, [] {
        if (test_switch("LSHKM_POW_HOST", "rn")) g_libm_pow = pow_rn;
        if (lshkm_pow_selfcheck(&bad, &tested) != 0) bad = -1;
    });
    if (bad == 0) return 0;
    set_error("this process's pow(x, 2) differs from the device restatement of glibc 2.35's __pow_fma on " +
              std::to_string(bad) + " of " + std::to_string(tested) +
              " self-check inputs (lshkm_pow_selfcheck): the reference's distances and similarities on this host "
              "cannot be reproduced bit for bit (csrc/gpow2.h)");
    return LSHKM_ERR_UNSUPPORTED;
}
}  // namespace lshkm

extern "C" {

int lshkm_pow2(lshkm_ctx ctx, const double* x_dev, int64_t n, double* out_dev) {
    LSHKM_CHECK(ctx && n >= 0 && (n == 0 || (x_dev && out_dev)), LSHKM_ERR_ARG, "bad arguments");
    if (n == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(pow2_kernel, dim3(grid), dim3(256), 0, ctx->stream, x_dev, n, out_dev);
    LSHKM_LAUNCH_CHECK();
    return 0;
}

int lshkm_pow_selfcheck(int64_t* mismatches_host, int64_t* tested_host) {
    LSHKM_CHECK(mismatches_host, LSHKM_ERR_ARG, "bad arguments");
    // 4096 squares within 2^-8 ulp of a rounding midpoint (about a fifth of
    // them differ from x*x under glibc), 1024 exact ties (27-bit mantissas),
    // and the special ranges (subnormal / overflowing squares, |x| near 1).
    int64_t bad = 0, tested = 0, near = 0;
    for (uint64_t j = 0; near < 4096; j++) {
        const uint64_t a = sc_mix(2 * j + 1), b = sc_mix(2 * j + 2);
        const double x = std::ldexp(gp_dbl(0x3ff0000000000000ull | (a >> 12)), (int)(b % 160) - 80);
        const double p = x * x, e = std::fma(x, x, -p);
        const double u = gp_dbl(gp_bits(p) & 0x7ff0000000000000ull) * 0x1p-52;
        if (!(std::fabs(std::fabs(e) - 0.5 * u) <= 0x1p-8 * u)) continue;
        near++;
        tested++;
        const double r = g_libm_pow(x, 2.0);
        bad += gp_bits(gp_sq(x)) != gp_bits(r) || gp_bits(gp_pow2_emul(x)) != gp_bits(r);
    }
    static const double base[] = {0x1p-537, 0x1p-520, 0x1p-511, 0x1p-369, 0x1p369, 0x1p511, 0x1p512,
                                  0x1p-40,  0x1p40,   1.0,      0x1p-1022, 0x1p-1074, 0x1p1023, -1.5};
    for (uint64_t j = 0; j < 2048; j++) {
        const uint64_t a = sc_mix(0x5eed0000 + j), b = sc_mix(0x5eed8000 + j);
        double x;
        if (j < 1024) {
            const uint64_t m = (a & ((1ull << 26) - 1)) << 26;
            x = std::ldexp(gp_dbl(0x3ff0000000000000ull | m), (int)(b % 200) - 100);
        } else {
            x = base[b % (sizeof base / sizeof base[0])] *
                (1.0 + std::ldexp((double)(int64_t)(a >> 11) - 0x1p52, -60 + (int)((b >> 8) % 58)));
        }
        tested++;
        const double r = g_libm_pow(x, 2.0);
        bad += gp_bits(gp_sq(x)) != gp_bits(r) || gp_bits(gp_pow2_emul(x)) != gp_bits(r);
    }
    *mismatches_host = bad;
    if (tested_host) *tested_host = tested;
    return 0;
}

}  // extern "C"
