// Cost of the pow(x, 2) forms in a lane chain: x*x, per-lane
// gp_sq, the wave-batched forms. hipcc -O3 -std=c++17 --offload-arch=gfx950
// -ffp-contract=off tools/sqbench.hip -o tools/sqbench; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../crypto-recommendation_amd/csrc/gpow2.h"

__device__ inline float hf(uint32_t h) {  // ~normal-ish float from a hash
    h ^= h >> 16; h *= 0x7feb352d; h ^= h >> 15; h *= 0x846ca68b; h ^= h >> 16;
    float u = (h & 0xffffff) * (1.0f / 16777216.0f);
    float v = ((h >> 8) & 0xffff) * (1.0f / 65536.0f);
    return (u - 0.5f) * 4.0f * v;
}

__device__ inline bool slow2(double x, double p) {
    const double e = fma(x, x, -p);
    const double r = __dadd_rn(p, __dmul_rn(e, 0x1.1111111111p+0));
    const uint32_t hx = (uint32_t)(gp_bits(x) >> 32) & 0x7fffffffu;
    const uint32_t hp = (uint32_t)(gp_bits(p) >> 32);
    const bool out = hx - 0x3D700000u >= 0x05000000u;
    const bool p2 = (hp & 0xFFFFFu) == 0u && e < 0.0;
    return (r != p || out || p2) && x != 0.0;
}

template <int NV, int TEST>
__device__ inline void sq_wave(const double (&x)[NV], double (&p)[NV], double* lds) {
    uint32_t need = 0;
    bool any = false;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        p[j] = __dmul_rn(x[j], x[j]);
        const bool s = TEST ? slow2(x[j], p[j]) : gp_sq_slow(x[j], p[j]);
        need |= (s ? 1u : 0u) << j;
    }
    if (__ballot(need != 0u) == 0ull) return;
    const int lane = (int)__lane_id();
    const int c = __popc(need);
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    const int total = __shfl(incl, 63);
    const int first = incl - c;
    for (int base = 0; base < total; base += 64) {
        int k = first;
#pragma unroll
        for (int j = 0; j < NV; j++)
            if ((need >> j) & 1u) {
                if (k >= base && k < base + 64) lds[k - base] = x[j];
                k++;
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < total - base) lds[lane] = gp_pow2_emul(lds[lane]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        k = first;
#pragma unroll
        for (int j = 0; j < NV; j++)
            if ((need >> j) & 1u) {
                if (k >= base && k < base + 64) p[j] = lds[k - base];
                k++;
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}


// ballot-prefix form: lds holds 64 * NV doubles
template <int NV>
__device__ inline void sq_wave2(const double (&x)[NV], double (&p)[NV], double* lds) {
    bool sl[NV];
    bool any = false;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        p[j] = __dmul_rn(x[j], x[j]);
        sl[j] = slow2(x[j], p[j]);
        any = any || sl[j];
    }
    if (__ballot(any) == 0ull) return;
    int pos[NV];
    int total = 0;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        const unsigned long long m = __ballot(sl[j]);
        pos[j] = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        total += __popcll(m);
        if (sl[j]) lds[pos[j]] = x[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int lane = (int)__lane_id();
    for (int b = 0; b < total; b += 64)
        if (b + lane < total) lds[b + lane] = gp_pow2_emul(lds[b + lane]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < NV; j++)
        if (sl[j]) p[j] = lds[pos[j]];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int V>
__global__ __launch_bounds__(256) void kern(int d, double* out, unsigned long long* nslow) {
    __shared__ double sqs[4 * 64 * 16];
    double* sq = sqs + (threadIdx.x >> 6) * 64 * 16;
    const uint32_t row = blockIdx.x * 256 + threadIdx.x;
    double acc = 0.0;
    unsigned ns = 0;
    for (int j0 = 0; j0 < d; j0 += 16) {
        double x[16], p[16];
#pragma unroll
        for (int t = 0; t < 16; t++) x[t] = (double)hf(row * 977u + j0 + t) - (double)hf(j0 + t + 0x9e3779b9u);
        if (V == 0) { for (int t = 0; t < 16; t++) p[t] = __dmul_rn(x[t], x[t]); }
        if (V == 1) { for (int t = 0; t < 16; t++) p[t] = gp_sq(x[t]); }
        if (V == 2) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                double xx[8], pp[8];
                for (int t = 0; t < 8; t++) xx[t] = x[8 * h + t];
                sq_wave<8, 0>(xx, pp, sq);
                for (int t = 0; t < 8; t++) p[8 * h + t] = pp[t];
            }
        }
        if (V == 3) { for (int t = 0; t < 16; t++) { const double q = __dmul_rn(x[t], x[t]); p[t] = slow2(x[t], q) ? gp_pow2_emul(x[t]) : q; } }
        if (V == 4) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                double xx[8], pp[8];
                for (int t = 0; t < 8; t++) xx[t] = x[8 * h + t];
                sq_wave<8, 1>(xx, pp, sq);
                for (int t = 0; t < 8; t++) p[8 * h + t] = pp[t];
            }
        }
        if (V == 5) sq_wave<16, 1>(x, p, sq);
        if (V == 8) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                double xx[8], pp[8];
                for (int t = 0; t < 8; t++) xx[t] = x[8 * h + t];
                sq_wave2<8>(xx, pp, sq);
                for (int t = 0; t < 8; t++) p[8 * h + t] = pp[t];
            }
        }
        if (V == 9) sq_wave2<16>(x, p, sq);
        if (V == 6) { for (int t = 0; t < 16; t++) ns += slow2(x[t], __dmul_rn(x[t], x[t])); }
        if (V == 7) { for (int t = 0; t < 16; t++) ns += gp_sq_slow(x[t], __dmul_rn(x[t], x[t])); }
#pragma unroll
        for (int t = 0; t < 16; t++) acc = __dadd_rn(acc, p[t]);
    }
    out[row] = acc;
    if (V >= 6) atomicAdd(nslow, (unsigned long long)ns);
}

int main() {
    const int nrow = 1 << 20, d = 128;
    double* out; unsigned long long* ns;
    hipMalloc(&out, (size_t)nrow * 8 * 10); hipMalloc(&ns, 16); hipMemset(ns, 0, 16);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    std::vector<double> h[10];
    auto run = [&](int v, auto k) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(nrow / 256), dim3(256), 0, 0, d, out + (size_t)v * nrow, ns);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("V%d %.3f ms\n", v, ms);
        }
        h[v].resize(nrow);
        hipMemcpy(h[v].data(), out + (size_t)v * nrow, nrow * 8, hipMemcpyDeviceToHost);
    };
    run(0, kern<0>); run(1, kern<1>); run(2, kern<2>); run(3, kern<3>); run(4, kern<4>); run(5, kern<5>); run(8, kern<8>); run(9, kern<9>);
    unsigned long long c[2];
    hipMemset(ns, 0, 16); hipLaunchKernelGGL(kern<6>, dim3(nrow / 256), dim3(256), 0, 0, d, out, ns); hipMemcpy(&c[0], ns, 8, hipMemcpyDeviceToHost);
    hipMemset(ns, 0, 16); hipLaunchKernelGGL(kern<7>, dim3(nrow / 256), dim3(256), 0, 0, d, out, ns); hipMemcpy(&c[1], ns, 8, hipMemcpyDeviceToHost);
    printf("slow frac new %.4f old %.4f\n", c[0] / (double)nrow / d, c[1] / (double)nrow / d);
    for (int v = 2; v <= 9; v++) {
        if (v == 6 || v == 7) continue;
        size_t bad = 0;
        for (int i = 0; i < nrow; i++) bad += memcmp(&h[v][i], &h[1][i], 8) != 0;
        printf("V%d vs V1 mismatches %zu\n", v, bad);
    }
    size_t d0 = 0;
    for (int i = 0; i < nrow; i++) d0 += memcmp(&h[0][i], &h[1][i], 8) != 0;
    printf("V0 (x*x) vs V1 rows differing %zu\n", d0);
    return 0;
}
