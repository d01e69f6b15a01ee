// Load-pattern microbench: 32-row MFMA-operand pattern vs coalesced, 10M x 128 fp32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int D = 128;
template <int PAT, int W>
__global__ __launch_bounds__(64 * W) void k(const float* X, int64_t N, float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31, h = lane >> 5;
    const int64_t ntiles = N / 32;
    float acc = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * W + wave; t < ntiles; t += (int64_t)gridDim.x * W) {
        float4 v[16];
        if (PAT == 0) {
            const float* xr = X + (t * 32 + col) * D + 8 * h;
#pragma unroll
            for (int s = 0; s < 8; s++) {
                v[2 * s] = *reinterpret_cast<const float4*>(xr + 16 * s);
                v[2 * s + 1] = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
            }
        } else {
            const float* xt = X + t * 32 * D;
#pragma unroll
            for (int i = 0; i < 16; i++) v[i] = *reinterpret_cast<const float4*>(xt + i * 256 + lane * 4);
        }
#pragma unroll
        for (int i = 0; i < 16; i++) acc += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    out[(int64_t)blockIdx.x * 64 * W + threadIdx.x] = acc;
}
template <int PAT, int W>
float run(const float* X, int64_t N, float* out, int bpc) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int nb = 256 * bpc;
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((k<PAT, W>), dim3(nb), dim3(64 * W), 0, 0, X, N, out);
    hipEventRecord(a);
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL((k<PAT, W>), dim3(nb), dim3(64 * W), 0, 0, X, N, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}
int main() {
    const int64_t N = 10000000;
    float *X, *out;
    hipMalloc(&X, N * D * 4);
    hipMalloc(&out, 256 * 16 * 256 * 4);
    hipMemset(X, 0, N * D * 4);
    const double gb = N * D * 4 / 1e9;
    for (int bpc : {2, 4, 8}) {
        float t0 = run<0, 4>(X, N, out, bpc), t1 = run<1, 4>(X, N, out, bpc);
        printf("W=4 bpc=%d  mfma-pattern %.3f ms (%.2f TB/s)   coalesced %.3f ms (%.2f TB/s)\n", bpc, t0, gb / t0, t1, gb / t1);
    }
    return 0;
}
