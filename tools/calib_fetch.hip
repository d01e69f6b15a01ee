// FETCH_SIZE calibration for the fused kernel's access pattern (profiling aid).
// Reads a 5.12 GB fp32 matrix [10M][128] once in two shapes and writes one
// float per wave, so FETCH_SIZE / bytes read gives the counter's scale factor:
//   coalesced: each wave reads 1 KiB contiguous per instruction (float4/lane)
//   fused:     lane (col, h) reads 2 x 16 B of row col at dims 16s + 8h (s < 8)
// build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr long N = 10000000, D = 128;

__global__ void coalesced(const float4* __restrict__ X, float* out, long n4) {
    float acc = 0.f;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
        const float4 v = X[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[0] = acc;   // never true for the zero-filled input; keeps the loads
}

__global__ void fused_shape(const float* __restrict__ X, float* out, long ntiles) {
    const int lane = threadIdx.x & 63, col = lane & 31, h = lane >> 5;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    float acc = 0.f;
    for (long t = wave; t < ntiles; t += nw) {
        const float* xr = X + (t * 32 + col) * D + 8 * h;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const float4 p0 = *reinterpret_cast<const float4*>(xr + 16 * s);
            const float4 p1 = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
            acc += p0.x + p0.y + p0.z + p0.w + p1.x + p1.y + p1.z + p1.w;
        }
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    float* X = nullptr;
    float* out = nullptr;
    const size_t bytes = (size_t)N * D * 4;
    if (hipMalloc(&X, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(X, 0, bytes);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(coalesced, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const float4*>(X), out, N * D / 4);
        hipLaunchKernelGGL(fused_shape, dim3(4096), dim3(256), 0, 0, X, out, N / 32);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("read %.3f GB per kernel launch\n", bytes / 1e9);
    (void)hipFree(X);
    (void)hipFree(out);
    return 0;
}
