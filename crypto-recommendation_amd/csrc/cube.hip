// cube.hip — randomized hypercube vertices with the lazy Euclidean-F coins.
//
// Replaces EuclideanFGen::generate (lib/generators/euclidean_f_gen.hpp:65-79)
// under HypercubeGen::generate (lib/generators/hypercube_gen.hpp:63-73):
// f_i(p) = memo_i[h_i(p)], where the first time a given h is seen for f_i a
// coin c ~ uniform_int_distribution<int>(1,2) is drawn from the ONE engine all
// f_i share (lsh_cube.hpp:112-126) and memo_i[h] = mod(h, c). Draw order is the
// global first-occurrence order over (row, f) — rows in insertion order, f_0
// first within a row — and queries continue the same stream.
// GPU form: every (row, f) does atomicMin(first_row[f][h]) on a dense memo
// window; the unseen (f, h) with a first row are collected, sorted by
// first_row * k + f (the stable radix sort), and a single lane draws the coins
// in that order with the restated minstd_rand0 / uniform_int (the only
// sequential step; a few hundred draws). Vertices are then a memo lookup.
#include "common.h"
#include "kernels.h"

namespace lshkm {

constexpr int32_t NO_ROW = 0x7F7F7F7F;   // the byte-memset fill of first_row

__global__ void h_minmax_kernel(const int32_t* __restrict__ h, int64_t n, int32_t* __restrict__ mm) {
    int32_t lo = 0x7FFFFFFF, hi = (int32_t)0x80000000;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = h[i];
        lo = min(lo, v);
        hi = max(hi, v);
    }
    for (int off = 32; off >= 1; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off));
        hi = max(hi, __shfl_xor(hi, off));
    }
    if ((threadIdx.x & 63) == 0) { atomicMin(mm, lo); atomicMax(mm + 1, hi); }
}

int launch_h_minmax(hipStream_t s, const int32_t* h, int64_t n, int32_t* mm_dev) {
    hipLaunchKernelGGL(h_minmax_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, s, h, n, mm_dev);
    return kstatus("cube.hip");
}

__global__ void coin_first_kernel(const int32_t* __restrict__ h, int64_t N, int k, int32_t hmin, int32_t hspan,
                                  const int32_t* __restrict__ memo, int32_t* __restrict__ first_row) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N * k; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = e / k;
        const int f = (int)(e - row * k);
        const int64_t off = (int64_t)f * hspan + (h[e] - hmin);
        if (memo[off] < 0) atomicMin(first_row + off, (int32_t)row);
    }
}

// Collect unseen (f, h) with a first row: key = first_row * k + f, val = flat memo offset.
__global__ void coin_collect_kernel(int32_t* __restrict__ first_row, int64_t total, int k, int32_t hspan,
                                    int32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                    unsigned int* __restrict__ count) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = first_row[e];
        if (r == NO_ROW) continue;
        const int f = (int)(e / hspan);
        const unsigned int slot = atomicAdd(count, 1u);
        keys[slot] = r * k + f;
        vals[slot] = (int32_t)e;
        first_row[e] = NO_ROW;
    }
}

__device__ inline uint32_t minstd_next(uint32_t& st) {
    st = (uint32_t)(((uint64_t)st * 16807ull) % 2147483647ull);
    return st;
}

// uniform_int_distribution<int>(1, 2) over minstd_rand0 (libstdc++-11 downscaling).
__device__ inline int coin_1_2(uint32_t& st) {
    const uint64_t scaling = 2147483645ull / 2ull, past = 2ull * scaling;
    uint64_t ret;
    do { ret = (uint64_t)minstd_next(st) - 1ull; } while (ret >= past);
    return (int)(ret / scaling) + 1;
}

__global__ void coin_draw_kernel(const int32_t* __restrict__ sorted_vals, const unsigned int* __restrict__ count,
                                 int32_t hmin, int32_t hspan, int32_t* __restrict__ memo, uint32_t* __restrict__ state) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t st = *state;
    const unsigned int n = *count;
    for (unsigned int i = 0; i < n; i++) {
        const int32_t off = sorted_vals[i];
        const int32_t hv = hmin + (off % hspan);
        const int c = coin_1_2(st);
        memo[off] = (hv % c + c) % c;          // mod(hash_num, c) (utils.hpp:97-98)
    }
    *state = st;
}

__global__ void coin_vertex_kernel(const int32_t* __restrict__ h, int64_t N, int k, int32_t hmin, int32_t hspan,
                                   const int32_t* __restrict__ memo, int32_t* __restrict__ vertex) {
    for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < N; row += (int64_t)gridDim.x * blockDim.x) {
        int v = 0;
        for (int f = 0; f < k; f++) v = (v << 1) + memo[(size_t)f * hspan + (h[row * k + f] - hmin)];
        vertex[row] = v;
    }
}

int launch_coin_first(hipStream_t s, const int32_t* h, int64_t N, int k, int32_t hmin, int32_t hspan,
                      const int32_t* memo, int32_t* first_row) {
    const int64_t n = N * k;
    hipLaunchKernelGGL(coin_first_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, s, h, N,
                       k, hmin, hspan, memo, first_row);
    return kstatus("cube.hip");
}

int launch_coin_collect(hipStream_t s, int32_t* first_row, int64_t total, int k, int32_t hspan, int32_t* keys,
                        int32_t* vals, unsigned int* count) {
    hipLaunchKernelGGL(coin_collect_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0, s,
                       first_row, total, k, hspan, keys, vals, count);
    return kstatus("cube.hip");
}

int launch_coin_draw(hipStream_t s, const int32_t* sorted_vals, const unsigned int* count, int32_t hmin, int32_t hspan,
                     int32_t* memo, uint32_t* state) {
    hipLaunchKernelGGL(coin_draw_kernel, dim3(1), dim3(64), 0, s, sorted_vals, count, hmin, hspan, memo, state);
    return kstatus("cube.hip");
}

int launch_coin_vertex(hipStream_t s, const int32_t* h, int64_t N, int k, int32_t hmin, int32_t hspan,
                       const int32_t* memo, int32_t* vertex) {
    hipLaunchKernelGGL(coin_vertex_kernel, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 8192)), dim3(256), 0, s, h, N,
                       k, hmin, hspan, memo, vertex);
    return kstatus("cube.hip");
}

// Imported coins (sharded builds): memo[off[i]] = bit[i].
__global__ void memo_scatter_kernel(const int32_t* __restrict__ off, const int32_t* __restrict__ bit, int64_t n,
                                    int32_t* __restrict__ memo) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        memo[off[i]] = bit[i];
}

int launch_memo_scatter(hipStream_t s, const int32_t* off, const int32_t* bit, int64_t n, int32_t* memo) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(memo_scatter_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s,
                       off, bit, n, memo);
    return kstatus("cube.hip");
}

// Re-center a memo window: copy memo[f][h - old_min] into a wider window.
__global__ void memo_rehome_kernel(const int32_t* __restrict__ old_memo, int32_t old_min, int32_t old_span,
                                   int32_t* __restrict__ new_memo, int32_t new_min, int32_t new_span, int k) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)k * new_span;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int f = (int)(e / new_span);
        const int32_t hv = new_min + (int32_t)(e - (int64_t)f * new_span);
        const int64_t o = (int64_t)hv - old_min;
        new_memo[e] = (old_memo && o >= 0 && o < old_span) ? old_memo[(size_t)f * old_span + o] : -1;
    }
}

int launch_memo_rehome(hipStream_t s, const int32_t* old_memo, int32_t old_min, int32_t old_span, int32_t* new_memo,
                       int32_t new_min, int32_t new_span, int k) {
    const int64_t n = (int64_t)k * new_span;
    hipLaunchKernelGGL(memo_rehome_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0, s,
                       old_memo, old_min, old_span, new_memo, new_min, new_span, k);
    return kstatus("cube.hip");
}

}  // namespace lshkm
