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
    // one atomic pair per block (contended single-word atomics serialise)
    __shared__ int32_t wlo[4], whi[4];
    if ((threadIdx.x & 63) == 0) { wlo[threadIdx.x >> 6] = lo; whi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) { lo = min(lo, wlo[w]); hi = max(hi, whi[w]); }
        atomicMin(mm, lo);
        atomicMax(mm + 1, hi);
    }
}

int launch_h_minmax(hipStream_t s, const int32_t* h, int64_t n, int32_t* mm_dev) {
    hipLaunchKernelGGL(h_minmax_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, s, h, n, mm_dev);
    return kstatus("cube.hip");
}

template <typename T>
__global__ void coin_first_kernel(const T* __restrict__ h, int64_t N, int k, int32_t hmin, int32_t hspan,
                                  const int32_t* __restrict__ memo, int32_t* __restrict__ first_row) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N * k; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = e / k;
        const int f = (int)(e - row * k);
        const int64_t off = (int64_t)f * hspan + ((int32_t)h[e] - hmin);
        // read first: most (f, h) have an earlier row already (the atomics on the
        // few popular entries otherwise serialise)
        if (memo[off] < 0 && first_row[off] > (int32_t)row) atomicMin(first_row + off, (int32_t)row);
    }
}

// Windows of at most CF_LDS_MAX entries: each block takes a contiguous run of
// rows and keeps its first rows per (f, h) in LDS (entries that already have a
// coin are marked), then merges them into first_row with one atomicMin per
// touched entry, skipped where first_row already holds an earlier row. A fresh
// 10M-row C4 cube: 34 ms -> well under 1 ms (every (row, f) hit one of ~400 hot
// global entries).
constexpr int CF_LDS_MAX = 12288;
constexpr int32_t CF_SEEN = -1;
constexpr int CF_KMAX = 32;          // functions per row held in registers (k <= 32)

// A wave's 64 consecutive rows of h are contiguous and 16-B aligned (chunks
// start at multiples of 64 rows): cf_fetch issues their coalesced 16-byte
// loads, cf_stash puts them in the wave's LDS buffer and reads this lane's row
// back (lane-per-row global loads touch ~k lines per instruction). The last chunk may read up to
// 15 B past the rows (WS_H keeps that slack).
// PF: 16-B pieces per lane, ceil(k * sizeof(T) / 16) (1, 2, 4 or 8). The
// loads are unconditional (clamped to the chunk's last piece) so the pieces
// stay in registers.
// (named registers, not an array: a loop-carried int4 array goes to scratch)
struct CfPre {
    int4 p0, p1, p2, p3, p4, p5, p6, p7;
};
template <typename T, int PF>
__device__ inline CfPre cf_fetch(const T* __restrict__ h, int64_t row0, int nrows, int k, int lane) {
    CfPre pre;
    const int q = (nrows * k * (int)sizeof(T) + 15) >> 4;
    const int4* src = reinterpret_cast<const int4*>(h + row0 * k);
    pre.p0 = src[min(lane, q - 1)];
    if constexpr (PF > 1) pre.p1 = src[min(lane + 64, q - 1)];
    if constexpr (PF > 2) { pre.p2 = src[min(lane + 128, q - 1)]; pre.p3 = src[min(lane + 192, q - 1)]; }
    if constexpr (PF > 4) {
        pre.p4 = src[min(lane + 256, q - 1)]; pre.p5 = src[min(lane + 320, q - 1)];
        pre.p6 = src[min(lane + 384, q - 1)]; pre.p7 = src[min(lane + 448, q - 1)];
    }
    return pre;
}
template <typename T, int PF>
__device__ inline void cf_stash(const CfPre pre, int nrows, int k, int32_t* __restrict__ buf, int lane,
                                int32_t (&v)[CF_KMAX]) {
    const int q = (nrows * k * (int)sizeof(T) + 15) >> 4;
    int4* b4 = reinterpret_cast<int4*>(buf);
    if (lane < q) b4[lane] = pre.p0;
    if constexpr (PF > 1) { if (lane + 64 < q) b4[lane + 64] = pre.p1; }
    if constexpr (PF > 2) {
        if (lane + 128 < q) b4[lane + 128] = pre.p2;
        if (lane + 192 < q) b4[lane + 192] = pre.p3;
    }
    if constexpr (PF > 4) {
        if (lane + 256 < q) b4[lane + 256] = pre.p4;
        if (lane + 320 < q) b4[lane + 320] = pre.p5;
        if (lane + 384 < q) b4[lane + 384] = pre.p6;
        if (lane + 448 < q) b4[lane + 448] = pre.p7;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    {   // lanes past nrows read stale buffer words (never used)
        if (sizeof(T) == 2 && (k & 1)) {
            const int16_t* p = reinterpret_cast<const int16_t*>(buf) + lane * k;
#pragma unroll
            for (int f = 0; f < CF_KMAX; f++)
                if (f < k) v[f] = p[f];
        } else if (sizeof(T) == 2) {
            const int32_t* p = buf + lane * (k >> 1);
#pragma unroll
            for (int f = 0; f < CF_KMAX; f += 2)
                if (f < k) {
                    const int32_t w = p[f >> 1];
                    v[f] = (int32_t)(int16_t)(w & 0xFFFF);
                    v[f + 1] = w >> 16;
                }
        } else {
            const int32_t* p = buf + lane * k;
#pragma unroll
            for (int f = 0; f < CF_KMAX; f++)
                if (f < k) v[f] = p[f];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// One row per lane (a wave takes 64 consecutive rows, staged through LDS),
// then a read-first LDS min per (f, h).
template <typename T, int PF>
__global__ __launch_bounds__(256) void coin_first_lds_kernel(const T* __restrict__ h, int64_t N, int k,
                                                             int32_t hmin, int32_t hspan, int64_t rows_per_block,
                                                             const int32_t* __restrict__ memo,
                                                             int32_t* __restrict__ first_row) {
    extern __shared__ int32_t lmin[];
    const int total = k * hspan;
    for (int e = threadIdx.x; e < total; e += 256) lmin[e] = memo[e] < 0 ? NO_ROW : CF_SEEN;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(N, r0 + rows_per_block);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // chunk starts are 64-row aligned (rows_per_block is a multiple of 64)
    int32_t* stage = lmin + ((total + 3) & ~3) + wave * (64 * k * (int)sizeof(T) / 4);
    for (int64_t c0 = r0 + 64 * wave; c0 < r1; c0 += 256) {
        const int64_t row = c0 + lane;
        const int nrows = (int)min((int64_t)64, r1 - c0);
        int32_t v[CF_KMAX];
        cf_stash<T, PF>(cf_fetch<T, PF>(h, c0, nrows, k, lane), nrows, k, stage, lane, v);
        if (row >= r1) continue;
#pragma unroll
        for (int f = 0; f < CF_KMAX; f++) {
            if (f >= k) break;
            const int off = f * hspan + (v[f] - hmin);
            const int32_t cur = lmin[off];
            if (cur != CF_SEEN && cur > (int32_t)row) atomicMin(lmin + off, (int32_t)row);
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < total; e += 256) {
        const int32_t v = lmin[e];
        if (v != CF_SEEN && v != NO_ROW && v < first_row[e]) atomicMin(first_row + e, v);
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

// minstd_rand0: st = st * 16807 mod (2^31 - 1), reduced with 2^31 = 1 (mod M)
// instead of a 64-bit division.
__device__ inline uint32_t minstd_next(uint32_t& st) {
    const uint64_t x = (uint64_t)st * 16807ull;          // < 2^46
    uint32_t r = (uint32_t)(x & 0x7FFFFFFFull) + (uint32_t)(x >> 31);
    if (r >= 2147483647u) r -= 2147483647u;
    st = r;
    return st;
}

// uniform_int_distribution<int>(1, 2) over minstd_rand0 (libstdc++-11 downscaling):
// ret / scaling is 0 or 1 for ret < past.
__device__ inline int coin_1_2(uint32_t& st) {
    constexpr uint32_t scaling = 2147483645u / 2u, past = 2u * scaling;
    uint32_t ret;
    do { ret = minstd_next(st) - 1u; } while (ret >= past);
    return ret >= scaling ? 2 : 1;
}

__device__ inline uint32_t minstd_mulmod(uint32_t a, uint32_t b) {
    const uint64_t x = (uint64_t)a * (uint64_t)b;        // < 2^62
    uint64_t r = (x & 0x7FFFFFFFull) + (x >> 31);         // < 2^32, = x (mod 2^31 - 1)
    r = (r & 0x7FFFFFFFull) + (r >> 31);
    if (r >= 2147483647ull) r -= 2147483647ull;
    return (uint32_t)r;
}

// The coins in draw order. The engine is an LCG, so draw i + 1 of a chunk is
// state * 16807^(i+1) mod M: 64 lanes take 64 consecutive draws at once. A
// draw that the uniform_int downscaling rejects (ret >= past: probability
// 2^-30) would shift every later coin by one engine step; a chunk that holds
// one is drawn again by one lane, in order.
__global__ void coin_draw_kernel(const int32_t* __restrict__ sorted_vals, const unsigned int* __restrict__ count,
                                 int32_t hmin, int32_t hspan, int32_t* __restrict__ memo, uint32_t* __restrict__ state) {
    if (blockIdx.x != 0) return;
    const int lane = threadIdx.x;                       // one wave
    constexpr uint32_t scaling = 2147483645u / 2u, past = 2u * scaling;
    uint32_t pw = 1, b = 16807u;                        // 16807^(lane+1)
    for (uint32_t e = (uint32_t)lane + 1u; e; e >>= 1) {
        if (e & 1u) pw = minstd_mulmod(pw, b);
        b = minstd_mulmod(b, b);
    }
    uint32_t st = *state;
    const unsigned int n = *count;
    for (unsigned int c0 = 0; c0 < n; c0 += 64) {
        const unsigned int m = min(64u, n - c0);
        const bool on = (unsigned int)lane < m;
        const uint32_t u = minstd_mulmod(st, pw);
        const bool rej = on && u - 1u >= past;
        if (__ballot(rej)) {                             // rare: this chunk one coin at a time
            if (lane == 0) {
                for (unsigned int i = c0; i < n; i++) {
                    const int32_t off = sorted_vals[i];
                    const int32_t hv = hmin + (off % hspan);
                    const int c = coin_1_2(st);
                    memo[off] = (hv % c + c) % c;
                }
            }
            st = __shfl(st, 0);
            break;
        }
        if (on) {
            const int c = u - 1u >= scaling ? 2 : 1;
            const int32_t off = sorted_vals[c0 + lane];
            const int32_t hv = hmin + (off % hspan);
            memo[off] = (hv % c + c) % c;              // mod(hash_num, c) (utils.hpp:97-98)
        }
        st = __shfl(u, (int)m - 1);
    }
    if (lane == 0) *state = st;
}

template <typename T>
__global__ void coin_vertex_kernel(const T* __restrict__ h, int64_t N, int k, int32_t hmin, int32_t hspan,
                                   const int32_t* __restrict__ memo, int32_t* __restrict__ vertex) {
    for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < N; row += (int64_t)gridDim.x * blockDim.x) {
        int v = 0;
        for (int f = 0; f < k; f++) v = (v << 1) + memo[(size_t)f * hspan + ((int32_t)h[row * k + f] - hmin)];
        vertex[row] = v;
    }
}

// Memo windows of at most CF_LDS_MAX entries: the memo in LDS, one row per
// lane from the staged rows.
template <typename T, int PF>
__global__ __launch_bounds__(256) void coin_vertex_lds_kernel(const T* __restrict__ h, int64_t N, int k,
                                                              int32_t hmin, int32_t hspan,
                                                              const int32_t* __restrict__ memo,
                                                              int32_t* __restrict__ vertex) {
    extern __shared__ int32_t lmemo[];          // [k * hspan], then the per-wave row stages
    const int total = k * hspan;
    for (int e = threadIdx.x; e < total; e += 256) lmemo[e] = memo[e];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int32_t* stage = lmemo + ((total + 3) & ~3) + wave * (64 * k * (int)sizeof(T) / 4);
    for (int64_t c0 = (int64_t)blockIdx.x * 256 + 64 * wave; c0 < N; c0 += (int64_t)gridDim.x * 256) {
        const int64_t row = c0 + lane;
        const int nrows = (int)min((int64_t)64, N - c0);
        int32_t v[CF_KMAX];
        cf_stash<T, PF>(cf_fetch<T, PF>(h, c0, nrows, k, lane), nrows, k, stage, lane, v);
        if (row >= N) continue;
        int x = 0;
#pragma unroll
        for (int f = 0; f < CF_KMAX; f++) {
            if (f >= k) break;
            x = (x << 1) + lmemo[f * hspan + (v[f] - hmin)];
        }
        vertex[row] = x;
    }
}

template <typename T>
static int launch_coin_first_t(hipStream_t s, const T* h, int64_t N, int k, int32_t hmin, int32_t hspan,
                               const int32_t* memo, int32_t* first_row) {
    const int64_t n = N * k;
    const int64_t total = (int64_t)k * hspan;
    if (total <= CF_LDS_MAX && k <= CF_KMAX) {
        static int cus[64] = {0};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return kstatus("hipGetDevice");
        if (dev < 64 && !cus[dev] &&
            hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return kstatus("hipDeviceGetAttribute");
        const int64_t ncu = dev < 64 && cus[dev] > 0 ? cus[dev] : 256;
        // >= 2048 rows per block so the LDS table's setup and merge stay small
        const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>(4 * ncu, (N + 2047) / 2048));
        const int64_t rpb = ((N + nblk - 1) / nblk + 63) & ~(int64_t)63;
        const size_t lds = (size_t)((total + 3) & ~3) * 4 + 4 * 64 * (size_t)k * sizeof(T);
        const int pf = (k * (int)sizeof(T) + 15) / 16;
#define CF_FIRST(P) hipLaunchKernelGGL((coin_first_lds_kernel<T, P>), dim3((unsigned)nblk), dim3(256), lds, s, h, N, k, hmin, hspan, rpb, memo, first_row)
        if (pf <= 1) CF_FIRST(1); else if (pf <= 2) CF_FIRST(2); else if (pf <= 4) CF_FIRST(4); else CF_FIRST(8);
#undef CF_FIRST
        return kstatus("cube.hip");
    }
    hipLaunchKernelGGL(coin_first_kernel<T>, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, s, h,
                       N, k, hmin, hspan, memo, first_row);
    return kstatus("cube.hip");
}

int launch_coin_first(hipStream_t s, const void* h, bool h16, int64_t N, int k, int32_t hmin, int32_t hspan,
                      const int32_t* memo, int32_t* first_row) {
    return h16 ? launch_coin_first_t(s, static_cast<const int16_t*>(h), N, k, hmin, hspan, memo, first_row)
               : launch_coin_first_t(s, static_cast<const int32_t*>(h), N, k, hmin, hspan, memo, first_row);
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

template <typename T>
static int launch_coin_vertex_t(hipStream_t s, const T* h, int64_t N, int k, int32_t hmin, int32_t hspan,
                                const int32_t* memo, int32_t* vertex) {
    if ((int64_t)k * hspan <= CF_LDS_MAX && k <= CF_KMAX) {
        const size_t lds = (size_t)((k * hspan + 3) & ~3) * 4 + 4 * 64 * (size_t)k * sizeof(T);
        const int pf = (k * (int)sizeof(T) + 15) / 16;
        const dim3 grid((unsigned)std::min<int64_t>((N + 255) / 256, 2048));
#define CF_VTX(P) hipLaunchKernelGGL((coin_vertex_lds_kernel<T, P>), grid, dim3(256), lds, s, h, N, k, hmin, hspan, memo, vertex)
        if (pf <= 1) CF_VTX(1); else if (pf <= 2) CF_VTX(2); else if (pf <= 4) CF_VTX(4); else CF_VTX(8);
#undef CF_VTX
        return kstatus("cube.hip");
    }
    hipLaunchKernelGGL(coin_vertex_kernel<T>, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 8192)), dim3(256), 0, s, h,
                       N, k, hmin, hspan, memo, vertex);
    return kstatus("cube.hip");
}

int launch_coin_vertex(hipStream_t s, const void* h, bool h16, int64_t N, int k, int32_t hmin, int32_t hspan,
                       const int32_t* memo, int32_t* vertex) {
    return h16 ? launch_coin_vertex_t(s, static_cast<const int16_t*>(h), N, k, hmin, hspan, memo, vertex)
               : launch_coin_vertex_t(s, static_cast<const int32_t*>(h), N, k, hmin, hspan, memo, vertex);
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
