// scatter.hip — stable bucket scatter (CSR build) on gfx950.
//
// Replaces the per-insert std::vector::emplace_back of
//   CustHashtable::insertVector  lib/data_structures/cust_hashtable.hpp:65-70
//   VectorBucket::insertVector   lib/data_structures/vector_bucket.hpp:41-44
// whose observable contract is: bucket b holds the rows with bucket ID b in
// insertion (= row) order. Built here as a stable LSD radix sort of
// (bucket ID, row) pairs, then a boundary pass that writes the CSR row
// pointers (empty buckets included). Also used for the k-means member lists
// (cluster-sorted rows, update.hpp:52-56 order) and the F-coin draw order.
//
// Per pass (<= 8 digit bits): upsweep (block digit histograms in LDS) ->
// exclusive scan of the [digit][block] matrix -> downsweep, where each wave
// ranks a contiguous quarter of the block's 4096-key tile: per 64-key round the
// lanes sharing a digit are found with DB ballots (AND of matching bit masks),
// rank = the wave's running count of that digit + popc(peers & lanemask_lt);
// the block then offsets each wave by the earlier waves' totals: a stable rank
// without sorting inside the tile.
// HBM per pass: 4 B key read (upsweep) + 8 B read + 8 B written (downsweep).
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace lshkm {

constexpr int RS_THREADS = 256;
constexpr int RS_TILE = 4096;

// Batched over T tables by blockIdx.y: table t's keys start at keys + t * k_ts,
// its histogram at hist + t * h_ts (likewise for every kernel below).
__global__ __launch_bounds__(RS_THREADS) void rs_upsweep(const int32_t* __restrict__ keys, int64_t kstride, int64_t N,
                                                        int shift, int nbins, int nblocks, uint32_t* __restrict__ hist,
                                                        int64_t k_ts, int64_t h_ts) {
    __shared__ uint32_t h[256];
    keys += blockIdx.y * k_ts;
    hist += blockIdx.y * h_ts;
    for (int b = threadIdx.x; b < nbins; b += RS_THREADS) h[b] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * RS_TILE;
    for (int e = threadIdx.x; e < RS_TILE; e += RS_THREADS) {
        const int64_t i = base + e;
        if (i < N) atomicAdd(&h[(keys[i * kstride] >> shift) & (nbins - 1)], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += RS_THREADS) hist[(size_t)b * nblocks + blockIdx.x] = h[b];
}

// Exclusive scan of M uint32 in place, one block of 1024 threads. For M <=
// 32768 the array is read as rows of 1024 (thread t: column t, all its loads
// in flight, each instruction coalesced): every row is scanned per wave by
// shuffles, the (row, wave) totals get one block scan, and the results are
// written back the same way. (A thread-per-contiguous-segment form touches 64
// cache lines per load instruction on the handful of CUs a few-table scan
// uses: 27-44 us for the C2 build's 5 x 31K counters.)
constexpr int RS_SEG = 32;
__device__ inline uint32_t rs_block_exclusive(uint32_t s, uint32_t* wsum) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    if (t < 64) {
        const uint32_t x = t < 16 ? wsum[t] : 0u;
        uint32_t y = x;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const uint32_t u = __shfl_up(y, o);
            if (lane >= o) y += u;
        }
        if (t < 16) wsum[16 + t] = y - x;              // exclusive wave offsets
    }
    __syncthreads();
    const uint32_t r = wsum[16 + w] + inc - s;
    __syncthreads();                                   // wsum reusable on return
    return r;
}
__global__ __launch_bounds__(1024) void rs_scan(uint32_t* __restrict__ a, int64_t M, int64_t a_ts) {
    __shared__ uint32_t wsum[32];
    __shared__ uint32_t rw[RS_SEG * 16];               // (row, wave) offsets
    a += blockIdx.y * a_ts;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (M <= (int64_t)RS_SEG * 1024) {                 // block-uniform
        const int rows = (int)((M + 1023) >> 10);
        uint32_t v[RS_SEG];
#pragma unroll
        for (int j = 0; j < RS_SEG; j++) v[j] = j < rows && ((int64_t)j << 10) + t < M ? a[((int64_t)j << 10) + t] : 0u;
        // per row: wave-exclusive prefix in v[j], the wave's row total to rw
#pragma unroll
        for (int j = 0; j < RS_SEG; j++) {               // branch-free: v stays in registers
            uint32_t inc = v[j];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(inc, o);
                if (lane >= o) inc += u;
            }
            if (lane == 63 && j < rows) rw[j * 16 + w] = inc;
            v[j] = inc - v[j];
        }
        __syncthreads();
        const uint32_t tot = t < rows * 16 ? rw[t] : 0u;
        const uint32_t ex = rs_block_exclusive(tot, wsum);
        if (t < rows * 16) rw[t] = ex;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RS_SEG; j++) {
            const int64_t i = ((int64_t)j << 10) + t;
            if (j < rows && i < M) a[i] = rw[j * 16 + w] + v[j];
        }
        return;
    }
    const int64_t seg = (M + 1023) / 1024;
    const int64_t lo = t * seg, hi = min(M, lo + seg);
    uint32_t s = 0;
    for (int64_t i = lo; i < hi; i++) s += a[i];
    uint32_t run = rs_block_exclusive(s, wsum);
    for (int64_t i = lo; i < hi; i++) { const uint32_t x = a[i]; a[i] = run; run += x; }
}

// Large histograms (the cube's 2^7 bins x N / 4096 tiles: 312K counters at
// N = 10M, 0.35-0.54 ms in the one-block scan): reduce-then-scan over
// RS_SC-element chunks, in place; the chunk totals go through rs_scan.
constexpr int RS_SC = 8192;
// up to this many counters the one-block scan (32 coalesced rows of 1024)
// beats the reduce-then-scan trio's two extra launches (the C2 build: 7-bit
// digits x 245 tiles x 5 tables)
constexpr int64_t RS_ONE_SCAN = 32768;
__global__ __launch_bounds__(1024) void rs_chunk_sum(const uint32_t* __restrict__ a, int64_t M, uint32_t* __restrict__ part,
                                                     int64_t a_ts, int64_t p_ts) {
    __shared__ uint32_t red[1024];
    a += blockIdx.y * a_ts;
    part += blockIdx.y * p_ts;
    const int64_t base = (int64_t)blockIdx.x * RS_SC;
    uint32_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int64_t i = base + u * 1024 + threadIdx.x;          // coalesced
        s += i < M ? a[i] : 0u;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ __launch_bounds__(1024) void rs_chunk_scan(uint32_t* __restrict__ a, int64_t M, const uint32_t* __restrict__ off,
                                                      int64_t a_ts, int64_t p_ts) {
    __shared__ uint32_t wsum[32];
    a += blockIdx.y * a_ts;
    off += blockIdx.y * p_ts;
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * RS_SC + t * 8;      // 8 consecutive per thread
    uint32_t v[8], s = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) { v[u] = base + u < M ? a[base + u] : 0u; s += v[u]; }
    uint32_t run = off[blockIdx.x] + rs_block_exclusive(s, wsum);
#pragma unroll
    for (int u = 0; u < 8; u++)
        if (base + u < M) { a[base + u] = run; run += v[u]; }
}

// Each wave ranks its own contiguous quarter of the tile (16 rounds of 64
// keys, the keys and their ranks kept in registers) against per-wave running
// digit counts in LDS; one barrier, the block turns the per-wave totals into
// per-wave digit offsets (global start + earlier waves), a second barrier, and
// every key is written. Two barriers per 4096-key tile (the round-per-256-keys
// form needed three per round).
constexpr int RS_R = RS_TILE / RS_THREADS;           // keys per lane
__global__ __launch_bounds__(RS_THREADS) void rs_downsweep(
    const int32_t* __restrict__ keys, int64_t kstride, const int32_t* __restrict__ vals, int64_t N, int shift,
    int dbits, int nblocks, const uint32_t* __restrict__ scanned, int32_t* __restrict__ keys_out,
    int32_t* __restrict__ vals_out, int64_t k_ts, int64_t v_ts, int64_t h_ts, int64_t o_ts) {
    __shared__ uint32_t wcnt[RS_THREADS / 64][256];
    keys += blockIdx.y * k_ts;
    if (vals) vals += blockIdx.y * v_ts;
    scanned += blockIdx.y * h_ts;
    keys_out += blockIdx.y * o_ts;
    vals_out += blockIdx.y * o_ts;
    const int nbins = 1 << dbits;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int b = t; b < nbins; b += RS_THREADS)
#pragma unroll
        for (int w2 = 0; w2 < RS_THREADS / 64; w2++) wcnt[w2][b] = 0;
    const int64_t base = (int64_t)blockIdx.x * RS_TILE + (int64_t)w * (RS_TILE / (RS_THREADS / 64));
    int32_t kk[RS_R], vv[RS_R];
#pragma unroll
    for (int r = 0; r < RS_R; r++) {
        const int64_t i = base + r * 64 + lane;
        kk[r] = i < N ? keys[i * kstride] : 0;
        vv[r] = i < N ? (vals ? vals[i] : (int32_t)i) : 0;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t rk[RS_R];
#pragma unroll
    for (int r = 0; r < RS_R; r++) {
        const bool valid = base + r * 64 + lane < N;
        const int digit = (kk[r] >> shift) & (nbins - 1);
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < dbits; b++) {
            const bool bit = (digit >> b) & 1;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t before = valid ? wcnt[w][digit] : 0u;   // this wave's earlier rounds
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        rk[r] = before + below;
        // the digit's first lane advances the wave's running count (LDS ops of
        // one wave complete in order: every peer has read 'before')
        if (valid && below == 0) wcnt[w][digit] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (int b = t; b < nbins; b += RS_THREADS) {
        uint32_t o = scanned[(size_t)b * nblocks + blockIdx.x];
#pragma unroll
        for (int w2 = 0; w2 < RS_THREADS / 64; w2++) {
            const uint32_t c = wcnt[w2][b];
            wcnt[w2][b] = o;
            o += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_R; r++) {
        if (base + r * 64 + lane < N) {
            const uint32_t pos = wcnt[w][(kk[r] >> shift) & (nbins - 1)] + rk[r];
            keys_out[pos] = kk[r];
            vals_out[pos] = vv[r];
        }
    }
}

__global__ void rs_copy(const int32_t* __restrict__ keys, int64_t kstride, const int32_t* __restrict__ vals, int64_t N,
                        int32_t* __restrict__ keys_out, int32_t* __restrict__ vals_out, int64_t k_ts, int64_t v_ts,
                        int64_t o_ts) {
    keys += blockIdx.y * k_ts;
    if (vals) vals += blockIdx.y * v_ts;
    keys_out += blockIdx.y * o_ts;
    vals_out += blockIdx.y * o_ts;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        keys_out[i] = keys[i * kstride];
        vals_out[i] = vals ? vals[i] : (int32_t)i;
    }
}

// Small sorts (n <= SP_MAX distinct int32 keys, e.g. the few hundred unseen
// coins of a cube build): one workgroup, a bitonic network over the keys padded
// to a power of two in LDS -- one launch instead of a multi-pass radix sort's
// dozen. Keys must be distinct (the order of equal keys is not kept).
constexpr int SP_MAX = 8192;
__global__ __launch_bounds__(1024) void sort_pairs_small_kernel(const int32_t* __restrict__ keys,
                                                                const int32_t* __restrict__ vals, int n, int P,
                                                                const unsigned int* __restrict__ n_dev,
                                                                int32_t* __restrict__ keys_out,
                                                                int32_t* __restrict__ vals_out) {
    __shared__ int32_t sk[SP_MAX], sv[SP_MAX];
    if (n_dev) {                        // count left on the device (<= SP_MAX: the host checks the caller's bound)
        n = (int)min(*n_dev, (unsigned int)SP_MAX);
        for (P = 1; P < n; P <<= 1) {}
    }
    for (int i = threadIdx.x; i < P; i += 1024) {
        sk[i] = i < n ? keys[i] : 0x7FFFFFFF;
        sv[i] = i < n ? vals[i] : 0;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P; i += 1024) {
                const int l = i ^ j;
                if (l > i) {
                    const int32_t a = sk[i], b = sk[l];
                    const bool up = (i & k) == 0;
                    if (up ? a > b : a < b) {
                        sk[i] = b; sk[l] = a;
                        const int32_t t = sv[i]; sv[i] = sv[l]; sv[l] = t;
                    }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < n; i += 1024) {
        keys_out[i] = sk[i];
        vals_out[i] = sv[i];
    }
}

// n_dev: the count is read on the device; n is then the caller's upper bound on
// it, checked here (a count past SP_MAX would drop keys silently).
int sort_pairs_small(hipStream_t s, const int32_t* keys, const int32_t* vals, int64_t n, int32_t* keys_out,
                     int32_t* vals_out, const unsigned int* n_dev) {
    if (n_dev) {
        if (n > SP_MAX) {
            set_error("sort_pairs_small: the device count's bound exceeds the one-workgroup sort");
            return -1;
        }
        hipLaunchKernelGGL(sort_pairs_small_kernel, dim3(1), dim3(1024), 0, s, keys, vals, 0, 1, n_dev, keys_out, vals_out);
        return kstatus("scatter.hip");
    }
    if (n <= 0) return 0;
    if (n > SP_MAX) {
        set_error("sort_pairs_small: too many keys");
        return -1;
    }
    int P = 1;
    while (P < n) P <<= 1;
    hipLaunchKernelGGL(sort_pairs_small_kernel, dim3(1), dim3(1024), 0, s, keys, vals, (int)n, P, nullptr, keys_out, vals_out);
    return kstatus("scatter.hip");
}

// row_ptr[b] = first position of key >= b in the sorted keys; row_ptr[nb] = N.
__global__ void csr_bounds(const int32_t* __restrict__ skeys, int64_t N, int64_t nb, int64_t* __restrict__ row_ptr) {
    skeys += blockIdx.y * N;
    row_ptr += blockIdx.y * (nb + 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= N; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t prev = i == 0 ? -1 : (int64_t)skeys[i - 1];
        const int64_t cur = i == N ? nb : (int64_t)skeys[i];
        for (int64_t b = prev + 1; b <= cur && b <= nb; b++) row_ptr[b] = i;
    }
}

static int key_bits(int64_t range) {
    int bits = 0;
    while (bits < 31 && ((int64_t)1 << bits) < range) bits++;
    return bits;
}

size_t sort_scratch_bytes(int64_t N, int64_t range, int T) {
    const int bits = key_bits(range);
    const int P = (bits + 7) / 8;
    const int DB = P ? (bits + P - 1) / P : 0;
    const int64_t nblocks = (N + RS_TILE - 1) / RS_TILE;
    const int64_t M = ((int64_t)1 << DB) * nblocks;
    return (size_t)T * ((size_t)(2 * N + 64) * 4 + (size_t)M * 4 + (size_t)((M + RS_SC - 1) / RS_SC + 2) * 4) + 256;
}

// T independent stable sorts in one set of launches (blockIdx.y = table): table
// t's keys at keys + t * key_ts (stride kstride), its values (or the row index
// when vals is null) at vals + t * val_ts; outputs at keys_out / vals_out + t * N.
int stable_sort_by_key_batched(hipStream_t s, const int32_t* keys, int64_t kstride, int64_t key_ts, const int32_t* vals,
                               int64_t val_ts, int T, int64_t N, int64_t range, int32_t* keys_out, int32_t* vals_out,
                               void* scratch) {
    if (N <= 0 || T <= 0) return 0;
    const int bits = key_bits(range);
    const int64_t nblocks = (N + RS_TILE - 1) / RS_TILE;
    if (bits == 0) {
        hipLaunchKernelGGL(rs_copy, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 4096), (unsigned)T), dim3(256), 0,
                           s, keys, kstride, vals, N, keys_out, vals_out, key_ts, val_ts, N);
        return kstatus("scatter.hip");
    }
    const int P = (bits + 7) / 8;
    const int DB = (bits + P - 1) / P;
    const int nbins = 1 << DB;
    const int64_t M = (int64_t)nbins * nblocks;
    const int64_t nch = (M + RS_SC - 1) / RS_SC;
    int32_t* k2 = reinterpret_cast<int32_t*>(scratch);          // [T][N]
    int32_t* v2 = k2 + (size_t)T * N;                            // [T][N] (+64)
    uint32_t* hist = reinterpret_cast<uint32_t*>(v2 + (size_t)T * N + 64);   // [T][M]
    uint32_t* part = hist + (size_t)T * M;                       // [T][nch + 2]
    const int32_t* kin = keys;
    const int32_t* vin = vals;
    int64_t kst = kstride, kts = key_ts, vts = val_ts;
    for (int p = 0; p < P; p++) {
        const bool to_out = ((P - 1 - p) % 2) == 0;
        int32_t* ko = to_out ? keys_out : k2;
        int32_t* vo = to_out ? vals_out : v2;
        const int shift = p * DB;
        hipLaunchKernelGGL(rs_upsweep, dim3((unsigned)nblocks, (unsigned)T), dim3(RS_THREADS), 0, s, kin, kst, N, shift,
                           nbins, (int)nblocks, hist, kts, M);
        if (M <= RS_ONE_SCAN) {
            hipLaunchKernelGGL(rs_scan, dim3(1, (unsigned)T), dim3(1024), 0, s, hist, M, M);
        } else {
            hipLaunchKernelGGL(rs_chunk_sum, dim3((unsigned)nch, (unsigned)T), dim3(1024), 0, s, hist, M, part, M, nch + 2);
            hipLaunchKernelGGL(rs_scan, dim3(1, (unsigned)T), dim3(1024), 0, s, part, nch, nch + 2);
            hipLaunchKernelGGL(rs_chunk_scan, dim3((unsigned)nch, (unsigned)T), dim3(1024), 0, s, hist, M, part, M,
                               nch + 2);
        }
        hipLaunchKernelGGL(rs_downsweep, dim3((unsigned)nblocks, (unsigned)T), dim3(RS_THREADS), 0, s, kin, kst, vin, N,
                           shift, DB, (int)nblocks, hist, ko, vo, kts, vts, M, N);
        kin = ko; vin = vo; kst = 1; kts = N; vts = N;
    }
    return kstatus("scatter.hip");
}

int stable_sort_by_key(hipStream_t s, const int32_t* keys, int64_t kstride, const int32_t* vals, int64_t N,
                       int64_t range, int32_t* keys_out, int32_t* vals_out, void* scratch) {
    return stable_sort_by_key_batched(s, keys, kstride, 0, vals, 0, 1, N, range, keys_out, vals_out, scratch);
}

int launch_csr_bounds(hipStream_t s, const int32_t* sorted_keys, int64_t N, int64_t nb, int64_t* row_ptr, int T) {
    const int64_t threads = N + 1;
    hipLaunchKernelGGL(csr_bounds, dim3((unsigned)std::min<int64_t>((threads + 255) / 256, 8192), (unsigned)T), dim3(256),
                       0, s, sorted_keys, N, nb, row_ptr);
    return kstatus("scatter.hip");
}

}  // namespace lshkm
