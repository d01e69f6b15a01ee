// query.hip — batched bucket queries on gfx950.
//
// LSH: get_LSH_filtered_combined_buckets / get_LSH_combined_buckets
// (lib/lsh_cube.hpp:77-106) over CustHashtable::getFilteredBucketFor /
// getBucketFor (lib/data_structures/cust_hashtable.hpp:73-113). Per query the
// result is the union of its L buckets (filtered: members whose stored k-tuple
// equals the query's), deduplicated and sorted by row (std::set<CustVector*>
// over one contiguous std::vector orders by row index).
//   1. candidates per (query, table) = its bucket size; exclusive scan;
//   2. one wave per (query, table) streams its bucket (already row-sorted),
//      keeps a member iff it passes table l and fails every table l' < l
//      (O(1): bucket[m][l'] == qbucket[l'] plus the tuple test) — so the kept
//      lists are disjoint — and compacts them with ballot/popc, order kept;
//   3. per-query totals -> output offsets (two-phase API);
//   4. merge: an element at position p of kept list l lands at
//      p + sum_{l' != l} lower_bound(kept list l', e).
// Hypercube: get_hypercube_combined_buckets (lib/lsh_cube.hpp:139-177): main
// bucket, then the probe buckets in get_num_hamming_dist_from order
// (lib/utils.cpp:22-50), concatenated without dedup; the probe masks are the
// same for every query and are built on the host.
#include "common.h"
#include "kernels.h"

namespace lshkm {

// Exclusive scan of M int64 -> out[0..M] (out[M] = total). One block.
__global__ __launch_bounds__(1024) void scan_i64_kernel(const int64_t* __restrict__ a, int64_t M, int64_t* __restrict__ out) {
    __shared__ int64_t part[1024];
    const int t = threadIdx.x;
    const int64_t seg = (M + 1023) / 1024;
    const int64_t lo = t * seg, hi = min(M, lo + seg);
    int64_t s = 0;
    for (int64_t i = lo; i < hi; i++) s += a[i];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int64_t run = t ? part[t - 1] : 0;
    for (int64_t i = lo; i < hi; i++) { const int64_t v = a[i]; out[i] = run; run += v; }
    if (t == 1023) out[M] = part[1023];
}

// Large M: reduce-then-scan over SC_CH-element chunks (one block each, 8
// consecutive elements per thread), the chunk totals scanned by one block.
constexpr int SC_CH = 8192;
__global__ __launch_bounds__(1024) void scan_chunk_sum_kernel(const int64_t* __restrict__ a, int64_t M,
                                                             int64_t* __restrict__ part) {
    __shared__ int64_t red[1024];
    const int64_t base = (int64_t)blockIdx.x * SC_CH + threadIdx.x * 8;
    int64_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) s += base + u < M ? a[base + u] : 0;
    red[threadIdx.x] = s;
    __syncthreads();
    for (int off = 512; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(1024) void scan_chunk_kernel(const int64_t* __restrict__ a, int64_t M,
                                                         const int64_t* __restrict__ part_off, int64_t* __restrict__ out) {
    __shared__ int64_t sh[1024];
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * SC_CH + t * 8;
    int64_t v[8], s = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) { v[u] = base + u < M ? a[base + u] : 0; s += v[u]; }
    sh[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {          // Hillis-Steele inclusive scan of the thread sums
        const int64_t w = t >= off ? sh[t - off] : 0;
        __syncthreads();
        sh[t] += w;
        __syncthreads();
    }
    int64_t run = part_off[blockIdx.x] + (t ? sh[t - 1] : 0);
#pragma unroll
    for (int u = 0; u < 8; u++)
        if (base + u < M) { out[base + u] = run; run += v[u]; }
    if (blockIdx.x == gridDim.x - 1 && t == 1023) out[M] = part_off[gridDim.x];
}

size_t scan_ws_bytes(int64_t M) { return (size_t)(2 * ((M + SC_CH - 1) / SC_CH + 1)) * 8; }

// scratch: scan_ws_bytes(M) bytes, or NULL (then one block scans everything)
int launch_scan_i64(hipStream_t s, const int64_t* a, int64_t M, int64_t* out, int64_t* scratch) {
    if (M <= 4 * SC_CH || !scratch) {
        hipLaunchKernelGGL(scan_i64_kernel, dim3(1), dim3(1024), 0, s, a, M, out);
        return kstatus("query.hip");
    }
    const int64_t nb = (M + SC_CH - 1) / SC_CH;
    hipLaunchKernelGGL(scan_chunk_sum_kernel, dim3((unsigned)nb), dim3(1024), 0, s, a, M, scratch);
    hipLaunchKernelGGL(scan_i64_kernel, dim3(1), dim3(1024), 0, s, scratch, nb, scratch + nb + 1);
    hipLaunchKernelGGL(scan_chunk_kernel, dim3((unsigned)nb), dim3(1024), 0, s, a, M, scratch + nb + 1, out);
    return kstatus("query.hip");
}

__global__ void lq_sizes(const int32_t* __restrict__ qbucket, int64_t nq, int L, int64_t nb,
                         const int64_t* __restrict__ row_ptr, int64_t* __restrict__ sizes) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq * L; e += (int64_t)gridDim.x * blockDim.x) {
        const int l = (int)(e % L);
        const int64_t b = qbucket[e];
        const int64_t* rp = row_ptr + (size_t)l * (nb + 1);
        sizes[e] = rp[b + 1] - rp[b];
    }
}

__device__ inline bool tuple_eq(const int32_t* __restrict__ a, const int32_t* __restrict__ b, int k) {
    for (int i = 0; i < k; i++)
        if (a[i] != b[i]) return false;
    return true;
}

// Four (query, table) pairs per wave, 16 lanes each: a pair's work is a short
// chain of dependent loads (bucket id -> bucket bounds -> member ids -> their
// tuples), so the wave keeps four chains in flight instead of one.
constexpr int LQ_U = 4;          // 16-member chunks per round, loads in flight together
constexpr int LQ_G = 16;         // lanes per pair
__global__ __launch_bounds__(256) void lq_mark(
    const int32_t* __restrict__ qbucket, const int32_t* __restrict__ qtuple, const int32_t* __restrict__ alias,
    int64_t nq, int L, int k, int64_t nb, int filtered, int64_t N, const int32_t* __restrict__ tuples,
    const int32_t* __restrict__ bucket, const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ idx,
    const int64_t* __restrict__ cand_off, int32_t* __restrict__ klist, int64_t* __restrict__ kcount,
    const int32_t* __restrict__ mt0) {
    const int lane = threadIdx.x & 63, gl = lane & (LQ_G - 1), grp = lane / LQ_G;
    const int64_t pair = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LQ_G) + grp;
    if (pair >= nq * L) return;                          // whole groups (pair is uniform in a group)
    const unsigned long long gmask = ((1ull << LQ_G) - 1ull) << (grp * LQ_G);
    const unsigned long long lt = (1ull << lane) - 1ull;
    const int64_t q = pair / L;
    const int l = (int)(pair - q * L);
    const int32_t* qt = nullptr;
    if (filtered && tuples) {
        const int64_t a = alias ? alias[q] : -1;   // first-write-wins ID map (euclidean_phi_gen.hpp:94)
        qt = a >= 0 ? tuples + (size_t)a * L * k : qtuple + (size_t)q * L * k;
    }
    const int32_t* qb = qbucket + (size_t)q * L;
    const int64_t* rp = row_ptr + (size_t)l * (nb + 1);
    const int64_t beg = rp[qb[l]], end = rp[qb[l] + 1];
    const int32_t* members = idx + (size_t)l * N;
    int64_t out = cand_off[pair];
    const int32_t q0 = qt ? qt[l * k] : 0;
    // LQ_U chunks of 16 members: the member ids, then the first tuple value of
    // each (a random member's tuple almost always differs there), in flight
    // together; the rest of the tuple and the earlier-table dedup only for the
    // lanes still in; compaction in member order within the group
    for (int64_t p0 = beg; p0 < end; p0 += LQ_G * LQ_U) {
        int32_t m[LQ_U], t0[LQ_U];
#pragma unroll
        for (int u = 0; u < LQ_U; u++) {
            const int64_t p = p0 + LQ_G * u + gl;
            m[u] = p < end ? members[p] : 0;
        }
#pragma unroll
        for (int u = 0; u < LQ_U; u++) {
            const int64_t p = p0 + LQ_G * u + gl;
            t0[u] = !qt || p >= end ? 0 : mt0 ? mt0[(size_t)l * N + p] : tuples[(size_t)m[u] * L * k + l * k];
        }
#pragma unroll
        for (int u = 0; u < LQ_U; u++) {
            const int64_t p = p0 + LQ_G * u + gl;
            bool keep = p < end && (!qt || t0[u] == q0);
            if (keep && qt) {
                const int32_t* mt = tuples + (size_t)m[u] * L * k;
                keep = tuple_eq(mt + l * k + 1, qt + l * k + 1, k - 1);
            }
            if (keep) {
                const int32_t* mt = tuples ? tuples + (size_t)m[u] * L * k : nullptr;
                for (int l2 = 0; keep && l2 < l; l2++) {
                    const bool in2 = bucket[(size_t)m[u] * L + l2] == qb[l2] && (!qt || tuple_eq(mt + l2 * k, qt + l2 * k, k));
                    if (in2) keep = false;
                }
            }
            const unsigned long long bal = __ballot(keep) & gmask;
            if (keep) klist[out + __popcll(bal & lt)] = m[u];
            out += __popcll(bal);
        }
    }
    if (gl == 0) kcount[pair] = out - cand_off[pair];
}

__global__ void lq_qsizes(const int64_t* __restrict__ kcount, int64_t nq, int L, int64_t* __restrict__ qsz) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = 0;
        for (int l = 0; l < L; l++) s += kcount[q * L + l];
        qsz[q] = s;
    }
}

__global__ __launch_bounds__(256) void lq_merge(const int64_t* __restrict__ cand_off, const int64_t* __restrict__ kcount,
                                                const int32_t* __restrict__ klist, int64_t nq, int L,
                                                const int64_t* __restrict__ out_ptr, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t pair = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pair >= nq * L) return;
    const int64_t q = pair / L;
    const int l = (int)(pair - q * L);
    const int64_t n = kcount[pair];
    const int32_t* mine = klist + cand_off[pair];
    for (int64_t p = lane; p < n; p += 64) {
        const int32_t e = mine[p];
        int64_t rank = p;
        for (int l2 = 0; l2 < L; l2++) {
            if (l2 == l) continue;
            const int32_t* other = klist + cand_off[q * L + l2];
            int64_t lo = 0, hi = kcount[q * L + l2];
            while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (other[mid] < e) lo = mid + 1; else hi = mid; }
            rank += lo;
        }
        out[out_ptr[q] + rank] = e;
    }
}

int launch_lsh_query(hipStream_t s, const int32_t* qbucket, const int32_t* qtuple, const int32_t* alias, int64_t nq,
                     int L, int k, int64_t nb, int filtered, int64_t N, const int32_t* tuples, const int32_t* bucket,
                     const int64_t* row_ptr, const int32_t* idx, int64_t* sizes, int64_t* cand_off,
                     int32_t* klist, int64_t* kcount, int64_t* qsz, int64_t* out_ptr, int32_t* out, int phase,
                     int64_t* scan_ws, const int32_t* mt0) {
    const int64_t pairs = nq * L;
    if (phase == 0) {          // candidate counts -> cand_off[pairs + 1]
        hipLaunchKernelGGL(lq_sizes, dim3((unsigned)std::min<int64_t>((pairs + 255) / 256, 4096)), dim3(256), 0, s, qbucket,
                           nq, L, nb, row_ptr, sizes);
        if (launch_scan_i64(s, sizes, pairs, cand_off, scan_ws)) return -2;
    } else if (phase == 1) {   // filter + dedup + compact -> out_ptr[nq + 1]
        hipLaunchKernelGGL(lq_mark, dim3((unsigned)((pairs + 4 * (64 / LQ_G) - 1) / (4 * (64 / LQ_G)))), dim3(256), 0, s,
                           qbucket, qtuple, alias, nq, L, k,
                           nb, filtered, N, tuples, bucket, row_ptr, idx, cand_off, klist, kcount, mt0);
        hipLaunchKernelGGL(lq_qsizes, dim3((unsigned)std::min<int64_t>((nq + 255) / 256, 4096)), dim3(256), 0, s, kcount,
                           nq, L, qsz);
        if (launch_scan_i64(s, qsz, nq, out_ptr, scan_ws)) return -2;
    } else {                   // merge into the caller's output
        hipLaunchKernelGGL(lq_merge, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, s, cand_off, kcount, klist, nq, L,
                           out_ptr, out);
    }
    return kstatus("query.hip");
}

// mt0[l * N + pos] = the first tuple value of table l's member at CSR position pos
__global__ void lq_gather_t0(const int32_t* __restrict__ tuples, const int32_t* __restrict__ idx, int64_t N, int L,
                             int k, int32_t* __restrict__ mt0) {
    const int l = blockIdx.y;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (int64_t)gridDim.x * blockDim.x)
        mt0[(size_t)l * N + p] = tuples[(size_t)idx[(size_t)l * N + p] * L * k + l * k];
}
int launch_lsh_gather_t0(hipStream_t s, const int32_t* tuples, const int32_t* idx, int64_t N, int L, int k, int32_t* mt0) {
    if (N <= 0) return 0;
    hipLaunchKernelGGL(lq_gather_t0, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 4096), (unsigned)L), dim3(256), 0, s,
                       tuples, idx, N, L, k, mt0);
    return kstatus("query.hip");
}

// ------------------------------------------------------------------ hypercube
__global__ void cq_sizes(const int32_t* __restrict__ qvert, int64_t nq, const int32_t* __restrict__ masks, int S,
                         const int64_t* __restrict__ row_ptr, int64_t* __restrict__ sizes) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq * S; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = e / S;
        const int64_t v = qvert[q] ^ masks[e - q * S];
        sizes[e] = row_ptr[v + 1] - row_ptr[v];
    }
}

__global__ void cq_qptr(const int64_t* __restrict__ slot_off, int64_t nq, int S, int64_t* __restrict__ out_ptr) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q <= nq; q += (int64_t)gridDim.x * blockDim.x)
        out_ptr[q] = slot_off[q * S];
}

// Per-slot source offset idx position of the slot's bucket, written over the
// sizes array once the scan has consumed it.
__global__ void cq_beg(const int32_t* __restrict__ qvert, int64_t nq, const int32_t* __restrict__ masks, int S,
                       const int64_t* __restrict__ row_ptr, int64_t* __restrict__ beg) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nq * S; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = e / S;
        beg[e] = row_ptr[qvert[q] ^ masks[e - q * S]];
    }
}

// Last s in [0, hi] with a[s] <= x (a non-decreasing, a[0] <= x): a 64-ary
// search, one probe per lane per round (log64 of the slot count rounds of
// L2-resident loads), wave-uniform result.
__device__ inline int64_t last_le64(const int64_t* __restrict__ a, int64_t hi, int64_t x, int lane) {
    int64_t lo = 0;
    while (hi - lo >= 64) {
        const int64_t step = (hi - lo + 62) / 63;            // lo + 63 step >= hi
        const int64_t pj = min(lo + (int64_t)lane * step, hi);
        const unsigned long long b = __ballot(a[pj] <= x);   // a prefix of the lanes
        const int m = __popcll(b);                           // >= 1 (lane 0 probes lo)
        const int64_t nlo = min(lo + (int64_t)(m - 1) * step, hi);
        hi = m < 64 ? min(lo + (int64_t)m * step, hi) - 1 : hi;
        lo = nlo;
    }
    const unsigned long long b = __ballot(lo + lane <= hi && a[min(lo + lane, hi)] <= x);
    return lo + __popcll(b) - 1;
}

// Load-balanced copy: waves own contiguous CQ_CH-element chunks of the OUTPUT
// (not slots), so a skewed bucket-size distribution (a few huge vertices)
// spreads over every CU. A chunk finds its first slot by the 64-ary search and
// walks the slots it spans; within a slot the lanes copy 512 elements per
// round with 8 loads in flight, stores contiguous.
constexpr int64_t CQ_CH = 4096;
__global__ __launch_bounds__(256) void cq_copy(const int64_t* __restrict__ slot_off, int64_t slots,
                                               const int64_t* __restrict__ beg, const int32_t* __restrict__ idx,
                                               int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t total = slot_off[slots];
    const int64_t nch = (total + CQ_CH - 1) / CQ_CH;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += nw) {
        int64_t p = c * CQ_CH;
        const int64_t oe = min(p + CQ_CH, total);
        int64_t s = last_le64(slot_off, slots, p, lane);     // slot_off[s] <= p < slot_off[s + 1]
        int64_t so = slot_off[s];
        while (p < oe) {
            const int64_t send = slot_off[s + 1];
            const int64_t stop = min(send, oe);
            const int32_t* src = idx + (beg[s] - so);        // output i <- idx[beg[s] + i - slot_off[s]]
            for (int64_t i = p + lane; i < stop; i += 512) {
                int32_t w[8];
#pragma unroll
                for (int u = 0; u < 8; u++) w[u] = i + 64 * u < stop ? src[i + 64 * u] : 0;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (i + 64 * u < stop) out[i + 64 * u] = w[u];
            }
            p = stop;
            so = send;
            s++;
        }
    }
}

int launch_cube_query(hipStream_t s, const int32_t* qvert, int64_t nq, const int32_t* masks, int S,
                      const int64_t* row_ptr, const int32_t* idx, int64_t* sizes, int64_t* slot_off,
                      int64_t* out_ptr, int32_t* out, int64_t* scan_ws) {
    const int64_t slots = nq * S;
    hipLaunchKernelGGL(cq_sizes, dim3((unsigned)std::min<int64_t>((slots + 255) / 256, 4096)), dim3(256), 0, s, qvert, nq,
                       masks, S, row_ptr, sizes);
    if (launch_scan_i64(s, sizes, slots, slot_off, scan_ws)) return -2;
    hipLaunchKernelGGL(cq_qptr, dim3((unsigned)std::min<int64_t>((nq + 256) / 256, 4096)), dim3(256), 0, s, slot_off, nq, S,
                       out_ptr);
    if (out) {
        // sizes[] is dead after the scan: it now holds each slot's bucket start
        hipLaunchKernelGGL(cq_beg, dim3((unsigned)std::min<int64_t>((slots + 255) / 256, 4096)), dim3(256), 0, s, qvert, nq,
                           masks, S, row_ptr, sizes);
        hipLaunchKernelGGL(cq_copy, dim3(2048), dim3(256), 0, s, slot_off, slots, sizes, idx, out);
    }
    return kstatus("query.hip");
}

}  // namespace lshkm
