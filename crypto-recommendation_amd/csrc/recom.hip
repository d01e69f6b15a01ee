// recom.hip — the recommend step on gfx950:
//   get_P_closest          lib/crypto_rec.hpp:213-231
//   parallel_quickSort     lib/crypto_rec.hpp:234-277 (Lomuto, pivot = last, '>=')
//   get_predicted_user_sim lib/crypto_rec.hpp:280-302
//   get_top_N_recom        lib/crypto_rec.hpp:305-325
// for a batch of users, each with its candidate neighbour rows (the output of
// an LSH / hypercube query). Vectors are fp64 rows.
//
// Ordering. With distinct, non-NaN keys the reference's quicksort yields the
// keys in descending order, so the first P positions are the P largest. Equal
// keys are permuted by Lomuto's swap sequence and NaNs fail every '>='; the
// order then depends on the whole array. One wave per user therefore extracts
// the top P+1 similarities in parallel and, only if a NaN is present or two of
// the first P+1 are equal (a tie touching the first P positions), hands the user
// to lomuto_sort, which replays the reference's quicksort exactly (one lane per
// user; disjoint subarrays, so the order they are sorted in does not matter).
#include <climits>

#include "../../include/lshkm.h"
#include "common.h"
#include "kernels.h"
#include "exact.h"

namespace lshkm {

constexpr int RC_WAVES = 4;
constexpr int RC_MAXV = 8;       // candidates per lane held in registers (n <= 512 per user)

// CustVector::cosineSimilarity (cust_vector.hpp:158-174), this = neighbour x,
// in = user u: long-double inner product of double products, fp64 norms
// (xa, ub: sum of squares in dim order), long-double division, then double.
__device__ inline double rc_cos_sim(const double* __restrict__ x, const double* __restrict__ u, int d, double xa,
                                    double ub) {
    X87acc ip;
    ip.init();
    for (int j = 0; j < d; j++) ip.add(__dmul_rn(x[j], u[j]));
    return x87_quot(ip.value(), __dmul_rn(sqrt(xa), sqrt(ub)));
}

__device__ inline double rc_sumsq(const double* __restrict__ x, int d) {
    double a = 0.0;
    for (int j = 0; j < d; j++) a = __dadd_rn(a, gp_sq(x[j]));
    return a;
}

__global__ __launch_bounds__(256) void rc_norm_kernel(const double* __restrict__ X, int64_t N, int d,
                                                      double* __restrict__ xa) {
    for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < N; r += (int64_t)gridDim.x * 256)
        xa[r] = rc_sumsq(X + r * d, d);
}

// The reference's quicksort on key/val[0..n), exactly (crypto_rec.hpp:234-277).
// Explicit stack, smaller part first: depth <= log2(n) + 1.
__device__ void lomuto_sort(double* key, int32_t* val, int n) {
    int lo_s[64], hi_s[64];
    int sp = 0;
    if (n > 1) { lo_s[0] = 0; hi_s[0] = n - 1; sp = 1; }
    while (sp > 0) {
        sp--;
        int low = lo_s[sp], high = hi_s[sp];
        while (low < high) {
            const double pivot = key[high];
            int i = low - 1;
            for (int j = low; j <= high - 1; j++) {
                const double kj = key[j];
                if (kj >= pivot) {
                    i++;
                    const double tk = key[i]; key[i] = kj; key[j] = tk;
                    const int32_t tv = val[i]; val[i] = val[j]; val[j] = tv;
                }
            }
            const double tk = key[i + 1]; key[i + 1] = key[high]; key[high] = tk;
            const int32_t tv = val[i + 1]; val[i + 1] = val[high]; val[high] = tv;
            const int pi = i + 1;
            // parts [low, pi-1] and [pi+1, high]: push the larger, continue with the smaller
            if (pi - low < high - pi) {
                if (pi + 1 < high) { lo_s[sp] = pi + 1; hi_s[sp] = high; sp++; }
                high = pi - 1;
            } else {
                if (low < pi - 1) { lo_s[sp] = low; hi_s[sp] = pi - 1; sp++; }
                low = pi + 1;
            }
        }
    }
}

// One wave per user: similarities (sim, in candidate order), then the top P+1
// by repeated wave-wide max over a work copy (key). Users with a NaN or a tie
// in the first P+1 go to the exact replay list.
__global__ __launch_bounds__(64 * RC_WAVES) void rc_p_closest_kernel(
    const double* __restrict__ X, const double* __restrict__ xa, int d, const double* __restrict__ U, int64_t nq,
    const int64_t* __restrict__ cand_ptr, const int32_t* __restrict__ cand_idx, int P, double* __restrict__ sim,
    double* __restrict__ key, int32_t* __restrict__ out_idx, double* __restrict__ out_sim,
    int32_t* __restrict__ out_cnt, int32_t* __restrict__ replay, unsigned int* __restrict__ replay_count) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * RC_WAVES + (threadIdx.x >> 6);
    for (int64_t q = w0; q < nq; q += (int64_t)gridDim.x * RC_WAVES) {
        const int64_t o = cand_ptr[q];
        const int n = (int)(cand_ptr[q + 1] - o);
        const double* u = U + q * d;
        const double ub = rc_sumsq(u, d);
        bool nan = false;
        unsigned inexact = 0;            // this lane's candidates still held as intervals
        if (n <= 64 * RC_MAXV) {
            // Certified similarities first (exact.h IpAcc: q exact, or the exact
            // value within q +- qr); the soft-x87 chain only for candidates whose
            // interval reaches T, the (P+1)-th largest lower bound -- nothing
            // below T can enter the top P+1 -- and for declined ones (zero
            // vectors, NaN/inf). A replayed user (NaN or tie) gets every value exact.
            double qv[RC_MAXV], qr[RC_MAXV];
#pragma unroll
            for (int k = 0; k < RC_MAXV; k++) {
                qv[k] = -__builtin_inf(); qr[k] = 0.0;
                const int i = lane + 64 * k;
                if (i < n) {
                    const int32_t r = cand_idx[o + i];
                    const double* x = X + (int64_t)r * d;
                    IpAcc ip;
                    for (int j = 0; j < d; j++) ip.add(__dmul_rn(x[j], u[j]));
                    const int st = ip.quot_status(__dmul_rn(sqrt(xa[r]), sqrt(ub)), qv[k], qr[k]);
                    if (st == 2) { qv[k] = rc_cos_sim(x, u, d, xa[r], ub); qr[k] = 0.0; }
                    else if (st == 0) qr[k] = 0.0;
                    nan |= qv[k] != qv[k];
                }
            }
            const bool any_nan = __ballot(nan) != 0;
            double T = -__builtin_inf();
            if (!any_nan) {
                // T: the (P+1)-th largest lower bound (repeated wave max, first position)
                double lo[RC_MAXV];
#pragma unroll
                for (int k = 0; k < RC_MAXV; k++) lo[k] = lane + 64 * k < n ? qv[k] - qr[k] : -__builtin_inf();
                const int ext0 = n < P + 1 ? n : P + 1;
                for (int e = 0; e < ext0; e++) {
                    double best = -__builtin_inf();
                    int bk = -1;
#pragma unroll
                    for (int k = 0; k < RC_MAXV; k++)
                        if (lo[k] > best || bk < 0) { best = lo[k]; bk = k; }
                    int bl = lane;
                    for (int off = 32; off >= 1; off >>= 1) {
                        const double ob = __shfl_xor(best, off);
                        const int ol = __shfl_xor(bl, off);
                        if (ob > best || (ob == best && ol < bl)) { best = ob; bl = ol; }
                    }
                    T = best;
                    if (lane == bl) {
#pragma unroll
                        for (int k = 0; k < RC_MAXV; k++)
                            if (k == bk) lo[k] = -__builtin_inf();
                    }
                }
                if (n <= P + 1) T = -__builtin_inf();     // every candidate is in the top P+1
            }
#pragma unroll
            for (int k = 0; k < RC_MAXV; k++) {
                const int i = lane + 64 * k;
                if (i < n && qr[k] != 0.0 && (any_nan || qv[k] + qr[k] >= T)) {
                    const int32_t r = cand_idx[o + i];
                    qv[k] = rc_cos_sim(X + (int64_t)r * d, u, d, xa[r], ub);
                    qr[k] = 0.0;
                }
                if (i < n) {
                    sim[o + i] = qv[k];
                    key[o + i] = qv[k];
                }
            }
            // a tie found below makes this user a replay: its values must all be exact
#pragma unroll
            for (int k = 0; k < RC_MAXV; k++)
                if (qr[k] != 0.0) inexact |= 1u << k;
        } else {
            for (int i = lane; i < n; i += 64) {
                const int32_t r = cand_idx[o + i];
                const double s = rc_cos_sim(X + (int64_t)r * d, u, d, xa[r], ub);
                sim[o + i] = s;
                key[o + i] = s;
                nan |= s != s;
            }
        }
        const int c = n < P ? n : P;
        if (lane == 0) out_cnt[q] = c;
        for (int i = c + lane; i < P; i += 64) {
            out_idx[q * P + i] = -1;
            out_sim[q * P + i] = 0.0;
        }
        bool replay_me = __ballot(nan) != 0;
        const int ext = n < P + 1 ? n : P + 1;
        double prev = 0.0;
        for (int k = 0; k < ext && !replay_me; k++) {
            double best = -__builtin_inf();
            int bpos = 0x7fffffff;
            for (int i = lane; i < n; i += 64) {
                const double v = key[o + i];
                if (v > best) { best = v; bpos = i; }
            }
            for (int off = 32; off >= 1; off >>= 1) {
                const double ob = __shfl_xor(best, off);
                const int op = __shfl_xor(bpos, off);
                if (ob > best || (ob == best && op < bpos)) { best = ob; bpos = op; }
            }
            if (k > 0 && best == prev) {          // a tie touching the first P positions
                replay_me = true;
                break;
            }
            prev = best;
            if (k < c && lane == 0) {
                out_idx[q * P + k] = cand_idx[o + bpos];
                out_sim[q * P + k] = best;
            }
            if (lane == (bpos & 63)) key[o + bpos] = -__builtin_inf();
            wave_sync();
        }
        if (replay_me && __ballot(inexact != 0u)) {
            for (int k = 0; k < RC_MAXV; k++)
                if ((inexact >> k) & 1u) {
                    const int i = lane + 64 * k;
                    const int32_t r = cand_idx[o + i];
                    sim[o + i] = rc_cos_sim(X + (int64_t)r * d, u, d, xa[r], ub);
                }
        }
        if (replay_me && lane == 0) replay[atomicAdd(replay_count, 1u)] = (int32_t)q;
    }
}

// Exact replay of the reference's quicksort for the listed users (one lane each).
__global__ __launch_bounds__(64) void rc_replay_kernel(const int64_t* __restrict__ cand_ptr,
                                                       const int32_t* __restrict__ cand_idx, int P,
                                                       const double* __restrict__ sim, double* __restrict__ key,
                                                       int32_t* __restrict__ pos, const int32_t* __restrict__ replay,
                                                       const unsigned int* __restrict__ replay_count,
                                                       int32_t* __restrict__ out_idx, double* __restrict__ out_sim) {
    const unsigned int total = *replay_count;
    for (unsigned int t = blockIdx.x * 64 + threadIdx.x; t < total; t += gridDim.x * 64) {
        const int64_t q = replay[t];
        const int64_t o = cand_ptr[q];
        const int n = (int)(cand_ptr[q + 1] - o);
        for (int i = 0; i < n; i++) {
            key[o + i] = sim[o + i];
            pos[o + i] = cand_idx[o + i];
        }
        lomuto_sort(key + o, pos + o, n);
        const int c = n < P ? n : P;
        for (int i = 0; i < c; i++) {
            out_idx[q * P + i] = pos[o + i];
            out_sim[q * P + i] = key[o + i];
        }
    }
}

// get_top_N_recom with get_predicted_user_sim: one wave per user, lane per
// unknown index (sums over the neighbours in their sorted order), then the
// exact quicksort of the predictions by lane 0 and the first n_top, 0-padded.
__global__ __launch_bounds__(64 * RC_WAVES) void rc_top_n_kernel(
    const double* __restrict__ X, const double* __restrict__ x_mean, int d, const double* __restrict__ u_mean,
    int64_t nq, const int64_t* __restrict__ unk_ptr, const int32_t* __restrict__ unk_idx,
    const int32_t* __restrict__ nb_idx, const double* __restrict__ nb_sim, const int32_t* __restrict__ nb_cnt, int P,
    int n_top, double* __restrict__ pred, int32_t* __restrict__ pidx, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * RC_WAVES + (threadIdx.x >> 6);
    for (int64_t q = w0; q < nq; q += (int64_t)gridDim.x * RC_WAVES) {
        const int64_t o = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - o);
        const int cnt = nb_cnt[q];
        const double um = u_mean[q];
        for (int e = lane; e < m; e += 64) {
            const int index = unk_idx[o + e];
            double main_sum = 0.0, abs_sum = 0.0;
            for (int i = 0; i < cnt; i++) {
                const double cs = nb_sim[q * P + i];
                abs_sum = __dadd_rn(abs_sum, fabs(cs));
                const int32_t r = nb_idx[q * P + i];
                main_sum = __dadd_rn(main_sum, __dmul_rn(cs, __dsub_rn(X[(int64_t)r * d + index], x_mean[r])));
            }
            pred[o + e] = __dadd_rn(__ddiv_rn(main_sum, abs_sum), um);
            pidx[o + e] = index;
        }
        __threadfence_block();
        wave_sync();
        if (lane == 0) {
            lomuto_sort(pred + o, pidx + o, m);
            for (int i = 0; i < n_top; i++) out[q * n_top + i] = i < m ? pidx[o + i] : 0;
        }
    }
}

// ---------------------------------------------------------------------------
// The clustering recommenders' get_top_N_recom(neighbors, user, N) -- the
// 3-argument overload (crypto_rec.hpp:327-345) over the user's whole cluster
// (main.cpp:260-269 Part A: the user's own cluster; :353-373 Part B: the
// cluster of the nearest centroid). One wave per user:
//   phase 1: cosineSimilarity(member, user) of every member, lane per member,
//     certified by IpAcc (exact.h; ~3% decline), the declined members queued
//     in LDS and run through the X87acc chain 64 at a time (all lanes busy),
//     sims into the wave's scratch row in member order;
//   phase 2: get_predicted_user_sim (:280-306): lane per unknown index (CR_MI
//     per lane), the member loop in order, 64 members per chunk read coalesced
//     (sim, mean, row id) and broadcast by readlane, the row values of the next
//     8 members loaded ahead of the dependent fp64 chains;
//   the Lomuto quicksort of the predictions (lane 0, :341) and the first n_top,
//   0-padded (:343). Users of an empty cluster get -1 (main.cpp skips them).
constexpr int CR_MI = 4;          // unknown indexes per lane per pass (256 per pass)
constexpr int CR_Q = 128;         // LDS queue of declined members per wave

__device__ inline double cr_rl(double v, int t) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), t);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), t);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <typename T>
__device__ inline double cr_sumsq(const T* __restrict__ x, int d) {
    double a = 0.0;
    for (int j = 0; j < d; j++) {
        const double v = (double)x[j];
        a = __dadd_rn(a, sq_of<T>(v));
    }
    return a;
}

// IpAcc certificate of cosineSimilarity(x, u) (cust_vector.hpp:158-174);
// false: the x87 chain must decide (declined, or a zero denominator)
template <typename T>
__device__ inline bool cr_sim_cert(const T* __restrict__ x, const T* __restrict__ u, int d, double ub, double& s,
                                   double& denom) {
    IpAcc ip;
    double xa = 0.0;
    for (int j = 0; j < d; j++) {
        const double xj = (double)x[j], uj = (double)u[j];
        ip.add(__dmul_rn(xj, uj));
        xa = __dadd_rn(xa, sq_of<T>(xj));
    }
    denom = __dmul_rn(sqrt(xa), sqrt(ub));
    double qr;
    return ip.quot_status(denom, s, qr) == 0;
}

template <typename T>
__device__ inline double cr_sim_x87(const T* __restrict__ x, const T* __restrict__ u, int d, double denom) {
    X87acc ip;
    ip.init();
    for (int j = 0; j < d; j++) ip.add(__dmul_rn((double)x[j], (double)u[j]));
    return x87_quot(ip.value(), denom);
}

// Phase 1 for one user: sim[i] = cosineSimilarity(member i, user) for the n
// members mem[0 .. n) (dataset rows), in member order. Declined certificates
// are queued (queue / qden: this wave's CR_Q LDS slots) and decided by the x87
// chain 64 at a time. Counts the x87-chain members in `soft`.
template <typename T>
__device__ inline void cr_sims(const T* __restrict__ X, const int32_t* __restrict__ mem, int n, const T* __restrict__ u,
                               int d, double* __restrict__ sim, int32_t* queue, double* qden, int lane,
                               unsigned long long& soft) {
    const double ub = cr_sumsq(u, d);
    int nqd = 0;                                    // queued declines
    auto drain = [&](int cnt) {                     // the x87 chain for queue[0 .. cnt)
        if (lane < cnt) {
            const int i = queue[lane];
            sim[i] = cr_sim_x87(X + (int64_t)mem[i] * d, u, d, qden[lane]);
        }
        soft += (unsigned long long)cnt;
    };
    for (int b = 0; b < n; b += 64) {
        const int i = b + lane;
        bool dec = false;
        double s = 0.0, den = 0.0;
        if (i < n) {
            dec = !cr_sim_cert(X + (int64_t)mem[i] * d, u, d, ub, s, den);
            if (!dec) sim[i] = s;
        }
        const unsigned long long mask = __ballot(dec);
        const int pos = nqd + __popcll(mask & ((1ull << lane) - 1ull));
        if (dec) { queue[pos] = i; qden[pos] = den; }
        nqd += __popcll(mask);
        wave_sync();
        if (nqd >= 64) {
            drain(64);
            const int rest = nqd - 64;
            int32_t qi = 0; double qd = 0.0;
            if (lane < rest) { qi = queue[64 + lane]; qd = qden[64 + lane]; }
            wave_sync();
            if (lane < rest) { queue[lane] = qi; qden[lane] = qd; }
            nqd = rest;
            wave_sync();
        }
    }
    if (nqd > 0) drain(nqd);
    __threadfence_block();
    wave_sync();
}

// Phase 2 for one user (get_predicted_user_sim, crypto_rec.hpp:285-303): over
// the members mem[0 .. n) in order, abs_sum += |sim| and, per unknown index e
// (uidx[0 .. m)), main_sum[e] += sim * (x[index] - mean), every sum continuing
// from its carry (main_in / abs_in: 0 for the first shard). Writes the running
// sums (main_out[e], *abs_out by lane 0) or, with pred != NULL, the
// predictions main / abs + um and the index list.
template <typename T>
__device__ inline void cr_chains(const T* __restrict__ X, const double* __restrict__ x_mean,
                                 const int32_t* __restrict__ mem, int n, int d, const double* __restrict__ sim,
                                 const int32_t* __restrict__ uidx, int m, const double* __restrict__ main_in,
                                 double abs_in, double* __restrict__ main_out, double* __restrict__ abs_out, double um,
                                 double* __restrict__ pred, int32_t* __restrict__ pidx, int lane) {
    for (int g0 = 0; g0 < m; g0 += 64 * CR_MI) {
        int idx[CR_MI];
        bool ok[CR_MI];
        double acc[CR_MI];
#pragma unroll
        for (int k = 0; k < CR_MI; k++) {
            const int e = g0 + lane + 64 * k;
            ok[k] = e < m;
            idx[k] = ok[k] ? uidx[e] : 0;
            acc[k] = ok[k] && main_in ? main_in[e] : 0.0;
        }
        double abs_sum = abs_in;
        for (int b = 0; b < n; b += 64) {
            const int cnt = n - b < 64 ? n - b : 64;
            int32_t r = 0;
            double sv = 0.0, mv = 0.0;
            if (lane < cnt) {
                r = mem[b + lane];
                sv = sim[b + lane];
                mv = x_mean[r];
            }
            for (int t0 = 0; t0 < cnt; t0 += 8) {
                double xv[8][CR_MI];
#pragma unroll
                for (int tt = 0; tt < 8; tt++) {
                    const int64_t rr = (int64_t)__builtin_amdgcn_readlane(r, t0 + tt);
#pragma unroll
                    for (int k = 0; k < CR_MI; k++)
                        xv[tt][k] = (t0 + tt < cnt && ok[k]) ? (double)X[rr * d + idx[k]] : 0.0;
                }
#pragma unroll
                for (int tt = 0; tt < 8; tt++) {
                    if (t0 + tt >= cnt) break;
                    const double cs = cr_rl(sv, t0 + tt), nm = cr_rl(mv, t0 + tt);
                    abs_sum = __dadd_rn(abs_sum, fabs(cs));
#pragma unroll
                    for (int k = 0; k < CR_MI; k++)
                        acc[k] = __dadd_rn(acc[k], __dmul_rn(cs, __dsub_rn(xv[tt][k], nm)));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < CR_MI; k++)
            if (ok[k]) {
                const int e = g0 + lane + 64 * k;
                if (pred) {
                    pred[e] = __dadd_rn(__ddiv_rn(acc[k], abs_sum), um);    // crypto_rec.hpp:299-302
                    pidx[e] = idx[k];
                } else {
                    main_out[e] = acc[k];
                }
            }
        if (!pred && g0 == 0 && lane == 0) *abs_out = abs_sum;
    }
    if (!pred && m == 0 && lane == 0) {
        // no unknown index: only the |sim| chain (its count decides "skipped")
        double abs_sum = abs_in;
        for (int i = 0; i < n; i++) abs_sum = __dadd_rn(abs_sum, fabs(sim[i]));
        *abs_out = abs_sum;
    }
    __threadfence_block();
    wave_sync();
}

// Lane 0: the reference's quicksort of the predictions (:341) and the first
// n_top unknown indexes, 0-padded (:343).
__device__ inline void cr_top(double* pred, int32_t* pidx, int m, int n_top, int32_t* out, int lane) {
    if (lane == 0) {
        if (m > 0) lomuto_sort(pred, pidx, m);
        for (int i = 0; i < n_top; i++) out[i] = i < m ? pidx[i] : 0;
    }
    wave_sync();
}

template <typename T>
__global__ __launch_bounds__(64 * RC_WAVES) void rc_cluster_top_n_kernel(
    const T* __restrict__ X, const double* __restrict__ x_mean, int d, const int64_t* __restrict__ crow,
    const int32_t* __restrict__ crows, int K, const T* __restrict__ U, const double* __restrict__ u_mean, int64_t nq,
    const int32_t* __restrict__ ucl, const int64_t* __restrict__ unk_ptr, const int32_t* __restrict__ unk_idx,
    int n_top, double* __restrict__ scratch, int64_t scratch_row, double* __restrict__ pred, int32_t* __restrict__ pidx,
    int32_t* __restrict__ out, unsigned long long* __restrict__ soft_count) {
    __shared__ int32_t queue[RC_WAVES][CR_Q];
    __shared__ double qden[RC_WAVES][CR_Q];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t w0 = (int64_t)blockIdx.x * RC_WAVES + wv;
    const int64_t nw = (int64_t)gridDim.x * RC_WAVES;
    double* sim = scratch + w0 * scratch_row;       // this wave's similarities, member order
    unsigned long long soft = 0;
    for (int64_t q = w0; q < nq; q += nw) {
        const int c = ucl[q];
        const int64_t base = (c >= 0 && c < K) ? crow[c] : 0;
        const int n = (c >= 0 && c < K) ? (int)(crow[c + 1] - base) : 0;
        if (n == 0) {                                   // main.cpp:262 / :366 skip the user
            for (int i = lane; i < n_top; i += 64) out[q * n_top + i] = -1;
            continue;
        }
        const int64_t o = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - o);
        if (m > 0) {
            const T* u = U + q * d;
            cr_sims(X, crows + base, n, u, d, sim, queue[wv], qden[wv], lane, soft);
            cr_chains(X, x_mean, crows + base, n, d, sim, unk_idx + o, m, (const double*)nullptr, 0.0,
                      (double*)nullptr, (double*)nullptr, u_mean[q], pred + o, pidx + o, lane);
        }
        cr_top(pred + o, pidx + o, m, n_top, out + q * n_top, lane);
    }
    if (soft_count && lane == 0 && soft) atomicAdd(soft_count, soft);     // one atomic per wave
}

// Sharded form, phase 1: every user's similarities to THIS shard's members of
// its cluster into sims[soff[q] .. soff[q+1]) (member order).
template <typename T>
__global__ __launch_bounds__(64 * RC_WAVES) void rc_shard_sims_kernel(
    const T* __restrict__ X, int d, const int64_t* __restrict__ crow, const int32_t* __restrict__ crows, int K,
    const T* __restrict__ U, int64_t nq, const int32_t* __restrict__ ucl, const int64_t* __restrict__ unk_ptr,
    const int64_t* __restrict__ soff, double* __restrict__ sims, unsigned long long* __restrict__ soft_count) {
    __shared__ int32_t queue[RC_WAVES][CR_Q];
    __shared__ double qden[RC_WAVES][CR_Q];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long soft = 0;
    for (int64_t q = (int64_t)blockIdx.x * RC_WAVES + wv; q < nq; q += (int64_t)gridDim.x * RC_WAVES) {
        const int c = ucl[q];
        const int64_t base = (c >= 0 && c < K) ? crow[c] : 0;
        const int n = (c >= 0 && c < K) ? (int)(crow[c + 1] - base) : 0;
        if (n > 0) cr_sims(X, crows + base, n, U + q * d, d, sims + soff[q], queue[wv], qden[wv], lane, soft);
    }
    if (soft_count && lane == 0 && soft) atomicAdd(soft_count, soft);
}

// Sharded form, phase 2: the chains over this shard's members, continued from
// the carry (carry_main [total unknowns], carry_abs / carry_cnt [nq]; NULL on
// the first shard); the running sums out, or (out != NULL) the final step.
template <typename T>
__global__ __launch_bounds__(64 * RC_WAVES) void rc_shard_chain_kernel(
    const T* __restrict__ X, const double* __restrict__ x_mean, int d, const int64_t* __restrict__ crow,
    const int32_t* __restrict__ crows, int K, int64_t nq, const int32_t* __restrict__ ucl,
    const double* __restrict__ u_mean, const int64_t* __restrict__ unk_ptr, const int32_t* __restrict__ unk_idx,
    const int64_t* __restrict__ soff, const double* __restrict__ sims, const double* __restrict__ carry_main,
    const double* __restrict__ carry_abs, const int64_t* __restrict__ carry_cnt, double* __restrict__ main_out,
    double* __restrict__ abs_out, int64_t* __restrict__ cnt_out, int n_top, double* __restrict__ pred,
    int32_t* __restrict__ pidx, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t q = (int64_t)blockIdx.x * RC_WAVES + wv; q < nq; q += (int64_t)gridDim.x * RC_WAVES) {
        const int c = ucl[q];
        const int64_t base = (c >= 0 && c < K) ? crow[c] : 0;
        const int n = (c >= 0 && c < K) ? (int)(crow[c + 1] - base) : 0;
        const int64_t o = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - o);
        const int64_t total = (carry_cnt ? carry_cnt[q] : 0) + n;
        const double* min = carry_main ? carry_main + o : nullptr;
        const double ain = carry_abs ? carry_abs[q] : 0.0;
        if (!out) {                                     // pass the running sums on
            if (n > 0) {
                cr_chains(X, x_mean, crows + base, n, d, sims + soff[q], unk_idx + o, m, min, ain, main_out + o,
                          abs_out + q, u_mean[q], (double*)nullptr, (int32_t*)nullptr, lane);
            } else {                                    // no member here: the carry unchanged
                for (int e = lane; e < m; e += 64) main_out[o + e] = min ? min[e] : 0.0;
                if (lane == 0) abs_out[q] = ain;
            }
            if (lane == 0) cnt_out[q] = total;
            continue;
        }
        if (total == 0) {                               // an empty cluster on every shard: skipped
            for (int i = lane; i < n_top; i += 64) out[q * n_top + i] = -1;
            continue;
        }
        if (m > 0) {
            if (n > 0) {
                cr_chains(X, x_mean, crows + base, n, d, sims + soff[q], unk_idx + o, m, min, ain, (double*)nullptr,
                          (double*)nullptr, u_mean[q], pred + o, pidx + o, lane);
            } else {
                for (int e = lane; e < m; e += 64) {
                    pred[o + e] = __dadd_rn(__ddiv_rn(min ? min[e] : 0.0, ain), u_mean[q]);
                    pidx[o + e] = unk_idx[o + e];
                }
                __threadfence_block();
                wave_sync();
            }
        }
        cr_top(pred + o, pidx + o, m, n_top, out + q * n_top, lane);
    }
}

int launch_rc_cluster_top_n(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow,
                            const int32_t* crows, int K, Pts U, const double* u_mean, int64_t nq, const int32_t* ucl,
                            const int64_t* unk_ptr, const int32_t* unk_idx, int n_top, double* scratch,
                            int64_t scratch_row, int nwaves, double* pred, int32_t* pidx, int32_t* out,
                            unsigned long long* soft_count) {
    if (nq <= 0) return 0;
    const unsigned grid = (unsigned)((nwaves + RC_WAVES - 1) / RC_WAVES);
    if (X.f64)
        hipLaunchKernelGGL(rc_cluster_top_n_kernel<double>, dim3(grid), dim3(64 * RC_WAVES), 0, s, X.d(), x_mean, d,
                           crow, crows, K, U.d(), u_mean, nq, ucl, unk_ptr, unk_idx, n_top, scratch, scratch_row, pred,
                           pidx, out, soft_count);
    else
        hipLaunchKernelGGL(rc_cluster_top_n_kernel<float>, dim3(grid), dim3(64 * RC_WAVES), 0, s, X.f(), x_mean, d,
                           crow, crows, K, U.f(), u_mean, nq, ucl, unk_ptr, unk_idx, n_top, scratch, scratch_row, pred,
                           pidx, out, soft_count);
    return kstatus("rc_cluster_top_n_kernel");
}

int launch_rc_shard_sims(hipStream_t s, Pts X, int d, const int64_t* crow, const int32_t* crows, int K, Pts U,
                        int64_t nq, const int32_t* ucl, const int64_t* unk_ptr, const int64_t* soff, double* sims,
                        unsigned long long* soft_count) {
    if (nq <= 0) return 0;
    const dim3 grid(gsz(nq, RC_WAVES, 2048));
    if (X.f64)
        hipLaunchKernelGGL(rc_shard_sims_kernel<double>, grid, dim3(64 * RC_WAVES), 0, s, X.d(), d, crow, crows, K,
                           U.d(), nq, ucl, unk_ptr, soff, sims, soft_count);
    else
        hipLaunchKernelGGL(rc_shard_sims_kernel<float>, grid, dim3(64 * RC_WAVES), 0, s, X.f(), d, crow, crows, K,
                           U.f(), nq, ucl, unk_ptr, soff, sims, soft_count);
    return kstatus("rc_shard_sims_kernel");
}

int launch_rc_shard_chain(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow, const int32_t* crows,
                          int K, int64_t nq, const int32_t* ucl, const double* u_mean, const int64_t* unk_ptr,
                          const int32_t* unk_idx, const int64_t* soff, const double* sims, const double* carry_main,
                          const double* carry_abs, const int64_t* carry_cnt, double* main_out, double* abs_out,
                          int64_t* cnt_out, int n_top, double* pred, int32_t* pidx, int32_t* out) {
    if (nq <= 0) return 0;
    const dim3 grid(gsz(nq, RC_WAVES, 2048));
    if (X.f64)
        hipLaunchKernelGGL(rc_shard_chain_kernel<double>, grid, dim3(64 * RC_WAVES), 0, s, X.d(), x_mean, d, crow,
                           crows, K, nq, ucl, u_mean, unk_ptr, unk_idx, soff, sims, carry_main, carry_abs, carry_cnt,
                           main_out, abs_out, cnt_out, n_top, pred, pidx, out);
    else
        hipLaunchKernelGGL(rc_shard_chain_kernel<float>, grid, dim3(64 * RC_WAVES), 0, s, X.f(), x_mean, d, crow,
                           crows, K, nq, ucl, u_mean, unk_ptr, unk_idx, soff, sims, carry_main, carry_abs, carry_cnt,
                           main_out, abs_out, cnt_out, n_top, pred, pidx, out);
    return kstatus("rc_shard_chain_kernel");
}

// ------------------------------------------------- terms form (round 4)
// The clustering recommender as two data-parallel phases instead of one wave
// per user (which walked ~10K members with lane-per-member row loads touching
// 64 lines per instruction, then the chains with 8 lanes of 64 busy):
//   rc_terms_cl_kernel: every (user, member) pair at once, 64 members of a
//     cluster per wave for all of the cluster's users (below);
//   rc_chain_terms_kernel: one thread per (user, unknown index) adds its terms
//     and the |sim| in member order (the reference's sequential chains,
//     :290-296), 64 values in flight, continued from / into the rank carry;
//   rc_top_kernel: one thread per user, the division, the quicksort and the
//     first N (:299-302, :341-343).
constexpr int CT_STAGE = 64;      // member rows staged per wave

// The certified similarity of the lane's staged row (8-B units, in dim order)
// against user row u8 (LDS when the wave's members share one user, else the
// lane's own global row); ok = false where the certificate declines.
// ub: the user's sum_j pow(u_j, 2) (rc_user_norm_kernel: the same chain, once
// per user instead of once per member). Called with u8 in LDS or in global
// memory, never a generic pointer (flat loads wait on both counters).
template <typename T>
__device__ inline double ct_sim(const uint64_t* myrow8, const uint64_t* u8, int nunit, double ub, bool& ok) {
    constexpr int PER = 8 / (int)sizeof(T);
    double xa = 0.0;
    IpAcc ip;
    auto step = [&](uint64_t xw, uint64_t uw) {
        T xv[PER], uv[PER];
        memcpy(xv, &xw, 8);
        memcpy(uv, &uw, 8);
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const double xj = (double)xv[k], uj = (double)uv[k];
            ip.add(__dmul_rn(xj, uj));
            xa = __dadd_rn(xa, sq_of<T>(xj));
        }
    };
    int w = 0;
    for (; w + 4 <= nunit; w += 4) {                // four units' reads in flight
        uint64_t xw[4], uw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { xw[k] = myrow8[w + k]; uw[k] = u8[w + k]; }
#pragma unroll
        for (int k = 0; k < 4; k++) step(xw[k], uw[k]);
    }
    for (; w < nunit; w++) step(myrow8[w], u8[w]);
    const double denom = __dmul_rn(sqrt(xa), sqrt(ub));
    double sv, qr;
    ok = ip.quot_status(denom, sv, qr) == 0;        // declined: rc_terms_fix_kernel decides
    return sv;
}

// The users' sum_j pow(u_j, 2) in j order (cosineSimilarity's |u|^2,
// cust_vector.hpp:166-170), lane per user.
template <typename T>
__global__ __launch_bounds__(256) void rc_user_norm_kernel(const T* __restrict__ U, int64_t nq, int d,
                                                           double* __restrict__ ub) {
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
        double b = 0.0;
        for (int j = 0; j < d; j++) b = __dadd_rn(b, sq_of<T>((double)U[q * d + j]));
        ub[q] = b;
    }
}

// Member g's user and dataset row (the pair space g = soff[q] + i; rc_terms_fix_kernel's lookups).
__global__ __launch_bounds__(256) void rc_member_map_kernel(int64_t nq, const int64_t* __restrict__ soff,
                                                            const int32_t* __restrict__ ucl,
                                                            const int64_t* __restrict__ crow,
                                                            const int32_t* __restrict__ crows,
                                                            int32_t* __restrict__ mem_q, int32_t* __restrict__ mem_r) {
    for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t b = soff[q], n = soff[q + 1] - b;
        if (n == 0) continue;
        const int32_t* cr = crows + crow[ucl[q]];
        for (int64_t i = threadIdx.x; i < n; i += 256) {
            mem_q[b + i] = (int32_t)q;
            mem_r[b + i] = cr[i];
        }
    }
}

// rc_terms_cl_kernel: a wave takes 64 members of one cluster, stages their
// rows through LDS by coalesced row loads once for every user of that cluster
// on this shard -- users sharing a cluster read its rows once, not once each
// (~1.6 users per distinct cluster at C5: 38 % fewer row bytes than one pass
// per (user, member) pair); per user and lane: cosineSimilarity (IpAcc
// certificate; declined ones listed for rc_terms_fix_kernel's x87 chain) and
// the terms of get_predicted_user_sim's main sums, t = sim * (x[index] - mean)
// (crypto_rec.hpp:296), one fp64 per (member, unknown index), at the pair
// index soff[q] + i (i = the member's index in its cluster).
// Item it: rc_item_meta_kernel's record (its group's cluster chunk and users);
// user k of the work list: rc_user_meta_kernel's record (its pair and term
// offsets, unknown indexes and |u|^2).
// Rows of at most 64 units (fp32 d <= 128) run as a software pipeline over the
// wave's items it_j = blockIdx.x + j * gridDim.x: every global load an item
// consumes is issued while the item before it is computed -- its member rows
// (unit `lane` of each), its mean values, its first CT_UMAX users' rows and
// unknown-index lists and its user records -- and the rest one or two items
// earlier (member row indexes, user records, item records). The vector memory
// counter retires in order, so a load issued after the next item's rows and
// consumed by this item would wait on all of them: the round-5 form issued
// this item's user rows and means after the next item's row loads and waited
// on those (45 % of its cycles waiting, profiles/round5_sq_c5_terms_v1.txt).
// Users past the first CT_UMAX of a group, or with more than 64 unknown
// indexes, take direct loads (correct, not pipelined).
constexpr int CT_UMAX = 4;        // users per item staged ahead
struct RcItem {
    int64_t mem0;      // crows index of the item's first member
    int32_t cnt;       // members in the item (1..64)
    int32_t i0;        // index of its first member in the cluster
    int32_t kb, ke;    // the group's users: work-list positions kb .. ke
    int32_t pad0, pad1;
};
static_assert(sizeof(RcItem) == 32, "RcItem: two 16-B loads");
struct RcUser {
    int64_t soff, toff, o;   // pair offset, term offset, unk_idx offset
    double unorm;            // sum_j pow(u_j, 2)
    int32_t q, m;            // user index, unknown indexes
    int32_t qlow, pad;       // min_j lowbit_exp(u_j) (exact.h; LOWBIT_NONE: an all-zero row)
};
static_assert(sizeof(RcUser) == 48, "RcUser: three 16-B loads");

__global__ __launch_bounds__(256) void rc_item_meta_kernel(const int32_t* __restrict__ ioff, int ngroups, int64_t nitems,
                                                           const int32_t* __restrict__ gcl,
                                                           const int32_t* __restrict__ gptr,
                                                           const int64_t* __restrict__ crow, RcItem* __restrict__ items) {
    for (int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x; it < nitems; it += (int64_t)gridDim.x * 256) {
        int lo = 0, hi = ngroups;                    // the last g with ioff[g] <= it
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (ioff[mid] <= it) lo = mid; else hi = mid;
        }
        const int i0 = (int)(it - ioff[lo]) * CT_STAGE;
        const int64_t cb = crow[gcl[lo]], n = crow[gcl[lo] + 1] - cb;
        RcItem m;
        m.mem0 = cb + i0;
        m.cnt = (int32_t)(n - i0 < CT_STAGE ? n - i0 : CT_STAGE);
        m.i0 = i0;
        m.kb = gptr[lo];
        m.ke = gptr[lo + 1];
        m.pad0 = m.pad1 = 0;
        items[it] = m;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void rc_user_meta_kernel(const T* __restrict__ U, int d,
                                                           const int32_t* __restrict__ gusr, int64_t nusers,
                                                           const int64_t* __restrict__ soff,
                                                           const int64_t* __restrict__ toff,
                                                           const int64_t* __restrict__ unk_ptr,
                                                           const double* __restrict__ unorm, RcUser* __restrict__ users) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nusers; k += (int64_t)gridDim.x * 256) {
        const int q = gusr[k];
        RcUser u;
        u.soff = soff[q];
        u.toff = toff[q];
        u.o = unk_ptr[q];
        u.m = (int32_t)(unk_ptr[q + 1] - u.o);
        u.unorm = unorm[q];
        u.q = q;
        int ql = LOWBIT_NONE;
        for (int j = 0; j < d; j++) ql = min(ql, lowbit_exp(U[(int64_t)q * d + j]));
        u.qlow = ql;
        u.pad = 0;
        users[k] = u;
    }
}

// ct_sim with the row reads one 4-unit block ahead of the arithmetic (the
// round-5 loop waited on each block's LDS reads), and the member's |x|^2 taken
// from the item's first user (XA) instead of recomputed per user.
// The member's lowest-bit bound qx (XA pass, with |x|^2) and the user's qu
// certify a never-rounding x87 chain (exact.h ip_never_rounds): then the
// quotient's status drops the chain's rounding bound, which alone declined
// ~6-12 % of pairs (a 2^-58 relative R against a 2^-53 half ulp).
// Plain fp64 chain (ct_exact53): when every partial sum of the products is a
// multiple of 2^(qx + qu) below 2^T with T - (qx + qu) <= 53 -- T from the
// Cauchy-Schwarz bound sqrt(xa ub) >= sum_j |x_j u_j| >= max_k |S_k| -- every
// add of the chain is exact in fp64 as it is in the x87 chain: the sum is
// exact in one fma per element (fp32 rows: the products are exact doubles)
// instead of IpAcc's TwoSum (~10 fp64 ops), and it is ip87 itself.
template <typename T>
__device__ inline bool ct_exact53(double xa, double ub, int qx, int qu, double& bnd) {
    // fp64 rows: the rounded products |RN(x u)| <= |x u| (1 + 2^-53)
    bnd = sqrt(xa) * sqrt(ub) * (1.0 + 0x1p-40);
    if (qx >= LOWBIT_NONE || qu >= LOWBIT_NONE) return true;     // a zero row: every product 0
    if (!(bnd > 0.0 && bnd < 0x1p1000)) return false;
    return ilogb(bnd) + 1 - (qx + qu) <= 53;
}

template <typename T, bool XA>
__device__ inline double ct_sim_pl(const uint64_t* myrow8, const uint64_t* u8, int nunit, double ub, double& xa,
                                   int& qx, int qu, bool& ok) {
    constexpr int PER = 8 / (int)sizeof(T);
    if (XA) {
        // the member's sum_j pow(x_j, 2) in j order and its lowest set bit, once per member
        double xs = 0.0;
        int ql = LOWBIT_NONE;
        auto xstep = [&](uint64_t xw) {
            T xv[PER];
            memcpy(xv, &xw, 8);
#pragma unroll
            for (int k = 0; k < PER; k++) {
                xs = __dadd_rn(xs, sq_of<T>((double)xv[k]));
                ql = min(ql, lowbit_exp(xv[k]));
            }
        };
        int w = 0;
        for (; w + 4 <= nunit; w += 4) {
            uint64_t xw[4];
#pragma unroll
            for (int k = 0; k < 4; k++) xw[k] = myrow8[w + k];
#pragma unroll
            for (int k = 0; k < 4; k++) xstep(xw[k]);
        }
        for (; w < nunit; w++) xstep(myrow8[w]);
        xa = xs;
        qx = ql;
    }
    const double denom = __dmul_rn(sqrt(xa), sqrt(ub));
    double bnd;
    double sv = 0.0, qr;
    if (ct_exact53<T>(xa, ub, qx, qu, bnd)) {
        double s = 0.0;
        auto step = [&](uint64_t xw, uint64_t uw) {
            T xv[PER], uv[PER];
            memcpy(xv, &xw, 8);
            memcpy(uv, &uw, 8);
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const double xj = (double)xv[k], uj = (double)uv[k];
                if constexpr (sizeof(T) == 4) s = fma(xj, uj, s);          // exact product, exact sum
                else s = __dadd_rn(s, __dmul_rn(xj, uj));                  // the reference's rounded product
            }
        };
        int w = 0;
        for (; w + 4 <= nunit; w += 4) {
            uint64_t xw[4], uw[4];
#pragma unroll
            for (int k = 0; k < 4; k++) { xw[k] = myrow8[w + k]; uw[k] = u8[w + k]; }
#pragma unroll
            for (int k = 0; k < 4; k++) step(xw[k], uw[k]);
        }
        for (; w < nunit; w++) step(myrow8[w], u8[w]);
        IpAcc ip;
        ip.sh = s;
        ip.mx = bnd;
        ok = ip.quot_status(denom, sv, qr, true) == 0;
        return sv;
    }
    IpAcc ip;
    auto step = [&](uint64_t xw, uint64_t uw) {
        T xv[PER], uv[PER];
        memcpy(xv, &xw, 8);
        memcpy(uv, &uw, 8);
#pragma unroll
        for (int k = 0; k < PER; k++) ip.add(__dmul_rn((double)xv[k], (double)uv[k]));
    };
    int w = 0;
    if (nunit >= 4) {
        uint64_t xc[4], uc[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { xc[k] = myrow8[k]; uc[k] = u8[k]; }
        for (; w + 8 <= nunit; w += 4) {
            uint64_t xn[4], un[4];
#pragma unroll
            for (int k = 0; k < 4; k++) { xn[k] = myrow8[w + 4 + k]; un[k] = u8[w + 4 + k]; }
#pragma unroll
            for (int k = 0; k < 4; k++) step(xc[k], uc[k]);
#pragma unroll
            for (int k = 0; k < 4; k++) { xc[k] = xn[k]; uc[k] = un[k]; }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) step(xc[k], uc[k]);
        w += 4;
    }
    for (; w < nunit; w++) step(myrow8[w], u8[w]);
    const bool exact = ip_never_rounds(ip.mx, min(qx, LOWBIT_NONE) + min(qu, LOWBIT_NONE));
    ok = ip.quot_status(denom, sv, qr, exact) == 0;     // declined: rc_terms_fix_kernel decides
    return sv;
}

__device__ inline int64_t rl64(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l);
    const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline double rld(double v, int l) { return __longlong_as_double(rl64(__double_as_longlong(v), l)); }

template <typename T>
__global__ __launch_bounds__(64) void rc_terms_cl_kernel(
    const T* __restrict__ X, const double* __restrict__ x_mean, int d, const T* __restrict__ U,
    const RcItem* __restrict__ items, int64_t nitems, const RcUser* __restrict__ users,
    const int32_t* __restrict__ crows, const int32_t* __restrict__ unk_idx, double* __restrict__ sims,
    double* __restrict__ terms, int stride8, int64_t* __restrict__ fix_region, const int64_t* __restrict__ fix_cap,
    int64_t* __restrict__ fix_cnt) {
    constexpr int SB = 16;                          // rows per staging batch (loads in flight)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x;
    const int nunit = (int)((int64_t)d * (int64_t)sizeof(T) / 8);
    uint64_t* stage = reinterpret_cast<uint64_t*>(smem);
    uint64_t* ustage = stage + (size_t)CT_STAGE * stride8;      // CT_UMAX + 1 user rows
    const uint64_t* myrow8 = stage + (size_t)lane * stride8;
    const int64_t G = gridDim.x;
    const bool pfok = nunit <= 64;
    const int ul = lane < nunit ? lane : nunit - 1;              // this lane's unit (clamped: no branch per load)
    auto meta = [&](int64_t it_) { return items[it_ < nitems ? it_ : nitems - 1]; };
    auto member_row = [&](const RcItem& m) { return crows[m.mem0 + (lane < m.cnt ? lane : m.cnt - 1)]; };
    // lane u: the record of the item's user u (clamped to its last)
    auto user_rec = [&](const RcItem& m) { return users[m.kb + (lane < m.ke - m.kb ? lane : m.ke - m.kb - 1)]; };
    uint64_t pf[CT_STAGE];
    auto issue_pf = [&](int32_t rr) {
#pragma unroll
        for (int t = 0; t < CT_STAGE; t++) {
            const int rt = __builtin_amdgcn_readlane(rr, t);
            pf[t] = reinterpret_cast<const uint64_t*>(X + (int64_t)rt * d)[ul];
        }
    };
    // the first CT_UMAX users' rows (unit `lane`) and unknown-index lists (lane e: index e)
    uint64_t up0[CT_UMAX], up1[CT_UMAX];
    int32_t ux0[CT_UMAX], ux1[CT_UMAX];
    auto issue_users = [&](const RcItem& m, const RcUser& ur, uint64_t (&up)[CT_UMAX], int32_t (&ux)[CT_UMAX]) {
#pragma unroll
        for (int u = 0; u < CT_UMAX; u++) {
            const int uu = u < m.ke - m.kb ? u : 0;
            const int q = __builtin_amdgcn_readlane(ur.q, uu);
            const int mm = __builtin_amdgcn_readlane(ur.m, uu);
            const int64_t o = rl64(ur.o, uu);
            if (pfok) up[u] = reinterpret_cast<const uint64_t*>(U + (int64_t)q * d)[ul];
            ux[u] = terms && mm > 0 ? unk_idx[o + (lane < mm ? lane : mm - 1)] : 0;
        }
    };
    const int64_t it0 = blockIdx.x;
    if (it0 >= nitems) return;
    // this block's private decline list: fix_region[rbase ..), its capacity the
    // pairs of its items (rc_block_cap_kernel) -- no shared counter: one atomic
    // per (item, user) pass on a single word serialised at ~12 ns each, ~1.9 ms
    // over the ~160K passes of a C5 call, was the round-5 kernel's floor
    int64_t rbase = 0;
    for (int b = lane; b < (int)blockIdx.x; b += 64) rbase += fix_cap[b];
    for (int off = 32; off >= 1; off >>= 1) rbase += __shfl_xor(rbase, off);
    int64_t nloc = 0;
    // pipeline fill: item 0's loads, then item 1's that the loop expects in flight
    RcItem m0 = meta(it0), m1 = meta(it0 + G), m2 = meta(it0 + 2 * G);
    int32_t r0 = member_row(m0), r1 = member_row(m1);
    RcUser ub0 = user_rec(m0), ub1 = user_rec(m1);
    if (pfok) issue_pf(r0);
    issue_users(m0, ub0, up0, ux0);
    double mean0 = x_mean[r0];
    for (int64_t it = it0; it < nitems; it += G) {
        const bool on = lane < m0.cnt;
        const bool more = it + G < nitems;
        const int nu = m0.ke - m0.kb;
        __syncthreads();                            // the previous item's reads of the stage are done
        if (pfok) {
#pragma unroll
            for (int t = 0; t < CT_STAGE; t++)
                if (lane < nunit) stage[(size_t)t * stride8 + lane] = pf[t];
#pragma unroll
            for (int u = 0; u < CT_UMAX; u++)
                if (u < nu && lane < nunit) ustage[(size_t)u * stride8 + lane] = up0[u];
        } else {
            for (int t0 = 0; t0 < CT_STAGE; t0 += SB) {
                for (int u0 = 0; u0 < nunit; u0 += 64) {
                    const bool uon = u0 + lane < nunit;
                    uint64_t v[SB];
#pragma unroll
                    for (int k = 0; k < SB; k++) {
                        const int rt = __builtin_amdgcn_readlane(r0, t0 + k);
                        v[k] = uon ? reinterpret_cast<const uint64_t*>(X + (int64_t)rt * d)[u0 + lane] : 0ull;
                    }
#pragma unroll
                    for (int k = 0; k < SB; k++)
                        if (uon) stage[(size_t)(t0 + k) * stride8 + u0 + lane] = v[k];
                }
            }
        }
        // loads for the items ahead (consumed an item or more later; see above)
        if (pfok && more) issue_pf(r1);
        if (more) issue_users(m1, ub1, up1, ux1);
        const double mean1 = x_mean[r1];
        const int32_t r2 = member_row(m2);
        const RcUser ub2 = user_rec(m2);
        const RcItem m3 = meta(it + 3 * G);
        const T* xr = reinterpret_cast<const T*>(myrow8);
        double xa = 0.0;
        int qx = LOWBIT_NONE;
        for (int u = 0; u < nu; u++) {
            const int q = __builtin_amdgcn_readlane(ub0.q, u < 64 ? u : 0);
            const uint64_t* urow = ustage + (size_t)(pfok && u < CT_UMAX ? u : CT_UMAX) * stride8;
            int64_t soffq, toffq, o;
            double unq;
            int m, qu;
            if (u < 64) {
                soffq = rl64(ub0.soff, u); toffq = rl64(ub0.toff, u); o = rl64(ub0.o, u);
                unq = rld(ub0.unorm, u); m = __builtin_amdgcn_readlane(ub0.m, u);
                qu = __builtin_amdgcn_readlane(ub0.qlow, u);
            } else {
                const RcUser r = users[m0.kb + u];
                soffq = r.soff; toffq = r.toff; o = r.o; unq = r.unorm; m = r.m; qu = r.qlow;
            }
            const int qq = u < 64 ? q : users[m0.kb + u].q;
            if (u >= CT_UMAX || !pfok) {            // direct: the row into the spare slot
                __syncthreads();
                for (int u0 = lane; u0 < nunit; u0 += 64)
                    ustage[(size_t)CT_UMAX * stride8 + u0] = reinterpret_cast<const uint64_t*>(U + (int64_t)qq * d)[u0];
            }
            __syncthreads();
            bool ok;
            const double sv = u == 0 ? ct_sim_pl<T, true>(myrow8, urow, nunit, unq, xa, qx, qu, ok)
                                     : ct_sim_pl<T, false>(myrow8, urow, nunit, unq, xa, qx, qu, ok);
            const int64_t i = m0.i0 + lane;
            const int64_t g = soffq + i;
            const unsigned long long dm = __ballot(on && !ok);
            if (on && !ok) fix_region[rbase + nloc + __popcll(dm & ((1ull << lane) - 1ull))] = g;
            nloc += __popcll(dm);
            const bool wr = on && ok;
            if (wr) sims[g] = sv;
            if (terms) {
                // the index list is read across lanes (readlane ignores EXEC, so
                // every lane's copy is selected and read in uniform control flow;
                // only the stores are predicated)
                double* tq = terms + toffq + i * m;             // member-major: the pair's m terms together
                int32_t uxv = ux0[0];
#pragma unroll
                for (int uu = 1; uu < CT_UMAX; uu++)
                    if (uu == u) uxv = ux0[uu];
                if (u < CT_UMAX && m <= 64) {
                    for (int e = 0; e < m; e++) {
                        const double t = __dmul_rn(sv, __dsub_rn((double)xr[__builtin_amdgcn_readlane(uxv, e)], mean0));
                        if (wr) tq[e] = t;
                    }
                } else {
                    for (int e = 0; e < m; e++) {
                        const double t = __dmul_rn(sv, __dsub_rn((double)xr[unk_idx[o + e]], mean0));
                        if (wr) tq[e] = t;
                    }
                }
            }
        }
        m0 = m1; m1 = m2; m2 = m3;
        r0 = r1; r1 = r2;
        ub0 = ub1; ub1 = ub2;
        mean0 = mean1;
#pragma unroll
        for (int u = 0; u < CT_UMAX; u++) { up0[u] = up1[u]; ux0[u] = ux1[u]; }
    }
    if (lane == 0) fix_cnt[blockIdx.x] = nloc;
}

// Block b of the terms grid (G blocks): the pairs of its items it = b, b + G, ...
// -- the capacity of its private decline list.
__global__ __launch_bounds__(256) void rc_block_cap_kernel(const RcItem* __restrict__ items, int64_t nitems, int G,
                                                           int64_t* __restrict__ cap) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= G) return;
    int64_t c = 0;
    for (int64_t it = b; it < nitems; it += G) {
        const RcItem m = items[it];
        c += (int64_t)m.cnt * (m.ke - m.kb);
    }
    cap[b] = c;
}

// The blocks' private lists into one dense list in block order (fix_list,
// *fix_count), for rc_terms_fix_kernel: block b (one wave) copies its count.
__global__ __launch_bounds__(64) void rc_fix_gather_kernel(const int64_t* __restrict__ cap,
                                                           const int64_t* __restrict__ cnt, int G,
                                                           const int64_t* __restrict__ region,
                                                           int64_t* __restrict__ fix_list,
                                                           unsigned long long* __restrict__ fix_count) {
    const int b = blockIdx.x, lane = threadIdx.x;
    int64_t rs = 0, ds = 0, tot = 0;
    for (int k = lane; k < G; k += 64) {
        const int64_t c = cnt[k];
        if (k < b) { rs += cap[k]; ds += c; }
        tot += c;
    }
    for (int off = 32; off >= 1; off >>= 1) {
        rs += __shfl_xor(rs, off);
        ds += __shfl_xor(ds, off);
        tot += __shfl_xor(tot, off);
    }
    if (b == 0 && lane == 0) *fix_count = (unsigned long long)tot;
    const int64_t n = cnt[b];
    for (int64_t i = lane; i < n; i += 64) fix_list[ds + i] = region[rs + i];
}

// The listed members: cosineSimilarity by the x87 chain (softx87.h X87acc),
// lane per member, 64 members per wave with their rows and their users' rows
// staged through LDS (coalesced row loads, as rc_terms_cl_kernel), then the terms;
// soft_count += the list length.
template <typename T>
__global__ __launch_bounds__(64) void rc_terms_fix_kernel(
    const T* __restrict__ X, const double* __restrict__ x_mean, int d, const T* __restrict__ U,
    const int32_t* __restrict__ mem_q, const int32_t* __restrict__ mem_r, const int64_t* __restrict__ soff,
    const int64_t* __restrict__ unk_ptr, const int32_t* __restrict__ unk_idx, const int64_t* __restrict__ toff,
    double* __restrict__ sims, double* __restrict__ terms, const int64_t* __restrict__ fix_list,
    const unsigned long long* __restrict__ fix_count, int stride8, unsigned long long* __restrict__ soft_count,
    const double* __restrict__ unorm) {
    constexpr int SB = 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x;
    const int nunit = (int)((int64_t)d * (int64_t)sizeof(T) / 8);
    uint64_t* xs = reinterpret_cast<uint64_t*>(smem);
    uint64_t* us = xs + (size_t)CT_STAGE * stride8;
    const T* myx = reinterpret_cast<const T*>(xs + (size_t)lane * stride8);
    const T* myu = reinterpret_cast<const T*>(us + (size_t)lane * stride8);
    const int64_t nfix = (int64_t)*fix_count;
    if (blockIdx.x == 0 && lane == 0 && soft_count && nfix) atomicAdd(soft_count, (unsigned long long)nfix);
    for (int64_t k0 = (int64_t)blockIdx.x * CT_STAGE; k0 < nfix; k0 += (int64_t)gridDim.x * CT_STAGE) {
        const bool on = k0 + lane < nfix;
        const int64_t g = fix_list[min(k0 + lane, nfix - 1)];
        const int q = mem_q[g];
        const int32_t r = mem_r[g];
        __syncthreads();
        for (int t0 = 0; t0 < CT_STAGE; t0 += SB) {
            for (int u0 = 0; u0 < nunit; u0 += 64) {
                const bool uon = u0 + lane < nunit;
                uint64_t vx[SB], vu[SB];
#pragma unroll
                for (int k = 0; k < SB; k++) {
                    const int rt = __builtin_amdgcn_readlane(r, t0 + k), qt = __builtin_amdgcn_readlane(q, t0 + k);
                    vx[k] = uon ? reinterpret_cast<const uint64_t*>(X + (int64_t)rt * d)[u0 + lane] : 0ull;
                    vu[k] = uon ? reinterpret_cast<const uint64_t*>(U + (int64_t)qt * d)[u0 + lane] : 0ull;
                }
#pragma unroll
                for (int k = 0; k < SB; k++)
                    if (uon) {
                        xs[(size_t)(t0 + k) * stride8 + u0 + lane] = vx[k];
                        us[(size_t)(t0 + k) * stride8 + u0 + lane] = vu[k];
                    }
            }
        }
        __syncthreads();
        double xa = 0.0;
        const double ub = unorm[q];
        X87acc ip;
        ip.init();
        for (int j = 0; j < d; j++) {
            const double xj = (double)myx[j], uj = (double)myu[j];
            ip.add(__dmul_rn(xj, uj));
            xa = __dadd_rn(xa, sq_of<T>(xj));
        }
        const double sv = x87_quot(ip.value(), __dmul_rn(sqrt(xa), sqrt(ub)));
        if (!on) continue;
        sims[g] = sv;
        if (terms) {
            const int64_t o = unk_ptr[q];
            const int m = (int)(unk_ptr[q + 1] - o);
            const int64_t i = g - soff[q];
            const double mean = x_mean[r];
            double* tq = terms + toff[q] + i * m;
            for (int e = 0; e < m; e++) tq[e] = __dmul_rn(sv, __dsub_rn((double)myx[unk_idx[o + e]], mean));
        }
    }
}

// One wave per user q: its get_predicted_user_sim chains (crypto_rec.hpp:290-296)
// -- per unknown index e, main_e = sum_i sim_i * (x_i[e] - mean_i), and the
// |sim| sum -- each one sequential fp64 adds in member order, as the
// reference's. The wave streams 64 members at a time (the sims coalesced, the
// block's terms member-major: 64 x m contiguous doubles per user), transposes
// the block through LDS, and lane k adds chain k's 64 values in order (lane
// RC_CH: the |sim| chain), the next block's loads in flight meanwhile (the
// round-4 form, one thread per chain reading its own stream, waited on ~20K
// dependent loads per thread with 128 waves on the chip). Users with more than
// RC_CH unknown indexes run their chains in groups (|sim| with the first).
// carry_*: the previous rank's sums (NULL: first rank); pred == NULL: the
// running sums out, else the predictions (:299-302).
constexpr int RC_CH = 8;                  // chains per group
constexpr int RC_LS = 65;                 // LDS row stride (doubles; reads run to t0 + 15 <= 63)
constexpr int RC_PF = 4;                  // blocks of 64 members in flight
__global__ __launch_bounds__(64) void rc_chain_user_kernel(
    int64_t nq, const int64_t* __restrict__ soff, const int64_t* __restrict__ unk_ptr,
    const int64_t* __restrict__ toff, const double* __restrict__ sims, const double* __restrict__ terms,
    const double* __restrict__ carry_main, const double* __restrict__ carry_abs,
    const int64_t* __restrict__ carry_cnt, const double* __restrict__ u_mean, double* __restrict__ main_out,
    double* __restrict__ abs_out, int64_t* __restrict__ cnt_out, double* __restrict__ pred, int64_t long_min) {
    __shared__ double blk[(RC_CH + 1) * RC_LS];
    __shared__ double as_sh;
    const int lane = threadIdx.x;
    for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t b0 = soff[q], n = soff[q + 1] - b0;
        if (n >= long_min) continue;                   // a huge cluster: the segmented chains (rc_long_*)
        const int64_t u0 = unk_ptr[q];
        const int m = (int)(unk_ptr[q + 1] - u0);
        const double* sp = sims + b0;
        const double* tq = terms + toff[q];
        for (int c0 = 0; c0 < (m > 0 ? m : 1); c0 += RC_CH) {
            const int nc = min(RC_CH, m - c0);                 // chains of this group (<= 0: none)
            const bool first = c0 == 0;
            const bool mine = lane < nc;
            const bool absl = lane == RC_CH && first;
            double acc = 0.0;
            if (mine) acc = carry_main ? carry_main[u0 + c0 + lane] : 0.0;
            if (absl) acc = carry_abs ? carry_abs[q] : 0.0;
            // v[k]: chain c0 + k's value of member i0 + lane (k < nc); v[RC_CH]: its sim
            auto load_blk = [&](int64_t i0, double (&v)[RC_CH + 1]) {
                const int64_t i = min(i0 + lane, n - 1);
#pragma unroll
                for (int k = 0; k < RC_CH; k++) v[k] = k < nc ? tq[i * m + c0 + k] : 0.0;
                v[RC_CH] = first ? sp[i] : 0.0;
            };
            if (n > 0) {
                // a ring of RC_PF blocks in flight (one block's adds take ~0.5 us,
                // a load round trip several); the LDS reads of a chain in
                // batches of 16 ahead of their dependent adds
                double ring[RC_PF][RC_CH + 1];
#pragma unroll
                for (int p = 0; p < RC_PF; p++)
                    if ((int64_t)p * 64 < n) load_blk((int64_t)p * 64, ring[p]);
                for (int64_t i0 = 0; i0 < n; i0 += 64 * RC_PF) {
#pragma unroll
                    for (int p = 0; p < RC_PF; p++) {
                        const int64_t ib = i0 + (int64_t)p * 64;
                        if (ib >= n) break;                       // wave-uniform
#pragma unroll
                        for (int k = 0; k <= RC_CH; k++) blk[k * RC_LS + lane] = ring[p][k];
                        __syncthreads();
                        if (ib + 64 * RC_PF < n) load_blk(ib + 64 * RC_PF, ring[p]);
                        const int cnt = (int)min((int64_t)64, n - ib);
                        if (mine || absl) {
                            const double* row = blk + lane * RC_LS;
                            for (int t0 = 0; t0 < cnt; t0 += 16) {
                                double v[16];
#pragma unroll
                                for (int k = 0; k < 16; k++) v[k] = row[t0 + k];   // < RC_LS: in the row
#pragma unroll
                                for (int k = 0; k < 16; k++)
                                    if (t0 + k < cnt) acc = __dadd_rn(acc, mine ? v[k] : fabs(v[k]));
                            }
                        }
                        __syncthreads();
                    }
                }
            }
            // the |sim| sum to every lane (each prediction divides by it)
            if (absl) as_sh = acc;
            __syncthreads();
            const double as = as_sh;
            if (pred) {
                if (mine) pred[u0 + c0 + lane] = __dadd_rn(__ddiv_rn(acc, as), u_mean[q]);
            } else {
                if (mine) main_out[u0 + c0 + lane] = acc;
                if (absl) {
                    abs_out[q] = acc;
                    cnt_out[q] = (carry_cnt ? carry_cnt[q] : 0) + n;
                }
            }
            __syncthreads();
        }
    }
}

// A user of a huge cluster (n >= RC_LONG_MIN members on this shard): its chains
// were evaluated by binade segments (launch_seg_columns: the terms block [n][m]
// -> sums [m], the |sim| copy [n][1] -> its sum); the same outputs as
// rc_chain_user_kernel from them.
// V [rows][D]: user k's member r at row off_k + r -- its m_k terms, zeros, then
// |sim| in column D - 1 (blockIdx.y = k)
__global__ void rc_long_pack_kernel(const RcLongUser* __restrict__ tab, int D, const double* __restrict__ sims,
                                    const double* __restrict__ terms, double* __restrict__ V) {
    const RcLongUser u = tab[blockIdx.y];
    const int64_t tot = u.n * D;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / D;
        const int e = (int)(i - r * D);
        const double v = e < u.m ? terms[u.toff + r * u.m + e] : (e == D - 1 ? fabs(sims[u.b0 + r]) : 0.0);
        V[(u.off + r) * D + e] = v;
    }
}

__global__ void rc_long_carry_kernel(const RcLongUser* __restrict__ tab, int64_t nlong, int D,
                                     const double* __restrict__ carry_main, const double* __restrict__ carry_abs,
                                     double* __restrict__ carry) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlong * D) return;
    const RcLongUser u = tab[i / D];
    const int e = (int)(i % D);
    carry[i] = e < u.m ? carry_main[u.u0 + e] : (e == D - 1 ? carry_abs[u.q] : 0.0);
}

// user k = blockIdx.x: rc_chain_user_kernel's outputs from its column sums
__global__ void rc_long_finish_kernel(const RcLongUser* __restrict__ tab, int D, const double* __restrict__ sums,
                                      const int64_t* __restrict__ carry_cnt, const double* __restrict__ u_mean,
                                      double* __restrict__ main_out, double* __restrict__ abs_out,
                                      int64_t* __restrict__ cnt_out, double* __restrict__ pred) {
    const RcLongUser u = tab[blockIdx.x];
    const double* sk = sums + (size_t)blockIdx.x * D;
    const double as = sk[D - 1];
    for (int e = threadIdx.x; e < u.m; e += blockDim.x) {
        if (pred) pred[u.u0 + e] = __dadd_rn(__ddiv_rn(sk[e], as), u_mean[u.q]);
        else main_out[u.u0 + e] = sk[e];
    }
    if (!pred && threadIdx.x == 0) {
        abs_out[u.q] = as;
        cnt_out[u.q] = (carry_cnt ? carry_cnt[u.q] : 0) + u.n;
    }
}

// One thread per user: the quicksort of its predictions (:341) and the first
// n_top unknown indexes, 0-padded (:343); -1 rows for users whose cluster is
// empty on every rank (main.cpp:262 / :366 skip them).
__global__ __launch_bounds__(64) void rc_top_kernel(int64_t nq, const int64_t* __restrict__ soff,
                                                    const int64_t* __restrict__ carry_cnt,
                                                    const int64_t* __restrict__ unk_ptr,
                                                    const int32_t* __restrict__ unk_idx, double* __restrict__ pred,
                                                    int32_t* __restrict__ pidx, int n_top, int32_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (q >= nq) return;
    const int64_t cnt = (carry_cnt ? carry_cnt[q] : 0) + soff[q + 1] - soff[q];
    if (cnt == 0) {
        for (int i = 0; i < n_top; i++) out[q * n_top + i] = -1;
        return;
    }
    const int64_t o = unk_ptr[q];
    const int m = (int)(unk_ptr[q + 1] - o);
    for (int e = 0; e < m; e++) pidx[o + e] = unk_idx[o + e];
    if (m > 0) lomuto_sort(pred + o, pidx + o, m);
    for (int i = 0; i < n_top; i++) out[q * n_top + i] = i < m ? pidx[o + i] : 0;
}

int rc_terms_stride8(int d, int elem) { return (int)(((int64_t)d * elem + 7) / 8) + 1; }

int launch_rc_terms(hipStream_t s, Pts X, const double* x_mean, int d, const int64_t* crow, const int32_t* crows,
                    int K, Pts U, int64_t nq, const int32_t* ucl, const int64_t* soff, int64_t total,
                    const int64_t* unk_ptr, const int32_t* unk_idx, const int64_t* toff, double* sims, double* terms,
                    int32_t* mem_q, int32_t* mem_r, int64_t* fix_list, unsigned long long* fix_count,
                    unsigned long long* soft_count, double* unorm, const RcGroups* groups, int64_t* fix_region,
                    int64_t* fix_aux) {
    if (nq <= 0 || total <= 0) return 0;
    const int elem = X.f64 ? 8 : 4;
    const int stride8 = rc_terms_stride8(d, elem);
    const size_t lds = (size_t)(CT_STAGE + 1) * stride8 * 8;
    const size_t lds_cl = (size_t)(CT_STAGE + CT_UMAX + 1) * stride8 * 8;   // rows | the users' rows | a spare
    // every check before the first launch: a refused call enqueues nothing
    if (((int64_t)d * elem) % 8 != 0 || 2 * lds > 160 * 1024 || lds_cl > 160 * 1024) {
        set_error("launch_rc_terms: rows must be a multiple of 8 B and stage in LDS");
        return LSHKM_ERR_ARG;
    }
    if (!groups || groups->nitems <= 0 || groups->nusers <= 0 || !groups->items || !groups->users ||
        ((uintptr_t)groups->items & 15) != 0 || ((uintptr_t)groups->users & 15) != 0 || !fix_region || !fix_aux) {
        set_error("launch_rc_terms: empty cluster-major work list (or no 16-B aligned item records) for a nonzero member total");
        return LSHKM_ERR_ARG;
    }
    hipLaunchKernelGGL(rc_member_map_kernel, dim3((unsigned)std::min<int64_t>(nq, 4096)), dim3(256), 0, s, nq, soff, ucl,
                       crow, crows, mem_q, mem_r);
    if (X.f64)
        hipLaunchKernelGGL(rc_user_norm_kernel<double>, dim3(gsz(nq, 256, 1024)), dim3(256), 0, s, U.d(), nq, d, unorm);
    else
        hipLaunchKernelGGL(rc_user_norm_kernel<float>, dim3(gsz(nq, 256, 1024)), dim3(256), 0, s, U.f(), nq, d, unorm);
    // persistent: the resident waves (LDS-limited) times 2, each walking its
    // items as a pipeline (a grid of 65,536 one-item blocks would pay the
    // pipeline's fill per block)
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return kstatus("launch_rc_terms (device)");
    if (dev < 64 && !cus[dev] &&
        hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return kstatus("launch_rc_terms (CU count)");
    const int64_t per_cu = std::max<int64_t>(1, (int64_t)(160 * 1024) / (int64_t)lds_cl);
    const int64_t resident = (dev < 64 && cus[dev] > 0 ? cus[dev] : 256) * per_cu;
    const dim3 cgrid((unsigned)std::min<int64_t>(
        {groups->nitems, (int64_t)RC_TERMS_GMAX, test_switch("LSHKM_TERMS_GRID", "r4") ? 4 * resident : 2 * resident}));
    RcItem* items = reinterpret_cast<RcItem*>(groups->items);
    RcUser* users = reinterpret_cast<RcUser*>(groups->users);
    hipLaunchKernelGGL(rc_item_meta_kernel, dim3(gsz(groups->nitems, 256, 4096)), dim3(256), 0, s, groups->ioff,
                       groups->ngroups, groups->nitems, groups->gcl, groups->gptr, crow, items);
    if (X.f64)
        hipLaunchKernelGGL(rc_user_meta_kernel<double>, dim3(gsz(groups->nusers, 256, 1024)), dim3(256), 0, s, U.d(), d,
                           groups->gusr, groups->nusers, soff, toff, unk_ptr, unorm, users);
    else
        hipLaunchKernelGGL(rc_user_meta_kernel<float>, dim3(gsz(groups->nusers, 256, 1024)), dim3(256), 0, s, U.f(), d,
                           groups->gusr, groups->nusers, soff, toff, unk_ptr, unorm, users);
    const int G = (int)cgrid.x;
    int64_t* fcap = fix_aux;
    int64_t* fcnt = fix_aux + RC_TERMS_GMAX;
    hipLaunchKernelGGL(rc_block_cap_kernel, dim3((unsigned)((G + 255) / 256)), dim3(256), 0, s, items, groups->nitems, G,
                       fcap);
    if (X.f64)
        hipLaunchKernelGGL(rc_terms_cl_kernel<double>, cgrid, dim3(64), lds_cl, s, X.d(), x_mean, d, U.d(), items,
                           groups->nitems, users, crows, unk_idx, sims, terms, stride8, fix_region, fcap, fcnt);
    else
        hipLaunchKernelGGL(rc_terms_cl_kernel<float>, cgrid, dim3(64), lds_cl, s, X.f(), x_mean, d, U.f(), items,
                           groups->nitems, users, crows, unk_idx, sims, terms, stride8, fix_region, fcap, fcnt);
    hipLaunchKernelGGL(rc_fix_gather_kernel, dim3((unsigned)G), dim3(64), 0, s, fcap, fcnt, G, fix_region, fix_list,
                       fix_count);
    // the list length is on the device: a grid for up to ~1/4 of the pairs, looping beyond
    const dim3 fgrid(gsz(total / 4 + 1, CT_STAGE, 2048));
    const size_t flds = 2 * lds;
    if (X.f64)
        hipLaunchKernelGGL(rc_terms_fix_kernel<double>, fgrid, dim3(64), flds, s, X.d(), x_mean, d, U.d(), mem_q, mem_r,
                           soff, unk_ptr, unk_idx, toff, sims, terms, fix_list, fix_count, stride8, soft_count, unorm);
    else
        hipLaunchKernelGGL(rc_terms_fix_kernel<float>, fgrid, dim3(64), flds, s, X.f(), x_mean, d, U.f(), mem_q, mem_r,
                           soff, unk_ptr, unk_idx, toff, sims, terms, fix_list, fix_count, stride8, soft_count, unorm);
    return kstatus("rc_terms_cl_kernel");
}

int launch_rc_chain_terms(hipStream_t s, int64_t nq, const int64_t* soff, const int64_t* unk_ptr, const int64_t* toff,
                          const double* sims, const double* terms, const double* carry_main, const double* carry_abs,
                          const int64_t* carry_cnt, const double* u_mean, double* main_out, double* abs_out,
                          int64_t* cnt_out, double* pred, int64_t long_min) {
    if (nq <= 0) return 0;
    hipLaunchKernelGGL(rc_chain_user_kernel, dim3((unsigned)std::min<int64_t>(nq, 65536)), dim3(64), 0, s, nq, soff,
                       unk_ptr, toff, sims, terms, carry_main, carry_abs, carry_cnt, u_mean, main_out, abs_out, cnt_out,
                       pred, long_min);
    return kstatus("rc_chain_user_kernel");
}

// The users of huge clusters (lng: one batch of them), by segments: their chain
// would be one wave's ~n dependent adds (4.9 ms for the 206,926 members of the
// first C5 iteration's largest cluster).
int launch_rc_long(hipStream_t s, const double* sims, const double* terms, const double* carry_main,
                   const double* carry_abs, const int64_t* carry_cnt, const double* u_mean, double* main_out,
                   double* abs_out, int64_t* cnt_out, double* pred, const RcLong& L) {
    const RcLong* lng = &L;
    {
        int rc;
        const int D = lng->D;
        hipLaunchKernelGGL(rc_long_pack_kernel, dim3(gsz(lng->rows * D / lng->nlong, 256, 2048), (unsigned)lng->nlong),
                           dim3(256), 0, s, lng->tab, D, sims, terms, lng->V);
        if (carry_main)
            hipLaunchKernelGGL(rc_long_carry_kernel, dim3(gsz(lng->nlong * D, 256, 65535)), dim3(256), 0, s, lng->tab,
                               lng->nlong, D, carry_main, carry_abs, lng->carry);
        if ((rc = launch_seg_iota(s, lng->iota, lng->rows)) ||
            (rc = launch_seg_columns(s, lng->V, lng->rows, (int)lng->nlong, D, lng->iota, lng->crow,
                                     carry_main ? lng->carry : nullptr, lng->sums, lng->ws)))
            return rc;
        hipLaunchKernelGGL(rc_long_finish_kernel, dim3((unsigned)lng->nlong), dim3(64), 0, s, lng->tab, D, lng->sums,
                           carry_cnt, u_mean, main_out, abs_out, cnt_out, pred);
    }
    return kstatus("rc_long");
}

int launch_rc_top(hipStream_t s, int64_t nq, const int64_t* soff, const int64_t* carry_cnt, const int64_t* unk_ptr,
                  const int32_t* unk_idx, double* pred, int32_t* pidx, int n_top, int32_t* out) {
    if (nq <= 0) return 0;
    hipLaunchKernelGGL(rc_top_kernel, dim3((unsigned)((nq + 63) / 64)), dim3(64), 0, s, nq, soff, carry_cnt, unk_ptr,
                       unk_idx, pred, pidx, n_top, out);
    return kstatus("rc_top_kernel");
}

int launch_rc_norms(hipStream_t s, const double* X, int64_t N, int d, double* xa) {
    hipLaunchKernelGGL(rc_norm_kernel, dim3(gsz(N, 256, 4096)), dim3(256), 0, s, X, N, d, xa);
    return kstatus("recom.hip");
}

int launch_rc_p_closest(hipStream_t s, const double* X, const double* xa, int d, const double* U, int64_t nq,
                        const int64_t* cand_ptr, const int32_t* cand_idx, int P, double* sim, double* key,
                        int32_t* pos, int32_t* out_idx, double* out_sim, int32_t* out_cnt, int32_t* replay,
                        unsigned int* replay_count) {
    if (nq <= 0) return 0;
    if (hipMemsetAsync(replay_count, 0, sizeof(unsigned int), s) != hipSuccess) return kstatus("recom.hip");
    hipLaunchKernelGGL(rc_p_closest_kernel, dim3(gsz(nq, RC_WAVES, 8192)), dim3(64 * RC_WAVES), 0, s, X, xa, d, U, nq,
                       cand_ptr, cand_idx, P, sim, key, out_idx, out_sim, out_cnt, replay, replay_count);
    hipLaunchKernelGGL(rc_replay_kernel, dim3(gsz(nq, 64, 1024)), dim3(64), 0, s, cand_ptr, cand_idx, P, sim, key, pos,
                       replay, replay_count, out_idx, out_sim);
    return kstatus("recom.hip");
}

int launch_rc_top_n(hipStream_t s, const double* X, const double* x_mean, int d, const double* u_mean, int64_t nq,
                    const int64_t* unk_ptr, const int32_t* unk_idx, const int32_t* nb_idx, const double* nb_sim,
                    const int32_t* nb_cnt, int P, int n_top, double* pred, int32_t* pidx, int32_t* out) {
    if (nq <= 0) return 0;
    hipLaunchKernelGGL(rc_top_n_kernel, dim3(gsz(nq, RC_WAVES, 8192)), dim3(64 * RC_WAVES), 0, s, X, x_mean, d, u_mean,
                       nq, unk_ptr, unk_idx, nb_idx, nb_sim, nb_cnt, P, n_top, pred, pidx, out);
    return kstatus("recom.hip");
}

}  // namespace lshkm
