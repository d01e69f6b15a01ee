// api_index.cpp — C ABI for index build / query (LSH, hypercube) and the
// k-means update. Stream-ordered; host syncs only where a device-computed size
// decides an allocation (query totals, coin counts, the continue flag).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/lshkm.h"
#include "common.h"
#include "index.h"
#include "kernels.h"

using namespace lshkm;

// Hashing of a batch: the split-f16 MFMA kernel where it applies (fp32 rows,
// d = 128, L*k <= 32), else the fp64 kernel (hash.hip). mm (cube euclidean):
// the h range, into a pair the caller pre-set. LSHKM_HASH_PATH=fp64 forces the
// fp64 kernel (tests compare the two).
int lshkm::hash_rows(lshkm_ctx ctx, int mode, Pts X, int64_t N, const ProjTable& pj, int64_t nb, int32_t* out_h,
                     int32_t* out_phi, int32_t* out_bucket, int32_t* mm, bool* h16) {
    const bool want16 = h16 && *h16;
    if (h16) *h16 = false;
    if (N <= 0) return 0;
    const bool force64 = test_switch("LSHKM_HASH_PATH", "fp64");
    unsigned long long* stats = (unsigned long long*)ctx->stats.p;
    int rc;
    if (!X.f64 && pj.mfma_ok && !force64) {
        const int64_t cap = N + FUSED_LIST_SLACK;
        // the fix-up pass rebuilds a table's phi from the stored tuples
        if (mode == HM_LSH_EUCLID && !out_h) {
            if ((rc = ctx->ws_tuples.reserve((size_t)N * pj.LK * 4))) return rc;
            out_h = ctx->ws_tuples.as<int32_t>();
        }
        if ((rc = ctx->ws_hfix.reserve((size_t)cap * 8)) || (rc = ctx->ws_seg.reserve((size_t)FUSED_MAX_SEGS * 2 * 4)))
            return rc;
        const bool w16 = want16 && mode == HM_CUBE_EUCLID_H;
        if ((rc = launch_hash_mfma(ctx->stream, mode, X.f(), N, pj.mfma_params(nb), out_h, out_phi, out_bucket, mm,
                                   (unsigned long long*)ctx->ws_hfix.p, cap, (int32_t*)ctx->ws_seg.p, FUSED_MAX_SEGS * 2,
                                   stats, w16)))
            return rc;
        if (h16) *h16 = w16;
        return 0;
    }
    if ((rc = launch_proj_hash(ctx->stream, mode, X, N, pj.params(nb), out_h, out_phi, out_bucket, stats))) return rc;
    if (mode == HM_CUBE_EUCLID_H && mm) return launch_h_minmax(ctx->stream, out_h, N * pj.k, mm);
    return 0;
}

namespace {

// ctx->ws slot map
enum { WS_QTUP = 0, WS_QBKT, WS_SIZES, WS_COFF, WS_KLIST, WS_KCNT, WS_QSZ, WS_SORT, WS_SKEYS, WS_ROWS, WS_CROW,
       WS_SUMS, WS_CNTS, WS_FLAG, WS_H, WS_MASKS };

template <typename T> T* slot(lshkm_ctx ctx, int i) { return ctx->ws[i].as<T>(); }

int reserve(lshkm_ctx ctx, int i, size_t bytes) {
    ctx->ws_epoch++;
    return ctx->ws[i].reserve(std::max<size_t>(bytes, 64));
}

// the scan workspace is context state too: its users bump the epoch as well
int reserve_scan(lshkm_ctx ctx, size_t bytes) {
    ctx->ws_epoch++;
    return ctx->ws_scan.reserve(bytes);
}

// batches beyond this go straight to their (pageable) destinations
constexpr size_t PIN_BATCH_MAX = (size_t)16 << 20;

int d2h_batch_impl(lshkm_ctx ctx, const D2H* r, int n) {
    size_t tot = 0;
    for (int i = 0; i < n; i++) tot += (r[i].bytes + 255) & ~(size_t)255;
    if (tot > PIN_BATCH_MAX || lshkm_ctx_s::pin_grow(ctx->rb_buf, ctx->rb_cap, tot)) {
        for (int i = 0; i < n; i++)
            if (r[i].bytes) LSHKM_HIP(hipMemcpyAsync(r[i].dst, r[i].src, r[i].bytes, hipMemcpyDeviceToHost, ctx->stream));
        LSHKM_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    }
    char* b = static_cast<char*>(ctx->rb_buf);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        if (r[i].bytes) LSHKM_HIP(hipMemcpyAsync(b + off, r[i].src, r[i].bytes, hipMemcpyDeviceToHost, ctx->stream));
        off += (r[i].bytes + 255) & ~(size_t)255;
    }
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    off = 0;
    for (int i = 0; i < n; i++) {
        if (r[i].bytes) std::memcpy(r[i].dst, b + off, r[i].bytes);
        off += (r[i].bytes + 255) & ~(size_t)255;
    }
    return 0;
}

int h2d_batch_impl(lshkm_ctx ctx, const H2D* r, int n) {
    size_t tot = 0;
    for (int i = 0; i < n; i++) tot += (r[i].bytes + 255) & ~(size_t)255;
    if (ctx->ub_pending) {                           // the previous batch's copies still read ub_buf
        LSHKM_HIP(hipEventSynchronize(ctx->ub_ev));
        ctx->ub_pending = false;
    }
    if (!ctx->ub_ev && hipEventCreateWithFlags(&ctx->ub_ev, hipEventDisableTiming) != hipSuccess) ctx->ub_ev = nullptr;
    if (!ctx->ub_ev || tot > PIN_BATCH_MAX || lshkm_ctx_s::pin_grow(ctx->ub_buf, ctx->ub_cap, tot)) {
        // pageable sources: copied before return (the caller's buffers may go)
        for (int i = 0; i < n; i++)
            if (r[i].bytes) LSHKM_HIP(hipMemcpyAsync(r[i].dst, r[i].src, r[i].bytes, hipMemcpyHostToDevice, ctx->stream));
        LSHKM_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    }
    char* b = static_cast<char*>(ctx->ub_buf);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        if (r[i].bytes) {
            std::memcpy(b + off, r[i].src, r[i].bytes);
            LSHKM_HIP(hipMemcpyAsync(r[i].dst, b + off, r[i].bytes, hipMemcpyHostToDevice, ctx->stream));
        }
        off += (r[i].bytes + 255) & ~(size_t)255;
    }
    LSHKM_HIP(hipEventRecord(ctx->ub_ev, ctx->stream));
    ctx->ub_pending = true;
    return 0;
}

int d2h(lshkm_ctx ctx, void* dst, const void* src, size_t bytes) {
    const D2H r{dst, src, bytes};
    return d2h_batch_impl(ctx, &r, 1);
}

// Stable scatter of keys[i * kstride] in [0, nb) -> idx (row order kept) + row_ptr.
// T bucket CSRs at once: table t's keys at keys + t (stride kstride), its
// members at idx + t * N, its row pointers at row_ptr + t * (nb + 1).
int build_csr(lshkm_ctx ctx, const int32_t* keys, int64_t kstride, int64_t N, int64_t nb, int32_t* idx,
              int64_t* row_ptr, int T = 1) {
    int rc;
    if ((rc = reserve(ctx, WS_SORT, sort_scratch_bytes(N, nb, T))) || (rc = reserve(ctx, WS_SKEYS, (size_t)N * T * 4)))
        return rc;
    if (N > 0 && (rc = stable_sort_by_key_batched(ctx->stream, keys, kstride, 1, nullptr, 0, T, N, nb,
                                                  slot<int32_t>(ctx, WS_SKEYS), idx, ctx->ws[WS_SORT].p))) { LSHKM_LAUNCH_CHECK(); return rc; }
    if ((rc = launch_csr_bounds(ctx->stream, slot<int32_t>(ctx, WS_SKEYS), N, nb, row_ptr, T))) { LSHKM_LAUNCH_CHECK(); return rc; }
    return 0;
}

// Probe masks of get_hypercube_combined_buckets: 0 first (main bucket), then
// Hamming distance 1 (bit 0..k-1), 2 (lexicographic i<j), ... ; probes == 1
// starts at distance 2 (lsh_cube.hpp:148-150); stops when the cube is exhausted.
std::vector<int32_t> probe_masks(int probes, int k) {
    std::vector<int32_t> m(1, 0);
    int remaining = probes;
    int dist = probes > 1 ? 1 : 2;
    std::vector<int> comb(64);
    while (remaining > 0 && dist <= k) {
        for (int i = 0; i < dist; i++) comb[i] = i;
        for (;;) {
            int mask = 0;
            for (int i = 0; i < dist; i++) mask |= 1 << comb[i];
            m.push_back(mask);
            if (--remaining == 0) break;
            int p = dist - 1;
            while (p >= 0 && comb[p] == k - dist + p) p--;
            if (p < 0) break;
            comb[p]++;
            for (int q = p + 1; q < dist; q++) comb[q] = comb[q - 1] + 1;
        }
        dist++;
    }
    return m;
}

}  // namespace

// ----------------------------------------------------------------------- LSH
static int lsh_build_impl(lshkm_lsh lsh, Pts X, int64_t N) {
    LSHKM_CHECK(lsh && (X.p || N == 0) && N >= 0 && N < (1ll << 31), LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = lsh->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    const int L = lsh->proj.L, k = lsh->proj.k;
    const int64_t nb = lsh->nb;
    int rc;
    if ((rc = lsh->bucket.reserve((size_t)std::max<int64_t>(N, 1) * L * 4)) ||
        (rc = lsh->row_ptr.reserve((size_t)L * (nb + 1) * 8)) || (rc = lsh->idx.reserve((size_t)std::max<int64_t>(N, 1) * L * 4)))
        return rc;
    if (lsh->metric == LSHKM_METRIC_EUCLIDEAN && (rc = lsh->tuples.reserve((size_t)std::max<int64_t>(N, 1) * L * k * 4))) return rc;
    const int mode = lsh->metric == LSHKM_METRIC_EUCLIDEAN ? HM_LSH_EUCLID : HM_LSH_COSINE;
    if ((rc = hash_rows(ctx, mode, X, N, lsh->proj, nb, mode == HM_LSH_EUCLID ? lsh->tuples.as<int32_t>() : nullptr,
                        nullptr, lsh->bucket.as<int32_t>(), nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
    if ((rc = build_csr(ctx, lsh->bucket.as<int32_t>(), L, N, nb, lsh->idx.as<int32_t>(), lsh->row_ptr.as<int64_t>(), L)))
        return rc;
    lsh->N = N;
    lsh->built = 1;
    lsh->mt0_valid = false;
    return 0;
}

extern "C" {

int lshkm_lsh_build(lshkm_lsh lsh, const float* X, int64_t N) { return lsh_build_impl(lsh, X, N); }
int lshkm_lsh_build_f64(lshkm_lsh lsh, const double* X, int64_t N) { return lsh_build_impl(lsh, X, N); }

int lshkm_lsh_get_buckets(lshkm_lsh lsh, int table, int64_t* row_ptr, int32_t* idx) {
    LSHKM_CHECK(lsh && lsh->built && table >= 0 && table < lsh->proj.L, LSHKM_ERR_ARG, "not built / bad table");
    lshkm_ctx ctx = lsh->ctx;
    const int64_t nb = lsh->nb, N = lsh->N;
    int rc;
    if (row_ptr && (rc = d2h(ctx, row_ptr, lsh->row_ptr.as<int64_t>() + (size_t)table * (nb + 1), (size_t)(nb + 1) * 8))) return rc;
    if (idx && N > 0 && (rc = d2h(ctx, idx, lsh->idx.as<int32_t>() + (size_t)table * N, (size_t)N * 4))) return rc;
    return 0;
}

int lshkm_lsh_device_views(lshkm_lsh lsh, const int64_t** row_ptr, const int32_t** idx, const int32_t** tuples,
                           const int32_t** bucket) {
    LSHKM_CHECK(lsh && lsh->built, LSHKM_ERR_STATE, "index not built");
    if (row_ptr) *row_ptr = lsh->row_ptr.as<int64_t>();
    if (idx) *idx = lsh->idx.as<int32_t>();
    if (tuples) *tuples = lsh->metric == LSHKM_METRIC_EUCLIDEAN ? lsh->tuples.as<int32_t>() : nullptr;
    if (bucket) *bucket = lsh->bucket.as<int32_t>();
    return 0;
}

}  // extern "C"

static int lsh_query_impl(lshkm_lsh lsh, Pts Q, int64_t nq, const int32_t* alias, int filtered, int64_t* out_ptr,
                          int32_t* out_idx, int64_t out_cap, int64_t* total_host) {
    LSHKM_CHECK(lsh && lsh->built, LSHKM_ERR_STATE, "index not built (lshkm_lsh_build)");
    LSHKM_CHECK((Q.p || nq == 0) && nq >= 0 && out_ptr && total_host, LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = lsh->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int L = lsh->proj.L, k = lsh->proj.k;
    const int64_t nb = lsh->nb, pairs = nq * L;
    const bool eu = lsh->metric == LSHKM_METRIC_EUCLIDEAN;
    int rc;
    // the filling call of the two-phase protocol (same Q, nq, alias, filtered
    // and out_ptr buffer -- whose prefix offsets the sizing call just wrote --,
    // nothing else on the context's slots in between): only the merge runs again
    const bool reuse = out_idx && lsh->q_valid && lsh->q_epoch == ctx->ws_epoch && lsh->q_Q == Q.p &&
                       lsh->q_f64 == Q.f64 && lsh->q_nq == nq && lsh->q_alias == alias &&
                       lsh->q_filtered == filtered && lsh->q_out_ptr == out_ptr;
    lsh->q_valid = false;
    if (nq == 0) {
        LSHKM_HIP(hipMemsetAsync(out_ptr, 0, 8, s));
        *total_host = 0;
        return 0;
    }
    if (reuse) {
        *total_host = lsh->q_total;
        if (lsh->q_total <= out_cap && lsh->q_total > 0 &&
            (rc = launch_lsh_query(s, slot<int32_t>(ctx, WS_QBKT), slot<int32_t>(ctx, WS_QTUP), alias, nq, L, k, nb,
                                   eu && filtered ? 1 : 0, lsh->N, eu ? lsh->tuples.as<int32_t>() : nullptr,
                                   lsh->bucket.as<int32_t>(), lsh->row_ptr.as<int64_t>(), lsh->idx.as<int32_t>(),
                                   slot<int64_t>(ctx, WS_SIZES), slot<int64_t>(ctx, WS_COFF), slot<int32_t>(ctx, WS_KLIST),
                                   slot<int64_t>(ctx, WS_KCNT), slot<int64_t>(ctx, WS_QSZ), out_ptr, out_idx, 2,
                                   nullptr, lsh->mt0_valid ? lsh->mt0.as<int32_t>() : nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
        return 0;
    }
    if ((rc = reserve(ctx, WS_QTUP, (size_t)pairs * k * 4)) || (rc = reserve(ctx, WS_QBKT, (size_t)pairs * 4)) ||
        (rc = reserve(ctx, WS_SIZES, (size_t)pairs * 8)) || (rc = reserve(ctx, WS_COFF, (size_t)(pairs + 1) * 8)) ||
        (rc = reserve(ctx, WS_KCNT, (size_t)pairs * 8)) || (rc = reserve(ctx, WS_QSZ, (size_t)nq * 8)))
        return rc;
    if (nq > 0 && (rc = hash_rows(ctx, eu ? HM_LSH_EUCLID : HM_LSH_COSINE, Q, nq, lsh->proj, nb,
                                  eu ? slot<int32_t>(ctx, WS_QTUP) : nullptr, nullptr, slot<int32_t>(ctx, WS_QBKT),
                                  nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
    auto run = [&](int phase, int32_t* out) {
        if (reserve_scan(ctx, scan_ws_bytes(nq * L + nq))) return LSHKM_ERR_NOMEM;
        return launch_lsh_query(s, slot<int32_t>(ctx, WS_QBKT), slot<int32_t>(ctx, WS_QTUP), alias, nq, L, k, nb,
                                eu && filtered ? 1 : 0, lsh->N, eu ? lsh->tuples.as<int32_t>() : nullptr,
                                lsh->bucket.as<int32_t>(), lsh->row_ptr.as<int64_t>(), lsh->idx.as<int32_t>(),
                                slot<int64_t>(ctx, WS_SIZES), slot<int64_t>(ctx, WS_COFF), slot<int32_t>(ctx, WS_KLIST),
                                slot<int64_t>(ctx, WS_KCNT), slot<int64_t>(ctx, WS_QSZ), out_ptr, out, phase,
                                ctx->ws_scan.as<int64_t>(), lsh->mt0_valid ? lsh->mt0.as<int32_t>() : nullptr);
    };
    if (eu && filtered && !lsh->mt0_valid && lsh->N > 0) {
        if ((rc = lsh->mt0.reserve((size_t)lsh->N * L * 4))) return rc;
        if ((rc = launch_lsh_gather_t0(s, lsh->tuples.as<int32_t>(), lsh->idx.as<int32_t>(), lsh->N, L, k,
                                       lsh->mt0.as<int32_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
        lsh->mt0_valid = true;
    }
    if ((rc = run(0, nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
    int64_t cand = 0;
    if ((rc = d2h(ctx, &cand, slot<int64_t>(ctx, WS_COFF) + pairs, 8))) return rc;
    if ((rc = reserve(ctx, WS_KLIST, (size_t)cand * 4))) return rc;
    if ((rc = run(1, nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
    int64_t total = 0;
    if ((rc = d2h(ctx, &total, out_ptr + nq, 8))) return rc;
    *total_host = total;
    if (out_idx && total <= out_cap && total > 0)
        if ((rc = run(2, out_idx))) { LSHKM_LAUNCH_CHECK(); return rc; }
    if (!out_idx) {
        lsh->q_valid = true; lsh->q_epoch = ctx->ws_epoch; lsh->q_Q = Q.p; lsh->q_f64 = Q.f64; lsh->q_nq = nq;
        lsh->q_alias = alias; lsh->q_filtered = filtered; lsh->q_total = total; lsh->q_out_ptr = out_ptr;
    }
    return 0;
}

extern "C" {

int lshkm_lsh_query(lshkm_lsh lsh, const float* Q, int64_t nq, const int32_t* alias, int filtered, int64_t* out_ptr,
                    int32_t* out_idx, int64_t out_cap, int64_t* total_host) {
    return lsh_query_impl(lsh, Q, nq, alias, filtered, out_ptr, out_idx, out_cap, total_host);
}

int lshkm_lsh_query_f64(lshkm_lsh lsh, const double* Q, int64_t nq, const int32_t* alias, int filtered,
                        int64_t* out_ptr, int32_t* out_idx, int64_t out_cap, int64_t* total_host) {
    return lsh_query_impl(lsh, Q, nq, alias, filtered, out_ptr, out_idx, out_cap, total_host);
}

// ----------------------------------------------------------------- hypercube
int lshkm_cube_create(lshkm_ctx ctx, int metric, int d, int k, float w, const float* V, const float* t, const double* R,
                      uint32_t rng_state, lshkm_cube* out) {
    LSHKM_CHECK(ctx && out && d > 0 && d <= 1024 && k > 0 && k <= 30, LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN ? (V && t && w > 0.f) : (metric == LSHKM_METRIC_COSINE && R),
                LSHKM_ERR_ARG, "euclidean cube needs V, t, w > 0; cosine cube needs R");
    LSHKM_HIP(hipSetDevice(ctx->device));
    lshkm_cube c = new lshkm_cube_s();
    c->ctx = ctx; c->metric = metric; c->k = k;
    std::vector<int32_t> r0(k, 0);
    int rc = c->proj.upload(ctx->stream, metric, d, 1, k, w, V, t, r0.data(), R);
    if (!rc) rc = c->rng_d.reserve(64);
    if (!rc) rc = c->mm.reserve(64);
    if (!rc) rc = c->cnt.reserve(64);
    if (rc) { delete c; return rc; }
    if (hipMemcpy(c->rng_d.p, &rng_state, 4, hipMemcpyHostToDevice) != hipSuccess) { delete c; set_error("copy failed"); return LSHKM_ERR_HIP; }
    *out = c;
    return 0;
}

int lshkm_cube_destroy(lshkm_cube cube) {
    if (!cube) return 0;
    (void)hipDeviceSynchronize();
    delete cube;
    return 0;
}

// Dense coin-memo window: grow (re-home) it so that [lo, hi] is covered.
static int cube_ensure_window(lshkm_cube cube, int32_t lo_h, int32_t hi_h) {
    lshkm_ctx ctx = cube->ctx;
    hipStream_t s = ctx->stream;
    const int k = cube->k;
    int rc;
    const int32_t mm[2] = {lo_h, hi_h};
    if (cube->hspan == 0 || mm[0] < cube->hmin || mm[1] >= cube->hmin + cube->hspan) {
        const int64_t lo = cube->hspan ? std::min<int64_t>(cube->hmin, mm[0]) : mm[0];
        const int64_t hi = cube->hspan ? std::max<int64_t>((int64_t)cube->hmin + cube->hspan - 1, mm[1]) : mm[1];
        const int64_t margin = std::max<int64_t>(64, (hi - lo) / 2);
        const int64_t nlo = lo - margin, nspan = hi - lo + 1 + 2 * margin;
        LSHKM_CHECK(nspan < (1 << 26), LSHKM_ERR_UNSUPPORTED, "h range too wide for the dense coin memo");
        if ((rc = cube->memo2.reserve((size_t)k * nspan * 4))) return rc;
        if ((rc = launch_memo_rehome(s, cube->hspan ? cube->memo.as<int32_t>() : nullptr, cube->hmin, cube->hspan,
                                     cube->memo2.as<int32_t>(), (int32_t)nlo, (int32_t)nspan, k))) { LSHKM_LAUNCH_CHECK(); return rc; }
        std::swap(cube->memo.p, cube->memo2.p);
        std::swap(cube->memo.cap, cube->memo2.cap);
        cube->hmin = (int32_t)nlo;
        cube->hspan = (int32_t)nspan;
        if ((rc = cube->first_row.reserve((size_t)k * nspan * 4))) return rc;
        LSHKM_HIP(hipMemsetAsync(cube->first_row.p, 0x7F, (size_t)k * nspan * 4, s));   // 0x7F7F7F7F > any row
    }
    return 0;
}

// h of a batch (EuclideanH, k per row) into WS_H, and the memo window over it.
// h is int16 (*h16) when the MFMA kernel wrote it and the range fits, else
// int32 (the batch is hashed again when the int16 values saturated).
static int cube_h_batch(lshkm_cube cube, Pts X, int64_t N, const void** h_out, bool* h16) {
    lshkm_ctx ctx = cube->ctx;
    hipStream_t s = ctx->stream;
    const int k = cube->k;
    int rc;
    LSHKM_CHECK(N * k < (1ll << 31), LSHKM_ERR_UNSUPPORTED, "rows * k must be < 2^31");
    if ((rc = reserve(ctx, WS_H, (size_t)N * k * 4 + 16))) return rc;   // + the staged loads' slack (cube.hip)
    int32_t* h = slot<int32_t>(ctx, WS_H);
    const int32_t init_mm[2] = {0x7FFFFFFF, (int32_t)0x80000000};
    int32_t mm[2];
    bool narrow = true;
    for (int pass = 0; pass < 2; pass++) {
        if ((rc = ctx->pin_stage(8))) return rc;
        std::memcpy(ctx->pinned, init_mm, 8);
        LSHKM_HIP(hipMemcpyAsync(cube->mm.p, ctx->pinned, 8, hipMemcpyHostToDevice, s));
        LSHKM_HIP(hipEventRecord(ctx->pinned_ev, s));
        if ((rc = hash_rows(ctx, HM_CUBE_EUCLID_H, X, N, cube->proj, 1ll << k, h, nullptr, nullptr,
                            cube->mm.as<int32_t>(), &narrow))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if ((rc = d2h(ctx, mm, cube->mm.p, 8))) return rc;
        if (!narrow || (mm[0] >= -32768 && mm[1] <= 32767)) break;
        narrow = false;                      // saturated: hash again as int32
    }
    if ((rc = cube_ensure_window(cube, mm[0], mm[1]))) return rc;
    *h_out = h;
    *h16 = narrow;
    return 0;
}

// First occurrence of every (f, h) of the batch that has no coin yet, as
// (key = row * k + f, memo offset) pairs in WS_SIZES / WS_COFF; count in
// cube->cnt on the device and, when n is given, in *n.
static int cube_unseen_impl(lshkm_cube cube, const void* h, bool h16, int64_t N, unsigned int* n) {
    lshkm_ctx ctx = cube->ctx;
    hipStream_t s = ctx->stream;
    const int k = cube->k;
    int rc;
    const int64_t total = (int64_t)k * cube->hspan;
    LSHKM_HIP(hipMemsetAsync(cube->first_row.p, 0x7F, (size_t)total * 4, s));
    if ((rc = launch_coin_first(s, h, h16, N, k, cube->hmin, cube->hspan, cube->memo.as<int32_t>(), cube->first_row.as<int32_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
    LSHKM_HIP(hipMemsetAsync(cube->cnt.p, 0, 4, s));
    const int64_t maxe = std::min<int64_t>(total, N * k);
    if ((rc = reserve(ctx, WS_SIZES, (size_t)maxe * 4)) || (rc = reserve(ctx, WS_COFF, (size_t)maxe * 4)) ||
        (rc = reserve(ctx, WS_KLIST, (size_t)maxe * 4)) || (rc = reserve(ctx, WS_KCNT, (size_t)maxe * 4)))
        return rc;
    if ((rc = launch_coin_collect(s, cube->first_row.as<int32_t>(), total, k, cube->hspan, slot<int32_t>(ctx, WS_SIZES),
                                  slot<int32_t>(ctx, WS_COFF), cube->cnt.as<unsigned int>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
    return n ? d2h(ctx, n, cube->cnt.p, 4) : 0;
}

static int cube_vertices_impl(lshkm_cube cube, Pts X, int64_t N, int32_t* vertex) {
    lshkm_ctx ctx = cube->ctx;
    hipStream_t s = ctx->stream;
    const int k = cube->k;
    int rc;
    if (N == 0) return 0;
    if (cube->metric == LSHKM_METRIC_COSINE) {
        if ((rc = hash_rows(ctx, HM_CUBE_COSINE, X, N, cube->proj, 1ll << k, vertex, nullptr, nullptr, nullptr))) {
            LSHKM_LAUNCH_CHECK();
            return rc;
        }
        return 0;
    }
    const void* h = nullptr;
    bool h16 = false;
    if ((rc = cube_h_batch(cube, X, N, &h, &h16))) return rc;
    // first occurrence of each unseen (f, h), then the draw in (row, f) order
    const int64_t bound = std::min<int64_t>((int64_t)k * cube->hspan, N * k);
    if (bound <= 8192) {
        // the count cannot pass the one-workgroup sort's limit: it stays on the
        // device (sort and draw read it there), no host round trip
        if ((rc = cube_unseen_impl(cube, h, h16, N, nullptr))) return rc;
        if ((rc = sort_pairs_small(s, slot<int32_t>(ctx, WS_SIZES), slot<int32_t>(ctx, WS_COFF), bound,
                                   slot<int32_t>(ctx, WS_KLIST), slot<int32_t>(ctx, WS_KCNT), cube->cnt.as<unsigned int>())) ||
            (rc = launch_coin_draw(s, slot<int32_t>(ctx, WS_KCNT), cube->cnt.as<unsigned int>(), cube->hmin, cube->hspan,
                                   cube->memo.as<int32_t>(), cube->rng_d.as<uint32_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if ((rc = launch_coin_vertex(s, h, h16, N, k, cube->hmin, cube->hspan, cube->memo.as<int32_t>(), vertex))) { LSHKM_LAUNCH_CHECK(); return rc; }
        return 0;
    }
    unsigned int ncoins = 0;
    if ((rc = cube_unseen_impl(cube, h, h16, N, &ncoins))) return rc;
    if (ncoins > 0) {
        // the draw order: keys row * k + f are distinct, so a few thousand sort in
        // one workgroup (a multi-pass radix sort is a dozen launches)
        if (ncoins <= 8192) {
            if ((rc = sort_pairs_small(s, slot<int32_t>(ctx, WS_SIZES), slot<int32_t>(ctx, WS_COFF), ncoins,
                                       slot<int32_t>(ctx, WS_KLIST), slot<int32_t>(ctx, WS_KCNT)))) { LSHKM_LAUNCH_CHECK(); return rc; }
        } else {
            if ((rc = reserve(ctx, WS_SORT, sort_scratch_bytes(ncoins, N * k)))) return rc;
            if ((rc = stable_sort_by_key(s, slot<int32_t>(ctx, WS_SIZES), 1, slot<int32_t>(ctx, WS_COFF), ncoins, N * k,
                                         slot<int32_t>(ctx, WS_KLIST), slot<int32_t>(ctx, WS_KCNT), ctx->ws[WS_SORT].p))) { LSHKM_LAUNCH_CHECK(); return rc; }
        }
        if ((rc = launch_coin_draw(s, slot<int32_t>(ctx, WS_KCNT), cube->cnt.as<unsigned int>(), cube->hmin, cube->hspan,
                                   cube->memo.as<int32_t>(), cube->rng_d.as<uint32_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
    }
    if ((rc = launch_coin_vertex(s, h, h16, N, k, cube->hmin, cube->hspan, cube->memo.as<int32_t>(), vertex))) { LSHKM_LAUNCH_CHECK(); return rc; }
    return 0;
}

// ---- sharded EuclideanF coins: export, host draw, import
static int cube_unseen_api(lshkm_cube cube, Pts X, int64_t N, int32_t* f_host, int32_t* h_host, int64_t* row_host,
                           int64_t cap, int64_t* count_host) {
    LSHKM_CHECK(cube && (X.p || N == 0) && N >= 0 && N < (1ll << 31) && count_host && (cap == 0 || (f_host && h_host && row_host)),
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(cube->metric == LSHKM_METRIC_EUCLIDEAN, LSHKM_ERR_ARG, "coins exist only for the euclidean cube");
    lshkm_ctx ctx = cube->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    *count_host = 0;
    if (N == 0) return 0;
    int rc;
    const void* h = nullptr;
    bool h16 = false;
    if ((rc = cube_h_batch(cube, X, N, &h, &h16))) return rc;
    unsigned int n = 0;
    if ((rc = cube_unseen_impl(cube, h, h16, N, &n))) return rc;
    *count_host = n;
    if (n == 0 || (int64_t)n > cap) return 0;
    std::vector<int32_t> keys(n), offs(n);
    if ((rc = d2h(ctx, keys.data(), ctx->ws[WS_SIZES].p, (size_t)n * 4)) || (rc = d2h(ctx, offs.data(), ctx->ws[WS_COFF].p, (size_t)n * 4)))
        return rc;
    for (unsigned int i = 0; i < n; i++) {
        f_host[i] = keys[i] % cube->k;
        row_host[i] = keys[i] / cube->k;
        h_host[i] = cube->hmin + offs[i] % cube->hspan;
    }
    return 0;
}

int lshkm_cube_unseen(lshkm_cube cube, const float* X, int64_t N, int32_t* f_host, int32_t* h_host,
                      int64_t* row_host, int64_t cap, int64_t* count_host) {
    return cube_unseen_api(cube, X, N, f_host, h_host, row_host, cap, count_host);
}

int lshkm_cube_unseen_f64(lshkm_cube cube, const double* X, int64_t N, int32_t* f_host, int32_t* h_host,
                          int64_t* row_host, int64_t cap, int64_t* count_host) {
    return cube_unseen_api(cube, X, N, f_host, h_host, row_host, cap, count_host);
}

int lshkm_cube_import_coins(lshkm_cube cube, const int32_t* f_host, const int32_t* h_host, const int32_t* bit_host,
                            int64_t n, uint32_t rng_state) {
    LSHKM_CHECK(cube && n >= 0 && (n == 0 || (f_host && h_host && bit_host)), LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(cube->metric == LSHKM_METRIC_EUCLIDEAN, LSHKM_ERR_ARG, "coins exist only for the euclidean cube");
    lshkm_ctx ctx = cube->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if (n > 0) {
        int32_t lo = h_host[0], hi = h_host[0];
        for (int64_t i = 0; i < n; i++) {
            LSHKM_CHECK(f_host[i] >= 0 && f_host[i] < cube->k && (bit_host[i] == 0 || bit_host[i] == 1), LSHKM_ERR_ARG,
                        "bad coin entry");
            lo = std::min(lo, h_host[i]);
            hi = std::max(hi, h_host[i]);
        }
        if ((rc = cube_ensure_window(cube, lo, hi))) return rc;
        // memo is device-resident: patch it through a host image of the entries
        std::vector<int32_t> off(n), bit(n);
        for (int64_t i = 0; i < n; i++) {
            off[i] = f_host[i] * cube->hspan + (h_host[i] - cube->hmin);
            bit[i] = bit_host[i];
        }
        if ((rc = reserve(ctx, WS_KLIST, (size_t)n * 4)) || (rc = reserve(ctx, WS_KCNT, (size_t)n * 4))) return rc;
        LSHKM_HIP(hipMemcpyAsync(ctx->ws[WS_KLIST].p, off.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
        LSHKM_HIP(hipMemcpyAsync(ctx->ws[WS_KCNT].p, bit.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
        if ((rc = launch_memo_scatter(ctx->stream, slot<int32_t>(ctx, WS_KLIST), slot<int32_t>(ctx, WS_KCNT), n,
                                      cube->memo.as<int32_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
        LSHKM_HIP(hipStreamSynchronize(ctx->stream));      // the host images go out of scope
    }
    LSHKM_HIP(hipMemcpyAsync(cube->rng_d.p, &rng_state, 4, hipMemcpyHostToDevice, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

static int cube_build_impl(lshkm_cube cube, Pts X, int64_t N) {
    LSHKM_CHECK(cube && (X.p || N == 0) && N >= 0 && N < (1ll << 31), LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = cube->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    const int64_t nb = 1ll << cube->k;
    int rc;
    if ((rc = cube->vertex.reserve((size_t)std::max<int64_t>(N, 1) * 4)) || (rc = cube->idx.reserve((size_t)std::max<int64_t>(N, 1) * 4)) ||
        (rc = cube->row_ptr.reserve((size_t)(nb + 1) * 8)))
        return rc;
    if ((rc = cube_vertices_impl(cube, X, N, cube->vertex.as<int32_t>()))) return rc;
    if ((rc = build_csr(ctx, cube->vertex.as<int32_t>(), 1, N, nb, cube->idx.as<int32_t>(), cube->row_ptr.as<int64_t>()))) return rc;
    cube->N = N;
    cube->built = 1;
    return 0;
}

int lshkm_cube_build(lshkm_cube cube, const float* X, int64_t N) { return cube_build_impl(cube, X, N); }
int lshkm_cube_build_f64(lshkm_cube cube, const double* X, int64_t N) { return cube_build_impl(cube, X, N); }

static int cube_vertices_api(lshkm_cube cube, Pts Q, int64_t nq, int32_t* vertex) {
    LSHKM_CHECK(cube && (Q.p || nq == 0) && nq >= 0 && (vertex || nq == 0), LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(cube->ctx->device));
    return cube_vertices_impl(cube, Q, nq, vertex);
}

int lshkm_cube_vertices(lshkm_cube cube, const float* Q, int64_t nq, int32_t* vertex) {
    return cube_vertices_api(cube, Q, nq, vertex);
}

int lshkm_cube_vertices_f64(lshkm_cube cube, const double* Q, int64_t nq, int32_t* vertex) {
    return cube_vertices_api(cube, Q, nq, vertex);
}

int lshkm_cube_get_buckets(lshkm_cube cube, int64_t* row_ptr, int32_t* idx) {
    LSHKM_CHECK(cube && cube->built, LSHKM_ERR_STATE, "cube not built");
    int rc;
    if (row_ptr && (rc = d2h(cube->ctx, row_ptr, cube->row_ptr.p, (size_t)((1ll << cube->k) + 1) * 8))) return rc;
    if (idx && cube->N > 0 && (rc = d2h(cube->ctx, idx, cube->idx.p, (size_t)cube->N * 4))) return rc;
    return 0;
}

static int cube_query_impl(lshkm_cube cube, Pts Q, int64_t nq, int probes, int64_t* out_ptr, int32_t* out_idx,
                           int64_t out_cap, int64_t* total_host) {
    LSHKM_CHECK(cube && cube->built, LSHKM_ERR_STATE, "cube not built (lshkm_cube_build)");
    LSHKM_CHECK((Q.p || nq == 0) && nq >= 0 && out_ptr && total_host, LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = cube->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const std::vector<int32_t> masks = probe_masks(probes, cube->k);
    const int S = (int)masks.size();
    int rc;
    if (nq == 0) {
        LSHKM_HIP(hipMemsetAsync(out_ptr, 0, 8, s));
        *total_host = 0;
        return 0;
    }
    if ((rc = reserve(ctx, WS_QBKT, (size_t)nq * 4)) || (rc = reserve(ctx, WS_MASKS, (size_t)S * 4)) ||
        (rc = reserve(ctx, WS_QSZ, (size_t)nq * S * 8)) || (rc = reserve(ctx, WS_CROW, (size_t)(nq * S + 1) * 8)) ||
        (rc = reserve_scan(ctx, scan_ws_bytes(nq * S))))
        return rc;
    if ((rc = cube_vertices_impl(cube, Q, nq, slot<int32_t>(ctx, WS_QBKT)))) return rc;
    LSHKM_HIP(hipMemcpyAsync(ctx->ws[WS_MASKS].p, masks.data(), (size_t)S * 4, hipMemcpyHostToDevice, s));
    if ((rc = launch_cube_query(s, slot<int32_t>(ctx, WS_QBKT), nq, slot<int32_t>(ctx, WS_MASKS), S, cube->row_ptr.as<int64_t>(),
                                cube->idx.as<int32_t>(), slot<int64_t>(ctx, WS_QSZ), slot<int64_t>(ctx, WS_CROW), out_ptr,
                                nullptr, ctx->ws_scan.as<int64_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
    int64_t total = 0;
    if ((rc = d2h(ctx, &total, out_ptr + nq, 8))) return rc;
    *total_host = total;
    if (out_idx && total <= out_cap && total > 0)
        if ((rc = launch_cube_query(s, slot<int32_t>(ctx, WS_QBKT), nq, slot<int32_t>(ctx, WS_MASKS), S,
                                    cube->row_ptr.as<int64_t>(), cube->idx.as<int32_t>(), slot<int64_t>(ctx, WS_QSZ),
                                    slot<int64_t>(ctx, WS_CROW), out_ptr, out_idx, ctx->ws_scan.as<int64_t>()))) { LSHKM_LAUNCH_CHECK(); return rc; }
    return 0;
}

int lshkm_cube_query(lshkm_cube cube, const float* Q, int64_t nq, int probes, int64_t* out_ptr, int32_t* out_idx,
                     int64_t out_cap, int64_t* total_host) {
    return cube_query_impl(cube, Q, nq, probes, out_ptr, out_idx, out_cap, total_host);
}

int lshkm_cube_query_f64(lshkm_cube cube, const double* Q, int64_t nq, int probes, int64_t* out_ptr,
                         int32_t* out_idx, int64_t out_cap, int64_t* total_host) {
    return cube_query_impl(cube, Q, nq, probes, out_ptr, out_idx, out_cap, total_host);
}

int lshkm_cube_get_memo(lshkm_cube cube, int32_t* f, int32_t* h, int32_t* bit, int64_t cap, int64_t* count,
                        uint32_t* rng_state) {
    LSHKM_CHECK(cube && count, LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = cube->ctx;
    int rc;
    uint32_t st = 0;
    if ((rc = d2h(ctx, &st, cube->rng_d.p, 4))) return rc;
    if (rng_state) *rng_state = st;
    std::vector<int32_t> memo((size_t)cube->k * cube->hspan);
    if (!memo.empty() && (rc = d2h(ctx, memo.data(), cube->memo.p, memo.size() * 4))) return rc;
    int64_t n = 0;
    for (int fi = 0; fi < cube->k; fi++)
        for (int32_t o = 0; o < cube->hspan; o++) {
            const int32_t b = memo[(size_t)fi * cube->hspan + o];
            if (b < 0) continue;
            if (n < cap) {
                if (f) f[n] = fi;
                if (h) h[n] = cube->hmin + o;
                if (bit) bit[n] = b;
            }
            n++;
        }
    *count = n;
    return 0;
}

// ------------------------------------------------------------------- k-means
// csr_crow / csr_rows: the cluster CSR of this assignment from lshkm_clusters
// (the caller's; NULL: built here into the context's slots).
static int km_sums(lshkm_ctx ctx, Pts X, int64_t N, int d, const int32_t* assign, int K, double* sums,
                   int64_t* counts, const double* carry = nullptr, const int64_t* carry_counts = nullptr,
                   const int64_t* csr_crow = nullptr, const int32_t* csr_rows = nullptr) {
    int rc;
    const int32_t* rows_p = csr_rows;
    const int64_t* crow_p = csr_crow;
    if (!crow_p) {
        if ((rc = reserve(ctx, WS_ROWS, (size_t)std::max<int64_t>(N, 1) * 4)) ||
            (rc = reserve(ctx, WS_CROW, (size_t)(K + 1) * 8)))
            return rc;
        if ((rc = build_csr(ctx, assign, 1, N, K, slot<int32_t>(ctx, WS_ROWS), slot<int64_t>(ctx, WS_CROW)))) return rc;
        rows_p = slot<int32_t>(ctx, WS_ROWS);
        crow_p = slot<int64_t>(ctx, WS_CROW);
    }
    // Parallel exact sums (fixed point where the chain provably never rounds);
    // test switch LSHKM_KM_PATH=chain runs every (c, j) chain sequentially.
    const bool force_chain = test_switch("LSHKM_KM_PATH", "chain");
    // fp64 rows: binade segments (update.hip / kmseg.h; the fp64 update of 1M x
    // 100 rows, K = 256: 0.93 ms vs 2.68 ms for fixed point + the wide chains);
    // test switch LSHKM_KM_PATH=fx: the fixed-point form. The segment workspace
    // is ~5 B per row element plus 2.5 KB per (cluster, dim): past KM_SEG_WS_CAP
    // (or when it cannot be reserved, or K exceeds the composition grid's y
    // limit) the fixed-point form runs instead -- the same exact sums.
    if (X.f64 && !force_chain && !test_switch("LSHKM_KM_PATH", "fx") && K <= 65535) {
        const size_t wsb = km_seg_ws_bytes(N, K, d);
        if (wsb <= KM_SEG_WS_CAP && ctx->ws_range[11].reserve(wsb) == 0) {
            if ((rc = launch_km_sums_seg(ctx->stream, X, d, rows_p, crow_p, K, N, sums, counts, carry, carry_counts,
                                         ctx->ws_range[11].p))) {
                LSHKM_LAUNCH_CHECK();
                return rc;
            }
            return 0;
        }
        (void)hipGetLastError();          // a failed reservation leaves no sticky error
    }
    if (!force_chain) {
        if ((rc = ctx->ws_range[11].reserve(km_fx_ws_bytes(K, d)))) return rc;
        // the chains the never-rounds test flags: by segments (fp32 rows of
        // general values: ~5 % of the chains of 10K N(0,1) values, most of 40K),
        // sequential where the segment workspace does not fit
        void* seg_ws = nullptr;
        if (!X.f64 && K <= 65535) {
            const size_t wsb = km_seg_ws_bytes(N, K, d);
            if (wsb <= KM_SEG_WS_CAP && ctx->ws_km_seg.reserve(wsb) == 0) seg_ws = ctx->ws_km_seg.p;
            else (void)hipGetLastError();
        }
        if ((rc = launch_km_sums_fx(ctx->stream, X, d, rows_p, crow_p, K, N, sums, counts, carry, carry_counts,
                                    ctx->ws_range[11].p, (unsigned long long*)ctx->stats.p + STAT_KM_SEQ, seg_ws))) {
            LSHKM_LAUNCH_CHECK();
            return rc;
        }
        return 0;
    }
    if ((rc = launch_km_chain(ctx->stream, X, d, rows_p, crow_p, K, sums, counts,
                              carry, carry_counts))) { LSHKM_LAUNCH_CHECK(); return rc; }
    return 0;
}

static int km_finalize(lshkm_ctx ctx, const double* sums, const int64_t* counts, int K, int d, const double* C_old,
                       int metric, double min_dist, double* C_new, int* cont) {
    int rc;
    if ((rc = reserve(ctx, WS_FLAG, 64))) return rc;
    LSHKM_HIP(hipMemsetAsync(ctx->ws[WS_FLAG].p, 0, 4, ctx->stream));
    if ((rc = launch_km_finalize(ctx->stream, sums, counts, K, d, C_old, metric, min_dist, C_new, slot<int>(ctx, WS_FLAG)))) { LSHKM_LAUNCH_CHECK(); return rc; }
    int moved = 0;
    if ((rc = d2h(ctx, &moved, ctx->ws[WS_FLAG].p, 4))) return rc;
    if (cont) *cont = moved ? 1 : 0;
    return 0;
}

static int kmeans_update_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int32_t* assign, const double* C_old,
                              int K, int metric, double min_dist, double* C_new, int64_t* counts, int* cont) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && assign && C_old && C_new && N >= 0 && N < (1ll << 31) && d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = reserve(ctx, WS_SUMS, (size_t)K * d * 8)) || (rc = reserve(ctx, WS_CNTS, (size_t)K * 8))) return rc;
    int64_t* cnt = counts ? counts : slot<int64_t>(ctx, WS_CNTS);
    if ((rc = km_sums(ctx, X, N, d, assign, K, slot<double>(ctx, WS_SUMS), cnt))) return rc;
    return km_finalize(ctx, slot<double>(ctx, WS_SUMS), cnt, K, d, C_old, metric, min_dist, C_new, cont);
}

static int kmeans_partial_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int32_t* assign, int K, double* sums,
                               int64_t* counts) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && assign && sums && counts && N >= 0 && N < (1ll << 31) && d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return km_sums(ctx, X, N, d, assign, K, sums, counts);
}

static int kmeans_partial_carry_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int32_t* assign, int K,
                                     const double* carry_sums, const int64_t* carry_counts, double* sums,
                                     int64_t* counts) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && (assign || N == 0) && sums && counts && N >= 0 && N < (1ll << 31) && d > 0 &&
                    K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(sums != carry_sums, LSHKM_ERR_ARG, "sums must not alias carry_sums");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return km_sums(ctx, X, N, d, assign, K, sums, counts, carry_sums, carry_counts);
}

int lshkm_kmeans_update(lshkm_ctx ctx, const float* X, int64_t N, int d, const int32_t* assign, const double* C_old,
                        int K, int metric, double min_dist, double* C_new, int64_t* counts, int* cont) {
    return kmeans_update_impl(ctx, X, N, d, assign, C_old, K, metric, min_dist, C_new, counts, cont);
}

int lshkm_kmeans_update_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int32_t* assign,
                            const double* C_old, int K, int metric, double min_dist, double* C_new, int64_t* counts,
                            int* cont) {
    return kmeans_update_impl(ctx, X, N, d, assign, C_old, K, metric, min_dist, C_new, counts, cont);
}

int lshkm_kmeans_partial(lshkm_ctx ctx, const float* X, int64_t N, int d, const int32_t* assign, int K, double* sums,
                         int64_t* counts) {
    return kmeans_partial_impl(ctx, X, N, d, assign, K, sums, counts);
}

int lshkm_kmeans_partial_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int32_t* assign, int K,
                             double* sums, int64_t* counts) {
    return kmeans_partial_impl(ctx, X, N, d, assign, K, sums, counts);
}

static int kmeans_partial_csr_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int64_t* crow, const int32_t* rows,
                                   int K, double* sums, int64_t* counts) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && crow && (rows || N == 0) && sums && counts && N >= 0 && N < (1ll << 31) &&
                    d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return km_sums(ctx, X, N, d, nullptr, K, sums, counts, nullptr, nullptr, crow, rows);
}

int lshkm_kmeans_partial_csr(lshkm_ctx ctx, const float* X, int64_t N, int d, const int64_t* crow, const int32_t* rows,
                             int K, double* sums, int64_t* counts) {
    return kmeans_partial_csr_impl(ctx, X, N, d, crow, rows, K, sums, counts);
}

int lshkm_kmeans_partial_csr_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int64_t* crow,
                                 const int32_t* rows, int K, double* sums, int64_t* counts) {
    return kmeans_partial_csr_impl(ctx, X, N, d, crow, rows, K, sums, counts);
}

int lshkm_kmeans_partial_carry(lshkm_ctx ctx, const float* X, int64_t N, int d, const int32_t* assign, int K,
                               const double* carry_sums, const int64_t* carry_counts, double* sums, int64_t* counts) {
    return kmeans_partial_carry_impl(ctx, X, N, d, assign, K, carry_sums, carry_counts, sums, counts);
}

int lshkm_kmeans_partial_carry_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int32_t* assign, int K,
                                   const double* carry_sums, const int64_t* carry_counts, double* sums,
                                   int64_t* counts) {
    return kmeans_partial_carry_impl(ctx, X, N, d, assign, K, carry_sums, carry_counts, sums, counts);
}

// ------------------------------------------------------- sharded k-means sums
static int shard_begin_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int64_t* crow, const int32_t* rows, int K,
                            double* sums, double* asum, int32_t* qt, int64_t* counts) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && crow && (rows || N == 0) && sums && asum && qt && counts && N >= 0 &&
                    N < (1ll << 31) && d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ctx->ws_range[11].reserve(km_fx_ws_bytes(K, d)))) return rc;
    if ((rc = launch_km_shard_begin(ctx->stream, X, d, rows, crow, K, N, sums, asum, qt, counts, ctx->ws_range[11].p))) {
        LSHKM_LAUNCH_CHECK();
        return rc;
    }
    return 0;
}

static int shard_prepare_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int64_t* crow, const int32_t* rows, int K,
                              const double* start, const int32_t* flag, const uint8_t* mask, void* ws,
                              int64_t ws_bytes) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && crow && (rows || N == 0) && start && flag && mask && ws && N >= 0 &&
                    N < (1ll << 31) && d > 0 && K > 0 && K <= 65535,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(ws_bytes >= (int64_t)km_shard_ws_bytes(N, K, d), LSHKM_ERR_ARG,
                "workspace smaller than lshkm_kmeans_shard_ws_bytes");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = launch_km_shard_prepare(ctx->stream, X, d, rows, crow, K, N, start, flag, mask, ws))) {
        LSHKM_LAUNCH_CHECK();
        return rc;
    }
    return 0;
}

static int shard_chain_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int64_t* crow, const int32_t* rows, int K,
                            const int32_t* flag, const uint8_t* mask, const double* carry, void* ws, int64_t ws_bytes,
                            double* sums) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && crow && (rows || N == 0) && flag && mask && ws && sums && N >= 0 &&
                    N < (1ll << 31) && d > 0 && K > 0 && K <= 65535,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(ws_bytes >= (int64_t)km_shard_ws_bytes(N, K, d), LSHKM_ERR_ARG,
                "workspace smaller than lshkm_kmeans_shard_ws_bytes");
    LSHKM_CHECK(carry != sums, LSHKM_ERR_ARG, "sums must not alias carry");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = launch_km_shard_chain(ctx->stream, X, d, rows, crow, K, N, flag, mask, carry, ws, sums))) {
        LSHKM_LAUNCH_CHECK();
        return rc;
    }
    return 0;
}

int lshkm_kmeans_shard_begin(lshkm_ctx ctx, const float* X, int64_t N, int d, const int64_t* crow, const int32_t* rows,
                             int K, double* sums, double* asum, int32_t* qt, int64_t* counts) {
    return shard_begin_impl(ctx, X, N, d, crow, rows, K, sums, asum, qt, counts);
}

int lshkm_kmeans_shard_begin_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int64_t* crow,
                                 const int32_t* rows, int K, double* sums, double* asum, int32_t* qt, int64_t* counts) {
    return shard_begin_impl(ctx, X, N, d, crow, rows, K, sums, asum, qt, counts);
}

int lshkm_kmeans_shard_certify(lshkm_ctx ctx, int K, int d, int world, int rank, const double* gathered,
                               const double* asum, const int32_t* qt, const int64_t* counts, double* sums_out,
                               double* start, int32_t* flag, uint8_t* mask, int64_t* n_flagged) {
    LSHKM_CHECK(ctx && K > 0 && d > 0 && world >= 1 && rank >= 0 && rank < world && gathered && asum && qt && counts &&
                    sums_out && flag && mask && n_flagged,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = reserve(ctx, WS_FLAG, 64))) return rc;
    unsigned long long* nf = slot<unsigned long long>(ctx, WS_FLAG);
    if ((rc = launch_km_shard_certify(ctx->stream, gathered, world, rank, asum, qt, counts, K, d, sums_out, start, flag,
                                      mask, nf))) {
        LSHKM_LAUNCH_CHECK();
        return rc;
    }
    unsigned long long h = 0;
    if ((rc = d2h(ctx, &h, nf, 8))) return rc;
    *n_flagged = (int64_t)h;
    return 0;
}

int lshkm_kmeans_shard_ws_bytes(int64_t N, int K, int d, int64_t* bytes) {
    LSHKM_CHECK(bytes && N >= 0 && K > 0 && d > 0, LSHKM_ERR_ARG, "bad arguments");
    *bytes = (int64_t)km_shard_ws_bytes(N, K, d);
    return 0;
}

int lshkm_kmeans_shard_prepare(lshkm_ctx ctx, const float* X, int64_t N, int d, const int64_t* crow,
                               const int32_t* rows, int K, const double* start, const int32_t* flag,
                               const uint8_t* mask, void* ws, int64_t ws_bytes) {
    return shard_prepare_impl(ctx, X, N, d, crow, rows, K, start, flag, mask, ws, ws_bytes);
}

int lshkm_kmeans_shard_prepare_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int64_t* crow,
                                   const int32_t* rows, int K, const double* start, const int32_t* flag,
                                   const uint8_t* mask, void* ws, int64_t ws_bytes) {
    return shard_prepare_impl(ctx, X, N, d, crow, rows, K, start, flag, mask, ws, ws_bytes);
}

int lshkm_kmeans_shard_chain(lshkm_ctx ctx, const float* X, int64_t N, int d, const int64_t* crow, const int32_t* rows,
                             int K, const int32_t* flag, const uint8_t* mask, const double* carry, void* ws,
                             int64_t ws_bytes, double* sums) {
    return shard_chain_impl(ctx, X, N, d, crow, rows, K, flag, mask, carry, ws, ws_bytes, sums);
}

int lshkm_kmeans_shard_chain_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int64_t* crow,
                                 const int32_t* rows, int K, const int32_t* flag, const uint8_t* mask,
                                 const double* carry, void* ws, int64_t ws_bytes, double* sums) {
    return shard_chain_impl(ctx, X, N, d, crow, rows, K, flag, mask, carry, ws, ws_bytes, sums);
}

int lshkm_kmeans_finalize(lshkm_ctx ctx, const double* sums, const int64_t* counts, int K, int d, const double* C_old,
                          int metric, double min_dist, double* C_new, int* cont) {
    LSHKM_CHECK(ctx && sums && counts && C_old && C_new && K > 0 && d > 0, LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return km_finalize(ctx, sums, counts, K, d, C_old, metric, min_dist, C_new, cont);
}

// separate_clusters_from_input (utils.hpp:150-158) as a CSR over the K clusters:
// members of cluster c = rows_dev[crow_dev[c] .. crow_dev[c+1]) in row order.
static int clusters_impl(lshkm_ctx ctx, const int32_t* assign, int64_t N, int K, int64_t* crow, int32_t* rows) {
    return build_csr(ctx, assign, 1, N, K, rows, crow);
}

int lshkm_clusters(lshkm_ctx ctx, const int32_t* assign_dev, int64_t N, int K, int64_t* crow_dev, int32_t* rows_dev) {
    LSHKM_CHECK(ctx && (assign_dev || N == 0) && crow_dev && (rows_dev || N == 0) && N >= 0 && N < (1ll << 31) &&
                    K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return clusters_impl(ctx, assign_dev, N, K, crow_dev, rows_dev);
}

static int silhouette_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int32_t* assign, const double* C, int K,
                           int metric, double* out_host, double* s_dev) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && (assign || N == 0) && C && out_host && N >= 0 && N < (1ll << 31) && d > 0 &&
                    K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN || metric == LSHKM_METRIC_COSINE, LSHKM_ERR_ARG, "unknown metric");
    LSHKM_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    int rc;
    lshkm::Buf& wn = ctx->ws_range[9];     // near [K] int32, then raw [K] + out [K+1] doubles
    lshkm::Buf& ws = ctx->ws_range[10];    // s [N] when the caller gives none
    if ((rc = reserve(ctx, WS_ROWS, (size_t)std::max<int64_t>(N, 1) * 4)) || (rc = reserve(ctx, WS_CROW, (size_t)(K + 1) * 8)) ||
        (rc = wn.reserve((size_t)K * 4 + 8 + (size_t)(2 * K + 1) * 8)) ||
        (!s_dev && (rc = ws.reserve((size_t)std::max<int64_t>(N, 1) * 8))))
        return rc;
    int32_t* near = (int32_t*)wn.p;
    double* raw = (double*)((char*)wn.p + ((size_t)K * 4 + 8) / 8 * 8);
    double* out = raw + K;
    double* sv = s_dev ? s_dev : (double*)ws.p;
    // separate_clusters_from_input (utils.hpp:150-158): members in row order
    if ((rc = build_csr(ctx, assign, 1, N, K, slot<int32_t>(ctx, WS_ROWS), slot<int64_t>(ctx, WS_CROW)))) return rc;
    if ((rc = launch_sil_near(s, C, K, d, metric, near))) return rc;
    // rows on a grid of <= 26 bits (every difference squares exactly): x*x for
    // pow(x, 2) without the per-square test (grid_exact_squares)
    bool exsq = false;
    if (metric == LSHKM_METRIC_EUCLIDEAN) {
        int qt[3];
        if ((rc = reserve(ctx, WS_FLAG, 64)) || (rc = launch_grid_bits(s, X, N * d, slot<int>(ctx, WS_FLAG)))) return rc;
        if ((rc = d2h(ctx, qt, ctx->ws[WS_FLAG].p, sizeof qt))) return rc;
        exsq = grid_exact_squares(qt);
    }
    if ((rc = launch_sil_points(s, X, d, metric, slot<int32_t>(ctx, WS_ROWS), slot<int64_t>(ctx, WS_CROW), assign, near,
                                N, sv, exsq)))
        return rc;
    if ((rc = launch_sil_sum(s, sv, slot<int32_t>(ctx, WS_ROWS), slot<int64_t>(ctx, WS_CROW), K, N, raw, out))) return rc;
    return d2h(ctx, out_host, out, (size_t)(K + 1) * 8);
}

int lshkm_silhouette(lshkm_ctx ctx, const float* X, int64_t N, int d, const int32_t* assign, const double* C, int K,
                     int metric, double* out_host, double* s_dev) {
    return silhouette_impl(ctx, X, N, d, assign, C, K, metric, out_host, s_dev);
}

int lshkm_silhouette_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int32_t* assign, const double* C,
                         int K, int metric, double* out_host, double* s_dev) {
    return silhouette_impl(ctx, X, N, d, assign, C, K, metric, out_host, s_dev);
}

}  // extern "C"

namespace lshkm {
int d2h_batch(lshkm_ctx_s* ctx, const D2H* r, int n) { return d2h_batch_impl(ctx, r, n); }
int h2d_batch(lshkm_ctx_s* ctx, const H2D* r, int n) { return h2d_batch_impl(ctx, r, n); }
}  // namespace lshkm
