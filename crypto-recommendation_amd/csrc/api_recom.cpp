// api_recom.cpp — C ABI of the recommend step (include/lshkm.h): batched
// get_P_closest and get_top_N_recom (lib/crypto_rec.hpp:213-325).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/lshkm.h"
#include "common.h"
#include "index.h"
#include "kernels.h"

using namespace lshkm;

static int read_i64(lshkm_ctx ctx, const int64_t* dev, int64_t* host) {
    const D2H r{host, dev, sizeof(int64_t)};
    return d2h_batch(ctx, &r, 1);
}

// Host vectors handed to hipMemcpyAsync must outlive the copy: declared after
// them, this waits for the stream on every exit path (its destructor runs
// before theirs).
struct StreamSyncOnExit {
    hipStream_t s;
    ~StreamSyncOnExit() { (void)hipStreamSynchronize(s); }
};

// The users' clusters on the host, each in [0, K): the reference indexes
// clusters[user.getCluster()] (main.cpp:261, :366), so an ID outside the
// clusters is a caller error here, not an empty neighbourhood.
static int read_ucl(lshkm_ctx ctx, const int32_t* ucl, int64_t nq, int K, std::vector<int32_t>& hu) {
    hu.resize((size_t)nq);
    if (nq == 0) return 0;
    const D2H r{hu.data(), ucl, sizeof(int32_t) * nq};
    int rc;
    if ((rc = d2h_batch(ctx, &r, 1))) return rc;
    for (int64_t q = 0; q < nq; q++)
        LSHKM_CHECK(hu[q] >= 0 && hu[q] < K, LSHKM_ERR_ARG, "ucl holds a cluster ID outside [0, K)");
    return 0;
}

extern "C" {

int lshkm_p_closest(lshkm_ctx ctx, const double* X, int64_t N, int d, const double* U, int64_t nq,
                    const int64_t* cand_ptr, const int32_t* cand_idx, int P, int32_t* out_idx, double* out_sim,
                    int32_t* out_cnt) {
    LSHKM_CHECK(ctx && X && U && cand_ptr && out_idx && out_sim && out_cnt && N >= 1 && d >= 1 && nq >= 0 && P >= 1,
                LSHKM_ERR_ARG, "bad arguments");
    if (nq == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    int64_t total = 0;
    int rc;
    if ((rc = read_i64(ctx, cand_ptr + nq, &total))) return rc;
    LSHKM_CHECK(total >= 0 && (total == 0 || cand_idx), LSHKM_ERR_ARG, "bad candidate lists");
    Buf &xa = ctx->ws_call[0], &sim = ctx->ws_call[1], &key = ctx->ws_call[2], &pos = ctx->ws_call[3],
        &replay = ctx->ws_call[4], &count = ctx->ws_call[5];
    const size_t T = (size_t)(total > 0 ? total : 1);
    if ((rc = xa.reserve(sizeof(double) * N)) || (rc = sim.reserve(sizeof(double) * T)) ||
        (rc = key.reserve(sizeof(double) * T)) || (rc = pos.reserve(sizeof(int32_t) * T)) ||
        (rc = replay.reserve(sizeof(int32_t) * nq)) || (rc = count.reserve(sizeof(unsigned int))))
        return rc;
    if ((rc = launch_rc_norms(ctx->stream, X, N, d, xa.as<double>())) ||
        (rc = launch_rc_p_closest(ctx->stream, X, xa.as<double>(), d, U, nq, cand_ptr, cand_idx, P, sim.as<double>(),
                                  key.as<double>(), pos.as<int32_t>(), out_idx, out_sim, out_cnt,
                                  replay.as<int32_t>(), count.as<unsigned int>()))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));   // the workspace is reused by the next call
    return 0;
}

int lshkm_top_n_recom(lshkm_ctx ctx, const double* X, const double* x_mean, int64_t N, int d, const double* u_mean,
                      int64_t nq, const int64_t* unk_ptr, const int32_t* unk_idx, const int32_t* nb_idx,
                      const double* nb_sim, const int32_t* nb_cnt, int P, int n_top, int32_t* out) {
    LSHKM_CHECK(ctx && X && x_mean && u_mean && unk_ptr && nb_idx && nb_sim && nb_cnt && out && N >= 1 && d >= 1 &&
                    nq >= 0 && P >= 1 && n_top >= 0,
                LSHKM_ERR_ARG, "bad arguments");
    if (nq == 0 || n_top == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    int64_t total = 0;
    int rc;
    if ((rc = read_i64(ctx, unk_ptr + nq, &total))) return rc;
    LSHKM_CHECK(total >= 0 && (total == 0 || unk_idx), LSHKM_ERR_ARG, "bad unknown-index lists");
    Buf &pred = ctx->ws_call[0], &pidx = ctx->ws_call[1];
    const size_t M = (size_t)(total > 0 ? total : 1);
    if ((rc = pred.reserve(sizeof(double) * M)) || (rc = pidx.reserve(sizeof(int32_t) * M))) return rc;
    if ((rc = launch_rc_top_n(ctx->stream, X, x_mean, d, u_mean, nq, unk_ptr, unk_idx, nb_idx, nb_sim, nb_cnt, P, n_top,
                              pred.as<double>(), pidx.as<int32_t>(), out))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"

static int terms_offsets(lshkm_ctx ctx, const int64_t* crow, int K, int64_t N, const int32_t* ucl, int64_t nq,
                         const int64_t* unk_ptr, std::vector<int64_t>& soff, std::vector<int64_t>& hup,
                         std::vector<int64_t>& toff, std::vector<int32_t>* hu_out = nullptr);
static int cluster_terms_impl(lshkm_ctx ctx, Pts X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                              const int32_t* crows, int K, Pts U, int64_t nq, const int32_t* ucl,
                              const int64_t* unk_ptr, const int32_t* unk_idx, int64_t* soff_dev, int64_t* toff_dev,
                              double* sims, double* terms, int64_t cap, int64_t tcap, int64_t* total_host,
                              int64_t* tterms_host);
static int chain_terms_impl(lshkm_ctx ctx, int64_t nq, const double* u_mean, const int64_t* unk_ptr,
                            const int32_t* unk_idx, const int64_t* soff, const int64_t* toff, const double* sims,
                            const double* terms, const double* carry_main, const double* carry_abs,
                            const int64_t* carry_cnt, double* main_out, double* abs_out, int64_t* cnt_out, int n_top,
                            int32_t* out);

// get_top_N_recom(neighbors, user, N), crypto_rec.hpp:327-345, over whole
// clusters (main.cpp:260-269, :353-373). The cluster sizes come to the host
// once to size the per-wave similarity scratch (waves x largest cluster).
static int cluster_top_n_impl(lshkm_ctx ctx, Pts X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                              const int32_t* crows, int K, Pts U, const double* u_mean, int64_t nq,
                              const int32_t* ucl, const int64_t* unk_ptr, const int32_t* unk_idx, int n_top,
                              int32_t* out) {
    LSHKM_CHECK(ctx && X.p && x_mean && crow && U.p && u_mean && ucl && unk_ptr && out && N >= 1 && d >= 1 &&
                    K >= 1 && nq >= 0 && n_top >= 0,
                LSHKM_ERR_ARG, "bad arguments");
    if (nq == 0 || n_top == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    {   // the terms form (recom.hip) when the rows stage and the terms fit 2 GiB
        const int64_t rb = (int64_t)d * (X.f64 ? 8 : 4);
        if (rb % 8 == 0 && rb <= 1016) {
            std::vector<int64_t> soff, hup, toff;
            int rc;
            if ((rc = terms_offsets(ctx, crow, K, N, ucl, nq, unk_ptr, soff, hup, toff))) return rc;
            if (toff[nq] <= (1ll << 28)) {
                Buf &bs = ctx->ws_call[0], &bt = ctx->ws_call[5], &bso = ctx->ws_call[6], &bto = ctx->ws_call[7];
                if ((rc = bs.reserve(8 * (size_t)std::max<int64_t>(soff[nq], 1))) ||
                    (rc = bt.reserve(8 * (size_t)std::max<int64_t>(toff[nq], 1))) ||
                    (rc = bso.reserve(8 * (size_t)(nq + 1))) || (rc = bto.reserve(8 * (size_t)(nq + 1))))
                    return rc;
                int64_t tot = 0, tt = 0;
                if ((rc = cluster_terms_impl(ctx, X, x_mean, N, d, crow, crows, K, U, nq, ucl, unk_ptr, unk_idx,
                                             bso.as<int64_t>(), bto.as<int64_t>(), bs.as<double>(), bt.as<double>(),
                                             soff[nq], toff[nq], &tot, &tt)))
                    return rc;
                return chain_terms_impl(ctx, nq, u_mean, unk_ptr, unk_idx, bso.as<int64_t>(), bto.as<int64_t>(),
                                        bs.as<double>(), bt.as<double>(), nullptr, nullptr, nullptr, nullptr, nullptr,
                                        nullptr, n_top, out);
            }
        }
    }
    std::vector<int64_t> hc((size_t)K + 1);
    std::vector<int32_t> hu;
    int64_t total = 0;
    {
        int rc;
        if ((rc = read_ucl(ctx, ucl, nq, K, hu))) return rc;
    }
    {
        const D2H rd[2] = {{hc.data(), crow, sizeof(int64_t) * (K + 1)}, {&total, unk_ptr + nq, sizeof(int64_t)}};
        int rc;
        if ((rc = d2h_batch(ctx, rd, 2))) return rc;
    }
    int64_t maxn = 0;
    bool ok = hc[0] == 0;
    for (int c = 0; c < K && ok; c++) {
        ok = hc[c + 1] >= hc[c];
        maxn = std::max<int64_t>(maxn, hc[c + 1] - hc[c]);
    }
    LSHKM_CHECK(ok && hc[K] <= N && (hc[K] == 0 || crows), LSHKM_ERR_ARG,
                "bad cluster CSR (crow must start at 0, not decrease, and hold at most N members)");
    LSHKM_CHECK(maxn < (1ll << 31), LSHKM_ERR_ARG, "a cluster of 2^31 members or more");
    LSHKM_CHECK(total >= 0 && (total == 0 || unk_idx), LSHKM_ERR_ARG, "bad unknown-index lists");
    // one wave per user in flight; the scratch row of a wave holds one cluster's
    // similarities (at most 1 GiB of scratch: fewer waves for huge clusters)
    const int64_t row = std::max<int64_t>(maxn, 1);
    int64_t nw = std::min<int64_t>(nq, 8192);
    nw = std::min<int64_t>(nw, std::max<int64_t>((int64_t)RC_CLUSTER_WAVES_PER_BLOCK, (1ll << 30) / (row * 8)));
    nw = (nw + RC_CLUSTER_WAVES_PER_BLOCK - 1) / RC_CLUSTER_WAVES_PER_BLOCK * RC_CLUSTER_WAVES_PER_BLOCK;
    Buf &scratch = ctx->ws_call[0], &pred = ctx->ws_call[1], &pidx = ctx->ws_call[2];
    const size_t M = (size_t)(total > 0 ? total : 1);
    int rc;
    if ((rc = scratch.reserve(sizeof(double) * (size_t)nw * row)) || (rc = pred.reserve(sizeof(double) * M)) ||
        (rc = pidx.reserve(sizeof(int32_t) * M)))
        return rc;
    if ((rc = launch_rc_cluster_top_n(ctx->stream, X, x_mean, d, crow, crows, K, U, u_mean, nq, ucl, unk_ptr, unk_idx,
                                      n_top, scratch.as<double>(), row, (int)nw, pred.as<double>(), pidx.as<int32_t>(),
                                      out, (unsigned long long*)ctx->stats.p + STAT_REC_SOFT))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));   // the workspace is reused by the next call
    return 0;
}

// Host view of the cluster CSR: every user's member count on this shard and
// the prefix offsets of its similarities.
// unk_ptr / hup (optional): the unknown-index CSR offsets, read in the same
// batch of copies (one stream synchronisation for all three)
static int shard_offsets(lshkm_ctx ctx, const int64_t* crow, int K, int64_t N, const int32_t* ucl, int64_t nq,
                         std::vector<int64_t>& soff, std::vector<int32_t>* hu_out = nullptr,
                         const int64_t* unk_ptr = nullptr, std::vector<int64_t>* hup = nullptr) {
    std::vector<int64_t> hc((size_t)K + 1);
    std::vector<int32_t> hu((size_t)nq);
    if (hup) hup->assign((size_t)nq + 1, 0);
    const D2H rd[3] = {{hc.data(), crow, sizeof(int64_t) * (K + 1)},
                       {hu.data(), ucl, sizeof(int32_t) * nq},
                       {hup ? hup->data() : nullptr, unk_ptr, hup ? sizeof(int64_t) * (nq + 1) : 0}};
    int rc;
    if ((rc = d2h_batch(ctx, rd, 3))) return rc;
    for (int64_t q = 0; q < nq; q++)
        LSHKM_CHECK(hu[q] >= 0 && hu[q] < K, LSHKM_ERR_ARG, "ucl holds a cluster ID outside [0, K)");
    bool ok = hc[0] == 0;
    for (int c = 0; c < K && ok; c++) ok = hc[c + 1] >= hc[c];
    LSHKM_CHECK(ok && hc[K] <= N, LSHKM_ERR_ARG, "bad cluster CSR");
    soff.assign((size_t)nq + 1, 0);
    for (int64_t q = 0; q < nq; q++) {
        const int64_t n = hc[hu[q] + 1] - hc[hu[q]];
        LSHKM_CHECK(n < (1ll << 31), LSHKM_ERR_ARG, "a cluster of 2^31 members or more");
        soff[q + 1] = soff[q] + n;
    }
    if (hu_out) hu_out->swap(hu);
    return 0;
}

static int cluster_sims_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const int64_t* crow, const int32_t* crows, int K,
                             Pts U, int64_t nq, const int32_t* ucl, const int64_t* unk_ptr, int64_t* soff_dev,
                             double* sims, int64_t cap, int64_t* total_host) {
    LSHKM_CHECK(ctx && X.p && crow && U.p && ucl && unk_ptr && soff_dev && total_host && N >= 1 && d >= 1 && K >= 1 &&
                    nq >= 0 && cap >= 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    std::vector<int64_t> soff;
    const StreamSyncOnExit sync_guard{ctx->stream};   // soff is copied before return
    int rc;
    if ((rc = shard_offsets(ctx, crow, K, N, ucl, nq, soff))) return rc;
    *total_host = soff[nq];
    const H2D up{soff_dev, soff.data(), sizeof(int64_t) * (nq + 1)};
    if ((rc = h2d_batch(ctx, &up, 1))) return rc;
    if (sims && soff[nq] <= cap && soff[nq] > 0) {
        LSHKM_CHECK(crows, LSHKM_ERR_ARG, "crows is NULL");
        if ((rc = launch_rc_shard_sims(ctx->stream, X, d, crow, crows, K, U, nq, ucl, unk_ptr, soff_dev, sims,
                                       (unsigned long long*)ctx->stats.p + STAT_REC_SOFT)))
            return rc;
    }
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

static int cluster_chain_impl(lshkm_ctx ctx, Pts X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                              const int32_t* crows, int K, int64_t nq, const int32_t* ucl, const double* u_mean,
                              const int64_t* unk_ptr, const int32_t* unk_idx, const int64_t* soff, const double* sims,
                              const double* carry_main, const double* carry_abs, const int64_t* carry_cnt,
                              double* main_out, double* abs_out, int64_t* cnt_out, int n_top, int32_t* out) {
    LSHKM_CHECK(ctx && X.p && x_mean && crow && ucl && u_mean && unk_ptr && soff && N >= 1 && d >= 1 && K >= 1 &&
                    nq >= 0 && n_top >= 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK((carry_main == nullptr) == (carry_abs == nullptr) && (carry_abs == nullptr) == (carry_cnt == nullptr),
                LSHKM_ERR_ARG, "carry_main / carry_abs / carry_cnt: all or none");
    LSHKM_CHECK(out || (main_out && abs_out && cnt_out), LSHKM_ERR_ARG, "either the carry outputs or out");
    if (nq == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    int64_t total = 0;
    int rc;
    std::vector<int32_t> hu;
    if ((rc = read_ucl(ctx, ucl, nq, K, hu))) return rc;
    if ((rc = read_i64(ctx, unk_ptr + nq, &total))) return rc;
    LSHKM_CHECK(total >= 0 && (total == 0 || unk_idx), LSHKM_ERR_ARG, "bad unknown-index lists");
    Buf &pred = ctx->ws_call[1], &pidx = ctx->ws_call[2];
    const size_t M = (size_t)(total > 0 ? total : 1);
    if (out && ((rc = pred.reserve(sizeof(double) * M)) || (rc = pidx.reserve(sizeof(int32_t) * M)))) return rc;
    if ((rc = launch_rc_shard_chain(ctx->stream, X, x_mean, d, crow, crows, K, nq, ucl, u_mean, unk_ptr, unk_idx, soff,
                                    sims, carry_main, carry_abs, carry_cnt, out ? nullptr : main_out,
                                    out ? nullptr : abs_out, out ? nullptr : cnt_out, n_top, pred.as<double>(),
                                    pidx.as<int32_t>(), out))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    if (out) LSHKM_HIP(hipStreamSynchronize(ctx->stream));   // pred / pidx workspace reused by the next call
    return 0;
}

// ----------------------------------------------------------- terms form
// Host offsets of the terms form: soff (members per user on this shard), the
// unknown-index CSR (hup) and toff (terms per user: members x unknown indexes).
static int terms_offsets(lshkm_ctx ctx, const int64_t* crow, int K, int64_t N, const int32_t* ucl, int64_t nq,
                         const int64_t* unk_ptr, std::vector<int64_t>& soff, std::vector<int64_t>& hup,
                         std::vector<int64_t>& toff, std::vector<int32_t>* hu_out) {
    int rc;
    if ((rc = shard_offsets(ctx, crow, K, N, ucl, nq, soff, hu_out, unk_ptr, &hup))) return rc;
    toff.assign((size_t)nq + 1, 0);
    bool ok = hup[0] == 0;
    for (int64_t q = 0; q < nq && ok; q++) {
        ok = hup[q + 1] >= hup[q];
        toff[q + 1] = toff[q] + (soff[q + 1] - soff[q]) * (hup[q + 1] - hup[q]);
    }
    LSHKM_CHECK(ok, LSHKM_ERR_ARG, "bad unknown-index lists (unk_ptr must start at 0 and not decrease)");
    return 0;
}

static int cluster_terms_impl(lshkm_ctx ctx, Pts X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                              const int32_t* crows, int K, Pts U, int64_t nq, const int32_t* ucl,
                              const int64_t* unk_ptr, const int32_t* unk_idx, int64_t* soff_dev, int64_t* toff_dev,
                              double* sims, double* terms, int64_t cap, int64_t tcap, int64_t* total_host,
                              int64_t* tterms_host) {
    LSHKM_CHECK(ctx && X.p && x_mean && crow && U.p && ucl && unk_ptr && soff_dev && toff_dev && total_host &&
                    tterms_host && N >= 1 && d >= 1 && K >= 1 && nq >= 0 && cap >= 0 && tcap >= 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(((int64_t)d * (X.f64 ? 8 : 4)) % 8 == 0 && (int64_t)d * (X.f64 ? 8 : 4) <= 1016, LSHKM_ERR_ARG,
                "the terms form stages rows of a multiple of 8 B up to 1016 B (use lshkm_cluster_sims)");
    LSHKM_HIP(hipSetDevice(ctx->device));
    std::vector<int64_t> soff, hup, toff;
    std::vector<int32_t> hu;                       // the users' clusters (host)
    std::vector<int32_t> pack;                     // the cluster-major work list (staged by h2d_batch)
    int rc;
    if ((rc = terms_offsets(ctx, crow, K, N, ucl, nq, unk_ptr, soff, hup, toff, &hu))) return rc;
    *total_host = soff[nq];
    *tterms_host = toff[nq];
    LSHKM_CHECK(toff[nq] == 0 || unk_idx, LSHKM_ERR_ARG, "unk_idx is NULL");
    const H2D offs[2] = {{soff_dev, soff.data(), sizeof(int64_t) * (nq + 1)},
                         {toff_dev, toff.data(), sizeof(int64_t) * (nq + 1)}};
    if (!(sims && terms && soff[nq] <= cap && toff[nq] <= tcap && soff[nq] > 0)) {
        if ((rc = h2d_batch(ctx, offs, 2))) return rc;
    } else {
        LSHKM_CHECK(crows, LSHKM_ERR_ARG, "crows is NULL");
        Buf& map = ctx->ws_call[8];                  // member -> (user, row); the declined-member list + count
        // mq | mr | the declined list | its count | unorm | the blocks' private lists | their capacities and counts
        if ((rc = map.reserve(24 * (size_t)soff[nq] + 16 + 8 * (size_t)nq + 16 * (size_t)RC_TERMS_GMAX))) return rc;
        int32_t* mq = map.as<int32_t>();
        int64_t* fl = reinterpret_cast<int64_t*>(map.as<char>() + 8 * (size_t)soff[nq]);
        double* unorm = reinterpret_cast<double*>(fl + soff[nq] + 1);     // the users' |u|^2
        int64_t* fregion = reinterpret_cast<int64_t*>(unorm + nq);
        int64_t* faux = fregion + soff[nq];
        // cluster-major work list: the users of each cluster (ascending) and the
        // 64-member chunks of the cluster's rows on this shard, each staged once
        // for all of them (rc_terms_cl_kernel)
        std::vector<int32_t> byc;
        byc.reserve((size_t)nq);
        for (int64_t q = 0; q < nq; q++)
            if (soff[q + 1] > soff[q]) byc.push_back((int32_t)q);
        std::stable_sort(byc.begin(), byc.end(), [&](int32_t a, int32_t b) { return hu[a] < hu[b]; });
        // one host buffer, one copy: ioff [G + 1] | gcl [G] | gptr [G + 1] | gusr
        std::vector<int32_t> gcl, gptr(1, 0), ioff(1, 0);
        for (size_t k = 0; k < byc.size(); k++) {
            const int32_t q = byc[k];
            if (k == 0 || hu[q] != hu[byc[k - 1]]) {
                if (k) gptr.push_back((int32_t)k);
                gcl.push_back(hu[q]);
                const int64_t n = soff[q + 1] - soff[q];
                ioff.push_back(ioff.back() + (int32_t)((n + 63) / 64));
            }
        }
        gptr.push_back((int32_t)byc.size());
        const size_t nG = gcl.size();
        pack.reserve(3 * nG + 2 + byc.size());
        pack.insert(pack.end(), ioff.begin(), ioff.end());
        pack.insert(pack.end(), gcl.begin(), gcl.end());
        pack.insert(pack.end(), gptr.begin(), gptr.end());
        pack.insert(pack.end(), byc.begin(), byc.end());
        Buf& gb = ctx->ws_call[9];
        const int64_t nitems = nG ? (int64_t)ioff.back() : 0;
        // the item and user records after the list
        const size_t item_off = (4 * std::max<size_t>(pack.size(), 1) + 255) / 256 * 256;
        const size_t user_off = item_off + (RC_ITEM_BYTES * (size_t)std::max<int64_t>(nitems, 1) + 255) / 256 * 256;
        if ((rc = gb.reserve(user_off + RC_USER_BYTES * std::max<size_t>(byc.size(), 1)))) return rc;
        int32_t* dp = gb.as<int32_t>();
        const H2D up[3] = {offs[0], offs[1], {dp, pack.data(), 4 * pack.size()}};
        if ((rc = h2d_batch(ctx, up, 3))) return rc;
        const RcGroups groups{dp, (int)nG, nitems, dp + nG + 1, dp + 2 * nG + 1, dp + 3 * nG + 2, gb.as<char>() + item_off,
                              (int64_t)byc.size(), gb.as<char>() + user_off};
        if ((rc = launch_rc_terms(ctx->stream, X, x_mean, d, crow, crows, K, U, nq, ucl, soff_dev, soff[nq], unk_ptr,
                                  unk_idx, toff_dev, sims, terms, mq, mq + soff[nq], fl,
                                  reinterpret_cast<unsigned long long*>(fl + soff[nq]),
                                  (unsigned long long*)ctx->stats.p + STAT_REC_SOFT, unorm, &groups, fregion, faux)))
            return rc;
    }
    // no host synchronisation: the uploads are staged (h2d_batch), the outputs
    // and the workspaces are ordered on the stream
    return 0;
}

static int chain_terms_impl(lshkm_ctx ctx, int64_t nq, const double* u_mean, const int64_t* unk_ptr,
                            const int32_t* unk_idx, const int64_t* soff, const int64_t* toff, const double* sims,
                            const double* terms, const double* carry_main, const double* carry_abs,
                            const int64_t* carry_cnt, double* main_out, double* abs_out, int64_t* cnt_out, int n_top,
                            int32_t* out) {
    LSHKM_CHECK(ctx && u_mean && unk_ptr && soff && toff && nq >= 0 && n_top >= 0, LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK((carry_main == nullptr) == (carry_abs == nullptr) && (carry_abs == nullptr) == (carry_cnt == nullptr),
                LSHKM_ERR_ARG, "carry_main / carry_abs / carry_cnt: all or none");
    LSHKM_CHECK(out || (main_out && abs_out && cnt_out), LSHKM_ERR_ARG, "either the carry outputs or out");
    if (nq == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc;
    // users whose cluster holds >= RC_LONG_MIN members here: their chains by
    // binade segments (the offsets come to the host to find them), in batches of
    // at most ~1 GiB of packed values; the unknown-index total is hu[nq] (one
    // batch of copies, one synchronisation)
    std::vector<int64_t> hs((size_t)nq + 1), ht((size_t)nq + 1), hu((size_t)nq + 1);
    {
        const D2H rd[3] = {{hs.data(), soff, sizeof(int64_t) * (nq + 1)},
                           {ht.data(), toff, sizeof(int64_t) * (nq + 1)},
                           {hu.data(), unk_ptr, sizeof(int64_t) * (nq + 1)}};
        if ((rc = d2h_batch(ctx, rd, 3))) return rc;
    }
    const int64_t total = hu[nq];
    LSHKM_CHECK(total == 0 || unk_idx, LSHKM_ERR_ARG, "unk_idx is NULL");
    Buf &pred = ctx->ws_call[1], &pidx = ctx->ws_call[2];
    const size_t M = (size_t)(total > 0 ? total : 1);
    if (out && ((rc = pred.reserve(sizeof(double) * M)) || (rc = pidx.reserve(sizeof(int32_t) * M)))) return rc;
    std::vector<RcLongUser> lus;
    for (int64_t q = 0; q < nq; q++) {
        const int64_t n = hs[q + 1] - hs[q];
        if (n >= RC_LONG_MIN) lus.push_back(RcLongUser{q, n, hs[q], ht[q], hu[q], hu[q + 1] - hu[q], 0, 0});
    }
    std::vector<int64_t> hcrow;                         // staged by h2d_batch with the user table
    const int64_t long_min = lus.empty() ? INT64_MAX : RC_LONG_MIN;
    for (size_t k0 = 0; k0 < lus.size();) {
        // a batch: users k0 .. k1-1, D = their max m + 1, rows * D * 8 <= 1 GiB (one user at least)
        size_t k1 = k0;
        int64_t rows = 0, D = 1;
        while (k1 < lus.size()) {
            const int64_t D2 = std::max<int64_t>(D, lus[k1].m + 1), rows2 = rows + lus[k1].n;
            if (k1 > k0 && (rows2 * D2 * 8 > (1ll << 30) || rows2 >= (1ll << 31))) break;
            D = D2;
            rows = rows2;
            k1++;
        }
        const int64_t nl = (int64_t)(k1 - k0);
        hcrow.assign(1, 0);
        for (size_t k = k0; k < k1; k++) {
            lus[k].off = hcrow.back();
            hcrow.push_back(hcrow.back() + lus[k].n);
        }
        const size_t wsb = (seg_columns_ws_bytes(rows, (int)nl, (int)D) + 255) / 256 * 256;
        const size_t vb = (size_t)rows * D * 8, cb = (size_t)nl * D * 8;
        const size_t tb = (size_t)nl * sizeof(RcLongUser), rb = (size_t)(nl + 1) * 8;
        const size_t nb = wsb + vb + 2 * cb + tb + rb + (size_t)rows * 4 + 256;
        if ((rc = ctx->ws_long.reserve(nb))) return rc;
        char* b = ctx->ws_long.as<char>();
        RcLong L{};
        L.ws = b;
        L.V = reinterpret_cast<double*>(b + wsb);
        L.carry = L.V + (size_t)rows * D;
        L.sums = L.carry + (size_t)nl * D;
        RcLongUser* tab = reinterpret_cast<RcLongUser*>(L.sums + (size_t)nl * D);
        int64_t* crow = reinterpret_cast<int64_t*>(tab + nl);
        L.iota = reinterpret_cast<int32_t*>(crow + nl + 1);
        L.tab = tab;
        L.crow = crow;
        L.nlong = nl;
        L.rows = rows;
        L.D = (int)D;
        const H2D up[2] = {{tab, lus.data() + k0, tb}, {crow, hcrow.data(), rb}};
        if ((rc = h2d_batch(ctx, up, 2))) return rc;
        if ((rc = launch_rc_long(ctx->stream, sims, terms, carry_main, carry_abs, carry_cnt, u_mean,
                                 out ? nullptr : main_out, out ? nullptr : abs_out, out ? nullptr : cnt_out,
                                 out ? pred.as<double>() : nullptr, L)))
            return rc;
        // a further batch may grow ws_long: not while this one's kernels run
        if (k1 < lus.size()) LSHKM_HIP(hipStreamSynchronize(ctx->stream));
        k0 = k1;
    }
    if ((rc = launch_rc_chain_terms(ctx->stream, nq, soff, unk_ptr, toff, sims, terms, carry_main, carry_abs, carry_cnt, u_mean,
                                    out ? nullptr : main_out, out ? nullptr : abs_out, out ? nullptr : cnt_out,
                                    out ? pred.as<double>() : nullptr, long_min))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    if (out && (rc = launch_rc_top(ctx->stream, nq, soff, carry_cnt, unk_ptr, unk_idx, pred.as<double>(),
                                   pidx.as<int32_t>(), n_top, out))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    // no host synchronisation: the pred / pidx workspace's next user is ordered
    // on the same stream (a reserve that grows it frees through hipFree)
    return 0;
}

extern "C" {

int lshkm_cluster_sims(lshkm_ctx ctx, const float* X, int64_t N, int d, const int64_t* crow, const int32_t* crows,
                       int K, const float* U, int64_t nq, const int32_t* ucl, const int64_t* unk_ptr,
                       int64_t* soff, double* sims, int64_t cap, int64_t* total) {
    return cluster_sims_impl(ctx, X, N, d, crow, crows, K, U, nq, ucl, unk_ptr, soff, sims, cap, total);
}

int lshkm_cluster_sims_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const int64_t* crow,
                           const int32_t* crows, int K, const double* U, int64_t nq, const int32_t* ucl,
                           const int64_t* unk_ptr, int64_t* soff, double* sims, int64_t cap, int64_t* total) {
    return cluster_sims_impl(ctx, X, N, d, crow, crows, K, U, nq, ucl, unk_ptr, soff, sims, cap, total);
}

int lshkm_cluster_chain(lshkm_ctx ctx, const float* X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                        const int32_t* crows, int K, int64_t nq, const int32_t* ucl, const double* u_mean,
                        const int64_t* unk_ptr, const int32_t* unk_idx, const int64_t* soff, const double* sims,
                        const double* carry_main, const double* carry_abs, const int64_t* carry_cnt,
                        double* main_out, double* abs_out, int64_t* cnt_out, int n_top, int32_t* out) {
    return cluster_chain_impl(ctx, X, x_mean, N, d, crow, crows, K, nq, ucl, u_mean, unk_ptr, unk_idx, soff, sims,
                              carry_main, carry_abs, carry_cnt, main_out, abs_out, cnt_out, n_top, out);
}

int lshkm_cluster_chain_f64(lshkm_ctx ctx, const double* X, const double* x_mean, int64_t N, int d,
                            const int64_t* crow, const int32_t* crows, int K, int64_t nq, const int32_t* ucl,
                            const double* u_mean, const int64_t* unk_ptr, const int32_t* unk_idx, const int64_t* soff,
                            const double* sims, const double* carry_main, const double* carry_abs,
                            const int64_t* carry_cnt, double* main_out, double* abs_out, int64_t* cnt_out, int n_top,
                            int32_t* out) {
    return cluster_chain_impl(ctx, X, x_mean, N, d, crow, crows, K, nq, ucl, u_mean, unk_ptr, unk_idx, soff, sims,
                              carry_main, carry_abs, carry_cnt, main_out, abs_out, cnt_out, n_top, out);
}

int lshkm_cluster_terms(lshkm_ctx ctx, const float* X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                        const int32_t* crows, int K, const float* U, int64_t nq, const int32_t* ucl,
                        const int64_t* unk_ptr, const int32_t* unk_idx, int64_t* soff, int64_t* toff, double* sims,
                        double* terms, int64_t cap, int64_t tcap, int64_t* total, int64_t* tterms) {
    return cluster_terms_impl(ctx, X, x_mean, N, d, crow, crows, K, U, nq, ucl, unk_ptr, unk_idx, soff, toff, sims,
                              terms, cap, tcap, total, tterms);
}

int lshkm_cluster_terms_f64(lshkm_ctx ctx, const double* X, const double* x_mean, int64_t N, int d,
                            const int64_t* crow, const int32_t* crows, int K, const double* U, int64_t nq,
                            const int32_t* ucl, const int64_t* unk_ptr, const int32_t* unk_idx, int64_t* soff,
                            int64_t* toff, double* sims, double* terms, int64_t cap, int64_t tcap, int64_t* total,
                            int64_t* tterms) {
    return cluster_terms_impl(ctx, X, x_mean, N, d, crow, crows, K, U, nq, ucl, unk_ptr, unk_idx, soff, toff, sims,
                              terms, cap, tcap, total, tterms);
}

int lshkm_cluster_chain_terms(lshkm_ctx ctx, int64_t nq, const double* u_mean, const int64_t* unk_ptr,
                              const int32_t* unk_idx, const int64_t* soff, const int64_t* toff, const double* sims,
                              const double* terms, const double* carry_main, const double* carry_abs,
                              const int64_t* carry_cnt, double* main_out, double* abs_out, int64_t* cnt_out,
                              int n_top, int32_t* out) {
    return chain_terms_impl(ctx, nq, u_mean, unk_ptr, unk_idx, soff, toff, sims, terms, carry_main, carry_abs,
                            carry_cnt, main_out, abs_out, cnt_out, n_top, out);
}

int lshkm_cluster_top_n(lshkm_ctx ctx, const float* X, const double* x_mean, int64_t N, int d, const int64_t* crow,
                        const int32_t* crows, int K, const float* U, const double* u_mean, int64_t nq,
                        const int32_t* ucl, const int64_t* unk_ptr, const int32_t* unk_idx, int n_top, int32_t* out) {
    return cluster_top_n_impl(ctx, X, x_mean, N, d, crow, crows, K, U, u_mean, nq, ucl, unk_ptr, unk_idx, n_top, out);
}

int lshkm_cluster_top_n_f64(lshkm_ctx ctx, const double* X, const double* x_mean, int64_t N, int d,
                            const int64_t* crow, const int32_t* crows, int K, const double* U, const double* u_mean,
                            int64_t nq, const int32_t* ucl, const int64_t* unk_ptr, const int32_t* unk_idx, int n_top,
                            int32_t* out) {
    return cluster_top_n_impl(ctx, X, x_mean, N, d, crow, crows, K, U, u_mean, nq, ucl, unk_ptr, unk_idx, n_top, out);
}

}  // extern "C"
