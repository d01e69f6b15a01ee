// api_recom.cpp — C ABI of the recommend step (include/lshkm.h): batched
// get_P_closest and get_top_N_recom (lib/crypto_rec.hpp:213-325).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/lshkm.h"
#include "common.h"
#include "index.h"
#include "kernels.h"

using namespace lshkm;

static int read_i64(lshkm_ctx ctx, const int64_t* dev, int64_t* host) {
    LSHKM_HIP(hipMemcpyAsync(host, dev, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
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
