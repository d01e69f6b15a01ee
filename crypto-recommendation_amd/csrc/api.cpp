// api.cpp — the C ABI (include/lshkm.h): contexts, handles, parameter
// generation in the reference's RNG draw order, and stream-ordered launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/lshkm.h"
#include "common.h"
#include "kernels.h"
#include "index.h"

namespace lshkm {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace lshkm

using namespace lshkm;

// ---------------------------------------------------------------- device buffers
namespace lshkm {

Buf::~Buf() { if (p) (void)hipFree(p); }
int Buf::reserve(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    if (hipMalloc(&p, bytes) != hipSuccess) { set_error("hipMalloc failed (" + std::to_string(bytes) + " B)"); p = nullptr; return LSHKM_ERR_NOMEM; }
    cap = bytes;
    return 0;
}

}  // namespace lshkm

extern "C" {

const char* lshkm_last_error(void) { return g_err.c_str(); }
const char* lshkm_version(void) { return "lshkm-gfx950 0.1"; }

int lshkm_ctx_create(int device, lshkm_ctx* out) {
    LSHKM_CHECK(out, LSHKM_ERR_ARG, "out is NULL");
    *out = nullptr;
    // the pow contract (gpow2.h), once per process, before any device work
    if (const int rc = pow_contract_check()) return rc;
    int n = 0;
    LSHKM_HIP(hipGetDeviceCount(&n));
    LSHKM_CHECK(device >= 0 && device < n, LSHKM_ERR_ARG, "device out of range");
    LSHKM_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    LSHKM_HIP(hipGetDeviceProperties(&prop, device));
    LSHKM_CHECK(std::string(prop.gcnArchName).find("gfx950") != std::string::npos, LSHKM_ERR_UNSUPPORTED,
                std::string("liblshkm is built for gfx950 only; device is ") + prop.gcnArchName);
    lshkm_ctx c = new lshkm_ctx_s();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) { delete c; set_error("stream create failed"); return LSHKM_ERR_HIP; }
    c->stream = c->own_stream;
    if (c->stats.reserve(sizeof(unsigned long long) * STAT_COUNT)) { delete c; return LSHKM_ERR_NOMEM; }
    (void)hipMemsetAsync(c->stats.p, 0, sizeof(unsigned long long) * STAT_COUNT, c->stream);
    *out = c;
    return 0;
}

int lshkm_ctx_set_stream(lshkm_ctx ctx, void* s) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    ctx->stream = (hipStream_t)s;   // verbatim: NULL is the default (null) stream
    return 0;
}

int lshkm_ctx_set_dist_mode(lshkm_ctx ctx, int mode) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    LSHKM_CHECK(mode == LSHKM_DIST_CERTIFIED || mode == LSHKM_DIST_EXACT, LSHKM_ERR_ARG,
                "unknown distance mode (LSHKM_DIST_CERTIFIED or LSHKM_DIST_EXACT)");
    ctx->dist_mode = mode;
    return 0;
}

int lshkm_ctx_get_dist_mode(lshkm_ctx ctx, int* mode) {
    LSHKM_CHECK(ctx && mode, LSHKM_ERR_ARG, "bad arguments");
    *mode = ctx->dist_mode;
    return 0;
}

int lshkm_ctx_sync(lshkm_ctx ctx) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

int lshkm_dev_alloc(lshkm_ctx ctx, int64_t bytes, void** out) {
    LSHKM_CHECK(ctx && out && bytes >= 0, LSHKM_ERR_ARG, "bad arguments");
    *out = nullptr;
    if (bytes == 0) return 0;
    LSHKM_HIP(hipSetDevice(ctx->device));
    if (hipMalloc(out, (size_t)bytes) != hipSuccess) {
        *out = nullptr;
        set_error("hipMalloc failed (" + std::to_string(bytes) + " B)");
        return LSHKM_ERR_NOMEM;
    }
    return 0;
}

int lshkm_dev_free(lshkm_ctx ctx, void* p) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    if (!p) return 0;
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));   // no launch on the stream may still read it
    LSHKM_HIP(hipFree(p));
    return 0;
}

int lshkm_memcpy_h2d(lshkm_ctx ctx, void* dst_dev, const void* src_host, int64_t bytes) {
    LSHKM_CHECK(ctx && bytes >= 0 && (bytes == 0 || (dst_dev && src_host)), LSHKM_ERR_ARG, "bad arguments");
    if (bytes == 0) return 0;
    LSHKM_HIP(hipMemcpyAsync(dst_dev, src_host, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));   // the host buffer may be reused on return
    return 0;
}

int lshkm_memcpy_d2h(lshkm_ctx ctx, void* dst_host, const void* src_dev, int64_t bytes) {
    LSHKM_CHECK(ctx && bytes >= 0 && (bytes == 0 || (dst_host && src_dev)), LSHKM_ERR_ARG, "bad arguments");
    if (bytes == 0) return 0;
    LSHKM_HIP(hipMemcpyAsync(dst_host, src_dev, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

int lshkm_ctx_destroy(lshkm_ctx ctx) {
    if (!ctx) return 0;
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return 0;
}

int lshkm_get_stat(lshkm_ctx ctx, int which, int64_t* v) {
    LSHKM_CHECK(ctx && v && which >= 0 && which < STAT_COUNT, LSHKM_ERR_ARG, "bad stat query");
    unsigned long long x = 0;
    LSHKM_HIP(hipMemcpyAsync(&x, (unsigned long long*)ctx->stats.p + which, sizeof(x), hipMemcpyDeviceToHost, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    *v = (int64_t)x;
    return 0;
}

int lshkm_ctx_enable_timing(lshkm_ctx ctx, int on) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    for (hipEvent_t& e : ctx->tev)
        if (!e) LSHKM_HIP(hipEventCreate(&e));
    ctx->timing = on != 0;
    return 0;
}

// The fused pass: from before the prep to the later of the main stream's last
// fused launch and the side stream's hash fix-up.
int lshkm_last_kernel_ms(lshkm_ctx ctx, float* ms) {
    LSHKM_CHECK(ctx && ms && ctx->tev[1], LSHKM_ERR_STATE, "timing not enabled");
    LSHKM_HIP(hipEventSynchronize(ctx->tev[1]));
    LSHKM_HIP(hipEventElapsedTime(ms, ctx->tev[0], ctx->tev[1]));
    if (ctx->tev_side) {
        float m2 = 0.f;
        LSHKM_HIP(hipEventSynchronize(ctx->tev[2]));
        LSHKM_HIP(hipEventElapsedTime(&m2, ctx->tev[0], ctx->tev[2]));
        *ms = std::max(*ms, m2);
    }
    return 0;
}

int lshkm_reset_stats(lshkm_ctx ctx) {
    LSHKM_CHECK(ctx, LSHKM_ERR_ARG, "ctx is NULL");
    LSHKM_HIP(hipMemsetAsync(ctx->stats.p, 0, sizeof(unsigned long long) * STAT_COUNT, ctx->stream));
    return 0;
}

// ------------------------------------------------------------ parameter generation
// The reference's generators draw from one std::default_random_engine seeded
// with the clock (lsh_cube.hpp:49-51); each EuclideanHGen owns a fresh
// normal_distribution<float> (euclidean_h_gen.hpp:58) so an odd d drops the
// cached second variate; CosineHGen likewise with double (cosine_h_gen.hpp:54).
static uint32_t engine_state(std::default_random_engine& g) {
    std::ostringstream os;
    os << g;
    return (uint32_t)std::stoul(os.str());
}

static void draw_euclid_h(std::default_random_engine& g, int d, float w, float* v, float* t) {
    std::normal_distribution<float> nd(0, 1);
    for (int j = 0; j < d; j++) v[j] = nd(g);
    std::uniform_real_distribution<float> ud(0, w);
    *t = ud(g);
}

static void draw_cosine_h(std::default_random_engine& g, int d, double* r) {
    std::normal_distribution<double> nd(0, 1);
    for (int j = 0; j < d; j++) r[j] = nd(g);
}

int lshkm_params_lsh_euclidean(uint64_t seed, int L, int k, int d, float w, float* V, float* t, int32_t* r,
                               uint32_t* state) {
    LSHKM_CHECK(L > 0 && k > 0 && d > 0 && V && t && r, LSHKM_ERR_ARG, "bad arguments");
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    for (int l = 0; l < L; l++) {
        std::uniform_int_distribution<int> uid(0, 100);   // euclidean_phi_gen.hpp:63
        for (int i = 0; i < k; i++) {
            const size_t li = (size_t)l * k + i;
            draw_euclid_h(g, d, w, V + li * d, t + li);
            r[li] = uid(g);
        }
    }
    if (state) *state = engine_state(g);
    return 0;
}

int lshkm_params_lsh_cosine(uint64_t seed, int L, int k, int d, double* R, uint32_t* state) {
    LSHKM_CHECK(L > 0 && k > 0 && d > 0 && R, LSHKM_ERR_ARG, "bad arguments");
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    for (int l = 0; l < L; l++)
        for (int i = 0; i < k; i++) draw_cosine_h(g, d, R + ((size_t)l * k + i) * d);
    if (state) *state = engine_state(g);
    return 0;
}

int lshkm_params_cube_euclidean(uint64_t seed, int k, int d, float w, float* V, float* t, uint32_t* state) {
    LSHKM_CHECK(k > 0 && d > 0 && V && t, LSHKM_ERR_ARG, "bad arguments");
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    for (int i = 0; i < k; i++) draw_euclid_h(g, d, w, V + (size_t)i * d, t + i);
    if (state) *state = engine_state(g);
    return 0;
}

// EuclideanF coins on the host (sharded builds): per entry in order,
// c = uniform_int_distribution<int>(1, 2) over the shared minstd_rand0
// (euclidean_f_gen.hpp:68-76), bit = mod(h, c) (utils.hpp:97-98). libstdc++'s
// own engine and distribution, resumed from the engine state value.
int lshkm_coins_draw(uint32_t* rng_state, const int32_t* h, int64_t n, int32_t* bit) {
    LSHKM_CHECK(rng_state && n >= 0 && (n == 0 || (h && bit)), LSHKM_ERR_ARG, "bad arguments");
    std::default_random_engine g;
    g.seed((unsigned long)*rng_state);
    LSHKM_CHECK(engine_state(g) == *rng_state, LSHKM_ERR_ARG, "rng_state is not a minstd_rand0 state");
    for (int64_t i = 0; i < n; i++) {
        std::uniform_int_distribution<int> coin(1, 2);
        const int c = coin(g);
        bit[i] = (h[i] % c + c) % c;
    }
    *rng_state = engine_state(g);
    return 0;
}

int lshkm_rand_selection(uint64_t seed, int64_t N, int K, int32_t* rows) {
    LSHKM_CHECK(rows && N >= 1 && N <= INT32_MAX && K >= 1 && K <= N, LSHKM_ERR_ARG,
                "bad arguments (need 1 <= K <= N < 2^31)");
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    std::uniform_int_distribution<int> uni(0, (int)(N - 1));
    rows[0] = uni(g);
    for (int i = 1; i < K; i++) {
        int r = uni(g), c = 0;
        while (c < i) {          // redraw on a repeat and check all again (initialization.hpp:53-61)
            if (rows[c] == r) { r = uni(g); c = 0; }
            else c++;
        }
        rows[i] = r;
    }
    return 0;
}

}  // extern "C"

static int kmeans_pp_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, int K, int metric, uint64_t seed, int32_t* rows) {
    LSHKM_CHECK(ctx && X.p && rows && N >= 1 && N <= INT32_MAX && d >= 1 && d <= 4096 && K >= 1, LSHKM_ERR_ARG,
                "bad arguments (need N < 2^31, 1 <= d <= 4096, K >= 1)");
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN || metric == LSHKM_METRIC_COSINE, LSHKM_ERR_ARG, "unknown metric");
    LSHKM_HIP(hipSetDevice(ctx->device));
    // every engine draw of k_means_pp up front (initialization.hpp:75-79,127-128):
    // they do not depend on the data. uniform_real<double>(0, total) is
    // canon * (total - 0) + 0 with canon = uniform_real<double>(0, 1).
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    std::uniform_int_distribution<int> uni(0, (int)(N - 1));
    std::vector<int32_t> chosen(K, 0);
    std::vector<double> canon(K, 0.0);
    chosen[0] = uni(g);
    for (int i = 1; i < K; i++) {
        std::uniform_real_distribution<double> unit(0.0, 1.0);
        canon[i] = unit(g);
    }
    Buf &ws = ctx->ws_call[0], &dch = ctx->ws_call[1], &dcanon = ctx->ws_call[2];
    int rc;
    if ((rc = ws.reserve(kmeans_pp_ws_bytes(N))) || (rc = dch.reserve(sizeof(int32_t) * K)) ||
        (rc = dcanon.reserve(sizeof(double) * K)))
        return rc;
    LSHKM_HIP(hipMemcpyAsync(dch.p, chosen.data(), sizeof(int32_t) * K, hipMemcpyHostToDevice, ctx->stream));
    LSHKM_HIP(hipMemcpyAsync(dcanon.p, canon.data(), sizeof(double) * K, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = launch_kmeans_pp(ctx->stream, X, N, d, K, metric, dcanon.as<double>(), dch.as<int32_t>(), ws.p,
                               (unsigned long long*)ctx->stats.p))) {
        (void)hipStreamSynchronize(ctx->stream);
        return rc;
    }
    LSHKM_HIP(hipMemcpyAsync(rows, dch.p, sizeof(int32_t) * K, hipMemcpyDeviceToHost, ctx->stream));
    LSHKM_HIP(hipStreamSynchronize(ctx->stream));
    return 0;
}

extern "C" {

int lshkm_kmeans_pp(lshkm_ctx ctx, const float* X, int64_t N, int d, int K, int metric, uint64_t seed,
                    int32_t* rows) {
    return kmeans_pp_impl(ctx, X, N, d, K, metric, seed, rows);
}

int lshkm_kmeans_pp_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, int K, int metric, uint64_t seed,
                        int32_t* rows) {
    return kmeans_pp_impl(ctx, X, N, d, K, metric, seed, rows);
}

int lshkm_params_cube_cosine(uint64_t seed, int k, int d, double* R, uint32_t* state) {
    LSHKM_CHECK(k > 0 && d > 0 && R, LSHKM_ERR_ARG, "bad arguments");
    std::default_random_engine g;
    g.seed((unsigned long)seed);
    for (int i = 0; i < k; i++) draw_cosine_h(g, d, R + (size_t)i * d);
    if (state) *state = engine_state(g);
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------ projection tables
namespace lshkm {

int ProjTable::upload(hipStream_t s, int metric_, int d_, int L_, int k_, float w_, const float* V, const float* t,
                      const int32_t* r, const double* R) {
    metric = metric_; d = d_; L = L_; k = k_; w = w_;
    LK = L * k;
    LKpad = hash_lkpad(LK);
    const int drows = (d + 3) / 4 * 4;    // zero pad rows: the kernel reads x in float4 steps
    std::vector<double> PT((size_t)drows * LKpad, 0.0), pn(LK, 0.0);
    std::vector<float> tt(LK, 0.f);
    std::vector<int32_t> rr(LK, 0);
    for (int f = 0; f < LK; f++) {
        long double n2 = 0.0L;
        for (int j = 0; j < d; j++) {
            const double v = metric == LSHKM_METRIC_EUCLIDEAN ? (double)V[(size_t)f * d + j] : R[(size_t)f * d + j];
            PT[(size_t)j * LKpad + f] = v;
            n2 += (long double)v * (long double)v;
        }
        pn[f] = (double)sqrtl(n2) * (1.0 + 0x1p-40);
        if (metric == LSHKM_METRIC_EUCLIDEAN) { tt[f] = t ? t[f] : 0.f; rr[f] = r ? r[f] : 0; }
    }
    int rc;
    if ((rc = PT_d.reserve(PT.size() * 8)) || (rc = t_d.reserve(LK * 4)) || (rc = pn_d.reserve(LK * 8)) ||
        (rc = r_d.reserve(LK * 4)))
        return rc;
    LSHKM_HIP(hipMemcpyAsync(PT_d.p, PT.data(), PT.size() * 8, hipMemcpyHostToDevice, s));
    LSHKM_HIP(hipMemcpyAsync(t_d.p, tt.data(), LK * 4, hipMemcpyHostToDevice, s));
    LSHKM_HIP(hipMemcpyAsync(pn_d.p, pn.data(), LK * 8, hipMemcpyHostToDevice, s));
    LSHKM_HIP(hipMemcpyAsync(r_d.p, rr.data(), LK * 4, hipMemcpyHostToDevice, s));
    // split-f16 image for the fused hash+assign kernel (euclidean) and the
    // MFMA hash (either metric; cosine splits the fp64 rows of R)
    // the fused kernels' phi arithmetic assumes the reference's r range
    // [0, 100] (euclidean_phi_gen.hpp:64; tile.h phi_term_small)
    bool r_small = true;
    for (int f = 0; f < LK; f++) r_small = r_small && rr[f] >= 0 && rr[f] <= 100;
    fused_ok = metric == LSHKM_METRIC_EUCLIDEAN && d == 128 && LK <= 32 && r_small;
    mfma_ok = d == 128 && LK <= 32;
    std::vector<_Float16> vh, vl;
    std::vector<double> v1;
    if (mfma_ok) {
        vh.assign(64 * 128, (_Float16)0.f);
        vl.assign(64 * 128, (_Float16)0.f);
        v1.assign(LK, 0.0);
        for (int f = 0; f < LK; f++) {
            long double s1 = 0.0L;
            for (int j = 0; j < 128; j++) {
                const double v = metric == LSHKM_METRIC_EUCLIDEAN ? (double)V[(size_t)f * d + j] : R[(size_t)f * d + j];
                const _Float16 hv = (_Float16)v;
                vh[f * 128 + j] = hv;
                vl[f * 128 + j] = (_Float16)(float)(v - (double)hv);   // v - hv is exact in fp64
                s1 += fabsl((long double)v);
            }
            v1[f] = (double)s1 * (1.0 + 0x1p-40);
        }
        if ((rc = vh_d.reserve(vh.size() * 2)) || (rc = vl_d.reserve(vl.size() * 2)) || (rc = v1_d.reserve(LK * 8)))
            return rc;
        LSHKM_HIP(hipMemcpyAsync(vh_d.p, vh.data(), vh.size() * 2, hipMemcpyHostToDevice, s));
        LSHKM_HIP(hipMemcpyAsync(vl_d.p, vl.data(), vl.size() * 2, hipMemcpyHostToDevice, s));
        LSHKM_HIP(hipMemcpyAsync(v1_d.p, v1.data(), LK * 8, hipMemcpyHostToDevice, s));
    }
    LSHKM_HIP(hipStreamSynchronize(s));   // host vectors go out of scope
    // host copies kept for introspection
    hV.assign(V ? V : (const float*)nullptr, V ? V + (size_t)LK * d : nullptr);
    return 0;
}

HashParams ProjTable::params(int64_t nb) const {
    HashParams p;
    p.PT = (const double*)PT_d.p;
    p.t = (const float*)t_d.p;
    p.pnorm = (const double*)pn_d.p;
    p.r = (const int32_t*)r_d.p;
    p.w = w;
    p.d = d; p.L = L; p.k = k; p.LK = LK; p.LKpad = LKpad;
    p.nb = nb;
    return p;
}

HashMfmaParams ProjTable::mfma_params(int64_t nb) const {
    HashMfmaParams p;
    p.Vh = vh_d.as<_Float16>(); p.Vl = vl_d.as<_Float16>();
    p.t = (const float*)t_d.p; p.pnorm = (const double*)pn_d.p; p.v1 = (const double*)v1_d.p;
    p.r = (const int32_t*)r_d.p; p.PT = (const double*)PT_d.p;
    p.w = w;
    p.d = d; p.L = L; p.k = k; p.LK = LK; p.LKpad = LKpad;
    p.nb = nb;
    return p;
}

}  // namespace lshkm

extern "C" {

// ----------------------------------------------------------------------- LSH
int lshkm_lsh_create(lshkm_ctx ctx, int metric, int d, int k, int L, int64_t nb, float w, const float* V,
                     const float* t, const int32_t* r, const double* R, lshkm_lsh* out) {
    LSHKM_CHECK(ctx && out, LSHKM_ERR_ARG, "ctx/out is NULL");
    LSHKM_CHECK(d > 0 && d <= 1024 && k > 0 && L > 0 && L * k <= 256, LSHKM_ERR_ARG, "unsupported d/k/L");
    LSHKM_CHECK(k <= 30, LSHKM_ERR_ARG, "k > 30");
    if (metric == LSHKM_METRIC_EUCLIDEAN) {
        LSHKM_CHECK(V && t && r, LSHKM_ERR_ARG, "euclidean LSH needs V, t, r");
        LSHKM_CHECK(nb > 0 && nb < (1ll << 31), LSHKM_ERR_ARG, "nb must be in [1, 2^31)");   // mod by 0 crashes the reference
        LSHKM_CHECK(w > 0.f, LSHKM_ERR_ARG, "w must be > 0");
    } else if (metric == LSHKM_METRIC_COSINE) {
        LSHKM_CHECK(R, LSHKM_ERR_ARG, "cosine LSH needs R");
        nb = (int64_t)1 << k;
    } else {
        set_error("unknown metric");
        return LSHKM_ERR_ARG;
    }
    LSHKM_HIP(hipSetDevice(ctx->device));
    lshkm_lsh h = new lshkm_lsh_s();
    h->ctx = ctx; h->metric = metric; h->nb = nb;
    int rc = h->proj.upload(ctx->stream, metric, d, L, k, w, V, t, r, R);
    if (rc) { delete h; return rc; }
    *out = h;
    return 0;
}

int lshkm_lsh_destroy(lshkm_lsh lsh) {
    if (!lsh) return 0;
    (void)hipDeviceSynchronize();   // never touches lsh->ctx: it may already be destroyed
    delete lsh;
    return 0;
}

}  // extern "C"

static int lsh_hash_impl(lshkm_lsh lsh, Pts X, int64_t N, int32_t* tuples, int32_t* phi, int32_t* bucket) {
    LSHKM_CHECK(lsh && (X.p || N == 0) && N >= 0, LSHKM_ERR_ARG, "bad arguments");
    lshkm_ctx ctx = lsh->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    const int mode = lsh->metric == LSHKM_METRIC_EUCLIDEAN ? HM_LSH_EUCLID : HM_LSH_COSINE;
    const int rc = hash_rows(ctx, mode, X, N, lsh->proj, lsh->nb, mode == HM_LSH_EUCLID ? tuples : nullptr, phi, bucket,
                             nullptr);
    if (rc) { LSHKM_LAUNCH_CHECK(); return rc; }
    return 0;
}

extern "C" {

int lshkm_lsh_hash(lshkm_lsh lsh, const float* X, int64_t N, int32_t* tuples, int32_t* phi, int32_t* bucket) {
    return lsh_hash_impl(lsh, X, N, tuples, phi, bucket);
}

int lshkm_lsh_hash_f64(lshkm_lsh lsh, const double* X, int64_t N, int32_t* tuples, int32_t* phi, int32_t* bucket) {
    return lsh_hash_impl(lsh, X, N, tuples, phi, bucket);
}

// ------------------------------------------------------------------- Lloyd
}  // extern "C"

// Kernel path for assignment: d = 128 takes the split-f16 fused kernel
// (persistent form, one launch per 256-centroid slice; cosine: normalised
// centroids), else the f32-MFMA kernel (d <= 256), else the exact pass.
// LSHKM_ASSIGN_PATH = "f32" / "exact" forces a path (tests compare them).
// fp64 rows and fp32 rows of d < 128 dims (d <= 128, K <= 512; either metric)
// take the hi-only form too (path 3: zero-padded dims); other
// fp64 rows the f32-MFMA kernel (rows rounded to f32 on load, the bound
// widened accordingly) or the exact pass.
static int assign_path(int metric, int d, int K, bool f64) {
    if (test_switch("LSHKM_ASSIGN_PATH", "exact")) return 2;
    const bool f32 = test_switch("LSHKM_ASSIGN_PATH", "f32");
    if (d == 128 && !f32 && !f64) {
        if (metric == LSHKM_METRIC_EUCLIDEAN || !test_switch("LSHKM_FUSED_FORM", "chunked")) return 0;
    }
    if (!f32 && d <= 128 && K <= 512 && !test_switch("LSHKM_FUSED_HI", "0")) return 3;
    return assign_dp(d) > 0 ? 1 : 2;
}

// Euclidean winner distances of the hi-only pass (fp32 rows), per context
// (lshkm_ctx_set_dist_mode): LSHKM_DIST_CERTIFIED (default) takes them from
// f32(c) in f32, certified to 2^-20 relative -- inside the 1e-5 relative the
// north star sets for float distances; cluster IDs stay bit-exact, and a row
// whose bound fails gets the reference-order fp64 chain. LSHKM_DIST_EXACT: the
// reference-order fp64 chain for every row (bit-exact distances). The context's
// mode alone decides (no environment override in the product library).
static bool fast_dist_on(const lshkm_ctx_s* ctx) {
    return ctx->dist_mode == LSHKM_DIST_CERTIFIED;
}

// K <= 1024, d <= 256: the exact pass scores every centroid in f32 first and
// runs the exact order only on the candidates the bound leaves (euclidean, and
// cosine on fp32 rows); LSHKM_EXACT_PASS=full: every centroid
static bool exact_pruned(Pts X, int d, int K, int metric) {
    return K <= 1024 && d <= 256 && !test_switch("LSHKM_EXACT_PASS", "full") &&
           (metric == LSHKM_METRIC_EUCLIDEAN || !X.f64);
}

// The pruned pass's centroid prep ahead of the fused pass (ws_ct): the listed
// rows' pass then starts as soon as the refinement ends.
static int exact_listed_prep(lshkm_ctx ctx, Pts X, int d, const double* C, int K, int metric) {
    int rc;
    if ((rc = ctx->ws_ct.reserve((size_t)d * ((K + 255) / 256 * 256) * 8))) return rc;
    return launch_assign_pruned_prep(ctx->stream, X.f64, d, C, K, (float*)ctx->ws_ct.p,
                                     metric == LSHKM_METRIC_EUCLIDEAN ? 0 : 1);
}

// Exact reference-order pass over the rows listed in ws_ambig (count on device).
// Segmented lists (seg_counts != NULL) come from the persistent fused form.
// prepped: exact_listed_prep ran for these centroids on this stream.
static int exact_listed(lshkm_ctx ctx, Pts X, int d, const double* C, int K, int metric,
                        const unsigned long long* cnt, int64_t N, int32_t* assign, double* dist,
                        const int32_t* seg_counts = nullptr, int64_t seg_rows = 0, int nseg = 0,
                        const int32_t* rows = nullptr, bool exact_dist = true, bool prepped = false,
                        const double* xn2 = nullptr, const double* nbv = nullptr) {
    if (!rows) rows = (const int32_t*)ctx->ws_ambig.p;
    const bool prune = exact_pruned(X, d, K, metric);
    if (!prune && (metric != LSHKM_METRIC_EUCLIDEAN || (!seg_counts && d > 256)))
        return launch_assign_exact(ctx->stream, X, N, d, C, K, metric, rows, cnt, N, assign, dist, seg_counts,
                                   seg_rows, nseg, xn2, nbv);
    int rc;
    if ((rc = ctx->ws_ct.reserve((size_t)d * ((K + 255) / 256 * 256) * 8))) return rc;
    if (prune)
        return launch_assign_pruned_list(ctx->stream, X, d, C, K, (float*)ctx->ws_ct.p, rows, cnt, N, assign, dist,
                                         seg_counts, seg_rows, nseg, metric == LSHKM_METRIC_EUCLIDEAN ? 0 : 1,
                                         exact_dist ? 1 : 0, prepped);
    return launch_assign_exact_list(ctx->stream, X, d, C, K, (double*)ctx->ws_ct.p, rows, cnt, N, assign, dist,
                                    seg_counts, seg_rows, nseg);
}

// force_exact: exact distances whatever the context's mode (range
// assignment's leftover rows: a range assignment is exact-order in either mode)
static int assign_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const double* C, int K, int metric,
                       const int32_t* src_rows_host, int32_t* assign, double* dist, lshkm_lsh lsh, int32_t* tuples,
                       int32_t* phi, int32_t* bucket, bool force_exact = false) {
    hipStream_t s = ctx->stream;
    const int DP = assign_dp(d);
    const int path = assign_path(metric, d, K, X.f64);
    // one pass for hashing + assignment: the euclidean index with euclidean
    // Lloyd (fused_ok: d = 128, L*k <= 32), or the cosine index with cosine Lloyd
    // on the hi-only form (k = 4)
    const bool hi_form = !test_switch("LSHKM_FUSED_HI", "0");
    const bool fuse_hash = lsh && path == 0 && lsh->metric == metric &&
                           (metric == LSHKM_METRIC_EUCLIDEAN ? lsh->proj.fused_ok
                                                             : (hi_form && lsh->proj.mfma_ok && lsh->proj.k == 4));
    int rc;
    if (lsh && !fuse_hash && (rc = hash_rows(ctx, lsh->metric == LSHKM_METRIC_EUCLIDEAN ? HM_LSH_EUCLID : HM_LSH_COSINE,
                                             X, N, lsh->proj, lsh->nb,
                                             lsh->metric == LSHKM_METRIC_EUCLIDEAN ? tuples : nullptr, phi, bucket,
                                             nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
    if (path == 0 || path == 3) {
        const int rows_kind = path == 3 ? (X.f64 ? 2 : 1) : 0;
        const int Kpad = (K + 63) / 64 * 64;
        const bool cosine = metric != LSHKM_METRIC_EUCLIDEAN;
        // hi-only scoring + 3-product refinement; test switch LSHKM_FUSED_HI=0: the 3-product form alone
        const bool hi = hi_form;
        // euclidean winner distances: the certified f32 form (default) or the
        // reference-order fp64 chain (LSHKM_DIST_EXACT)
        const bool fast = !cosine && rows_kind != 2 && !force_exact && fast_dist_on(ctx);
        // exact distances of the hi-only pass: rows whose chain met an inexact
        // square (glibc's pow(x, 2) may differ from x*x) are listed for the fix-up
        const bool pwfix = !cosine && hi && !fast;
        // ws_hfix regions: [hash fix-ups] then, cosine: [declines of the hi-only
        // pass][declines of the refinement]; euclidean exact: [pow fix-ups]
        const int nfix_regions = 1 + (cosine && hi ? 2 : 0) + (pwfix ? 1 : 0);
        const int64_t list_cap = N + FUSED_LIST_SLACK;
        const int64_t part_tiles = std::max<int64_t>((N + 31) / 32, (list_cap + 31) / 32 + FUSED_MAX_SEGS);
        if ((rc = ctx->ws_c32.reserve((size_t)Kpad * 128 * 2 * 2)) ||
            (rc = ctx->ws_cconst.reserve((size_t)(Kpad + 8) * 4 + (size_t)Kpad * 8)) ||
            (rc = ctx->ws_ambig.reserve((size_t)(N + FUSED_LIST_SLACK) * 4)) || (rc = ctx->ws_counter.reserve(64)) ||
            (rc = ctx->ws_seg.reserve((size_t)FUSED_MAX_SEGS * 2 * 4)) ||
            ((fuse_hash || cosine || pwfix) && (rc = ctx->ws_hfix.reserve((size_t)(N + FUSED_LIST_SLACK) * 8 * nfix_regions))) ||
            (((cosine && hi) || pwfix) && (rc = ctx->ws_seg3.reserve((size_t)FUSED_MAX_SEGS * 2 * 4))) ||
            (Kpad > 256 && (rc = ctx->ws_part.reserve((size_t)part_tiles * 64 * 16))) ||
            (hi && ((rc = ctx->ws_ambig2.reserve((size_t)list_cap * 4)) ||
                    (rc = ctx->ws_seg2.reserve((size_t)FUSED_MAX_SEGS * 2 * 4)))) ||
            (fuse_hash && !cosine && !tuples && (rc = ctx->ws_tuples.reserve((size_t)std::max<int64_t>(N, 1) * lsh->proj.LK * 4))))
            return rc;
        unsigned long long* cnt = (unsigned long long*)ctx->ws_counter.p;
        LSHKM_HIP(hipMemsetAsync(cnt, 0, 32, s));         // [0] ambiguous rows, [1] hash fix-up rows, [2] refined rows, [3] cosine declines / pow fix-ups
        _Float16* Ch = (_Float16*)ctx->ws_c32.p;
        _Float16* Cl = Ch + (size_t)Kpad * 128;
        float* cbound = (float*)ctx->ws_cconst.p;          // 4 floats, then cnh[Kpad]
        float* cnh = cbound + 8;
        double* nbv = (double*)(cnh + Kpad);               // cosine: [Kpad] sequential |c|^2 (Kpad % 64 == 0: aligned)
        float* C32 = nullptr;
        float* rn32 = nullptr;
        // the f32 image also serves the K <= 256 gather when every centroid value
        // is an f32 (dataset rows: the first Lloyd iteration), exact as doubles
        // (test switch LSHKM_GATHER32=0: the fp64 winner rows always)
        if (fast || (!cosine && rows_kind != 2 && Kpad <= 256 && !test_switch("LSHKM_GATHER32", "0"))) {
            if ((rc = ctx->ws_cf32.reserve((size_t)Kpad * 128 * 4 + (size_t)Kpad * 4))) return rc;
            C32 = (float*)ctx->ws_cf32.p;
            rn32 = C32 + (size_t)Kpad * 128;
        }
        double* C64p = nullptr;                            // d < 128: zero-padded fp64 centroids
        if (rows_kind != 0 && d != 128) {
            if ((rc = ctx->ws_c64p.reserve((size_t)Kpad * 128 * 8))) return rc;
            C64p = (double*)ctx->ws_c64p.p;
        }
        // the timed fused pass starts before the centroid prep
        if (ctx->timing) LSHKM_HIP(hipEventRecord(ctx->tev[0], s));
        if ((rc = launch_fused_prep(s, C, K, Kpad, Ch, Cl, cnh, cbound, cosine ? 1 : 0, nbv, C32, rn32, d, C64p))) { LSHKM_LAUNCH_CHECK(); return rc; }
        const bool xprep = exact_pruned(X, d, K, metric);
        if (xprep && (rc = exact_listed_prep(ctx, X, d, C, K, metric))) { LSHKM_LAUNCH_CHECK(); return rc; }
        FusedLaunch f;
        f.C32 = C32; f.rn32 = rn32; f.fast_dist = fast ? 1 : 0;
        f.rows = rows_kind; f.d = d; f.Cd = C;
        f.X = X.f64 ? nullptr : X.f(); f.X64 = X.f64 ? X.d() : nullptr;
        f.N = N; f.Ch = Ch; f.Cl = Cl; f.cnh = cnh; f.cbound = cbound; f.C64 = C64p ? C64p : C; f.Kpad = Kpad;
        f.assign = assign; f.dist = dist; f.ambig = (int32_t*)ctx->ws_ambig.p; f.ambig_count = cnt;
        f.stats = (unsigned long long*)ctx->stats.p;
        f.list_cap = N + FUSED_LIST_SLACK;
        f.seg_counts = (int32_t*)ctx->ws_seg.p;
        f.seg_cap = FUSED_MAX_SEGS;
        if (Kpad > 256) { f.part = ctx->ws_part.p; f.part_bytes = part_tiles * 64 * 16; }
        if (hi) {
            f.hi = true;
            f.list2 = (int32_t*)ctx->ws_ambig2.p;
            f.seg_counts2 = (int32_t*)ctx->ws_seg2.p;
            f.refined = cnt + 2;
        }
        if (pwfix) {
            f.cfix = (unsigned long long*)ctx->ws_hfix.p + (N + FUSED_LIST_SLACK);
            f.cfix_counts = (int32_t*)ctx->ws_seg3.p;
            f.cfix_count = cnt + 3;
        }
        if (cosine && rows_kind == 2) {
            if ((rc = ctx->ws_xn2.reserve((size_t)std::max<int64_t>(N, 1) * 8))) return rc;
            if ((rc = launch_row_sumsq(s, X.d(), N, d, (double*)ctx->ws_xn2.p))) { LSHKM_LAUNCH_CHECK(); return rc; }
            f.xn2 = (const double*)ctx->ws_xn2.p;
        }
        if (cosine) {
            f.metric = 1; f.nbv = nbv;
            f.hfix = (unsigned long long*)ctx->ws_hfix.p; f.hfix_count = hi ? cnt + 1 : cnt + 3;
            if (hi) {
                f.cfix = f.hfix + (N + FUSED_LIST_SLACK);
                f.cfix_counts = (int32_t*)ctx->ws_seg3.p;
                f.cfix_count = cnt + 3;
                f.hfix2 = f.cfix + (N + FUSED_LIST_SLACK);
            }
        }
        if (fuse_hash) {
            const ProjTable& pj = lsh->proj;
            f.Vh = pj.vh_d.as<_Float16>(); f.Vl = pj.vl_d.as<_Float16>(); f.PT = pj.PT_d.as<double>();
            f.tv = pj.t_d.as<float>(); f.pnorm = pj.pn_d.as<double>(); f.v1 = pj.v1_d.as<double>();
            f.rv = pj.r_d.as<int32_t>(); f.w = pj.w; f.L = pj.L; f.k = pj.k; f.LK = pj.LK; f.LKpad = pj.LKpad;
            f.nb = lsh->nb; f.phi = phi; f.bucket = bucket;
            f.tuples = cosine ? nullptr : tuples ? tuples : (int32_t*)ctx->ws_tuples.p;
            f.hfix = (unsigned long long*)ctx->ws_hfix.p; f.hfix_count = cnt + 1;
        }
        if (fuse_hash && ctx->side_init() == 0) {
            f.side = ctx->side_stream; f.fork = ctx->fork_ev; f.join = ctx->join_ev;
            f.defer_join = !cosine;        // euclidean: the exact pass also overlaps the fix-up
            if (ctx->timing) f.side_timing = ctx->tev[2];
        }
        ctx->tev_side = false;
        // the side stream's hash fix-up writes only tuples / phi / bucket: joined
        // before this call's last launch, and on every error path after the fork
        struct SideJoin {
            lshkm_ctx c;
            bool pending = false;
            ~SideJoin() { if (pending) (void)hipStreamSynchronize(c->side_stream); }
        } sj{ctx};
        rc = launch_fused(s, fuse_hash, f);
        sj.pending = f.join_pending;
        ctx->tev_side = f.side_timed;      // only a launch that recorded tev[2] extends the pass
        if (rc) { LSHKM_LAUNCH_CHECK(); return rc; }
        if (ctx->timing) LSHKM_HIP(hipEventRecord(ctx->tev[1], s));
        if ((rc = exact_listed(ctx, X, d, C, K, metric, cnt, N, assign, dist, f.nseg ? f.final_counts : nullptr,
                               f.seg_rows, f.nseg, f.nseg ? f.final_list : nullptr, !fast, xprep,
                               cosine ? f.xn2 : nullptr, cosine ? nbv : nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if (sj.pending) {
            LSHKM_HIP(hipStreamWaitEvent(s, f.join, 0));
            sj.pending = false;
        }
        {
            int di[3], n = 0;
            const unsigned long long* sp[3];
            if (hi) { di[n] = STAT_REFINED; sp[n++] = cnt + 2; }
            if (fuse_hash) { di[n] = STAT_HASH_FIX; sp[n++] = cnt + 1; }
            di[n] = STAT_ASSIGN_AMBIG; sp[n++] = cnt;
            if ((rc = launch_add_counters(s, (unsigned long long*)ctx->stats.p, n, di, sp))) { LSHKM_LAUNCH_CHECK(); return rc; }
        }
        if (cosine || pwfix) {
            if ((rc = launch_cos_fix_seg(s, X, d, C, f.ncos_lists, f.cos_list, f.cos_counts, f.seg_rows, f.nseg, assign,
                                         dist, cosine ? 1 : 0, cosine ? f.xn2 : nullptr, cosine ? nbv : nullptr))) { LSHKM_LAUNCH_CHECK(); return rc; }
            if ((rc = launch_add_counter(s, (unsigned long long*)ctx->stats.p + (cosine ? STAT_COS_FIX : STAT_POW_FIX), cnt + 3))) { LSHKM_LAUNCH_CHECK(); return rc; }
        }
    } else if (path == 1) {
        const int Kpad = (K + 63) / 64 * 64;
        if ((rc = ctx->ws_c32.reserve((size_t)Kpad * DP * 4)) || (rc = ctx->ws_cconst.reserve((size_t)3 * Kpad * 4)) ||
            (rc = ctx->ws_ambig.reserve((size_t)std::max<int64_t>(N, 1) * 2 * 4)) ||   // ambiguous rows | cosine fix-ups
            (rc = ctx->ws_counter.reserve(64)))
            return rc;
        unsigned long long* cnt = (unsigned long long*)ctx->ws_counter.p;
        LSHKM_HIP(hipMemsetAsync(cnt, 0, 16, s));
        if ((rc = launch_centroid_prep(s, C, K, Kpad, d, DP, metric, X.f64, (float*)ctx->ws_c32.p, (float*)ctx->ws_cconst.p))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if ((rc = launch_assign_mfma(s, X, N, d, DP, C, K, Kpad, metric, (const float*)ctx->ws_c32.p, (const float*)ctx->ws_cconst.p,
                                     assign, dist, (int32_t*)ctx->ws_ambig.p, cnt))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if ((rc = exact_listed(ctx, X, d, C, K, metric, cnt, N, assign, dist))) { LSHKM_LAUNCH_CHECK(); return rc; }
        if (metric != LSHKM_METRIC_EUCLIDEAN &&
            ((rc = launch_cos_fix(s, X, N, d, C, (const int32_t*)ctx->ws_ambig.p + N, cnt + 1, assign, dist)) ||
             (rc = launch_add_counter(s, (unsigned long long*)ctx->stats.p + STAT_COS_FIX, cnt + 1)))) { LSHKM_LAUNCH_CHECK(); return rc; }
        // ambiguous-count statistic
        if ((rc = launch_add_counter(s, (unsigned long long*)ctx->stats.p + STAT_ASSIGN_AMBIG, cnt))) { LSHKM_LAUNCH_CHECK(); return rc; }
    } else {
        // Exact reference-order pass over every centroid (cosine metric, or d > 256).
        if ((rc = launch_assign_exact(s, X, N, d, C, K, metric, nullptr, nullptr, N, assign, dist))) { LSHKM_LAUNCH_CHECK(); return rc; }
    }
    if (src_rows_host) {
        if ((rc = ctx->ws_src.reserve((size_t)K * 4))) return rc;
        // The same rows as the previous override already sit in ws_src (Lloyd
        // iterations and the bench pass one array repeatedly): no copy. A small
        // host->device copy blocked the host until the stream drained, so every
        // call waited for the previous one's tail: 2.05 ms of host enqueue per call vs 0.05).
        const bool same = ctx->src_cache_dev == ctx->ws_src.p && ctx->src_cache_cap == ctx->ws_src.cap &&
                          ctx->src_cache.size() == (size_t)K &&
                          std::memcmp(ctx->src_cache.data(), src_rows_host, (size_t)K * 4) == 0;
        if (!same) {
            // Stage through a pinned buffer so the caller's array may be freed at
            // once and no stream sync is needed (a ring of buffers, index.h).
            if ((rc = ctx->pin_stage((size_t)K * 4))) return rc;
            std::memcpy(ctx->pinned, src_rows_host, (size_t)K * 4);
            LSHKM_HIP(hipMemcpyAsync(ctx->ws_src.p, ctx->pinned, (size_t)K * 4, hipMemcpyHostToDevice, s));
            LSHKM_HIP(hipEventRecord(ctx->pinned_ev, s));
            ctx->src_cache.assign(src_rows_host, src_rows_host + K);
            ctx->src_cache_dev = ctx->ws_src.p;
            ctx->src_cache_cap = ctx->ws_src.cap;
        }
        if ((rc = launch_assign_override(s, (const int32_t*)ctx->ws_src.p, K, N, assign, dist))) { LSHKM_LAUNCH_CHECK(); return rc; }
    }
    return 0;
}

static int lloyd_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const double* C, int K, int metric,
                      const int32_t* src_rows_host, int32_t* assign, double* dist) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && C && (assign || N == 0) && (dist || N == 0) && N >= 0 && d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN || metric == LSHKM_METRIC_COSINE, LSHKM_ERR_ARG, "unknown metric");
    LSHKM_HIP(hipSetDevice(ctx->device));
    return assign_impl(ctx, X, N, d, C, K, metric, src_rows_host, assign, dist, nullptr, nullptr, nullptr, nullptr);
}

static int hash_assign_impl(lshkm_lsh lsh, Pts X, int64_t N, const double* C, int K, const int32_t* src_rows_host,
                            int32_t* tuples, int32_t* phi, int32_t* bucket, int32_t* assign, double* dist,
                            int metric = LSHKM_METRIC_EUCLIDEAN) {
    LSHKM_CHECK(lsh && (X.p || N == 0) && C && (assign || N == 0) && (dist || N == 0) && N >= 0 && K > 0, LSHKM_ERR_ARG,
                "bad arguments");
    lshkm_ctx ctx = lsh->ctx;
    LSHKM_HIP(hipSetDevice(ctx->device));
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN || metric == LSHKM_METRIC_COSINE, LSHKM_ERR_ARG, "unknown metric");
    return assign_impl(ctx, X, N, lsh->proj.d, C, K, metric, src_rows_host, assign, dist, lsh, tuples, phi, bucket);
}

static int range_impl(lshkm_ctx ctx, Pts X, int64_t N, int d, const double* C, int K, int metric,
                      const int64_t* comb_ptr, const int32_t* comb_idx, const int32_t* key_host,
                      const int32_t* src_rows_host, int32_t* assign, double* dist, int* passes_host) {
    LSHKM_CHECK(ctx && (X.p || N == 0) && C && comb_ptr && (assign || N == 0) && (dist || N == 0) && N >= 0 &&
                    N < (1ll << 31) && d > 0 && K > 0,
                LSHKM_ERR_ARG, "bad arguments");
    LSHKM_CHECK(metric == LSHKM_METRIC_EUCLIDEAN || metric == LSHKM_METRIC_COSINE, LSHKM_ERR_ARG, "unknown metric");
    LSHKM_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    lshkm::Buf* w = ctx->ws_range;
    int rc;
    int64_t M = 0;
    LSHKM_HIP(hipMemcpyAsync(&M, comb_ptr + K, 8, hipMemcpyDeviceToHost, s));
    LSHKM_HIP(hipStreamSynchronize(s));
    LSHKM_CHECK(M >= 0 && (M == 0 || comb_idx), LSHKM_ERR_ARG, "bad combined-bucket CSR");
    const size_t scratch = sort_scratch_bytes(std::max<int64_t>(M, 1), std::max<int64_t>(N, 1));
    if ((rc = w[0].reserve(64)) || (rc = w[1].reserve((size_t)std::max<int64_t>(M, 1) * 4 * 4)) ||
        (rc = w[2].reserve(scratch)) || (rc = w[3].reserve((size_t)(N + 1) * 8)) ||
        (rc = w[4].reserve((size_t)std::max<int64_t>(M, 1) * 9)) || (rc = w[5].reserve((size_t)K * 4)))
        return rc;
    double* r0 = (double*)w[0].p;                          // [0] r0, [1] pass count, [2] unassigned count
    unsigned long long* cnt = (unsigned long long*)w[0].p + 1;
    int32_t* rows = (int32_t*)w[1].p;
    int32_t* cents = rows + std::max<int64_t>(M, 1);
    int32_t* rows_s = cents + std::max<int64_t>(M, 1);
    int32_t* cents_s = rows_s + std::max<int64_t>(M, 1);
    int64_t* vptr = (int64_t*)w[3].p;
    double* cache = (double*)w[4].p;
    int8_t* cached = (int8_t*)(cache + std::max<int64_t>(M, 1));
    const int32_t* key = nullptr;
    if (key_host) {
        LSHKM_HIP(hipMemcpyAsync(w[5].p, key_host, (size_t)K * 4, hipMemcpyHostToDevice, s));
        key = (const int32_t*)w[5].p;
    }
    if ((rc = launch_range_radius(s, C, K, d, metric, r0, (unsigned long long*)w[0].p + 4))) return rc;
    if ((rc = launch_range_init(s, N, assign, dist))) return rc;
    int passes = 0;
    if (M > 0 && N > 0) {
        if ((rc = launch_range_pairs(s, comb_ptr, comb_idx, K, rows, cents))) return rc;
        if ((rc = stable_sort_by_key(s, rows, 1, cents, M, N, rows_s, cents_s, w[2].p))) return rc;
        if ((rc = launch_csr_bounds(s, rows_s, M, N, vptr))) return rc;
        LSHKM_HIP(hipMemsetAsync(cached, 0, (size_t)M, s));
        // the do-while of assignment.hpp:160-216, one launch per pass
        for (;;) {
            unsigned long long assigned = 0;
            LSHKM_HIP(hipMemsetAsync(cnt, 0, 8, s));
            if ((rc = launch_range_pass(s, X, d, C, K, metric, key, vptr, cents_s, cache, cached, N, r0, passes,
                                        assign, dist, cnt)))
                return rc;
            passes++;
            LSHKM_HIP(hipMemcpyAsync(&assigned, cnt, 8, hipMemcpyDeviceToHost, s));
            LSHKM_HIP(hipStreamSynchronize(s));
            if (!assigned) break;
        }
    } else {
        passes = 1;     // one pass over empty buckets assigns nothing
    }
    // lloyds_for_remaining (assignment.hpp:83-104): the Lloyd path on the rows left unassigned
    if (N > 0) {
        if ((rc = w[6].reserve((size_t)N * 4))) return rc;
        int32_t* list = (int32_t*)w[6].p;
        unsigned long long* ucnt = cnt + 1;
        unsigned long long U = 0;
        LSHKM_HIP(hipMemsetAsync(ucnt, 0, 8, s));
        if ((rc = launch_range_unassigned(s, assign, N, list, ucnt))) return rc;
        LSHKM_HIP(hipMemcpyAsync(&U, ucnt, 8, hipMemcpyDeviceToHost, s));
        LSHKM_HIP(hipStreamSynchronize(s));
        if (U > 0) {
            if ((rc = w[7].reserve((size_t)U * d * X.esize())) || (rc = w[8].reserve((size_t)U * 12))) return rc;
            double* dr = (double*)w[8].p;
            int32_t* ar = (int32_t*)(dr + U);
            if ((rc = launch_range_gather(s, X, d, list, (int64_t)U, w[7].p))) return rc;
            const Pts Xr = X.f64 ? Pts(w[7].as<double>()) : Pts(w[7].as<float>());
            // the range pass's distances are the exact chain; the leftover rows
            // get the same (a range assignment is exact-order in either mode)
            rc = assign_impl(ctx, Xr, (int64_t)U, d, C, K, metric, nullptr, ar, dr, nullptr, nullptr, nullptr, nullptr,
                             true);
            if (rc) return rc;
            if ((rc = launch_range_scatter(s, list, (int64_t)U, ar, dr, assign, dist))) return rc;
        }
    }
    // the centroid override (assignment.hpp:125-127, :143-145)
    if (src_rows_host) {
        if ((rc = ctx->ws_src.reserve((size_t)K * 4))) return rc;
        ctx->src_cache_dev = nullptr;            // ws_src overwritten outside the cache
        LSHKM_HIP(hipMemcpyAsync(ctx->ws_src.p, src_rows_host, (size_t)K * 4, hipMemcpyHostToDevice, s));
        if ((rc = launch_assign_override(s, (const int32_t*)ctx->ws_src.p, K, N, assign, dist))) return rc;
        LSHKM_HIP(hipStreamSynchronize(s));     // the host arrays may be freed on return
    }
    if (key_host) LSHKM_HIP(hipStreamSynchronize(s));
    if (passes_host) *passes_host = passes;
    return 0;
}

extern "C" {

int lshkm_lloyd_assign(lshkm_ctx ctx, const float* X, int64_t N, int d, const double* C, int K, int metric,
                       const int32_t* src_rows_host, int32_t* assign, double* dist) {
    return lloyd_impl(ctx, X, N, d, C, K, metric, src_rows_host, assign, dist);
}

int lshkm_lloyd_assign_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const double* C, int K, int metric,
                           const int32_t* src_rows_host, int32_t* assign, double* dist) {
    return lloyd_impl(ctx, X, N, d, C, K, metric, src_rows_host, assign, dist);
}

int lshkm_hash_assign(lshkm_lsh lsh, const float* X, int64_t N, const double* C, int K, const int32_t* src_rows_host,
                      int32_t* tuples, int32_t* phi, int32_t* bucket, int32_t* assign, double* dist) {
    return hash_assign_impl(lsh, X, N, C, K, src_rows_host, tuples, phi, bucket, assign, dist);
}

int lshkm_hash_assign_f64(lshkm_lsh lsh, const double* X, int64_t N, const double* C, int K,
                          const int32_t* src_rows_host, int32_t* tuples, int32_t* phi, int32_t* bucket,
                          int32_t* assign, double* dist) {
    return hash_assign_impl(lsh, X, N, C, K, src_rows_host, tuples, phi, bucket, assign, dist);
}

int lshkm_hash_assign_metric(lshkm_lsh lsh, const float* X, int64_t N, const double* C, int K, int metric,
                             const int32_t* src_rows_host, int32_t* tuples, int32_t* phi, int32_t* bucket,
                             int32_t* assign, double* dist) {
    return hash_assign_impl(lsh, X, N, C, K, src_rows_host, tuples, phi, bucket, assign, dist, metric);
}

int lshkm_hash_assign_metric_f64(lshkm_lsh lsh, const double* X, int64_t N, const double* C, int K, int metric,
                                 const int32_t* src_rows_host, int32_t* tuples, int32_t* phi, int32_t* bucket,
                                 int32_t* assign, double* dist) {
    return hash_assign_impl(lsh, X, N, C, K, src_rows_host, tuples, phi, bucket, assign, dist, metric);
}

int lshkm_range_assign(lshkm_ctx ctx, const float* X, int64_t N, int d, const double* C, int K, int metric,
                       const int64_t* comb_ptr, const int32_t* comb_idx, const int32_t* key_host,
                       const int32_t* src_rows_host, int32_t* assign, double* dist, int* passes_host) {
    return range_impl(ctx, X, N, d, C, K, metric, comb_ptr, comb_idx, key_host, src_rows_host, assign, dist,
                      passes_host);
}

int lshkm_range_assign_f64(lshkm_ctx ctx, const double* X, int64_t N, int d, const double* C, int K, int metric,
                           const int64_t* comb_ptr, const int32_t* comb_idx, const int32_t* key_host,
                           const int32_t* src_rows_host, int32_t* assign, double* dist, int* passes_host) {
    return range_impl(ctx, X, N, d, C, K, metric, comb_ptr, comb_idx, key_host, src_rows_host, assign, dist,
                      passes_host);
}

int lshkm_synth(lshkm_ctx ctx, uint64_t seed, int64_t row0, int64_t rows, int d, float* X) {
    LSHKM_CHECK(ctx && (X || rows == 0) && rows >= 0 && d > 0, LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc = launch_synth(ctx->stream, seed, row0, rows, d, X);
    if (rc) { LSHKM_LAUNCH_CHECK(); }
    return rc;
}

int lshkm_synth_normal(lshkm_ctx ctx, uint64_t seed, int64_t row0, int64_t rows, int d, float* X) {
    LSHKM_CHECK(ctx && (X || rows == 0) && rows >= 0 && d > 0, LSHKM_ERR_ARG, "bad arguments");
    LSHKM_HIP(hipSetDevice(ctx->device));
    int rc = launch_synth(ctx->stream, seed, row0, rows, d, X, 1);
    if (rc) { LSHKM_LAUNCH_CHECK(); }
    return rc;
}

}  // extern "C"
