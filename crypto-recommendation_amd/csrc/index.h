// index.h — handle types behind the opaque C ABI pointers.
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "kernels.h"

namespace lshkm {

// Growable device buffer (never shrinks; freed with its owner).
struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    ~Buf();
    int reserve(size_t bytes);
    template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};

// Device copy of a projection family: transposed fp64 projections + per-row
// constants, as the hash kernel reads them.
struct ProjTable {
    int metric = 0, d = 0, L = 0, k = 0, LK = 0, LKpad = 0;
    float w = 0.f;
    Buf PT_d, t_d, pn_d, r_d;
    // split-f16 image for the fused kernel (euclidean, d == 128, L*k <= 32):
    // Vh/Vl [64][128] f16 (rows >= LK zero), v1 = ||v||_1 rounded up
    bool fused_ok = false;
    bool mfma_ok = false;        // split image present (either metric): hash_mfma.hip
    Buf vh_d, vl_d, v1_d;
    std::vector<float> hV;
    int upload(hipStream_t s, int metric, int d, int L, int k, float w, const float* V, const float* t,
               const int32_t* r, const double* R);
    HashParams params(int64_t nb) const;
    HashMfmaParams mfma_params(int64_t nb) const;
};

}  // namespace lshkm

struct lshkm_ctx_s;
namespace lshkm {
// Hashing of a batch on the split-f16 MFMA kernel where it applies, else the
// fp64 kernel (api_index.cpp).
// h16 (cube euclidean): in, int16 h wanted; out, whether int16 was written
// (only the MFMA kernel writes it).
int hash_rows(lshkm_ctx_s* ctx, int mode, Pts X, int64_t N, const ProjTable& pj, int64_t nb, int32_t* out_h,
              int32_t* out_phi, int32_t* out_bucket, int32_t* mm, bool* h16 = nullptr);

}  // namespace lshkm

struct lshkm_ctx_s {
    int device = 0;
    // LSHKM_DIST_CERTIFIED (default) / LSHKM_DIST_EXACT: lshkm_ctx_set_dist_mode
    int dist_mode = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    lshkm::Buf stats;            // STAT_COUNT x u64
    // assignment workspace
    lshkm::Buf ws_c32, ws_cconst, ws_ambig, ws_counter, ws_src, ws_hfix, ws_ct, ws_seg, ws_tuples, ws_part;
    lshkm::Buf ws_cf32;     // fast distances: f32(c) [Kpad][128] + |c - f32(c)| [Kpad]
    lshkm::Buf ws_c64p;     // general rows (d < 128): the zero-padded fp64 centroids [Kpad][128]
    lshkm::Buf ws_ambig2, ws_seg2;   // the hi-only form's refinement output list
    lshkm::Buf ws_seg3;              // hi-only cosine: segment counts of the declined winner distances (euclidean exact: of the pow fix-ups)
    lshkm::Buf ws_xn2;               // cosine on fp64 rows: [N] sum_j pow(x_j, 2)
    // scatter / query / update workspace (see api_index.cpp for the slot map)
    lshkm::Buf ws[16];
    // range assignment workspace (lshkm_range_assign)
    lshkm::Buf ws_range[12];
    lshkm::Buf ws_long;          // the recommender's chains of huge clusters (RcLong)
    lshkm::Buf ws_km_seg;        // k-means: the segment records of the chains the never-rounds test flags (fp32 rows)
    lshkm::Buf ws_scan;          // multi-block scans of large query size arrays
    // workspaces of the entry points that synchronise their stream before
    // returning (kmeans_pp, p_closest, top_n_recom): reused across calls
    lshkm::Buf ws_call[10];
    uint64_t ws_epoch = 0;       // bumped by every user of the ws[] slots (api_index.cpp reserve)
    // optional HIP-event timing of the dominant kernel launch (lshkm_last_kernel_ms)
    bool timing = false;
    hipEvent_t tev[3] = {nullptr, nullptr, nullptr};   // [2]: the side stream's end (hash fix-up)
    bool tev_side = false;       // the last timed call recorded tev[2]
    // a side stream for work independent of the main stream's next kernels
    // (the hash fix-up beside the LIST refinement), forked / joined by events
    hipStream_t side_stream = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    int side_init() {
        if (side_stream) return 0;
        if (hipStreamCreateWithFlags(&side_stream, hipStreamNonBlocking) != hipSuccess) return -2;
        if (hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&join_ev, hipEventDisableTiming) != hipSuccess)
            return -2;
        return 0;
    }
    // pinned host staging for small host->device inputs: a ring of PIN_SLOTS
    // buffers, each reused only after the copy from it PIN_SLOTS stagings ago
    // has landed (one slot made every call wait for the previous call's tail:
    // the host then re-fed an idle GPU). Callers fill `pinned`, copy from it and
    // record `pinned_ev` on their stream.
    static constexpr int PIN_SLOTS = 4;
    void* pin_buf[PIN_SLOTS] = {};
    size_t pin_cap[PIN_SLOTS] = {};
    hipEvent_t pin_ev[PIN_SLOTS] = {};
    bool pin_used[PIN_SLOTS] = {};
    int pin_cur = -1;
    void* pinned = nullptr;
    hipEvent_t pinned_ev = nullptr;
    // the centroid-override rows last copied into ws_src (valid while ws_src
    // keeps that allocation): a repeated override needs no copy
    std::vector<int32_t> src_cache;
    void* src_cache_dev = nullptr;
    size_t src_cache_cap = 0;
    int pin_stage(size_t bytes) {
        const int i = (pin_cur + 1) % PIN_SLOTS;
        if (!pin_ev[i] && hipEventCreateWithFlags(&pin_ev[i], hipEventDisableTiming) != hipSuccess) return -2;
        if (pin_used[i]) (void)hipEventSynchronize(pin_ev[i]);
        if (bytes > pin_cap[i]) {
            if (pin_buf[i]) (void)hipHostFree(pin_buf[i]);
            pin_buf[i] = nullptr; pin_cap[i] = 0;
            if (hipHostMalloc(&pin_buf[i], bytes, hipHostMallocDefault) != hipSuccess) return -3;
            pin_cap[i] = bytes;
        }
        pin_cur = i;
        pin_used[i] = true;              // the caller records pin_ev[i] after its copy
        pinned = pin_buf[i];
        pinned_ev = pin_ev[i];
        return 0;
    }
    // pinned host buffers of the entry points that synchronise their stream
    // before returning: rb_buf receives device->host reads (d2h_batch: async
    // copies, one synchronisation per batch -- into pageable memory every copy
    // was its own blocking round trip, ~20 us each), ub_buf stages host->device
    // uploads (h2d_batch; reused only after the calling entry point's sync)
    void* rb_buf = nullptr;
    size_t rb_cap = 0;
    void* ub_buf = nullptr;
    size_t ub_cap = 0;
    hipEvent_t ub_ev = nullptr;      // recorded after each upload batch: ub_buf is rewritten only after it
    bool ub_pending = false;
    static int pin_grow(void*& b, size_t& cap, size_t bytes) {
        if (bytes <= cap) return 0;
        if (b) (void)hipHostFree(b);
        b = nullptr;
        cap = 0;
        const size_t nb = std::max<size_t>(bytes, 64 << 10);
        if (hipHostMalloc(&b, nb, hipHostMallocDefault) != hipSuccess) return -3;
        cap = nb;
        return 0;
    }
    ~lshkm_ctx_s() {
        if (rb_buf) (void)hipHostFree(rb_buf);
        if (ub_ev) {
            if (ub_pending) (void)hipEventSynchronize(ub_ev);
            (void)hipEventDestroy(ub_ev);
        }
        if (ub_buf) (void)hipHostFree(ub_buf);
        for (hipEvent_t& e : tev)
            if (e) (void)hipEventDestroy(e);
        if (side_stream) (void)hipStreamSynchronize(side_stream), (void)hipStreamDestroy(side_stream);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        if (join_ev) (void)hipEventDestroy(join_ev);
        for (int i = 0; i < PIN_SLOTS; i++) {
            if (pin_ev[i]) (void)hipEventSynchronize(pin_ev[i]), (void)hipEventDestroy(pin_ev[i]);
            if (pin_buf[i]) (void)hipHostFree(pin_buf[i]);
        }
    }
};

namespace lshkm {
// Device->host reads / host->device uploads in one batch (api_index.cpp):
// d2h_batch returns after every read landed in its destination; h2d_batch
// stages the sources in ctx->ub_buf and only issues the copies (the host
// buffers may go at once; the next batch waits for this one's copies before it
// rewrites ub_buf).
struct D2H { void* dst; const void* src; size_t bytes; };
struct H2D { void* dst; const void* src; size_t bytes; };
int d2h_batch(lshkm_ctx_s* ctx, const D2H* r, int n);
int h2d_batch(lshkm_ctx_s* ctx, const H2D* r, int n);
}  // namespace lshkm

struct lshkm_lsh_s {
    lshkm_ctx_s* ctx = nullptr;
    int metric = 0;
    int64_t nb = 0;
    lshkm::ProjTable proj;
    // built index (lshkm_lsh_build)
    int built = 0;
    int64_t N = 0;
    lshkm::Buf tuples, bucket, row_ptr, idx;
    // filtered queries: each table's members' first tuple value in CSR order
    // (mt0[l * N + pos]), gathered once after a build by the first filtered
    // query, so the marking pass reads it coalesced instead of one random
    // tuple line per member
    lshkm::Buf mt0;
    bool mt0_valid = false;
    // two-phase query: the sizing call's device state, reused by the filling
    // call when nothing else touched the context's slots in between
    bool q_valid = false;
    uint64_t q_epoch = 0;
    const void* q_Q = nullptr;
    bool q_f64 = false;
    const void* q_alias = nullptr;
    const int64_t* q_out_ptr = nullptr;
    int64_t q_nq = 0, q_total = 0;
    int q_filtered = 0;
};

struct lshkm_cube_s {
    lshkm_ctx_s* ctx = nullptr;
    int metric = 0;
    int k = 0;
    lshkm::ProjTable proj;
    // lazy EuclideanF coin memo: memo[f][h - hmin] in {-1 (unseen), 0, 1}
    int32_t hmin = 0, hspan = 0;
    lshkm::Buf memo, memo2, first_row;
    lshkm::Buf rng_d;             // device copy of the engine state (uint32)
    lshkm::Buf mm, cnt;           // h min/max, collected-entry count
    int built = 0;
    int64_t N = 0;
    lshkm::Buf vertex, row_ptr, idx;
};
