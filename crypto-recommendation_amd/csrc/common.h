// common.h — shared internals of liblshkm (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#ifdef LSHKM_TEST_SWITCHES
#include <cstdlib>
#include <cstring>
#endif

namespace lshkm {

// Path switches for the tests' A/B comparisons (one kernel path forced against
// another, bit for bit). Compiled only into the test build liblshkm_test.so
// (-DLSHKM_TEST_SWITCHES, `make test`); the product library liblshkm.so reads
// no environment and always takes the default paths.
inline bool test_switch(const char* name, const char* value) {
#ifdef LSHKM_TEST_SWITCHES
    const char* e = std::getenv(name);
    return e && !std::strcmp(e, value);
#else
    (void)name;
    (void)value;
    return false;
#endif
}

// Thread-local last error, surfaced through lshkm_last_error().
void set_error(const std::string& msg);

#define LSHKM_HIP(expr)                                                              \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess) {                                                      \
            ::lshkm::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));   \
            return LSHKM_ERR_HIP;                                                    \
        }                                                                            \
    } while (0)

#define LSHKM_CHECK(cond, code, msg)                                                 \
    do {                                                                             \
        if (!(cond)) { ::lshkm::set_error(msg); return code; }                       \
    } while (0)

#define LSHKM_LAUNCH_CHECK() LSHKM_HIP(hipGetLastError())

// Status of the launches just issued by a launcher: 0, or -2 with the HIP
// error recorded for lshkm_last_error().
inline int kstatus(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return -2;
}

// Wave-scope LDS handoff: makes one lane's LDS writes visible to the other
// lanes of its wave (a fence the compiler cannot move loads across).
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Grid size for a grid-stride kernel: at least one block, at most cap.
inline unsigned gsz(int64_t work, int64_t per_block, int64_t cap) {
    int64_t b = (work + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (unsigned)b;
}

// Device counters kept per context (see lshkm_get_stat).
enum Stat {
    STAT_HASH_EXACT = 0,     // hash values resolved by the soft-x87 exact path
    STAT_ASSIGN_AMBIG = 1,   // points whose argmin the MFMA bound could not certify
    STAT_KPP_CHUNKS = 2,     // k-means++ prefix-walk chunks (KPP_CHUNK rows each) ...
    STAT_KPP_SEQ = 3,        // ... of which summed element by element (binade crossings, ties)
    STAT_COS_FIX = 4,        // cosine Lloyd winners whose distance took the soft-x87 chain
    STAT_REFINED = 5,        // rows the hi-only fused pass left to the 3-product refinement
    STAT_HASH_FIX = 6,       // rows the fused pass listed for the hash fix-up (an uncertified floor / sign)
    STAT_REC_SOFT = 7,       // clustering-recommender similarities decided by the x87 chain (IpAcc declined)
    STAT_POW_FIX = 8,        // euclidean winner distances redone with glibc's pow(x, 2) (an inexact square)
    STAT_KM_SEQ = 9,         // k-means (cluster, dim) sums whose never-rounds test failed (sequential / segment chain)
    STAT_COUNT = 10
};

constexpr int WAVE = 64;

}  // namespace lshkm
