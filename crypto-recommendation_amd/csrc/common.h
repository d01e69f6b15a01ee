// common.h — shared internals of liblshkm (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

namespace lshkm {

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

// Device counters kept per context (see lshkm_get_stat).
enum Stat {
    STAT_HASH_EXACT = 0,     // hash values resolved by the soft-x87 exact path
    STAT_ASSIGN_AMBIG = 1,   // points whose argmin the MFMA bound could not certify
    STAT_COUNT = 8
};

constexpr int WAVE = 64;

}  // namespace lshkm
