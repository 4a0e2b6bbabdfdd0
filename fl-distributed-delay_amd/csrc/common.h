// Shared helpers for the flsim HIP kernels (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#define FLSIM_WAVE 64

// ---- measurement switches ------------------------------------------------------------------
// The A/B switches behind the measurements DESIGN.md cites -- compile-time -DFLSIM_<X> overrides
// and the FLSIM_<X> environment overrides read through lab_env() -- act only in a lab build
// (make LAB=1 -> -DFLSIM_LAB).  The product build compiles their measured defaults, so its
// behaviour depends on no environment variable (FLSIM_DEBUG_BWD_STOP, the tests' stop of the
// backward pass after a given layer, excepted).
#if !defined(FLSIM_LAB) &&                                                                  \
    (defined(FLSIM_X6_FRESH) || defined(FLSIM_X6_PP_V) || defined(FLSIM_DG_FMS) ||          \
     defined(FLSIM_DIRECT_FENCES) || defined(FLSIM_DX6_FENCES) || defined(FLSIM_BUFLOAD) ||  \
     defined(FLSIM_SEQ_EARLY_EXIT) || defined(FLSIM_X6_FLUSH) || defined(FLSIM_WGRAD_X6) ||     \
     defined(FLSIM_ZL1F) || defined(FLSIM_SINGLE_BUF) || defined(FLSIM_DG3_FM) || defined(FLSIM_DX_FM))
#error "FLSIM_* measurement overrides need a lab build (make LAB=1)"
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace flsim {

// ---- error plumbing (thread-local last error, C-ABI returns int status) -------------------
void set_error(const char* fmt, ...);
const char* last_error();

#define FLSIM_CHECK_HIP(expr)                                                           \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            ::flsim::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                               __FILE__, __LINE__);                                     \
            return 2;                                                                   \
        }                                                                               \
    } while (0)

#define FLSIM_REQUIRE(cond, ...)                                                        \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            ::flsim::set_error(__VA_ARGS__);                                            \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

#define RC(x) do { int _r = (x); if (_r) return _r; } while (0)

// a measurement override from the environment (lab builds only; see the top of this file)
inline const char* lab_env(const char* name) {
#ifdef FLSIM_LAB
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

#define FLSIM_LAUNCH_CHECK()                                                            \
    do {                                                                                \
        hipError_t _e = hipGetLastError();                                              \
        if (_e != hipSuccess) {                                                         \
            ::flsim::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), \
                               __FILE__, __LINE__);                                     \
            return 2;                                                                   \
        }                                                                               \
    } while (0)

// ---- Philox4x32-10: the build's counter-based RNG spec (DESIGN.md "RNG spec") -------------
// word (e & 3) of philox(ctr = (e >> 2, t, worker, site), key = (seed_lo, seed_hi))
__host__ __device__ inline void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                              uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

__host__ __device__ inline uint32_t philox_word(uint64_t seed, uint32_t t, uint32_t worker,
                                                uint32_t site, uint32_t e) {
    uint32_t c0 = e >> 2, c1 = t, c2 = worker, c3 = site;
    philox4x32_10(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t w = e & 3;
    return w == 0 ? c0 : (w == 1 ? c1 : (w == 2 ? c2 : c3));
}

// RNG sites (must match oracle/oracle.py)
enum : uint32_t { SITE_DROP1 = 1, SITE_DROP2 = 2, SITE_DROP3 = 3, SITE_DROP4 = 4,
                  SITE_DROP5 = 5, SITE_DATA = 0x10 };

// keep iff u32 >= threshold; thresholds for p = 0.25 and p = 0.5
constexpr uint32_t THR_P25 = 0x40000000u;
constexpr uint32_t THR_P50 = 0x80000000u;

// torch: noise = bernoulli(1-p).div_(1-p) -> fp32(1/(1-p))
constexpr float SCALE_P25 = 1.33333337306976318359375f;  // fp32(1/0.75)
constexpr float SCALE_P50 = 2.0f;

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace flsim
