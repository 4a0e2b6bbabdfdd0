// Server step on the device: rule() (main.py:23-25) + Central.update_model (agents.py:9-21).
//
//   rule(weight_ups) = torch.stack(entries).mean(0) per parameter tensor, entries = the aliased
//   S_t of every fast worker (main.py:172) and the popped stale FIFO entries (main.py:161-165) in
//   append order; update_model = torch.optim.Adam (main.py:106).
//
// Arithmetic is bit-exact with torch 2.10 CPU: the sum over the stacked dim follows ATen's cascade
// (cascade.h: a host-built program per step, interpreted per element; multi_row_sum on whole
// 32-element column blocks of each tensor, row_sum on its last numel % 32 elements); mean =
// sum / (float)k; Adam m = fma(1-b1, g-m, m), v = fma((1-b2)*g, g, v*b2),
// den = sqrt(v)/sqrt(bc2) + eps, p += (-lr/bc1 * m) / den (correctly rounded sqrt; torch CPU's
// sqrt is not).  Compiled with -ffp-contract=off: the only fmas are explicit.
//
// Two kernels:
//   k_agg_stream  S_t already in a buffer (after the all-reduce at world > 1, or the facade):
//                 one float4 group per thread, 7 + distinct-array streams, HBM-bound;
//   k_slab_step   world = 1: the epoch's weight-gradient slabs are reduced to S_t in the same
//                 launch (slabstep.h), S_t never round-trips through HBM.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "flsim.h"
#include "probe.h"
#include "slabstep.h"

#ifndef FLSIM_SEQ_EARLY_EXIT
#define FLSIM_SEQ_EARLY_EXIT 1
#endif

namespace flsim {

constexpr int NYR = 8;          // entry arrays staged per thread (LDS); the rest load on demand
constexpr int MAX_TAILS = 8;    // tensor tails per streaming launch (host splits longer lists)
constexpr int AGG_GMAX = 2;     // float4 groups per thread of the register-array stream
constexpr int MAX_EDGE = 4 * AGG_GMAX * (2 * MAX_TAILS + 2);   // 256-element edge pieces per launch

// ---- element arithmetic -----------------------------------------------------------------------
// Correctly rounded fp32 sqrt.  v_sqrt_f32 is within 1 ulp; the exact residuals x - s'*s of the
// two neighbours s' = s -/+ 1 ulp (single-rounding fma: its sign is exact) pick the correctly
// rounded root.  Tiny inputs are scaled by 2^32 (root by 2^-16) so the residuals stay normal.
__device__ __forceinline__ float sqrt_rn(float x) {
    const bool tiny = x < 0x1p-96f;
    const float xs = tiny ? x * 0x1p+32f : x;
    float s = __builtin_amdgcn_sqrtf(xs);
    const int si = __float_as_int(s);
    const float s_dn = __int_as_float(si - 1);
    const float s_up = __int_as_float(si + 1);
    const float r_dn = __fmaf_rn(-s_dn, s, xs);
    const float r_up = __fmaf_rn(-s_up, s, xs);
    s = (r_dn <= 0.f) ? s_dn : s;
    s = (r_up > 0.f) ? s_up : s;
    s = tiny ? s * 0x1p-16f : s;
    // 0, +inf and NaN pass through unchanged (the correction above is only for finite x > 0)
    return (xs == 0.f || xs == __builtin_inff() || xs != xs) ? x : s;
}

// Correctly rounded a / b for a launch-constant divisor b with rb = RN(1/b) (Markstein: q0
// within 1 ulp, exact residual by fma, one correction).  Zero, tiny (near-subnormal) and
// non-finite quotients take the IEEE division so signs and subnormals stay exact.
__device__ __forceinline__ float div_const(float a, float b, float rb) {
    const float q0 = a * rb;
    const float r = __fmaf_rn(-q0, b, a);
    const float q = __fmaf_rn(r, rb, q0);
    const float aq = fabsf(q0);
    return (aq >= 0x1p-124f && aq <= 0x1p+124f) ? q : __fdiv_rn(a, b);
}

__device__ __forceinline__ void adam_elem(const AdamConst& A, float s, float& p, float& m,
                                          float& v) {
    const float g = div_const(s, A.fk, A.rk);               // rule(): mean = sum / k
    const float mi = __fmaf_rn(A.w1, g - m, m);
    float vi = v * A.b2;
    vi = __fmaf_rn(A.w2 * g, g, vi);
    const float den = div_const(sqrt_rn(vi), A.bc2s, A.rbc2s) + A.eps;
    p = p + __fdiv_rn(A.neg_ss * mi, den);
    m = mi;
    v = vi;
}

// Program access.  The interpreter reads one macro word (two dwords) per step at a uniform address,
// so the words must
// come through the scalar cache: the reference-order program rides in the kernel arguments; a
// general-order program is copied (device to device, stream-ordered, right before the launch)
// into this constant-address-space buffer.  A plain global buffer would be read with vector loads
// (the compiler cannot prove the kernel does not write it) and every op would wait on one.
constexpr int CASC_CONST_WORDS = 16384;
__constant__ int32_t g_casc_prog[CASC_CONST_WORDS];

template <bool INL>
struct ProgRef {
    const RuleProg& R;
    __device__ __forceinline__ uint32_t lo(int i) const {
        if constexpr (INL) return (uint32_t)R.iprog[2 * i];
        else return (uint32_t)g_casc_prog[2 * i];
    }
    __device__ __forceinline__ uint32_t hi(int i) const {
        if constexpr (INL) return (uint32_t)R.iprog[2 * i + 1];
        else return (uint32_t)g_casc_prog[2 * i + 1];
    }
};

// stage a general-order program into g_casc_prog on `stream` (no-op for inline programs)
static int stage_program(const RuleProg& R, hipStream_t stream) {
    if (R.prog == nullptr) return 0;
    FLSIM_REQUIRE(2 * (R.info.len + 1) <= CASC_CONST_WORDS, "rule program of %d macro words (max %d)",
                  R.info.len, CASC_CONST_WORDS / 2 - 1);
    static void* dst = nullptr;
    if (!dst) FLSIM_CHECK_HIP(hipGetSymbolAddress(&dst, HIP_SYMBOL(g_casc_prog)));
    FLSIM_CHECK_HIP(hipMemcpyAsync(dst, R.prog, (size_t)(R.info.len + 1) * 8,
                                   hipMemcpyDeviceToDevice, stream));
    return 0;
}

// ================================================================================================
// k_agg_stream: S_t from a buffer
// ================================================================================================
struct AggArgs {
    const float* S;
    float* S_out;                   // nullable: S_t also written here (the FIFO slot at a tick)
    float* p;
    float* m;
    float* v;
    long g0;                        // first float4 group of this launch
    long lo, hi;                    // element range [lo, hi)
    int ntail;
    int tail_lo[MAX_TAILS];         // [lo, hi) element ranges summed with row_sum
    int tail_hi[MAX_TAILS];
    int nedge;                      // blocks 0..nedge-1: 256-element edge pieces at edge_lo[b]
    long edge_lo[MAX_EDGE];
    AdamConst ac;
    RuleProg R;
};
static_assert(sizeof(AggArgs) <= 4096, "kernel argument block");

__device__ __forceinline__ bool in_tail(const AggArgs& A, long e) {
    bool r = false;
#pragma unroll
    for (int t = 0; t < MAX_TAILS; ++t)
        r |= (t < A.ntail) && e >= A.tail_lo[t] && e < A.tail_hi[t];
    return r;
}

__device__ __forceinline__ bool block_touch(const AggArgs& A, long blo, long span = 1024) {
    const long bhi = blo + span;
    bool touch = blo < A.lo || bhi > A.hi;
#pragma unroll
    for (int t = 0; t < MAX_TAILS; ++t)
        touch |= (t < A.ntail) && A.tail_lo[t] < bhi && A.tail_hi[t] > blo;
    return touch;
}

// Blocks [0, nedge) are 256-element edge pieces (launch edges, tensor tails): one element per
// thread; they run first and overlap the stream.  The other blocks stream one aligned float4 group
// per thread; a streaming block that is also an edge block returns at once.  Every load of a
// thread (S_t, the staged entry arrays, p, m, v) is issued before the arithmetic; loads and
// stores are non-temporal (each byte is touched once).
template <bool INL>
__global__ void __launch_bounds__(256) k_agg_stream(AggArgs A) {
    __shared__ f32x4 ys_lds[NYR * 256];
    const ProgRef<INL> prog{A.R};
    const int tid = threadIdx.x;
    if ((int)blockIdx.x < A.nedge) {
        const long e = A.edge_lo[blockIdx.x] + tid;
        if (e < A.lo || e >= A.hi) return;
        const float x = A.S[e];
        float p = A.p[e], m = A.m[e], v = A.v[e];
        auto yf = [&](int q) -> float { return A.R.arr[q] ? A.R.arr[q][e] : 0.f; };
        const CascVals<float> cv = casc_values(x, A.R.info.need, A.R.info.lp);
        const bool tail = in_tail(A, e);
        float s = 0.f;
        if (!tail) s = casc_run_macro(prog, 0, cv, yf);
        if (tail) s = casc_run_macro(prog, A.R.info.tail_off, cv, yf);
        adam_elem(A.ac, s, p, m, v);
        A.p[e] = p;
        A.m[e] = m;
        A.v[e] = v;
        if (A.S_out) A.S_out[e] = x;
        return;
    }
    const long e0 = 4 * (A.g0 + (long)(blockIdx.x - A.nedge) * 256) + 4 * tid;
    if (block_touch(A, e0 - 4 * tid)) return;
    auto ld = [](const float* ptr) -> f32x4 {
        return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ptr));
    };
    auto st = [](float* ptr, f32x4 val) {
        __builtin_nontemporal_store(val, reinterpret_cast<f32x4*>(ptr));
    };
    const int nst = A.R.narr < NYR ? A.R.narr : NYR;
    f32x4 ys[NYR];
#pragma unroll
    for (int q = 0; q < NYR; ++q)
        ys[q] = (q < nst && A.R.arr[q]) ? ld(A.R.arr[q] + e0) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 x = ld(A.S + e0);
    f32x4 p = ld(A.p + e0), m = ld(A.m + e0), v = ld(A.v + e0);
#pragma unroll
    for (int q = 0; q < NYR; ++q)
        if (q < nst) ys_lds[q * 256 + tid] = ys[q];
    auto yf = [&](int q) -> f32x4 {
        if (q < NYR) return ys_lds[q * 256 + tid];
        return A.R.arr[q] ? ld(A.R.arr[q] + e0) : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    const f32x4 sum = casc_run_macro<true>(
        prog, 0, casc_values(x, A.R.info.need, A.R.info.lp), yf);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        float pp = p[u], mm = m[u], vv = v[u];
        adam_elem(A.ac, sum[u], pp, mm, vv);
        p[u] = pp;
        m[u] = mm;
        v[u] = vv;
    }
    st(A.p + e0, p);
    st(A.m + e0, m);
    st(A.v + e0, v);
    if (A.S_out) st(A.S_out + e0, x);
}

// The reference-order stream with its few entry arrays (NY <= 2: the popped FIFO entries of the
// reference's one slow worker) held in registers instead of LDS, and G float4 groups per thread
// (block = 256 * G groups, group j of thread t at 256 j + t: each j is one coalesced sweep).  All
// of a thread's loads are issued before any arithmetic; no LDS, so 8 blocks of 4 waves fit a CU
// (the LDS-staged form above holds 32 KB per block: 5).  The interpreter runs once per thread on
// G * 4 elements in lock step (T = a 4G-wide vector; the program is uniform).  Edge pieces as
// k_agg_stream (a streaming block covers 1024 G elements).
template <int G>
struct AggVec;
template <>
struct AggVec<1> { typedef float T __attribute__((ext_vector_type(4))); };
template <>
struct AggVec<2> { typedef float T __attribute__((ext_vector_type(8))); };

template <int G, int NY>
__global__ void __launch_bounds__(256) k_agg_stream_reg(AggArgs A) {
    typedef typename AggVec<G>::T T;
    const ProgRef<true> prog{A.R};
    const int tid = threadIdx.x;
    if ((int)blockIdx.x < A.nedge) {
        const long e = A.edge_lo[blockIdx.x] + tid;
        if (e < A.lo || e >= A.hi) return;
        const float x = A.S[e];
        float p = A.p[e], m = A.m[e], v = A.v[e];
        auto yf = [&](int q) -> float { return A.R.arr[q] ? A.R.arr[q][e] : 0.f; };
        const CascVals<float> cv = casc_values(x, A.R.info.need, A.R.info.lp);
        const bool tail = in_tail(A, e);
        float s = 0.f;
        if (!tail) s = casc_run_macro(prog, 0, cv, yf);
        if (tail) s = casc_run_macro(prog, A.R.info.tail_off, cv, yf);
        adam_elem(A.ac, s, p, m, v);
        A.p[e] = p;
        A.m[e] = m;
        A.v[e] = v;
        if (A.S_out) A.S_out[e] = x;
        return;
    }
    const long b0 = 4 * (A.g0 + (long)(blockIdx.x - A.nedge) * 256 * G);   // block's first element
    if (block_touch(A, b0, 1024L * G)) return;
    auto ld = [](const float* ptr) -> f32x4 {
        return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ptr));
    };
    auto st = [](float* ptr, f32x4 val) {
        __builtin_nontemporal_store(val, reinterpret_cast<f32x4*>(ptr));
    };
    long e[G];
#pragma unroll
    for (int j = 0; j < G; ++j) e[j] = b0 + 1024L * j + 4 * tid;
    f32x4 xs[G], ps[G], ms[G], vs[G], ys[NY > 0 ? NY : 1][G];
#pragma unroll
    for (int q = 0; q < NY; ++q)
#pragma unroll
        for (int j = 0; j < G; ++j)
            ys[q][j] = A.R.arr[q] ? ld(A.R.arr[q] + e[j]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < G; ++j) {
        xs[j] = ld(A.S + e[j]);
        ps[j] = ld(A.p + e[j]);
        ms[j] = ld(A.m + e[j]);
        vs[j] = ld(A.v + e[j]);
    }
    auto widen = [](const f32x4 (&a)[G]) -> T {
        T t;
#pragma unroll
        for (int j = 0; j < G; ++j)
#pragma unroll
            for (int u = 0; u < 4; ++u) t[4 * j + u] = a[j][u];
        return t;
    };
    T yw[NY > 0 ? NY : 1];
#pragma unroll
    for (int q = 0; q < NY; ++q) yw[q] = widen(ys[q]);
    auto yf = [&](int q) -> T {
        if constexpr (NY == 0) return T(0.f);
        else if constexpr (NY == 1) return yw[0];
        else return q == 0 ? yw[0] : yw[1];
    };
    const T sum = casc_run_macro<true>(prog, 0, casc_values(widen(xs), A.R.info.need, A.R.info.lp),
                                       yf);
#pragma unroll
    for (int j = 0; j < G; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float pp = ps[j][u], mm = ms[j][u], vv = vs[j][u];
            adam_elem(A.ac, sum[4 * j + u], pp, mm, vv);
            ps[j][u] = pp;
            ms[j][u] = mm;
            vs[j][u] = vv;
        }
        st(A.p + e[j], ps[j]);
        st(A.m + e[j], ms[j]);
        st(A.v + e[j], vs[j]);
        if (A.S_out) st(A.S_out + e[j], xs[j]);
    }
}

// ================================================================================================
// k_slab_step: slabs -> S_t [-> S_out] [-> rule() + Adam], one launch
// ================================================================================================
struct StepArgs {
    float* base;                    // gradstate
    long cnt_off, part_off;         // tile counters (int32) / unit partials, floats from base
    float* S_out;
    float* p;
    float* m;
    float* v;
    int nseg, units;
    int u_lo;                       // first unit of this launch (block b runs unit u_lo + b)
    int il_lo, il_w, il_n;          // interleave units [il_lo, il_lo + il_n): il_w wide, then conv
    AdamConst ac;
    RuleProg R;
    SlabSeg seg[STEP_MAX_SEG];
};
static_assert(sizeof(StepArgs) <= 4096, "kernel argument block");

// LDS map (ONE __shared__ array, cdna_hip_programming.md §5 item 4(a)): z-lane partials f32x4[256]
// at 0, the tile's 256 sums at 1024, the last-arriver flag at 1280, staged entry arrays at 1536
constexpr int L_RED = 0, L_SUM = 1024, L_FLAG = 1280, L_Y = 1536;
// general-order tiles also stage x, p, m, v for the one-wave interpreter
constexpr int L_S = L_Y + NYR * 256, L_P = L_S + 256, L_M = L_P + 256, L_V = L_M + 256,
              L_END = L_V + 256;

// one unit's z-range of 256 slab columns -> this thread's column sum (thread t owns column t)
__device__ __forceinline__ float reduce_cols(const float* slab, const SlabSeg& g, int tile, int z0,
                                             int z1, float* lds) {
    const int tid = threadIdx.x;
    if ((g.n & 3) == 0) {
        const int tx = tid & 63, tz = tid >> 6;
        const long col = (long)tile * 256 + 4 * tx;
        f32x4 acc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (col < g.n) {
            const float* pz = slab + col;
            int z = z0 + tz;
            for (; z + 28 < z1; z += 32) {        // eight rows in flight per thread
                f32x4 x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    x[u] = __builtin_nontemporal_load(
                        reinterpret_cast<const f32x4*>(pz + (long)(z + 4 * u) * g.n));
#pragma unroll
                for (int u = 0; u < 8; ++u) acc[u & 3] += x[u];
            }
            for (; z + 12 < z1; z += 16) {
                f32x4 x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    x[u] = __builtin_nontemporal_load(
                        reinterpret_cast<const f32x4*>(pz + (long)(z + 4 * u) * g.n));
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[u] += x[u];
            }
            // at most three z-lanes rows left
            if (z < z1) acc[0] += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(pz + (long)z * g.n));
            if (z + 4 < z1) acc[1] += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(pz + (long)(z + 4) * g.n));
            if (z + 8 < z1) acc[2] += __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(pz + (long)(z + 8) * g.n));
        }
        f32x4 t = acc[0];
        t += acc[1];
        t += acc[2];
        t += acc[3];
        f32x4* red = reinterpret_cast<f32x4*>(lds + L_RED);
        red[tid] = t;
        __syncthreads();
        if (tz == 0) {
            t += red[64 + tx];
            t += red[128 + tx];
            t += red[192 + tx];
            reinterpret_cast<f32x4*>(lds + L_SUM)[tx] = t;
        }
        __syncthreads();
        return lds[L_SUM + tid];
    }
    // rows not a multiple of 4 floats (tiny tensors): one column per thread
    const long col = (long)tile * 256 + tid;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (col < g.n) {
        const float* pz = slab + col;
        int z = z0;
        for (; z + 3 < z1; z += 4) {
            a0 += pz[(long)z * g.n];
            a1 += pz[(long)(z + 1) * g.n];
            a2 += pz[(long)(z + 2) * g.n];
            a3 += pz[(long)(z + 3) * g.n];
        }
        if (z < z1) a0 += pz[(long)z * g.n];
        if (z + 1 < z1) a1 += pz[(long)(z + 1) * g.n];
        if (z + 2 < z1) a2 += pz[(long)(z + 2) * g.n];
    }
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

// finish-phase addressing of a slab column: packed conv [co][khkw*CIP + ci] -> torch
// [co][ci][kh][kw]; padding columns (ci >= CI, khkw >= 9, col >= n) carry nothing
__device__ __forceinline__ bool col_to_param(const SlabSeg& g, long col, long& tl) {
    tl = col;
    bool valid = col < g.n;
    if (g.CO) {
        const int co = (int)(col / g.KP);
        const int k = (int)(col - (long)co * g.KP);
        const int khkw = k / g.CIP, ci = k - khkw * g.CIP;
        valid = valid && khkw < 9 && ci < g.CI;
        tl = ((long)co * g.CI + ci) * 9 + khkw;
    }
    return valid;
}

// Identity-layout segments (the linear layers): tiles of 1024 elements, thread t owns the float4
// column 4t; it sums its Z slab rows itself (small Z, four accumulators) and finishes with 16-B
// parameter-side loads and stores; the parameter loads are issued before the slab reads.
template <bool ADAM, bool INL>
__device__ __forceinline__ void slab_step_wide(const StepArgs& A, const SlabSeg& g, int u, int ul,
                                               float* lds) {
    // entry arrays held in registers (the rest load on demand): all of a general-order program's
    // arrays up to 8 (configs[3] uses 6), so no Y word of the interpreter waits on a global load
    constexpr int NYW = 8;
    const int tid = threadIdx.x;
    const float* slab = A.base + g.slab_off;
    const ProgRef<INL> prog{A.R};
    int tile, t_end, j;
    if (g.nz == 1) {
        tile = ul * g.tpu;
        t_end = tile + g.tpu < g.tiles ? tile + g.tpu : g.tiles;
        j = 0;
    } else {
        tile = ul / g.nz;
        j = ul - tile * g.nz;
        t_end = tile + 1;
    }
    const int z0 = j * g.zc;
    int z1 = z0 + g.zc < g.Z ? z0 + g.zc : g.Z;
    if (z1 > g.zlim) z1 = g.zlim > z0 ? g.zlim : z0;     // rows past zlim are stale this epoch
    auto ld = [](const float* ptr) -> f32x4 {
        return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ptr));
    };
    for (; tile < t_end; ++tile) {
        const long c = (long)tile * 1024 + 4 * tid;
        const bool valid = c < g.n;
        const long e = g.toff + c;
        f32x4 p, m, v, ys[NYW];
        auto load_param_side = [&]() {
#pragma unroll
            for (int q = 0; q < NYW; ++q)
                ys[q] = (q < A.R.narr && A.R.arr[q]) ? ld(A.R.arr[q] + e) : f32x4{0.f, 0.f, 0.f, 0.f};
            p = ld(A.p + e);
            m = ld(A.m + e);
            v = ld(A.v + e);
        };
        // reference order: the parameter side is loaded ahead of the slab rows (both round trips
        // overlap); general order: after them, so the registers are free during the reduction and
        // more waves fit (the interpreter that follows hides the exposed load behind the other
        // resident waves)
        if (ADAM && INL && valid && g.nz == 1) load_param_side();
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
        if (valid) {
            const float* pz = slab + c;
            int z = z0;
            for (; z + 7 < z1; z += 8) {               // eight rows in flight
                f32x4 x[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) x[r] = ld(pz + (long)(z + r) * g.n);
                a0 += x[0];
                a1 += x[1];
                a2 += x[2];
                a3 += x[3];
                a0 += x[4];
                a1 += x[5];
                a2 += x[6];
                a3 += x[7];
            }
            for (; z + 3 < z1; z += 4) {
                const f32x4 x0 = ld(pz + (long)z * g.n), x1 = ld(pz + (long)(z + 1) * g.n);
                const f32x4 x2 = ld(pz + (long)(z + 2) * g.n), x3 = ld(pz + (long)(z + 3) * g.n);
                a0 += x0;
                a1 += x1;
                a2 += x2;
                a3 += x3;
            }
            if (z < z1) a0 += ld(pz + (long)z * g.n);
            if (z + 1 < z1) a1 += ld(pz + (long)(z + 1) * g.n);
            if (z + 2 < z1) a2 += ld(pz + (long)(z + 2) * g.n);
        }
        a0 += a1;
        a0 += a2;
        a0 += a3;
        if (ADAM && !INL && valid && g.nz == 1) load_param_side();
        if (g.nz > 1) {
            // the conv path's hand-off with 1024 floats per unit (sc1 stores / loads)
            float* part = A.base + A.part_off;
            float* mine = part + (long)u * 1024 + 4 * tid;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __hip_atomic_store(mine + k, a0[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            int* cnt = reinterpret_cast<int*>(A.base + A.cnt_off) + g.tile0 + tile;
            if (tid == 0) {
                const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                lds[L_FLAG] = __int_as_float(old);
            }
            __syncthreads();
            if (__float_as_int(lds[L_FLAG]) != g.nz - 1) return;
            if (ADAM && valid) load_param_side();
            float* pt = part + (long)(g.unit0 + tile * g.nz) * 1024 + 4 * tid;
            for (int jj = 0; jj < g.nz; ++jj) {
                f32x4 x;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    x[k] = __hip_atomic_load(pt + (long)jj * 1024 + k, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                if (jj == 0) a0 = x;
                else a0 += x;
            }
            if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!valid) continue;
        if (A.S_out) *reinterpret_cast<f32x4*>(A.S_out + e) = a0;
        if constexpr (ADAM) {
            auto yf = [&](int q) -> f32x4 {
                // q is uniform: a scalar switch picks the register, no indexed access
                static_assert(NYW == 8, "one case per register-held entry array");
                switch (q) {
                    case 0: return ys[0];
                    case 1: return ys[1];
                    case 2: return ys[2];
                    case 3: return ys[3];
                    case 4: return ys[4];
                    case 5: return ys[5];
                    case 6: return ys[6];
                    case 7: return ys[7];
                    default:
                        return A.R.arr[q] ? ld(A.R.arr[q] + e) : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            };
            const f32x4 sum = casc_run_macro<true>(
                prog, 0, casc_values(a0, A.R.info.need, A.R.info.lp), yf);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float pp = p[k], mm = m[k], vv = v[k];
                adam_elem(A.ac, sum[k], pp, mm, vv);
                p[k] = pp;
                m[k] = mm;
                v[k] = vv;
            }
            __builtin_nontemporal_store(p, reinterpret_cast<f32x4*>(A.p + e));
            __builtin_nontemporal_store(m, reinterpret_cast<f32x4*>(A.m + e));
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(A.v + e));
        }
    }
}

// Units are dispatched round-robin (block b -> unit b): consecutive units, hence every segment's
// mix of cheap and heavy units, are spread over all XCDs.  The partial hand-off uses sc1 stores /
// loads, whose cost does not depend on which XCD the last arriver sits on.  Each thread's
// parameter-side loads (p, m, v, staged entry arrays) are issued before the slab reduction (whole
// tiles) or together with the partial loads (split tiles), so the two memory round trips overlap.
template <bool ADAM, bool INL>
__device__ __forceinline__ void slab_step_body(const StepArgs& A, float* lds) {
    const int tid = threadIdx.x;
    // runs of XG consecutive units (a tile's z-units, neighbouring tiles: one parameter region)
    // share an XCD (blocks b and b + 8 do), the runs themselves go round-robin over the XCDs so
    // every XCD gets the same mix of segments
    constexpr int XG = 8;
    const int nb = (int)gridDim.x;
    const int b = (int)blockIdx.x;
    const int nfull = nb / (8 * XG) * (8 * XG);
    const int lb = b < nfull ? ((b >> 3) / XG * 8 + (b & 7)) * XG + (b >> 3) % XG : b;
    int u = A.u_lo + lb;
    if (u >= A.units) return;
    if (u >= A.il_lo && A.il_n > 0) {
        // position i of the interleaved run: wide unit f(i) when f steps, else conv unit i - f(i),
        // f(i) = floor(i * W / N) (the wide units spread evenly over the run)
        const long i = u - A.il_lo;
        const long f0 = i * A.il_w / A.il_n, f1 = (i + 1) * A.il_w / A.il_n;
        u = A.il_lo + (f1 > f0 ? (int)f0 : A.il_w + (int)(i - f0));
    }
    int si = 0;
    while (si + 1 < A.nseg && A.seg[si + 1].unit0 <= u) ++si;
    const SlabSeg& g = A.seg[si];
    const int ul = u - g.unit0;
    if (g.wide) {
        slab_step_wide<ADAM, INL>(A, g, u, ul, lds);
        return;
    }
    int tile, t_end, j;
    if (g.nz == 1) {
        tile = ul * g.tpu;
        t_end = tile + g.tpu < g.tiles ? tile + g.tpu : g.tiles;
        j = 0;
    } else {
        tile = ul / g.nz;
        j = ul - tile * g.nz;
        t_end = tile + 1;
    }
    const float* slab = A.base + g.slab_off;
    const int z0 = j * g.zc;
    int z1 = z0 + g.zc < g.Z ? z0 + g.zc : g.Z;
    if (z1 > g.zlim) z1 = g.zlim > z0 ? g.zlim : z0;     // rows past zlim are stale this epoch
    const ProgRef<INL> prog{A.R};
    const int nst = A.R.narr < NYR ? A.R.narr : NYR;
    for (; tile < t_end; ++tile) {
        long tl;
        const bool valid = col_to_param(g, (long)tile * 256 + tid, tl);
        const long e = g.toff + tl;
        float p = 0.f, m = 0.f, v = 0.f, ys[NYR];
        auto load_param_side = [&]() {
#pragma unroll
            for (int q = 0; q < NYR; ++q)
                ys[q] = (q < nst && A.R.arr[q]) ? A.R.arr[q][e] : 0.f;
            p = A.p[e];
            m = A.m[e];
            v = A.v[e];
        };
        if (ADAM && valid && g.nz == 1) load_param_side();
        __syncthreads();                       // LDS reuse across the unit's tiles
        float s = reduce_cols(slab, g, tile, z0, z1, lds);
        if (g.nz > 1) {
            // hand the partial to the tile's last-arriving unit: sc1 stores, every wave's vmcnt
            // drained, one agent-scope ticket; the last arriver reads all partials with sc1 loads
            float* part = A.base + A.part_off;
            __hip_atomic_store(part + (long)u * 1024 + tid, s, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            int* cnt = reinterpret_cast<int*>(A.base + A.cnt_off) + g.tile0 + tile;
            if (tid == 0) {
                const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                lds[L_FLAG] = __int_as_float(old);
            }
            __syncthreads();
            if (__float_as_int(lds[L_FLAG]) != g.nz - 1) return;
            if (ADAM && valid) load_param_side();
            // the nz partials in z order, eight loads in flight
            float* pt = part + (long)(g.unit0 + tile * g.nz) * 1024 + tid;
            s = 0.f;
            bool first = true;
            for (int j0 = 0; j0 < g.nz; j0 += 8) {
                float pv[8];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    pv[jj] = j0 + jj < g.nz ? __hip_atomic_load(pt + (long)(j0 + jj) * 1024,
                                                                __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT)
                                            : 0.f;
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    if (j0 + jj < g.nz) {
                        s = first ? pv[jj] : s + pv[jj];
                        first = false;
                    }
                }
            }
            if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (ADAM && !INL) {
            // general order: the tile's 256 elements go through the program as float4 lanes of
            // ONE wave (a quarter of the interpreter's scalar work per element); the tile is
            // staged in LDS (x, p, m, v, entry arrays) and written back by its owning threads.
            // Tiles holding row_sum tail elements, or more arrays than NYR, take the per-element
            // path below.
            if (valid && A.S_out) A.S_out[e] = s;
            const bool tail = valid && tl >= (long)(g.numel / 32) * 32;
            lds[L_S + tid] = valid ? s : 0.f;
            lds[L_P + tid] = p;
            lds[L_M + tid] = m;
            lds[L_V + tid] = v;
#pragma unroll
            for (int q = 0; q < NYR; ++q)
                if (q < nst) lds[L_Y + q * 256 + tid] = valid ? ys[q] : 0.f;
            if (!__syncthreads_or(tail) && A.R.narr <= NYR) {
#if FLSIM_SEQ_EARLY_EXIT
                if (tile + 1 == t_end) {
                    // the unit's last tile: waves 1..3 leave now (their slots go to the next
                    // streaming blocks instead of idling at a barrier through the program); wave
                    // 0 interprets and stores its four elements per lane itself
                    if (tid >= 64) return;
                    const f32x4* l4 = reinterpret_cast<const f32x4*>(lds);
                    auto yf4 = [&](int q) -> f32x4 { return l4[(L_Y + q * 256) / 4 + tid]; };
                    const f32x4 sum = casc_run_macro<true>(
                        prog, 0, casc_values(l4[L_S / 4 + tid], A.R.info.need, A.R.info.lp), yf4);
                    const f32x4 pp = l4[L_P / 4 + tid], mm = l4[L_M / 4 + tid],
                                vv = l4[L_V / 4 + tid];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        long tk;
                        if (!col_to_param(g, (long)tile * 256 + 4 * tid + k, tk)) continue;
                        float p1 = pp[k], m1 = mm[k], v1 = vv[k];
                        adam_elem(A.ac, sum[k], p1, m1, v1);
                        const long ek = g.toff + tk;
                        A.p[ek] = p1;
                        A.m[ek] = m1;
                        A.v[ek] = v1;
                    }
                    return;
                }
#endif
                if (tid < 64) {
                    const f32x4* l4 = reinterpret_cast<const f32x4*>(lds);
                    auto yf4 = [&](int q) -> f32x4 { return l4[(L_Y + q * 256) / 4 + tid]; };
                    const f32x4 sum = casc_run_macro<true>(
                        prog, 0, casc_values(l4[L_S / 4 + tid], A.R.info.need, A.R.info.lp), yf4);
                    f32x4 pp = l4[L_P / 4 + tid], mm = l4[L_M / 4 + tid], vv = l4[L_V / 4 + tid];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        float p1 = pp[k], m1 = mm[k], v1 = vv[k];
                        adam_elem(A.ac, sum[k], p1, m1, v1);
                        pp[k] = p1;
                        mm[k] = m1;
                        vv[k] = v1;
                    }
                    f32x4* w4 = reinterpret_cast<f32x4*>(lds);
                    w4[L_P / 4 + tid] = pp;
                    w4[L_M / 4 + tid] = mm;
                    w4[L_V / 4 + tid] = vv;
                }
                __syncthreads();
                if (valid) {
                    A.p[e] = lds[L_P + tid];
                    A.m[e] = lds[L_M + tid];
                    A.v[e] = lds[L_V + tid];
                }
                continue;
            }
        }
        if (!valid) continue;
        if (A.S_out && (INL || !ADAM)) A.S_out[e] = s;
        if constexpr (ADAM) {
#pragma unroll
            for (int q = 0; q < NYR; ++q)
                if (q < nst) lds[L_Y + q * 256 + tid] = ys[q];
            auto yf = [&](int q) -> float {
                if (q < NYR) return lds[L_Y + q * 256 + tid];
                return A.R.arr[q] ? A.R.arr[q][e] : 0.f;
            };
            const CascVals<float> cv = casc_values(s, A.R.info.need, A.R.info.lp);
            const bool tail = tl >= (long)(g.numel / 32) * 32;
            float sum = 0.f;
            if (!tail) sum = casc_run_macro(prog, 0, cv, yf);
            if (tail) sum = casc_run_macro(prog, A.R.info.tail_off, cv, yf);
            adam_elem(A.ac, sum, p, m, v);
            A.p[e] = p;
            A.m[e] = m;
            A.v[e] = v;
        }
    }
}

template <bool ADAM, bool INL>
__global__ void __launch_bounds__(256) k_slab_step(StepArgs A) {
    __shared__ float lds[L_Y + NYR * 256];
    slab_step_body<ADAM, INL>(A, lds);
}

// General-order programs: the interpreter's chains of dependent adds want many resident waves to
// hide their latency, so this instantiation is held to SEQ_WAVES waves per SIMD (register budget)
#ifndef SEQ_WAVES
#define SEQ_WAVES 4
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEQ_WAVES, 8)))
k_slab_step_seq(StepArgs A) {
    __shared__ float lds[L_END];
    slab_step_body<true, false>(A, lds);
}

// ================================================================================================
// host
// ================================================================================================
int make_adam_const(int divisor, long step, double lr, double beta1, double beta2, double eps,
                    AdamConst* ac) {
    FLSIM_REQUIRE(divisor > 0 && divisor < (1 << 24), "divisor %d out of range", divisor);
    FLSIM_REQUIRE(step >= 1, "step must be >= 1");
    ac->fk = (float)divisor;                         // rule(): mean = sum / k
    {
        volatile float one = 1.f, fk = (float)divisor;   // RN(1/k) in fp32, not via double
        ac->rk = one / fk;
    }
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    ac->w1 = (float)(1.0 - beta1);
    ac->b2 = (float)beta2;
    ac->w2 = (float)(1.0 - beta2);
    ac->bc2s = (float)sqrt(bc2);
    {
        volatile float one = 1.f, b = ac->bc2s;
        ac->rbc2s = one / b;
    }
    ac->eps = (float)eps;
    ac->neg_ss = (float)(-(lr / bc1));
    return 0;
}

int make_rule(const flsim_rule* r, RuleProg* R) {
    FLSIM_REQUIRE(r, "null rule");
    FLSIM_REQUIRE(r->n_arrays >= 0 && r->n_arrays <= RULE_MAX_ARR, "n_arrays = %d (max %d)",
                  r->n_arrays, RULE_MAX_ARR);
    memset(R, 0, sizeof(*R));
    R->narr = r->n_arrays;
    int distinct = 0;
    for (int q = 0; q < r->n_arrays; ++q) {
        R->arr[q] = r->arrays[q];
        bool seen = r->arrays[q] == nullptr;
        for (int s = 0; s < q && !seen; ++s) seen = r->arrays[s] == r->arrays[q];
        distinct += !seen;
    }
    R->distinct = distinct;
    if (r->prog == nullptr) {
        // reference order: [S] * c + arrays in order (main.py:161-172: the slow worker is last)
        FLSIM_REQUIRE(r->c >= 0 && r->c + r->n_arrays > 0,
                      "empty weight_ups (reference: IndexError in rule, main.py:25)");
        const int k = r->c + r->n_arrays;
        int32_t pos[RULE_MAX_ARR], arr[RULE_MAX_ARR];
        for (int q = 0; q < r->n_arrays; ++q) {
            pos[q] = r->c + q;
            arr[q] = q;
        }
        int32_t ops[RULE_INL_PROG];
        CascInfo oi;
        int len = build_cascade_program(k, pos, arr, r->n_arrays, ops, RULE_INL_PROG, &oi);
        FLSIM_REQUIRE(len > 0, "rule program for k = %d entries failed (%d)", k, len);
        len = build_macro_program(ops, oi, reinterpret_cast<uint32_t*>(R->iprog),
                                  RULE_INL_PROG / 2, &R->info);
        FLSIM_REQUIRE(len > 0, "rule macro program for k = %d entries failed (%d)", k, len);
        R->prog = nullptr;
    } else {
        R->prog = r->prog;
        R->info = CascInfo{r->info[0], r->info[1], r->info[2], r->info[3]};
        FLSIM_REQUIRE(R->info.len > 0 && R->info.tail_off > 0 && R->info.tail_off < R->info.len &&
                      R->info.lp >= 4, "bad program info");
    }
    return 0;
}

int slab_step_launch(float* gradstate, const StepPlan& plan, long cnt_off, long part_off,
                     float* S_out, const RuleProg* rule, const AdamConst* ac, float* p, float* m,
                     float* v, long P, hipStream_t stream) {
    StepArgs A{};
    A.base = gradstate;
    A.cnt_off = cnt_off;
    A.part_off = part_off;
    A.S_out = S_out;
    A.p = p;
    A.m = m;
    A.v = v;
    A.nseg = plan.nseg;
    A.units = plan.units;
    for (int i = 0; i < plan.nseg; ++i) A.seg[i] = plan.seg[i];
    if (rule) {
        FLSIM_REQUIRE(p && m && v && ac, "null pointer");
        A.R = *rule;
        A.ac = *ac;
    }
    // FLSIM_STEP_UNITS="lo,hi" (measurement only): run units [lo, hi) of the plan -- whole
    // segments, so every split tile completes and resets its counter
    A.u_lo = 0;
    int u_hi = plan.units;
    // general order only: interleave the wide and conv units (measured: reference order and
    // reduce-only steps are faster in plan order, profiles/r02f/step_bench_*.txt)
    A.il_lo = plan.u_wide;
    A.il_w = plan.u_conv - plan.u_wide;
    A.il_n = (rule && rule->prog != nullptr) ? plan.units - plan.u_wide : 0;
    if (const char* env = lab_env("FLSIM_STEP_UNITS")) {
        int lo = 0, hi = 0;
        if (sscanf(env, "%d,%d", &lo, &hi) == 2 && 0 <= lo && lo < hi && hi <= plan.units) {
            A.u_lo = lo;
            u_hi = hi;
            A.il_n = 0;             // measurement of a unit range: plan order, no interleave
        }
    }
    if (const char* env = lab_env("FLSIM_STEP_NO_INTERLEAVE"))
        if (atoi(env)) A.il_n = 0;
    const unsigned nblk = (unsigned)(u_hi - A.u_lo);
    // algorithmic HBM bytes: every slab byte once; S_out written; p, m, v read + written; each
    // distinct entry array read once
    double slab_read = 0.0;
    for (int i = 0; i < plan.nseg; ++i)
        slab_read += (double)(plan.seg[i].zlim < plan.seg[i].Z ? plan.seg[i].zlim : plan.seg[i].Z) *
                     plan.seg[i].n;
    double bytes = 4.0 * slab_read + (S_out ? 4.0 * P : 0.0);
    if (rule) bytes += 4.0 * (double)P * (6 + rule->distinct);
    const ProbeSlot ps = probe_begin();
    if (!rule) {
        hipExtLaunchKernelGGL(k_slab_step<false, true>, dim3(nblk), dim3(256), 0, stream, ps.start,
                              ps.stop, 0, A);
    } else if (rule->prog == nullptr) {
        hipExtLaunchKernelGGL(k_slab_step<true, true>, dim3(nblk), dim3(256), 0, stream, ps.start,
                              ps.stop, 0, A);
    } else {
        RC(stage_program(*rule, stream));
        hipExtLaunchKernelGGL(k_slab_step_seq, dim3(nblk), dim3(256), 0, stream, ps.start,
                              ps.stop, 0, A);
    }
    FLSIM_LAUNCH_CHECK();
    const int kid = !rule ? K_SLABSUM : (rule->prog == nullptr ? K_STEP : K_STEP_SEQ);
    return probe_end(ps, kid, bytes);
}

}  // namespace flsim

using namespace flsim;

extern "C" {

// ---- rule() + Adam from S_t in a buffer ---------------------------------------------------------
// tensor_sizes: numel of each parameter tensor in named_parameters order (the cascade's column
// rule is per tensor)
int flsim_aggregate_adam_rule(const float* S, const flsim_rule* rule, float* p, float* m, float* v,
                              long P, const long* tensor_sizes, int n_tensors, long step, double lr,
                              double beta1, double beta2, double eps, hipStream_t stream) {
    return flsim_aggregate_adam_rule_push(S, nullptr, rule, p, m, v, P, tensor_sizes, n_tensors,
                                          step, lr, beta1, beta2, eps, stream);
}

// the same, also writing S_t to S_out (the slow worker's FIFO slot at a tick, main.py:156,161)
// in the same pass: world > 1 after the all-reduce
int flsim_aggregate_adam_rule_push(const float* S, float* S_out, const flsim_rule* rule, float* p,
                                   float* m, float* v, long P, const long* tensor_sizes,
                                   int n_tensors, long step, double lr, double beta1, double beta2,
                                   double eps, hipStream_t stream) {
    FLSIM_REQUIRE(S && p && m && v && tensor_sizes && rule, "null pointer");
    FLSIM_REQUIRE(P > 0 && P < (1L << 31), "P = %ld out of range", P);
    const uintptr_t al = (uintptr_t)S | (uintptr_t)p | (uintptr_t)m | (uintptr_t)v |
                         (uintptr_t)S_out;
    FLSIM_REQUIRE((al & 15) == 0, "S/S_out/p/m/v must be 16-byte aligned");
    AggArgs A{};
    RC(make_rule(rule, &A.R));
    for (int q = 0; q < A.R.narr; ++q)
        FLSIM_REQUIRE(((uintptr_t)A.R.arr[q] & 15) == 0, "entry arrays must be 16-byte aligned");
    RC(make_adam_const(rule->k, step, lr, beta1, beta2, eps, &A.ac));
    // the register-array stream for the reference order with <= 2 entry arrays: 2 float4 groups
    // per thread without a stale array, 1 with (tools/agg_bench.py, profiles/r03a/agg_bench.txt:
    // 28.2 vs 28.4 us for k = 512; 32.0 vs 33.1 us for k = 513 with the stale S_{t-d});
    // FLSIM_AGG_G = 1 / 2 forces a form, 0 the LDS-staged k_agg_stream (measurement only)
    int agg_g = A.R.narr == 0 ? 2 : 1;
    if (const char* e = lab_env("FLSIM_AGG_G")) agg_g = atoi(e);
    if (agg_g < 0 || agg_g > AGG_GMAX) agg_g = 1;
    const bool reg = A.R.prog == nullptr && A.R.narr <= 2 && agg_g > 0;
    const int G = reg ? agg_g : 1;
    A.S = S;
    A.S_out = S_out;
    A.p = p;
    A.m = m;
    A.v = v;
    long off = 0;
    for (int t = 0; t < n_tensors; ++t) {
        FLSIM_REQUIRE(tensor_sizes[t] > 0, "tensor %d has size %ld", t, tensor_sizes[t]);
        off += tensor_sizes[t];
    }
    FLSIM_REQUIRE(off == P, "tensor sizes sum to %ld, P = %ld", off, P);
    // one launch per <= MAX_TAILS tensor tails (the last numel % 32 elements of each tensor)
    off = 0;
    long lo = 0;
    int t = 0;
    while (lo < P) {
        A.ntail = 0;
        long hi = lo;
        while (t < n_tensors) {
            const long n = tensor_sizes[t];
            const bool tail = (n % 32) != 0;
            if (tail && A.ntail == MAX_TAILS) break;
            if (tail) {
                A.tail_lo[A.ntail] = (int)(off + (n / 32) * 32);
                A.tail_hi[A.ntail] = (int)(off + n);
                A.ntail++;
            }
            off += n;
            hi = off;
            ++t;
        }
        A.lo = lo;
        A.hi = hi;
        A.g0 = lo / 4;
        const long groups = (hi + 3) / 4 - A.g0;
        const long gpb = 256L * G;                  // float4 groups per streaming block
        const long nblk = (groups + gpb - 1) / gpb;
        // edge pieces: the first and last block when they cross the launch range, and every
        // block holding a tail range (host copy of block_touch)
        A.nedge = 0;
        auto add_block = [&](long b) {
            const long blo = 4 * (A.g0 + b * gpb);
            for (int j = 0; j < A.nedge; j += 4 * G)
                if (A.edge_lo[j] == blo) return;
            for (int j = 0; j < 4 * G; ++j) A.edge_lo[A.nedge++] = blo + 256 * j;
        };
        for (long b : {0L, nblk - 1}) {
            const long blo = 4 * (A.g0 + b * gpb);
            if (blo < A.lo || blo + 4 * gpb > A.hi) add_block(b);
        }
        for (int j = 0; j < A.ntail; ++j) {
            const long b0 = (A.tail_lo[j] / 4 - A.g0) / gpb;
            const long b1 = ((A.tail_hi[j] - 1) / 4 - A.g0) / gpb;
            for (long b = b0; b <= b1; ++b) add_block(b);
        }
        // algorithmic HBM bytes: read S_t + the distinct entry arrays + p, m, v; write p, m, v
        // [+ S_out]
        const double bytes = 4.0 * (double)(hi - lo) * (7 + A.R.distinct + (S_out ? 1 : 0));
        const ProbeSlot ps = probe_begin();
        const dim3 grid((unsigned)(nblk + A.nedge));
        if (reg) {
            auto k = G == 2 ? (A.R.narr == 0 ? k_agg_stream_reg<2, 0>
                               : A.R.narr == 1 ? k_agg_stream_reg<2, 1> : k_agg_stream_reg<2, 2>)
                            : (A.R.narr == 0 ? k_agg_stream_reg<1, 0>
                               : A.R.narr == 1 ? k_agg_stream_reg<1, 1> : k_agg_stream_reg<1, 2>);
            hipExtLaunchKernelGGL(k, grid, dim3(256), 0, stream, ps.start, ps.stop, 0, A);
        } else if (A.R.prog == nullptr)
            hipExtLaunchKernelGGL(k_agg_stream<true>, grid, dim3(256),
                                  0, stream, ps.start, ps.stop, 0, A);
        else {
            RC(stage_program(A.R, stream));
            hipExtLaunchKernelGGL(k_agg_stream<false>, grid, dim3(256),
                                  0, stream, ps.start, ps.stop, 0, A);
        }
        FLSIM_LAUNCH_CHECK();
        if (probe_end(ps, A.R.prog == nullptr ? K_AGG : K_AGG_SEQ, bytes)) return 2;
        lo = hi;
    }
    return 0;
}

// reference order: weight_ups = [S] * c + stale[0 .. n_stale) (main.py:161-172)
int flsim_aggregate_adam(const float* S, int c, const float* const* stale, int n_stale,
                         float* p, float* m, float* v, long P, const long* tensor_sizes,
                         int n_tensors, long step, double lr, double beta1, double beta2,
                         double eps, hipStream_t stream) {
    FLSIM_REQUIRE(c >= 0 && n_stale >= 0 && n_stale <= 8, "bad entry counts c=%d ns=%d", c,
                  n_stale);
    FLSIM_REQUIRE(c + n_stale > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    flsim_rule r{};
    r.k = c + n_stale;
    r.c = c;
    r.n_arrays = n_stale;
    for (int q = 0; q < n_stale; ++q) r.arrays[q] = stale ? stale[q] : nullptr;
    return flsim_aggregate_adam_rule(S, &r, p, m, v, P, tensor_sizes, n_tensors, step, lr, beta1,
                                     beta2, eps, stream);
}

// independent-entry semantics: S already holds the sum of the k distinct entries
int flsim_aggregate_adam_sum(const float* S, int k, float* p, float* m, float* v, long P,
                             const long* tensor_sizes, int n_tensors, long step, double lr,
                             double beta1, double beta2, double eps, hipStream_t stream) {
    FLSIM_REQUIRE(k > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    flsim_rule r{};
    r.k = k;
    r.c = 1;
    return flsim_aggregate_adam_rule(S, &r, p, m, v, P, tensor_sizes, n_tensors, step, lr, beta1,
                                     beta2, eps, stream);
}

// host: rule()'s summation program for k entries with the non-S entries at pos[] (increasing)
// holding array arr[], in the device's macro-word form (cascade.h): prog[cap] int32 = pairs (lo,
// hi) + one fetch-pad pair; info[4] = {pairs, pair index of the row_sum part, need, lp}.
int flsim_cascade_program(int k, const int32_t* pos, const int32_t* arr, int n_events,
                          int32_t* prog, int cap, int32_t* info) {
    FLSIM_REQUIRE(prog && info && (n_events == 0 || (pos && arr)), "null pointer");
    FLSIM_REQUIRE(n_events >= 0 && n_events <= CASC_MAX_K, "n_events = %d", n_events);
    const int ocap = 72 + 40 * (n_events + 8);
    int32_t* ops = new int32_t[ocap];
    CascInfo ci{};
    int len = build_cascade_program(k, pos, arr, n_events, ops, ocap, &ci);
    CascInfo mi{};
    if (len > 0) len = build_macro_program(ops, ci, reinterpret_cast<uint32_t*>(prog), cap / 2, &mi);
    delete[] ops;
    FLSIM_REQUIRE(len != -3, "k = %d entries: supported 1 .. %d", k, CASC_MAX_K);
    FLSIM_REQUIRE(len != -1, "events must have increasing positions in [0, k) and arrays >= 0");
    FLSIM_REQUIRE(len > 0, "program longer than %d words (or an array index past 63)", cap);
    info[0] = mi.len;
    info[1] = mi.tail_off;
    info[2] = mi.need;
    info[3] = mi.lp;
    return 0;
}

// host interpreter of a macro program (testing): out[e] = the cascade sum of element e, x = S[e],
// entry arrays ys[q][e]; tail[e] != 0 selects the row_sum program
int flsim_cascade_eval_host(const int32_t* prog, const int32_t* info, const float* S,
                            const float* const* ys, int n_arrays, const uint8_t* tail, long n,
                            float* out) {
    FLSIM_REQUIRE(prog && info && S && out, "null pointer");
    struct HostPairs {
        const int32_t* w;
        uint32_t lo(int i) const { return (uint32_t)w[2 * i]; }
        uint32_t hi(int i) const { return (uint32_t)w[2 * i + 1]; }
    } hp{prog};
    for (long e = 0; e < n; ++e) {
        const CascVals<float> cv = casc_values(S[e], info[2], info[3]);
        auto yf = [&](int q) -> float {
            return (q < n_arrays && ys[q]) ? ys[q][e] : 0.f;
        };
        out[e] = casc_run_macro(hp, (tail && tail[e]) ? info[1] : 0, cv, yf);
    }
    return 0;
}

}  // extern "C"
