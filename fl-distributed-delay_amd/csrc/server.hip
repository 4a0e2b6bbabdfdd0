// Fused server step: aggregation rule + Central.update_model, streaming from HBM.
//
//   reference: main.py:23-25 rule() = torch.stack(weight_ups).mean(0) per parameter tensor, with
//              weight_ups = [S_t] * c_t (+ the stale FIFO entries, main.py:161-165), and
//              agents.py:9-21 update_model -> torch.optim.Adam (main.py:106).
//
// Arithmetic is bit-exact with torch 2.10 CPU:
//   * the sum over the stacked dim follows ATen's cascade (multi_row_sum, 4 levels, level step
//     2^max(4, ceil_log2(k)/4)) on whole 32-element column blocks of each tensor and the ILP-4
//     row_sum on the tensor's last P % 32 elements; the k entries are c_t copies of S_t followed
//     by the stale entries, so pure-S blocks are computed once per element and reused;
//   * mean = sum / (float)k;
//   * Adam: m = fma(1-b1, g-m, m); v = fma((1-b2)*g, g, v*b2); den = sqrt(v)/sqrt(bc2) + eps;
//     p += (-lr/bc1 * m) / den  (correctly rounded sqrt; torch CPU's sqrt is not).
// Compiled with -ffp-contract=off: the only fused multiply-adds are the explicit ones.
#include <stdio.h>
#include <stdlib.h>

#include "common.h"
#include "flsim.h"
#include "probe.h"

namespace flsim {

constexpr int MAX_STALE = 8;
constexpr int MAX_TAILS = 8;                  // tail ranges per launch (host splits longer lists)
constexpr int MAX_GROUPS = 4;                  // float4 groups per thread on the streaming path
constexpr int MAX_EDGE = 4 * MAX_GROUPS * (2 * MAX_TAILS + 2);  // 256-element element-path pieces

// Memoised multi_row_sum of k = c + ns rows whose first c rows are the same value x (S_t) and
// whose last ns rows are stale entries.  ATen's cascade: 4 accumulators, level step
// L = 2^lp with lp = max(4, ceil_log2(k) / 4); rows go into acc0; each full block of L rows
// closes with acc1 += acc0, every L blocks acc2 += acc1, every L^2 blocks acc3 += acc2; the last
// k % L rows stay in acc0; result acc0 + acc1 + acc2 + acc3.  Blocks made only of x give the
// same partial sums, so the first nbp = c >> lp blocks are summed once per element (bx = L
// copies of x, g1 = L copies of bx, ...) and only the remaining < L + ns rows are fed one by one.
// Every field is uniform, so all control flow below is scalar.
struct Casc {
    int c, ns, lp, nb, nbp, q1, q2, q3;
    int sbase;                      // row_sum streams: stale index of this stream's first stale
};                                  // row (stride 4); 0 for the plain multi_row_sum

struct AggArgs {
    const float* S;                 // running sum S_t (the c_t fast entries all alias it)
    const float* stale[MAX_STALE];  // stale entries (nullptr = zeros: torch-1.x semantics)
    float* p;
    float* m;
    float* v;
    long g0;                        // first float4 group of this launch
    long lo, hi;                    // element range [lo, hi) of this launch
    int ntail;
    int tail_lo[MAX_TAILS];         // [lo, hi) element ranges summed with row_sum
    int tail_hi[MAX_TAILS];
    int nedge;                      // blocks 0..nedge-1: 256-element edge pieces starting at
    long edge_lo[MAX_EDGE];         // edge_lo[b] (the 4G quarters of each edge block)
    long bspan;                     // elements per streaming block (1024 * G)
    int c, k;
    Casc main;                      // multi_row_sum over all k rows (tensor body)
    Casc rs[4];                     // row_sum: stream q = rows 4r + q, r < k / 4 (tensor tail)
    float w1, b2, w2, bc2s, rbc2s, eps, neg_ss, fk, rk;
};
static_assert(sizeof(AggArgs) <= 4096, "kernel argument block");

template <class T>
__device__ __forceinline__ T seq_sum(T v, int n) {
    T a = T(0.f);
    for (int j = 0; j < n; ++j) a += v;
    return a;
}

// T = float (one element) or f32x4 (four elements in lock step: the loop and branch overhead
// of the uniform block structure is paid once per four elements)
template <int LP, class T = float>
struct CascAcc {
    T a0 = T(0.f), a1 = T(0.f), a2 = T(0.f), a3 = T(0.f);
    int i, lp, L;
    // the first nbp full blocks, all made of x
    __device__ __forceinline__ CascAcc(T x, const Casc& C) {
        lp = LP ? LP : C.lp;
        L = 1 << lp;
        T bx = T(0.f);
        if constexpr (LP != 0) {
#pragma unroll
            for (int j = 0; j < (1 << LP); ++j) bx += x;
        } else {
            bx = seq_sum(x, L);
        }
        a1 = seq_sum(bx, C.q1);
        if (C.q2 | C.q3) {
            T g1 = T(0.f);
            if constexpr (LP != 0) {
#pragma unroll
                for (int j = 0; j < (1 << LP); ++j) g1 += bx;
            } else {
                g1 = seq_sum(bx, L);
            }
            a2 = seq_sum(g1, C.q2);
            if (C.q3) a3 = seq_sum(seq_sum(g1, L), C.q3);
        }
        i = C.nbp << lp;
    }
    __device__ __forceinline__ void feed(T val) {
        a0 += val;
        ++i;
        if ((i & (L - 1)) == 0) {   // never true past the last full block (k < (nb + 1) L)
            const int b = i >> lp;
            a1 += a0;
            a0 = T(0.f);
            if ((b & (L - 1)) == 0) {
                a2 += a1;
                a1 = T(0.f);
                if (((b >> lp) & (L - 1)) == 0) {
                    a3 += a2;
                    a2 = T(0.f);
                }
            }
        }
    }
    __device__ __forceinline__ T finish() {
        a0 += a1;
        a0 += a2;
        a0 += a3;
        return a0;
    }
};

// streaming path: four elements, stale values already in registers
template <int LP, int NSR>
__device__ __forceinline__ f32x4 multi_row_sum_regs4(f32x4 x, const f32x4 (&y)[NSR],
                                                     const Casc& C) {
    CascAcc<LP, f32x4> acc(x, C);
    while (acc.i < C.c) acc.feed(x);
#pragma unroll
    for (int q = 0; q < NSR; ++q)
        if (q < C.ns) acc.feed(y[q]);
    return acc.finish();
}

// y[q] for a uniform run-time q (select chain: keeps y in registers)
__device__ __forceinline__ float pick(const float (&y)[MAX_STALE], int q) {
    float r = 0.f;
#pragma unroll
    for (int j = 0; j < MAX_STALE; ++j) r = (j == q) ? y[j] : r;
    return r;
}

// element path: the stale rows of a stream are y[sbase], y[sbase + stride], ...
__device__ __forceinline__ float multi_row_sum_strided(float x, const float (&y)[MAX_STALE],
                                                       const Casc& C, int stride) {
    CascAcc<0> acc(x, C);
    while (acc.i < C.c) acc.feed(x);
    for (int j = 0; j < C.ns; ++j) acc.feed(pick(y, C.sbase + stride * j));
    return acc.finish();
}

// ATen row_sum (the last numel % 32 elements of a tensor): the k rows as (k/4, 4), stream q =
// rows 4r + q summed by multi_row_sum, leftover rows (k % 4) added to stream 0, then
// s0 + s1 + s2 + s3.
__device__ __forceinline__ float row_sum_regs(const AggArgs& A, float x,
                                              const float (&y)[MAX_STALE]) {
    float ps[4];
    for (int q = 0; q < 4; ++q) ps[q] = multi_row_sum_strided(x, y, A.rs[q], 4);
    for (int i = (A.k / 4) * 4; i < A.k; ++i) ps[0] += (i < A.c) ? x : pick(y, i - A.c);
    ps[0] += ps[1];
    ps[0] += ps[2];
    ps[0] += ps[3];
    return ps[0];
}

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

__device__ __forceinline__ void adam_elem(const AggArgs& A, float s, float& p, float& m, float& v) {
    const float g = div_const(s, A.fk, A.rk);               // rule(): mean = sum / k
    const float mi = __fmaf_rn(A.w1, g - m, m);
    float vi = v * A.b2;
    vi = __fmaf_rn(A.w2 * g, g, vi);
    const float den = div_const(sqrt_rn(vi), A.bc2s, A.rbc2s) + A.eps;
    p = p + __fdiv_rn(A.neg_ss * mi, den);
    m = mi;
    v = vi;
}

__device__ __forceinline__ bool in_tail(const AggArgs& A, long e) {
    bool r = false;
#pragma unroll
    for (int t = 0; t < MAX_TAILS; ++t)
        r |= (t < A.ntail) && e >= A.tail_lo[t] && e < A.tail_hi[t];
    return r;
}

__device__ __forceinline__ bool block_touch(const AggArgs& A, long blo) {
    const long bhi = blo + A.bspan;
    bool touch = blo < A.lo || bhi > A.hi;
#pragma unroll
    for (int t = 0; t < MAX_TAILS; ++t)
        touch |= (t < A.ntail) && A.tail_lo[t] < bhi && A.tail_hi[t] > blo;
    return touch;
}

// One launch per <= MAX_TAILS tensor tails.  Blocks [0, nedge) are the pieces of the edge blocks
// the host listed (launch edges, tail ranges): one element per thread, row_sum order on tail
// elements; they start first and overlap the stream.  The other blocks are the streaming path, one thread per
// aligned float4 group; a streaming block that is also an edge block returns at once.
// LP: 4 = the level step of every k < 2^20, 0 = read at run time.  NSR: stale entries held in
// registers by the streaming path (1 covers the reference's single slow worker).  G: float4
// groups per thread (a block streams 1024 G elements; every load of all G groups is issued
// before the arithmetic).  NT: non-temporal loads / stores (each byte is touched once).
template <int LP, int NSR, int G, bool NT>
__global__ void __launch_bounds__(256) k_aggregate_adam(AggArgs A) {
    if ((int)blockIdx.x < A.nedge) {
        // edge piece: 256 elements, one per thread, every load issued before the arithmetic
        const long e = A.edge_lo[blockIdx.x] + threadIdx.x;
        if (e < A.lo || e >= A.hi) return;
        float y[MAX_STALE];
#pragma unroll
        for (int q = 0; q < MAX_STALE; ++q)
            y[q] = (q < A.main.ns && A.stale[q]) ? A.stale[q][e] : 0.f;
        const float x = A.S[e];
        float p = A.p[e], m = A.m[e], v = A.v[e];
        const float s = in_tail(A, e) ? row_sum_regs(A, x, y) : multi_row_sum_strided(x, y, A.main, 1);
        adam_elem(A, s, p, m, v);
        A.p[e] = p;
        A.m[e] = m;
        A.v[e] = v;
        return;
    }
    const long blo = 4 * (A.g0 + (long)(blockIdx.x - A.nedge) * 256 * G);
    if (block_touch(A, blo)) return;
    auto ld = [](const float* ptr) -> f32x4 {
        if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ptr));
        else return *reinterpret_cast<const f32x4*>(ptr);
    };
    auto st = [](float* ptr, f32x4 val) {
        if constexpr (NT) __builtin_nontemporal_store(val, reinterpret_cast<f32x4*>(ptr));
        else *reinterpret_cast<f32x4*>(ptr) = val;
    };
    f32x4 xs[G], ys[G][NSR], p[G], m[G], v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const long e0 = blo + 1024 * g + 4 * threadIdx.x;
        xs[g] = ld(A.S + e0);
#pragma unroll
        for (int q = 0; q < NSR; ++q)
            ys[g][q] = (q < A.main.ns && A.stale[q]) ? ld(A.stale[q] + e0)
                                                     : f32x4{0.f, 0.f, 0.f, 0.f};
        p[g] = ld(A.p + e0);
        m[g] = ld(A.m + e0);
        v[g] = ld(A.v + e0);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const long e0 = blo + 1024 * g + 4 * threadIdx.x;
        const f32x4 sum = multi_row_sum_regs4<LP, NSR>(xs[g], ys[g], A.main);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float pp = p[g][u], mm = m[g][u], vv = v[g][u];
            adam_elem(A, sum[u], pp, mm, vv);
            p[g][u] = pp;
            m[g][u] = mm;
            v[g][u] = vv;
        }
        st(A.p + e0, p[g]);
        st(A.m + e0, m[g]);
        st(A.v + e0, v[g]);
    }
}

// streaming-path shape: float4 groups per thread and non-temporal access.  Default measured on
// MI355X inside the training step (tools/agg_instep.sh, theta/m/v/S cold in HBM): G=1 with
// non-temporal access 27.6 us, plain 29.0 us, G=2 28.5 us, G=4 29.8 us.  (Warm, back-to-back
// in tools/agg_bench.py the plain form is faster: 25.3 vs 26.5 us.)  FLSIM_AGG_VARIANT="G,NT"
// overrides the default for tuning.
struct AggVariant {
    int groups;
    bool nt;
};
static AggVariant agg_variant() {
    static AggVariant v = [] {
        AggVariant d{1, true};
        if (const char* s = getenv("FLSIM_AGG_VARIANT")) {
            int g = 1, nt = 0;
            if (sscanf(s, "%d,%d", &g, &nt) >= 1 && (g == 1 || g == 2 || g == 4)) d = {g, nt != 0};
        }
        return d;
    }();
    return v;
}

template <int LP, int NSR>
static auto pick_kernel(AggVariant v) {
    auto k = k_aggregate_adam<LP, NSR, 1, false>;
    if (v.groups == 2) k = v.nt ? k_aggregate_adam<LP, NSR, 2, true> : k_aggregate_adam<LP, NSR, 2, false>;
    else if (v.groups == 4) k = v.nt ? k_aggregate_adam<LP, NSR, 4, true> : k_aggregate_adam<LP, NSR, 4, false>;
    else if (v.nt) k = k_aggregate_adam<LP, NSR, 1, true>;
    return k;
}

// host: memo constants of a multi_row_sum over k rows, the first c of them copies of x
static Casc make_casc(int c, int k, int sbase) {
    Casc C{};
    int lp = 0;
    while ((1L << lp) < k) ++lp;     // ceil_log2(k)
    lp /= 4;
    if (lp < 4) lp = 4;
    C.c = c;
    C.ns = k - c;
    C.lp = lp;
    C.nb = k >> lp;
    C.nbp = (c >> lp) < C.nb ? (c >> lp) : C.nb;
    C.q1 = C.nbp & ((1 << lp) - 1);
    C.q2 = (C.nbp >> lp) & ((1 << lp) - 1);
    C.q3 = C.nbp >> (2 * lp);
    C.sbase = sbase;
    return C;
}

}  // namespace flsim

using namespace flsim;

extern "C" {

// tensor_sizes: numel of each parameter tensor in named_parameters order (the cascade's column
// rule is per tensor).  stale[i] == nullptr means a zero entry (torch-1.x stale semantics).
static int aggregate_adam_impl(const float* S, int c, const float* const* stale, int n_stale,
                               int divisor, float* p, float* m, float* v, long P,
                               const long* tensor_sizes, int n_tensors, long step, double lr,
                               double beta1, double beta2, double eps, hipStream_t stream);

int flsim_aggregate_adam(const float* S, int c, const float* const* stale, int n_stale,
                         float* p, float* m, float* v, long P, const long* tensor_sizes,
                         int n_tensors, long step, double lr, double beta1, double beta2,
                         double eps, hipStream_t stream) {
    return aggregate_adam_impl(S, c, stale, n_stale, c + n_stale, p, m, v, P, tensor_sizes,
                               n_tensors, step, lr, beta1, beta2, eps, stream);
}

// independent-entry semantics: S already holds the sum of the k distinct entries
int flsim_aggregate_adam_sum(const float* S, int k, float* p, float* m, float* v, long P,
                             const long* tensor_sizes, int n_tensors, long step, double lr,
                             double beta1, double beta2, double eps, hipStream_t stream) {
    FLSIM_REQUIRE(k > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    return aggregate_adam_impl(S, 1, nullptr, 0, k, p, m, v, P, tensor_sizes, n_tensors, step, lr,
                               beta1, beta2, eps, stream);
}

static int aggregate_adam_impl(const float* S, int c, const float* const* stale, int n_stale,
                               int divisor, float* p, float* m, float* v, long P,
                               const long* tensor_sizes, int n_tensors, long step, double lr,
                               double beta1, double beta2, double eps, hipStream_t stream) {
    FLSIM_REQUIRE(S && p && m && v && tensor_sizes, "null pointer");
    FLSIM_REQUIRE(c >= 0 && n_stale >= 0 && n_stale <= MAX_STALE, "bad entry counts c=%d ns=%d", c,
                  n_stale);
    FLSIM_REQUIRE(c + n_stale > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    FLSIM_REQUIRE(c + n_stale < (1 << 24), "k = %d entries: beyond exact fp32 integers", c + n_stale);
    FLSIM_REQUIRE(step >= 1, "step must be >= 1");
    FLSIM_REQUIRE(P > 0 && P < (1L << 31), "P = %ld out of range", P);
    const uintptr_t al = (uintptr_t)S | (uintptr_t)p | (uintptr_t)m | (uintptr_t)v;
    FLSIM_REQUIRE((al & 15) == 0, "S/p/m/v must be 16-byte aligned");
    AggArgs A{};
    A.S = S;
    for (int q = 0; q < n_stale; ++q) {
        A.stale[q] = stale ? stale[q] : nullptr;
        FLSIM_REQUIRE(((uintptr_t)A.stale[q] & 15) == 0, "stale entries must be 16-byte aligned");
    }
    A.p = p;
    A.m = m;
    A.v = v;
    const int k = c + n_stale;
    A.c = c;
    A.k = k;
    A.main = make_casc(c, k, 0);
    const int sz = k / 4;
    for (int q = 0; q < 4; ++q) {
        int cq = (c - q + 3) / 4;                 // rows r with 4r + q < c
        cq = cq < 0 ? 0 : (cq > sz ? sz : cq);
        A.rs[q] = make_casc(cq, sz, 4 * cq + q - c);
    }
    FLSIM_REQUIRE(divisor > 0 && divisor < (1 << 24), "divisor %d out of range", divisor);
    A.fk = (float)divisor;                         // rule(): mean = sum / k
    {
        volatile float one = 1.f, fk = (float)divisor;   // RN(1/k) in fp32, not via double
        A.rk = one / fk;
    }
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    A.w1 = (float)(1.0 - beta1);
    A.b2 = (float)beta2;
    A.w2 = (float)(1.0 - beta2);
    A.bc2s = (float)sqrt(bc2);
    {
        volatile float one = 1.f, b = A.bc2s;
        A.rbc2s = one / b;
    }
    A.eps = (float)eps;
    A.neg_ss = (float)(-(lr / bc1));
    // tail ranges (last numel % 32 elements of each tensor), split into launches of <= MAX_TAILS
    long off = 0;
    for (int t = 0; t < n_tensors; ++t) {
        FLSIM_REQUIRE(tensor_sizes[t] > 0, "tensor %d has size %ld", t, tensor_sizes[t]);
        off += tensor_sizes[t];
    }
    FLSIM_REQUIRE(off == P, "tensor sizes sum to %ld, P = %ld", off, P);
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
        const AggVariant var = agg_variant();
        const long G = var.groups;
        A.bspan = 1024 * G;
        const long groups = (hi + 3) / 4 - A.g0;
        const long nblk = (groups + 256 * G - 1) / (256 * G);
        // edge blocks: the first and last block when they cross the launch range, and every
        // block holding a tail range (host copy of block_touch)
        A.nedge = 0;
        auto add_block = [&](long b) {
            const long blo = 4 * (A.g0 + b * 256 * G);
            for (int j = 0; j < A.nedge; j += 4 * G)
                if (A.edge_lo[j] == blo) return;
            for (int j = 0; j < 4 * G; ++j) A.edge_lo[A.nedge++] = blo + 256 * j;
        };
        for (long b : {0L, nblk - 1}) {
            const long blo = 4 * (A.g0 + b * 256 * G);
            if (blo < A.lo || blo + A.bspan > A.hi) add_block(b);
        }
        for (int j = 0; j < A.ntail; ++j) {
            const long b0 = (A.tail_lo[j] / 4 - A.g0) / (256 * G);
            const long b1 = ((A.tail_hi[j] - 1) / 4 - A.g0) / (256 * G);
            for (long b = b0; b <= b1; ++b) add_block(b);
        }
        const dim3 grid((unsigned)(nblk + A.nedge));
        // algorithmic HBM bytes: read S_t + the distinct stale entries + p, m, v; write p, m, v
        int distinct = 0;
        for (int q = 0; q < n_stale; ++q) {
            bool seen = A.stale[q] == nullptr;
            for (int r = 0; r < q && !seen; ++r) seen = A.stale[r] == A.stale[q];
            distinct += !seen;
        }
        const double bytes = 4.0 * (double)(hi - lo) * (7 + distinct);
        const ProbeSlot ps = probe_begin();
        const bool lp4 = A.main.lp == 4, ns1 = n_stale <= 1;
        auto kern = lp4 ? (ns1 ? pick_kernel<4, 1>(var) : pick_kernel<4, MAX_STALE>(var))
                        : (ns1 ? pick_kernel<0, 1>(var) : pick_kernel<0, MAX_STALE>(var));
        hipExtLaunchKernelGGL(kern, grid, dim3(256), 0, stream, ps.start, ps.stop, 0, A);
        FLSIM_LAUNCH_CHECK();
        if (probe_end(ps, K_AGG, bytes)) return 2;
        lo = hi;
    }
    return 0;
}

}  // extern "C"

// =============================================================================================
// General entry order (heterogeneous-delay extension): weight_ups appended in
// worker-index order, so stale entries can sit anywhere among the c_t aliased S_t entries, and
// a step may pop many FIFOs.  The sequence is given as events (position, array) sorted by
// position; every other position is S_t.  Same cascade, memoised per pure block / level-1 group
// / level-2 group wherever no event falls inside; one element per thread; the event list is
// read with uniform (scalar) loads, so all control flow stays scalar.
// =============================================================================================
namespace flsim {

constexpr int SEQ_MAX_TAILS = 64;

struct SeqArgs {
    const float* S;
    const int32_t* ev;              // [n_events][2] = (entry position, array index), sorted
    const float* const* arrays;     // device table of stale arrays (nullptr = zeros)
    float* p;
    float* m;
    float* v;
    long P;
    int k, n_events, lp, nb;
    int ntail;
    int tail_lo[SEQ_MAX_TAILS], tail_hi[SEQ_MAX_TAILS];
    float w1, b2, w2, bc2s, rbc2s, eps, neg_ss, fk, rk;
};

__device__ __forceinline__ float seq_y(const SeqArgs& A, int j, long e) {
    const float* a = A.arrays[A.ev[2 * j + 1]];
    return a ? a[e] : 0.f;
}

// multi_row_sum over the entries of stream `q` of stride `str` (the whole sequence: q = 0,
// str = 1; row_sum stream q: positions 4r + q, r < kk) -- kk rows in the stream
__device__ float seq_cascade(const SeqArgs& A, float x, long e, int q, int str, int kk) {
    int lp = 0;
    while ((1 << lp) < kk) ++lp;
    lp /= 4;
    if (lp < 4) lp = 4;
    const int L = 1 << lp;
    const int nb = kk >> lp;
    const float bx = seq_sum(x, L);
    const float g1 = seq_sum(bx, L);
    const float g2 = seq_sum(g1, L);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int i = 0;                       // stream row
    int j = 0;                       // next event of the whole sequence
    auto next_row = [&]() -> int {   // stream row of the next event in this stream, or kk
        while (j < A.n_events) {
            const int pos = A.ev[2 * j];
            if (pos % str == q && pos / str < kk) return pos / str;
            if (pos / str >= kk && pos % str == q) return kk;
            ++j;
        }
        return kk;
    };
    auto close = [&]() {             // i just became a multiple of L
        const int b = i >> lp;
        a1 += a0;
        a0 = 0.f;
        if ((b & (L - 1)) == 0) {
            a2 += a1;
            a1 = 0.f;
            if (((b >> lp) & (L - 1)) == 0) {
                a3 += a2;
                a2 = 0.f;
            }
        }
    };
    const int full = nb << lp;       // rows inside full blocks
    while (i < kk) {
        const int nr = next_row();
        const int lim = nr < full ? nr : full;
        const int L2 = L * L, L3 = L * L * L;
        if ((i & (L3 - 1)) == 0 && i + L3 <= lim) {          // pure level-2 group
            a3 += g2;
            i += L3;
            continue;
        }
        if ((i & (L2 - 1)) == 0 && i + L2 <= lim) {          // pure level-1 group
            a2 += g1;
            i += L2;
            if ((((i >> lp) >> lp) & (L - 1)) == 0) {
                a3 += a2;
                a2 = 0.f;
            }
            continue;
        }
        if ((i & (L - 1)) == 0 && i + L <= lim) {            // pure block
            a1 += bx;
            i += L;
            const int b = i >> lp;
            if ((b & (L - 1)) == 0) {
                a2 += a1;
                a1 = 0.f;
                if (((b >> lp) & (L - 1)) == 0) {
                    a3 += a2;
                    a2 = 0.f;
                }
            }
            continue;
        }
        if (i == nr) {                                       // a stale entry
            a0 += seq_y(A, j, e);
            ++j;
        } else {
            a0 += x;
        }
        ++i;
        if ((i & (L - 1)) == 0 && i <= full) close();
    }
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

__global__ void __launch_bounds__(256) k_aggregate_adam_seq(SeqArgs A) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= A.P) return;
    bool tail = false;
#pragma unroll 1
    for (int t = 0; t < A.ntail; ++t) tail |= e >= A.tail_lo[t] && e < A.tail_hi[t];
    const float x = A.S[e];
    float s;
    if (!tail) {
        s = seq_cascade(A, x, e, 0, 1, A.k);
    } else {                         // row_sum: 4 streams of k/4 rows, leftovers into stream 0
        const int sz = A.k / 4;
        float ps[4];
        for (int q = 0; q < 4; ++q) ps[q] = seq_cascade(A, x, e, q, 4, sz);
        for (int i = sz * 4; i < A.k; ++i) {
            float val = x;
            for (int j = 0; j < A.n_events; ++j)
                if (A.ev[2 * j] == i) val = seq_y(A, j, e);
            ps[0] += val;
        }
        ps[0] += ps[1];
        ps[0] += ps[2];
        ps[0] += ps[3];
        s = ps[0];
    }
    const float g = div_const(s, A.fk, A.rk);
    float p = A.p[e], m = A.m[e], v = A.v[e];
    const float mi = __fmaf_rn(A.w1, g - m, m);
    float vi = v * A.b2;
    vi = __fmaf_rn(A.w2 * g, g, vi);
    const float den = div_const(sqrt_rn(vi), A.bc2s, A.rbc2s) + A.eps;
    A.p[e] = p + __fdiv_rn(A.neg_ss * mi, den);
    A.m[e] = mi;
    A.v[e] = vi;
}

}  // namespace flsim

extern "C" {

// weight_ups in general order: k entries, events[j] = (position, array index) of the non-S_t
// entries (sorted by position); arrays = device table of stale arrays (nullptr = zeros)
int flsim_aggregate_adam_seq(const float* S, int k, const int32_t* events, int n_events,
                             const float* const* arrays, int n_arrays, float* p, float* m, float* v, long P,
                             const long* tensor_sizes, int n_tensors, long step, double lr,
                             double beta1, double beta2, double eps, hipStream_t stream) {
    FLSIM_REQUIRE(S && p && m && v && tensor_sizes, "null pointer");
    FLSIM_REQUIRE(k > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    FLSIM_REQUIRE(k < (1 << 24) && n_events >= 0 && n_events <= k, "bad entry counts k=%d n=%d",
                  k, n_events);
    FLSIM_REQUIRE(n_events == 0 || (events && arrays), "null event table");
    FLSIM_REQUIRE(step >= 1 && P > 0 && P < (1L << 31), "bad step / P");
    SeqArgs A{};
    A.S = S;
    A.ev = events;
    A.arrays = arrays;
    A.p = p;
    A.m = m;
    A.v = v;
    A.P = P;
    A.k = k;
    A.n_events = n_events;
    long off = 0;
    for (int t = 0; t < n_tensors; ++t) {
        const long n = tensor_sizes[t];
        FLSIM_REQUIRE(n > 0, "tensor %d has size %ld", t, n);
        if (n % 32) {
            FLSIM_REQUIRE(A.ntail < SEQ_MAX_TAILS, "more than %d tensors with a row_sum tail",
                          SEQ_MAX_TAILS);
            A.tail_lo[A.ntail] = (int)(off + (n / 32) * 32);
            A.tail_hi[A.ntail] = (int)(off + n);
            A.ntail++;
        }
        off += n;
    }
    FLSIM_REQUIRE(off == P, "tensor sizes sum to %ld, P = %ld", off, P);
    A.fk = (float)k;
    {
        volatile float one = 1.f, fk = (float)k;
        A.rk = one / fk;
    }
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    A.w1 = (float)(1.0 - beta1);
    A.b2 = (float)beta2;
    A.w2 = (float)(1.0 - beta2);
    A.bc2s = (float)sqrt(bc2);
    {
        volatile float one = 1.f, b = A.bc2s;
        A.rbc2s = one / b;
    }
    A.eps = (float)eps;
    A.neg_ss = (float)(-(lr / bc1));
    // algorithmic HBM bytes: S_t + each distinct stale array once + p, m, v read and written
    const double bytes = 4.0 * (double)P * (7 + n_arrays);
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL(k_aggregate_adam_seq, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                          stream, ps.start, ps.stop, 0, A);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, K_AGG, bytes);
}

}  // extern "C"
