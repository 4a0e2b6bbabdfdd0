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
#include "common.h"
#include "flsim.h"

namespace flsim {

constexpr int MAX_STALE = 8;
constexpr int MAX_TAILS = 64;

struct AggArgs {
    const float* S;                 // running sum S_t (the c_t fast entries all alias it)
    const float* stale[MAX_STALE];  // stale entries (nullptr = zeros: torch-1.x semantics)
    int c;                          // copies of S_t
    int ns;                         // number of stale entries
    float* p;
    float* m;
    float* v;
    long P;
    int ntail;
    long tail_lo[MAX_TAILS];        // [lo, hi) element ranges summed with row_sum
    long tail_hi[MAX_TAILS];
    float w1, b2, w2, bc2s, eps, neg_ss;
};

__device__ __forceinline__ int ceil_log2_i(int x) {
    if (x <= 1) return 0;
    return 32 - __clz(x - 1);
}

__device__ __forceinline__ float seq_sum(float v, int n) {
    float a = 0.f;
    for (int j = 0; j < n; ++j) a += v;
    return a;
}

// k-entry value for one element: x for i < c, y[i - c] afterwards
__device__ __forceinline__ float entry(float x, const float (&y)[MAX_STALE], int c, int i) {
    if (i < c) return x;
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < MAX_STALE; ++q) r = (i - c == q) ? y[q] : r;
    return r;
}

// multi_row_sum over k rows whose first c are x and whose rows c.. are y[0..]: blocks made only
// of x are summed once; whole level-1 / level-2 groups of such blocks likewise.
__device__ __forceinline__ float multi_row_sum_rep(float x, const float (&y)[MAX_STALE], int c,
                                                   int k) {
    int lp = ceil_log2_i(k) / 4;
    if (lp < 4) lp = 4;
    const int L = 1 << lp;
    const int nb = k >> lp;              // full blocks
    int nbp = c >> lp;                   // blocks made only of x
    if (nbp > nb) nbp = nb;
    const float bx = seq_sum(x, L);      // acc0 after a pure block (acc0 is 0 at block start)
    const float g1 = seq_sum(bx, L);     // a1 total of a pure level-1 group
    const float g2 = seq_sum(g1, L);     // a2 total of a pure level-2 group
    const int q1 = nbp & (L - 1);
    const int q2 = (nbp >> lp) & (L - 1);
    const int q3 = nbp >> (2 * lp);
    float a0 = 0.f;
    float a1 = seq_sum(bx, q1);
    float a2 = seq_sum(g1, q2);
    float a3 = seq_sum(g2, q3);
    int i = nbp << lp;
    for (int b = nbp; b < nb; ++b) {
        for (int j = 0; j < L; ++j, ++i) a0 += entry(x, y, c, i);
        a1 += a0;
        a0 = 0.f;
        if (((b + 1) & (L - 1)) != 0) continue;
        a2 += a1;
        a1 = 0.f;
        if ((((b + 1) >> lp) & (L - 1)) != 0) continue;
        a3 += a2;
        a2 = 0.f;
    }
    for (; i < k; ++i) a0 += entry(x, y, c, i);
    a0 += a1;
    a0 += a2;
    a0 += a3;
    return a0;
}

// row_sum: the k entries viewed as (k/4, 4) -> stream q holds entries 4r+q.  Its first cq rows
// are S_t copies and the rest are stale entries, so each stream is itself a "c copies then a few
// others" multi_row_sum (memoised); leftovers (k % 4) go into stream 0, then s0 + s1 + s2 + s3.
__device__ __forceinline__ float row_sum_rep(float x, const float (&y)[MAX_STALE], int c, int k) {
    const int sz = k / 4;
    float ps[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        int cq = (c - q + 3) / 4;                 // rows r with 4r + q < c
        cq = cq < 0 ? 0 : (cq > sz ? sz : cq);
        float z[MAX_STALE];
#pragma unroll
        for (int j = 0; j < MAX_STALE; ++j) {
            const int i = 4 * (cq + j) + q;      // entry index (>= c when cq + j < sz)
            z[j] = (cq + j < sz) ? entry(x, y, c, i) : 0.f;
        }
        ps[q] = multi_row_sum_rep(x, z, cq, sz);
    }
    for (int i = sz * 4; i < k; ++i) ps[0] += entry(x, y, c, i);
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

__device__ __forceinline__ void adam_elem(const AggArgs& A, float g, float& p, float& m, float& v) {
    const float mi = __fmaf_rn(A.w1, g - m, m);
    float vi = v * A.b2;
    vi = __fmaf_rn(A.w2 * g, g, vi);
    const float den = __fdiv_rn(sqrt_rn(vi), A.bc2s) + A.eps;
    p = p + __fdiv_rn(A.neg_ss * mi, den);
    m = mi;
    v = vi;
}

__device__ __forceinline__ void do_elem(const AggArgs& A, long e, bool tail) {
    const int k = A.c + A.ns;
    float y[MAX_STALE];
#pragma unroll
    for (int q = 0; q < MAX_STALE; ++q)
        y[q] = (q < A.ns && A.stale[q]) ? A.stale[q][e] : 0.f;
    const float x = A.S[e];
    const float s = tail ? row_sum_rep(x, y, A.c, k) : multi_row_sum_rep(x, y, A.c, k);
    const float g = __fdiv_rn(s, (float)k);
    float p = A.p[e], m = A.m[e], v = A.v[e];
    adam_elem(A, g, p, m, v);
    A.p[e] = p;
    A.m[e] = m;
    A.v[e] = v;
}

__device__ __forceinline__ bool in_tail(const AggArgs& A, long e) {
    for (int t = 0; t < A.ntail; ++t)
        if (e >= A.tail_lo[t] && e < A.tail_hi[t]) return true;
    return false;
}

// one thread = 4 consecutive elements; blocks that touch no tail range take the float4 path
__global__ void __launch_bounds__(256) k_aggregate_adam(AggArgs A) {
    const long e0 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
    const long blo = (long)blockIdx.x * 1024;
    const long bhi = blo + 1024;
    bool touch = bhi > A.P;
    for (int t = 0; t < A.ntail; ++t) touch |= (A.tail_lo[t] < bhi && A.tail_hi[t] > blo);
    if (e0 >= A.P) return;
    if (!touch) {
        const int k = A.c + A.ns;
        const f32x4 xs = *reinterpret_cast<const f32x4*>(A.S + e0);
        f32x4 ys[MAX_STALE];
#pragma unroll
        for (int q = 0; q < MAX_STALE; ++q)
            ys[q] = (q < A.ns && A.stale[q]) ? *reinterpret_cast<const f32x4*>(A.stale[q] + e0)
                                             : f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 p = *reinterpret_cast<const f32x4*>(A.p + e0);
        f32x4 m = *reinterpret_cast<const f32x4*>(A.m + e0);
        f32x4 v = *reinterpret_cast<const f32x4*>(A.v + e0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float y[MAX_STALE];
#pragma unroll
            for (int q = 0; q < MAX_STALE; ++q) y[q] = ys[q][u];
            const float s = multi_row_sum_rep(xs[u], y, A.c, k);
            const float g = __fdiv_rn(s, (float)k);
            float pp = p[u], mm = m[u], vv = v[u];
            adam_elem(A, g, pp, mm, vv);
            p[u] = pp;
            m[u] = mm;
            v[u] = vv;
        }
        *reinterpret_cast<f32x4*>(A.p + e0) = p;
        *reinterpret_cast<f32x4*>(A.m + e0) = m;
        *reinterpret_cast<f32x4*>(A.v + e0) = v;
    } else {
        for (long e = e0; e < e0 + 4 && e < A.P; ++e) do_elem(A, e, in_tail(A, e));
    }
}

}  // namespace flsim

using namespace flsim;

extern "C" {

// tensor_sizes: numel of each parameter tensor in named_parameters order (the cascade's column
// rule is per tensor).  stale[i] == nullptr means a zero entry (torch-1.x stale semantics).
int flsim_aggregate_adam(const float* S, int c, const float* const* stale, int n_stale,
                         float* p, float* m, float* v, long P, const long* tensor_sizes,
                         int n_tensors, long step, double lr, double beta1, double beta2,
                         double eps, hipStream_t stream) {
    FLSIM_REQUIRE(S && p && m && v, "null pointer");
    FLSIM_REQUIRE(c >= 0 && n_stale >= 0 && n_stale <= MAX_STALE, "bad entry counts c=%d ns=%d", c,
                  n_stale);
    FLSIM_REQUIRE(c + n_stale > 0, "empty weight_ups (reference: IndexError in rule, main.py:25)");
    FLSIM_REQUIRE(step >= 1, "step must be >= 1");
    const uintptr_t al = (uintptr_t)S | (uintptr_t)p | (uintptr_t)m | (uintptr_t)v;
    FLSIM_REQUIRE((al & 15) == 0, "S/p/m/v must be 16-byte aligned");
    AggArgs A{};
    A.S = S;
    A.c = c;
    A.ns = n_stale;
    for (int q = 0; q < n_stale; ++q) {
        A.stale[q] = stale ? stale[q] : nullptr;
        FLSIM_REQUIRE(((uintptr_t)A.stale[q] & 15) == 0, "stale entries must be 16-byte aligned");
    }
    A.p = p;
    A.m = m;
    A.v = v;
    A.P = P;
    long off = 0;
    int nt = 0;
    for (int t = 0; t < n_tensors; ++t) {
        const long n = tensor_sizes[t];
        const long body = (n / 32) * 32;
        if (body < n) {
            FLSIM_REQUIRE(nt < MAX_TAILS, "too many tensors");
            A.tail_lo[nt] = off + body;
            A.tail_hi[nt] = off + n;
            nt++;
        }
        off += n;
    }
    FLSIM_REQUIRE(off == P, "tensor sizes sum to %ld, P = %ld", off, P);
    A.ntail = nt;
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    A.w1 = (float)(1.0 - beta1);
    A.b2 = (float)beta2;
    A.w2 = (float)(1.0 - beta2);
    A.bc2s = (float)sqrt(bc2);
    A.eps = (float)eps;
    A.neg_ss = (float)(-(lr / bc1));
    const long threads = (P + 3) / 4;
    hipLaunchKernelGGL(k_aggregate_adam, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream,
                       A);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

}  // extern "C"
