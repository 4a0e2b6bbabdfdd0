// The split-bf16 ("xs") form of an fp32 tensor, shared by its producers (GEMM epilogues, weight
// packing) and the split-bf16 GEMMs that consume it (gemm_x6.h).
//
// An fp32 value x is split into three bf16 parts, each rounded to nearest even:
//     h = bf16(x),  m = bf16(x - h),  l = bf16(x - h - m)
// x - h and x - h - m are exact in fp32, and x - h - m has at most 8 significant bits, so l holds
// it exactly and x = h + m + l exactly (and (h + m) + l in fp32 gives x back bit for bit).
//
// Layout of a tensor T whose element count is a multiple of 4, in units of 4 consecutive
// elements (4 channels of one NHWC pixel, 4 k of a row):
//     HM: 16-B units {h0 h1 h2 h3 | m0 m1 m2 m3} (bf16) at T's own byte offsets
//     L :  8-B units {l0 l1 l2 l3} at half T's byte offsets
// so HM is exactly as large as T and L half of it.  A split GEMM loads the parts it needs and
// never splits in its inner loop: the [h|m] unit is one of the bf16 MFMA's operand halves as it
// stands, and [h|l] / [l|h] are register moves of the HM and L units.
#pragma once
#include "common.h"

namespace flsim {

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct SplitBf16 {
    bf16x4v h, m, l;
};

__device__ __forceinline__ SplitBf16 split_bf16(f32x4 x) {
    SplitBf16 p;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const __bf16 h = (__bf16)x[e];
        const float r1 = x[e] - (float)h;
        const __bf16 m = (__bf16)r1;
        const float r2 = r1 - (float)m;
        p.h[e] = h;
        p.m[e] = m;
        p.l[e] = (__bf16)r2;
    }
    return p;
}

// two bf16x4 halves as one 16-B unit (f32x4 bits)
__device__ __forceinline__ f32x4 cat_bf16(bf16x4v a, bf16x4v b) {
    const bf16x8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(f32x4, v);
}

// one unit of the split form: the HM unit and the L unit
struct XsUnit {
    f32x4 hm;
    f32x2 l;
};

__device__ __forceinline__ XsUnit xs_of(f32x4 v) {
    const SplitBf16 p = split_bf16(v);
    return XsUnit{cat_bf16(p.h, p.m), __builtin_bit_cast(f32x2, p.l)};
}

// [h|l] and [l|h] 16-B operand units from the HM and L units (register moves only)
__device__ __forceinline__ f32x4 xs_hl(const XsUnit& u) { return f32x4{u.hm.x, u.hm.y, u.l.x, u.l.y}; }
__device__ __forceinline__ f32x4 xs_lh(const XsUnit& u) { return f32x4{u.l.x, u.l.y, u.hm.x, u.hm.y}; }

// the fp32 values of a unit: (h + m) + l, exact
__device__ __forceinline__ f32x4 xs_value(const XsUnit& u) {
    const bf16x8v hm = __builtin_bit_cast(bf16x8v, u.hm);
    const bf16x4v l = __builtin_bit_cast(bf16x4v, u.l);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = ((float)hm[e] + (float)hm[4 + e]) + (float)l[e];
    return v;
}

// x > 0 for the 4 values of a unit, from its h part alone: RNE keeps the sign, and a positive x rounds
// to a positive h unless x < 2^-134 (below bf16's smallest subnormal), which a ReLU output of
// these networks never is (its smallest positive values are fp32 sums of O(1e-3) products)
// (each h moved to the top half of a 32-bit word is > 0 as a signed integer iff h > 0).  The unit
// is bit-cast as a whole: __builtin_bit_cast(uint32_t, hm.y) of one vector element compiles to
// element x's bits with ROCm 7.2's clang (only one dword is even loaded), see DESIGN 6g
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t xs_pos4(f32x2 h) {     // h = the first 8 B of an HM unit
    const u32x2 w = __builtin_bit_cast(u32x2, h);
    const uint32_t a = w.x, b = w.y;
    return (uint32_t)((int32_t)(a << 16) > 0) | ((uint32_t)((int32_t)(a & 0xffff0000u) > 0) << 1) |
           ((uint32_t)((int32_t)(b << 16) > 0) << 2) |
           ((uint32_t)((int32_t)(b & 0xffff0000u) > 0) << 3);
}

// Unit index of channels 4 c4 .. 4 c4 + 3 of pixel m (pixels counted over all images, HW per image)
// of a split tensor of C channels: pixel-major [img][HW][C] (SM false), or channel-slice-major
// [img][C/16][HW][16] (SM true, loaders.h XsSrcSM)
template <int C, int HW, bool SM>
__device__ __forceinline__ long xs_unit(unsigned m, int c4) {
    if constexpr (!SM) {
        return (long)m * (C / 4) + c4;
    } else {
        static_assert(C % 16 == 0, "whole 16-channel slices");
        const unsigned img = m / (unsigned)HW, p = m - img * (unsigned)HW;
        return ((long)(img * (C / 16) + (c4 >> 2)) * HW + p) * 4 + (c4 & 3);
    }
}

// store the split form of 4 consecutive values (unit index u: elements 4u .. 4u + 3)
template <bool NT = true>
__device__ __forceinline__ void xs_store(float* hm, float* l, long u, f32x4 v) {
    const XsUnit x = xs_of(v);
    if constexpr (NT) {
        __builtin_nontemporal_store(x.hm, reinterpret_cast<f32x4*>(hm) + u);
        __builtin_nontemporal_store(x.l, reinterpret_cast<f32x2*>(l) + u);
    } else {
        reinterpret_cast<f32x4*>(hm)[u] = x.hm;
        reinterpret_cast<f32x2*>(l)[u] = x.l;
    }
}

// xs_store plus, when f is not null, the fp32 values themselves at the same unit index of f (a
// tensor laid out like the HM part: 4 B per element).  The layer inputs of PerformantNet1's fp32
// weight gradients (a1, d1, a3, d2, a5) get this copy: read as plain fp32 (BufSrc) it spares the
// weight gradients the L loads and the (h + m) + l recombination, 1.05-1.2x on conv2-6's
// (profiles/r06/r06q), for 4 B per element more written by the forward
__device__ __forceinline__ void xs_store_f(float* hm, float* l, float* f, long u, f32x4 v) {
    xs_store(hm, l, u, v);
    if (f) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(f) + u);
}

}  // namespace flsim
