// fp32 GEMM on the bf16 matrix cores at fp32 accuracy ("bf16x6"), for k-contiguous operand pairs.
//
// gfx950's fp32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16 rate.  Each fp32 operand
// x is split when it is staged into LDS: h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (round
// to nearest even; x - h and x - h - m are exact in fp32), so x = h + m + l to within 2^-25 |x|.
// A product a*b is the sum of six exact partial products
//     ah*bh + am*bh  +  ah*bm + am*bm  +  ah*bl + al*bh
// (the three dropped, am*bl + al*bm + al*bl, are below 2^-25 |a b|), accumulated in fp32.
// One v_mfma_f32_16x16x32_bf16 sums 32 products per lane slot, so the two terms of each pair above
// go into ONE instruction over the same 16-deep k-step: its 32 slots are (term, k) pairs.  A lane
// of the 16x16x32 MFMA supplies slots 8g .. 8g+7 (g = lane >> 4) of its row / column; with the
// k-contiguous LDS unit of 4 k values per lane (k = 4g .. 4g+3, gemm_core.h) the A operand is
// the 16-B unit [ah | am] (slots 8g..8g+3 = ah, 8g+4..8g+7 = am) and B is [bh | bh], etc.:
//     MFMA 1: A [h|m] x B [h|h]  = ah bh + am bh
//     MFMA 2: A [h|m] x B [m|m]  = ah bm + am bm
//     MFMA 3: A [h|l] x B [l|h]  = ah bl + al bh
// so the LDS holds two 16-B combination planes of the A tile and three of the B tile, each laid
// out and swizzled exactly like the fp32 KC tile, and every fragment is one ds_read_b128.
// Three 16-cycle bf16 MFMAs replace four 32-cycle fp32 ones per k-step (profiles/r03v:
// bf16x6 max error 1.0-3.1 x 2^-24 of sum |a b| against the fp32 MFMA's 1.6-3.3 on the same
// data, K = 1728 and 16384; pre-split operands run the inner loop at 312-316 fp32-equivalent
// TF/s against 148).
#pragma once
#include "gemm_core.h"

namespace flsim {

typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

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

// two bf16x4 halves as one 16-B LDS unit (f32x4 bits)
__device__ __forceinline__ f32x4 cat_bf16(bf16x4v a, bf16x4v b) {
    const bf16x8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(f32x4, v);
}

__device__ __forceinline__ f32x4 mfma_x32(f32x4 a, f32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, a),
                                                   __builtin_bit_cast(bf16x8v, b), c, 0, 0, 0);
}

// Same contract as gemm_kernel (gemm_core.h: 1-D XCD-aware grid, register-staged double buffer,
// one barrier per 16-deep k-step, STAGED / plain epilogues) for KC loaders that expose
// each_unit(); no ASUM epilogues (those need k-major tiles).
// BP = 3: B planes [h|h], [m|m], [l|h] (every fragment one ds_read_b128, no register moves);
// BP = 2: B planes [h|m], [l|h] and the pairing ah bh + am bm, ah bm + am bh (B [m|h] = the
// halves of [h|m] swapped in registers), ah bl + al bh: a third less LDS traffic for B.
template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI, int BP = 3>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_x6_kernel(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
               int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(AL::ROWS == BM && BL::ROWS == BN, "loader rows != tile");
    static_assert(AL::KC && BL::KC, "split-bf16 tiles are k-contiguous");
    static_assert(!EPI::ASUM, "no fused column sums on k-contiguous tiles");
    constexpr int A_FL = KCTile<BM>::FLOATS;      // one combination plane
    constexpr int B_FL = KCTile<BN>::FLOATS;
    constexpr int BUF = 2 * A_FL + BP * B_FL;     // one stage: A [h|m], [h|l]; B planes (BP)
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int STAGE_LD = BN + 4;
    constexpr int BASE_FL = 2 * BUF;
    constexpr int WROWS = 16 * FM;
    constexpr int WM_FIT = BASE_FL / (WROWS * STAGE_LD);
    constexpr int WM_PASS = WM_FIT < 1 ? 1 : (WM_FIT > WAVES_M ? WAVES_M : WM_FIT);
    constexpr int LDS_FL = STAGED && WM_PASS * WROWS * STAGE_LD > BASE_FL
                               ? WM_PASS * WROWS * STAGE_LD : BASE_FL;
    static_assert(LDS_FL * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WAVES_N;
    const int wn = wave % WAVES_N;
    const int gx = tiles_m, gy = tiles_n;
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % gy;
    const int tm = (L / gy) % gx;
    const int tz = L / (gx * gy);
    const int m0 = tm * BM;
    const int n0 = tn * BN;
    const int ks0 = tz * ksteps_per_split;
    int ks1 = ks0 + ksteps_per_split;
    if (ks1 > ksteps_total) ks1 = ksteps_total;

    al.setup(m0, tid);
    bl.setup(n0, tid);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    f32x4 ra[AL::UNITS];
    f32x4 rb[BL::UNITS];
    auto stage = [&](float* s) {
        al.each_unit(ra, [&](int row, int c, f32x4 v) {
            const SplitBf16 p = split_bf16(v);
            store_unit<true, BM>(s, row, c, cat_bf16(p.h, p.m));
            store_unit<true, BM>(s + A_FL, row, c, cat_bf16(p.h, p.l));
        });
        bl.each_unit(rb, [&](int row, int c, f32x4 v) {
            const SplitBf16 p = split_bf16(v);
            float* t = s + 2 * A_FL;
            if constexpr (BP == 3) {
                store_unit<true, BN>(t, row, c, cat_bf16(p.h, p.h));
                store_unit<true, BN>(t + B_FL, row, c, cat_bf16(p.m, p.m));
                store_unit<true, BN>(t + 2 * B_FL, row, c, cat_bf16(p.l, p.h));
            } else {
                store_unit<true, BN>(t, row, c, cat_bf16(p.h, p.m));
                store_unit<true, BN>(t + B_FL, row, c, cat_bf16(p.l, p.h));
            }
        });
    };

    if (ks0 < ks1) {
        al.load(ks0, ra);
        bl.load(ks0, rb);
        stage(lds);
        if (ks0 + 1 < ks1) {
            al.load(ks0 + 1, ra);
            bl.load(ks0 + 1, rb);
        }
    }
    __syncthreads();
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    int cur = 0;
    for (int ks = ks0; ks < ks1; ++ks) {
        if (ks + 1 < ks1) {
            stage(lds + (cur ^ 1) * BUF);
            if (ks + 2 < ks1) {
                al.load(ks + 2, ra);
                bl.load(ks + 2, rb);
            }
        }
        const float* A = lds + cur * BUF;
        const float* B = A + 2 * A_FL;
        f32x4 b0[FN], b1[FN], b2[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int c0 = wn * 16 * FN + 16 * j;
            if constexpr (BP == 3) {
                b0[j] = read_frag<true, BN>(B, c0, lane);                 // [h|h]
                b1[j] = read_frag<true, BN>(B + B_FL, c0, lane);          // [m|m]
                b2[j] = read_frag<true, BN>(B + 2 * B_FL, c0, lane);      // [l|h]
            } else {
                b0[j] = read_frag<true, BN>(B, c0, lane);                 // [h|m]
                b1[j] = f32x4{b0[j].z, b0[j].w, b0[j].x, b0[j].y};        // [m|h]
                b2[j] = read_frag<true, BN>(B + B_FL, c0, lane);          // [l|h]
            }
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r0 = wm * 16 * FM + 16 * i;
            const f32x4 ahm = read_frag<true, BM>(A, r0, lane);
            const f32x4 ahl = read_frag<true, BM>(A + A_FL, r0, lane);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                f32x4 c = acc[i][j];
                c = mfma_x32(ahl, b2[j], c);       // ah bl + al bh: smallest terms first
                if constexpr (BP == 3) {
                    c = mfma_x32(ahm, b1[j], c);   // ah bm + am bm
                    c = mfma_x32(ahm, b0[j], c);   // ah bh + am bh
                } else {
                    c = mfma_x32(ahm, b1[j], c);   // ah bm + am bh
                    c = mfma_x32(ahm, b0[j], c);   // ah bh + am bm
                }
                acc[i][j] = c;
            }
        }
        __syncthreads();
        cur ^= 1;
    }

    if constexpr (STAGED) {
        static_assert(BN == EPI::NCOL, "staged epilogue needs the full row in one block");
        constexpr int PASSES = (WAVES_M + WM_PASS - 1) / WM_PASS;
#pragma unroll 1
        for (int pass = 0; pass < PASSES; ++pass) {
            __syncthreads();
            if (wm / WM_PASS == pass) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const int ml = (wm - pass * WM_PASS) * WROWS + 16 * i + 4 * (lane >> 4);
                        const int nl = wn * 16 * FN + 16 * j + (lane & 15);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr)
                            lds[(ml + rr) * STAGE_LD + nl] = epi.value(nl, acc[i][j][rr]);
                    }
            }
            __syncthreads();
            const int wm_hi = (pass + 1) * WM_PASS < WAVES_M ? (pass + 1) * WM_PASS : WAVES_M;
            epi.store_rows(lds, STAGE_LD, m0 + pass * WM_PASS * WROWS,
                           (wm_hi - pass * WM_PASS) * WROWS, tid, 64 * WAVES_M * WAVES_N);
        }
    } else if constexpr (HasPre<EPI>::value) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
            const int nb0 = n0 + wn * 16 * FN + (lane & 15);
            f32x4 pre[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) pre[j] = epi.pre4(m, nb0 + 16 * j, tz);
#pragma unroll
            for (int j = 0; j < FN; ++j) epi.apply4p(m, nb0 + 16 * j, tz, acc[i][j], pre[j]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
                const int n = n0 + wn * 16 * FN + 16 * j + (lane & 15);
                epi.apply4(m, n, tz, acc[i][j]);
            }
    }
}

}  // namespace flsim
