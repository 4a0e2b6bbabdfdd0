// Direct-A split-bf16 GEMM for the convolutions' forward and data-gradient passes (gfx950).
//
// The operands arrive in the split form (split.h): every activation / dZ tensor is stored by its
// producer as HM + L parts, and the packed weights likewise, once per epoch.  So nothing is split
// in the GEMM.  As in gemm_direct.h, each wave owns 16*FM rows of the block tile and loads its A
// fragments straight from memory into registers, DEPTH k-steps ahead: lane l of the 16x16x32 bf16
// MFMA holds row (l & 15), k slots 8(l >> 4) .. +7 = the [h|m] unit of four consecutive input
// channels of one pixel (one 16-B load at the fp32 tensor's own byte offset), and [h|l] takes two
// dwords of the L unit (one 8-B load).  No LDS and no barrier for A.  Only B (the block's BN packed
// weight columns) goes through LDS, KB k-steps per stage, planes [h|m] and [l|h] ([m|h] too when
// NPLB = 3), each laid out like the fp32 KC tile.
//
// Per accumulator the MFMA sequence (k ascending; per k-step A[h|l] x B[l|h], A[h|m] x B[m|h],
// A[h|m] x B[h|m]) is gemm_x6_kernel's, and the parts are the same RNE split, so the results are
// bit-identical to gemm_x6_kernel over the fp32 operands.
#pragma once
#include "gemm_direct.h"
#include "gemm_x6.h"

namespace flsim {

// B staging for gemm_dx6_kernel: rows [n0, n0 + ROWS) of a row-major [NR][ld] matrix in the split
// form, one 16-deep k-step per load / store.  Per k-step the LDS holds NPL planes of KCTile<ROWS>
// (plane 0 [h|m], plane 1 [l|h], plane 2 [m|h]) and one spare 16-B chunk that takes the stores of
// units past the tile (rows >= NR read as zeros through the buffer bound).
template <int TR, int NT, int NPL>
struct RowsKCStageXs {
    using Unit = XsUnit;
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    static constexpr int PLANE = KCTile<ROWS>::FLOATS;
    static constexpr int SPARE = NPL * PLANE;
    static constexpr int FLOATS = NPL * PLANE + 4;
    static_assert(NPL == 2 || NPL == 3, "");
    const float* P;
    const float* PL;
    long ld;
    int NR;
    unsigned rowb[UNITS];
    int dst[UNITS];            // LDS float offset of the unit in plane 0, -1 for a surplus unit
    XsSrc buf;
    __device__ void setup(int r0, int tid) {
        buf.init(P, PL, (unsigned long)NR * ld * 4);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u0 = tid + j * NT;
            const bool real = u0 < TOTAL;
            const int u = real ? u0 : u0 % TOTAL;
            const int r = u >> 2, q = u & 3;
            rowb[j] = r0 + r < NR ? (unsigned)(((long)(r0 + r) * ld + 4 * q) * 4) : BUF_OOB;
            dst[j] = real ? KCTile<ROWS>::chunk_off(r, q) : -1;
        }
    }
    __device__ void load(int ks, Unit (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            r[j] = buf.ld(rowb[j] == BUF_OOB ? BUF_OOB : rowb[j] + (unsigned)(ks * GK * 4));
    }
    __device__ void store(float* lds, const Unit (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const bool real = TOTAL % NT == 0 || dst[j] >= 0;
            *reinterpret_cast<f32x4*>(lds + (real ? dst[j] : SPARE)) = r[j].hm;
            *reinterpret_cast<f32x4*>(lds + (real ? dst[j] + PLANE : SPARE)) = xs_lh(r[j]);
            if constexpr (NPL == 3)
                *reinterpret_cast<f32x4*>(lds + (real ? dst[j] + 2 * PLANE : SPARE)) =
                    f32x4{r[j].hm.z, r[j].hm.w, r[j].hm.x, r[j].hm.y};
        }
    }
};

// Block = WAVES waves stacked along M (each 16*FM rows) x all BN = 16*FN columns of its n-tile.
template <int FM, int FN, int WAVES, int KB, int DEPTH, class AD, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES)
gemm_dx6_kernel(AD ad, BL bl, EPI epi, int ksteps, int tiles_m, int tiles_n) {
    constexpr int BM = 16 * FM * WAVES;
    constexpr int BN = 16 * FN;
    static_assert(BL::ROWS == BN && BL::KC, "B loader: k-contiguous tile of BN rows");
    constexpr int BFL = BL::FLOATS;             // one k-step of B (+ the stager's spare chunk)
    constexpr int PLANE = BL::PLANE;
    constexpr int STG = KB * BFL;               // one stage
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int STAGE_LD = BN + 4;
    constexpr int BASE_FL = 2 * STG;
    constexpr int WROWS = 16 * FM;
    constexpr int WM_FIT = (BASE_FL > 8192 ? BASE_FL : 8192) / (WROWS * STAGE_LD);
    constexpr int WM_PASS = WM_FIT < 1 ? 1 : (WM_FIT > WAVES ? WAVES : WM_FIT);
    constexpr int LDS_FL = STAGED && WM_PASS * WROWS * STAGE_LD > BASE_FL
                               ? WM_PASS * WROWS * STAGE_LD : BASE_FL;
    static_assert(LDS_FL * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    // XCD-aware order as gemm_kernel: each XCD takes a contiguous range of tiles, n fastest
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % tiles_n;
    const int tm = L / tiles_n;
    const int m0 = tm * BM;
    const int n0 = tn * BN;

    ad.setup(m0 + wave * WROWS, lane);
    bl.setup(n0, tid);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // the A register ring and the unconditional loads past the end of K: as gemm_direct_kernel
    constexpr int R = DEPTH + 1;
    static_assert(KB % R == 0, "the A register ring index must be static");
    XsUnit ra[R][FM];
    typename BL::Unit rb[BL::UNITS];
    const int nst = ksteps / KB;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) ad.load(d, ra[d]);
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
        bl.load(kk, rb);
        bl.store(lds + kk * BFL, rb);
    }
    __syncthreads();
    if constexpr (WAVES == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    for (int s = 0; s < nst; ++s) {
        const float* Bs = lds + (s & 1) * STG;
        float* Bn = lds + ((s + 1) & 1) * STG;
        const int kn = (s + 1) * KB;
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            const int ks = s * KB + kk;
            if (kk > 0) bl.store(Bn + (kk - 1) * BFL, rb);
            bl.load(kn + kk, rb);
            ad.load(ks + DEPTH, ra[(kk + DEPTH) % R]);
            __builtin_amdgcn_sched_barrier(0);
            const float* Bk = Bs + kk * BFL;
            f32x4 a0[FM], a1[FM];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                a0[i] = ra[kk % R][i].hm;                 // [h|m]
                a1[i] = xs_hl(ra[kk % R][i]);             // [h|l]
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const f32x4 x0 = read_frag<true, BN>(Bk, 16 * j, lane);              // [h|m]
                const f32x4 x2 = read_frag<true, BN>(Bk + PLANE, 16 * j, lane);      // [l|h]
                f32x4 x1;                                                            // [m|h]
                if constexpr (BFL >= 3 * PLANE)
                    x1 = read_frag<true, BN>(Bk + 2 * PLANE, 16 * j, lane);
                else
                    x1 = f32x4{x0.z, x0.w, x0.x, x0.y};
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    acc[i][j] = x6_step<x6_fresh(true)>(acc[i][j], a0[i], a1[i], x0, x1, x2);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        bl.store(Bn + (KB - 1) * BFL, rb);
        __syncthreads();
    }

    if constexpr (STAGED) {
        static_assert(BN == EPI::NCOL || (IsPartial<EPI>::value && EPI::NCOL % BN == 0),
                      "staged epilogue needs the full row in one block");
        constexpr int PASSES = (WAVES + WM_PASS - 1) / WM_PASS;
#pragma unroll 1
        for (int pass = 0; pass < PASSES; ++pass) {
            __syncthreads();
            if (wave / WM_PASS == pass) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const int ml = (wave - pass * WM_PASS) * WROWS + 16 * i + 4 * (lane >> 4);
                        const int nl = 16 * j + (lane & 15);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr)
                            lds[(ml + rr) * STAGE_LD + nl] = epi.value(nl, acc[i][j][rr]);
                    }
            }
            __syncthreads();
            const int w_hi = (pass + 1) * WM_PASS < WAVES ? (pass + 1) * WM_PASS : WAVES;
            staged_store(epi, lds, STAGE_LD, m0 + pass * WM_PASS * WROWS,
                         (w_hi - pass * WM_PASS) * WROWS, n0, BN, tid, 64 * WAVES);
        }
    } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int m = m0 + wave * WROWS + 16 * i + 4 * (lane >> 4);
                const int n = n0 + 16 * j + (lane & 15);
                epi.apply4(m, n, 0, acc[i][j]);
            }
    }
}

}  // namespace flsim
