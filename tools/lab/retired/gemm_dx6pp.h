// Lab variant of gemm_dx6_kernel (development tool, not part of libflsim.so): the direct-A
// split-bf16 forward with its per-k-step scheduling fences replaced.  MODE 0: the product's
// fences; 1: no fences (the compiler's order); 2: sched_group_barrier interleave (per MFMA: an
// LDS read every 2nd, a global load every 4th, an LDS store every 4th, one VALU); 3: LDS reads in
// pairs every 3rd MFMA, loads / stores every 6th, two VALU.  Fresh accumulation off (the
// product's default level).
#pragma once
#include "gemm_dx6.h"

namespace flsim {

// Block = WAVES waves stacked along M (each 16*FM rows) x all BN = 16*FN columns of its n-tile.
template <int MODE, int FM, int FN, int WAVES, int KB, int DEPTH, class AD, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES)
gemm_dx6pp_kernel(AD ad, BL bl, EPI epi, int ksteps, int tiles_m, int tiles_n) {
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
            if constexpr (MODE == 0) __builtin_amdgcn_sched_barrier(0);
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
                    acc[i][j] = x6_step<false>(acc[i][j], a0[i], a1[i], x0, x1, x2);
                }
            }
            if constexpr (MODE == 2) {
#pragma unroll
                for (int n = 0; n < 3 * FM * FN; ++n) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (n % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    if (n % 4 == 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                    if (n % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
                }
            }
            if constexpr (MODE == 3) {
#pragma unroll
                for (int n = 0; n < 3 * FM * FN; ++n) {
                    if (n % 3 == 0) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (n % 6 == 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                    if (n % 6 == 4) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                }
            }
            if constexpr (MODE == 0) __builtin_amdgcn_sched_barrier(0);
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
