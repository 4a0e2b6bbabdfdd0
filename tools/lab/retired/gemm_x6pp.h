// Lab variant of gemm_x6_kernel (development tool, not part of libflsim.so): where the next
// k-step's LDS stores and global loads sit in the main loop.  MODE 0: first (the product's
// order); 1: after the first A fragment's MFMAs; 2: after half of them; 3: first, with the loop
// body branch-free (one basic block: the product's `if (ks + 1 < ks1)` around the staging splits
// the staging VALU and the MFMAs into separate blocks); 4: 3 plus sched_group_barrier
// interleaving (one MFMA, two VALU, every other MFMA one LDS store); 5: per MFMA V VALU, an LDS
// store every W, a global load every L, an LDS read every R MFMAs (template parameters).  A fragments are read one ahead.  Fresh accumulation off (the product's
// default level).
#pragma once
#include "gemm_x6.h"

namespace flsim {

template <int MODE, int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI,
          int V = 3, int W = 2, int LG = 4, int R = 0>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_x6pp_kernel(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
               int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(AL::ROWS == BM && BL::ROWS == BN, "loader rows != tile");
    using TA = X6Tile<AL::KC, BM, true, 4 * WAVES_M * WAVES_N>;
    using TB = X6Tile<BL::KC, BN, false, 4 * WAVES_M * WAVES_N>;
    static_assert(!EPI::ASUM || !AL::KC, "ASUM needs a k-major A tile");
    constexpr bool AMF = EPI::ASUM && AsumMfma<EPI>::value;
    constexpr int BUF = TA::FL + TB::FL;
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

    float asum = 0.f;
    f32x4 bacc[AMF ? FM : 1];
#pragma unroll
    for (int i = 0; i < (AMF ? FM : 1); ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool bwave = AMF && tn == 0 && wn == 0;     // wave-uniform
    typename AL::Unit ra[AL::UNITS];
    typename BL::Unit rb[BL::UNITS];
    auto stage = [&](float* s) {
        al.each_unit(ra, [&](int a, int c, const auto& v, bool ok) { TA::store(s, a, c, v, ok); });
        bl.each_unit(rb, [&](int a, int c, const auto& v, bool ok) {
            TB::store(s + TA::FL, a, c, v, ok);
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
    // The main loop in two compiled forms, chosen per wave before it starts: with the bias column
    // sum (ASUM: the waves that hold it in the tn = 0 blocks) and without.  With the sum behind a
    // branch inside the loop the weight gradients ran 2-9 % slower than with no sum at all
    // (conv6 9.76 against 8.93 ms, profiles/r04/r04h/lab_wg.txt); chosen per wave and taken on the
    // MFMA (AsumMfma) they run within 1.3 % of that, or faster (profiles/r04/r04i/lab_wg.txt)
    int cur = 0;
    auto main_loop = [&](auto with_sum) {
        constexpr bool WS = decltype(with_sum)::value;
        for (int ks = ks0; ks < ks1; ++ks) {
            const bool more = ks + 1 < ks1;
            auto next = [&]() {
                if constexpr (MODE >= 3) {
                    // branch-free: the last k-step stages into the buffer nobody reads again and
                    // the loads past the split re-read its last k-step
                    stage(lds + (cur ^ 1) * BUF);
                    const int kl = ks + 2 < ks1 ? ks + 2 : ks1 - 1;
                    al.load(kl, ra);
                    bl.load(kl, rb);
                } else if (more) {
                    stage(lds + (cur ^ 1) * BUF);
                    if (ks + 2 < ks1) {
                        al.load(ks + 2, ra);
                        bl.load(ks + 2, rb);
                    }
                }
            };
            if constexpr (MODE == 0 || MODE >= 3) next();
            const float* A = lds + cur * BUF;
            const float* B = A + TA::FL;
            if constexpr (WS && !AMF) {
                if (tid < BM) asum += TA::colsum(A, tid);
            }
            typename TB::Frag bf[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bf[j] = TB::frag(B, wn * 16 * FN + 16 * j, lane);
            typename TA::Frag af = TA::frag(A, wm * 16 * FM, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                typename TA::Frag an;
                if (i + 1 < FM) an = TA::frag(A, wm * 16 * FM + 16 * (i + 1), lane);
                if constexpr (WS && AMF) {
                    bacc[i] = mfma_x32(af.x1, bf16_ones(false, true), bacc[i]);   // l
                    bacc[i] = mfma_x32(af.x0, bf16_ones(true, true), bacc[i]);    // h + m
                }
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = x6_step<false>(acc[i][j], af.x0, af.x1, bf[j].x0, bf[j].x1, bf[j].x2);
                if constexpr (MODE == 1) {
                    if (i == 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        next();
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if constexpr (MODE == 2) {
                    if (i == (FM - 1) / 2) {
                        __builtin_amdgcn_sched_barrier(0);
                        next();
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                if (i + 1 < FM) af = an;
            }
            if constexpr (MODE == 4) {
                // interleave: one MFMA, two VALU, and every other MFMA one LDS store
#pragma unroll
                for (int n = 0; n < 3 * FM * FN; ++n) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                    if (n % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                }
            }
            if constexpr (MODE == 5) {
                // per MFMA: V VALU; every W-th MFMA one LDS store, every L-th one global load,
                // every R-th one LDS read (R = 0: LDS reads unconstrained)
#pragma unroll
                for (int n = 0; n < 3 * FM * FN; ++n) {
                    if constexpr (R > 0) {
                        if (n % R == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
                    if (n % W == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    if (n % LG == 1 % LG) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                }
            }
            __syncthreads();
            cur ^= 1;
        }
    };
    bool sum_wave = false;
    if constexpr (AMF) sum_wave = bwave;
    else if constexpr (EPI::ASUM) sum_wave = tn == 0 && wave * 64 < BM;
    if (sum_wave) main_loop(std::true_type{});
    else main_loop(std::false_type{});

    if constexpr (AMF) {
        // every column of the ones product is the row sum: lanes of column 0 store it
        if (bwave && (lane & 15) == 0) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    epi.asum(m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4) + rr, tz, bacc[i][rr]);
        }
    } else if constexpr (EPI::ASUM) {
        if (tn == 0 && tid < BM) epi.asum(m0 + tid, tz, asum);
    }
    if constexpr (STAGED) {
        static_assert(BN == EPI::NCOL || (IsPartial<EPI>::value && EPI::NCOL % BN == 0),
                      "staged epilogue needs the full row in one block");
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
            staged_store(epi, lds, STAGE_LD, m0 + pass * WM_PASS * WROWS,
                         (wm_hi - pass * WM_PASS) * WROWS, n0, BN, tid, 64 * WAVES_M * WAVES_N);
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
