// Experimental variants of flsim::gemm_kernel (lab only).
#pragma once
#include "loaders.h"

namespace flsim {

// KSUB 16-deep sub-steps per barrier (LDS stage = KSUB sub-tiles), PRIO: s_setprio 1 around the
// MFMA block.
template <int FM, int FN, int WAVES_M, int WAVES_N, int KSUB, int PRIO, int MINW, class AL,
          class BL, class EPI, int MODE = 0>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, MINW)
gemm_kernel_v(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
              int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    constexpr int A_FL = tile_floats<AL::KC, BM>();
    constexpr int B_FL = tile_floats<BL::KC, BN>();
    constexpr int SUB = A_FL + B_FL;
    constexpr int BUF = KSUB * SUB;
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF];

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
    f32x4 ra[KSUB][AL::UNITS];
    f32x4 rb[KSUB][BL::UNITS];

    // stage = KSUB consecutive k-steps (the last stage may be partial: missing sub-steps load
    // as whatever the loader gives for ks >= ks1 -- so guard them)
    auto load_stage = [&](int ks) {
#pragma unroll
        for (int s = 0; s < KSUB; ++s) {
            if (ks + s < ks1) {
                al.load(ks + s, ra[s]);
                bl.load(ks + s, rb[s]);
            }
        }
    };
    auto store_stage = [&](float* base, int ks) {
#pragma unroll
        for (int s = 0; s < KSUB; ++s) {
            if (ks + s < ks1) {
                al.store(base + s * SUB, ra[s]);
                bl.store(base + s * SUB + A_FL, rb[s]);
            }
        }
    };
    if (ks0 < ks1) {
        load_stage(ks0);
        store_stage(lds, ks0);
    }
    __syncthreads();
    int cur = 0;
    for (int ks = ks0; ks < ks1; ks += KSUB) {
        const bool more = ks + KSUB < ks1;
        if (MODE == 0 && more) load_stage(ks + KSUB);
        if (MODE == 3 && more) load_stage(ks0);
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < KSUB; ++s) {
            if (ks + s < ks1) {
                const float* A = lds + cur * BUF + s * SUB;
                const float* B = A + A_FL;
                if constexpr (EPI::ASUM) {
                    if (tn == 0 && tid < BM) {
#pragma unroll
                        for (int k = 0; k < GK; ++k) asum += A[k * KMTile<BM>::STRIDE + tid];
                    }
                }
                f32x4 af[FM], bf[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) af[i] = read_frag<AL::KC, BM>(A, wm * 16 * FM + 16 * i, lane);
#pragma unroll
                for (int j = 0; j < FN; ++j) bf[j] = read_frag<BL::KC, BN>(B, wn * 16 * FN + 16 * j, lane);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
            }
        }
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        if ((MODE == 0 || MODE == 3) && more) store_stage(lds + (cur ^ 1) * BUF, ks + KSUB);
        if (MODE != 2) __syncthreads();
        if (MODE == 0 || MODE == 3) cur ^= 1;
    }

    if constexpr (EPI::ASUM) {
        if (tn == 0 && tid < BM) epi.asum(m0 + tid, tz, asum);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
            const int n = n0 + wn * 16 * FN + 16 * j + (lane & 15);
            epi.apply4(m, n, tz, acc[i][j]);
        }
}

}  // namespace flsim
