// Lab: GEMM with LDS-DMA staging (global_load_lds_dwordx4) for KC x KC operands.
#pragma once
#include "loaders.h"

namespace flsim {

__device__ __forceinline__ void glds16(const float* src, float* lds_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// logical 16-B chunk a lane fetches so that the lane-linear LDS image is the XOR-swizzled KC
// tile: lane l lands at row 16p + l/4, slot l%4, which holds chunk (l%4) ^ kc_swz(row)
__device__ __forceinline__ int glds_chunk(int lane) { return (lane & 3) ^ ((4 - (lane >> 4)) & 3); }

template <int IH, int IW, int CI, int PAD, int TR, int NW, bool WIN = false>
struct Im2colGlds {
    static constexpr int ROWS = TR;
    static constexpr int OH = IH + 2 * PAD - 2, OW = IW + 2 * PAD - 2;
    static constexpr int PH = OH / 2, PW = OW / 2;
    static constexpr int ROWS_PER_IMG = WIN ? 4 * PH * PW : OH * OW;
    static constexpr int PIECES = TR / 16;
    static constexpr int PPW = (PIECES + NW - 1) / NW;
    static_assert(TR % 16 == 0 && CI % 16 == 0, "");
    const float* X;
    const float* zp;
    int M;
    long base[PPW];
    short mask[PPW];
    int c4;
    __device__ void setup(int m0, int wave, int lane) {
        c4 = 4 * glds_chunk(lane);
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
            const int p = wave + j * NW;
            const int m = m0 + 16 * p + (lane >> 2);
            base[j] = 0;
            mask[j] = 0;
            if (p < PIECES && m < M) {
                const int nimg = m / ROWS_PER_IMG;
                const int rem = m - nimg * ROWS_PER_IMG;
                int oh, ow;
                if constexpr (WIN) {
                    const int qq = rem >> 2;
                    const int ph = qq / PW;
                    oh = 2 * ph + ((rem >> 1) & 1);
                    ow = 2 * (qq - ph * PW) + (rem & 1);
                } else {
                    oh = rem / OW;
                    ow = rem - oh * OW;
                }
                base[j] = ((long)nimg * IH * IW + (long)(oh - PAD) * IW + (ow - PAD)) * CI + c4;
                int msk = 0;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int ih = oh + t / 3 - PAD, iw = ow + t % 3 - PAD;
                    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) msk |= 1 << t;
                }
                mask[j] = (short)msk;
            }
        }
    }
    __device__ void issue(int ks, float* tile, int wave) const {
        const int kk = ks * GK;
        const int khkw = kk / CI;
        const int ci0 = kk - khkw * CI;
        const int kh = khkw / 3;
        const long off = (long)(kh * IW + (khkw - 3 * kh)) * CI + ci0;
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
            const int p = wave + j * NW;
            if (p < PIECES) {
                const bool ok = khkw < 9 && ((mask[j] >> khkw) & 1);
                glds16(ok ? X + base[j] + off : zp, tile + 256 * p);
            }
        }
    }
};

template <int TR, int NW>
struct RowsGlds {
    static constexpr int ROWS = TR;
    static constexpr int PIECES = TR / 16;
    static constexpr int PPW = (PIECES + NW - 1) / NW;
    const float* P;
    const float* zp;
    long ld;
    int NR;
    const float* rowp[PPW];
    __device__ void setup(int r0, int wave, int lane) {
        const int c4 = 4 * glds_chunk(lane);
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
            const int p = wave + j * NW;
            const int r = r0 + 16 * p + (lane >> 2);
            rowp[j] = (p < PIECES && r < NR) ? P + (long)r * ld + c4 : nullptr;
        }
    }
    __device__ void issue(int ks, float* tile, int wave) const {
#pragma unroll
        for (int j = 0; j < PPW; ++j) {
            const int p = wave + j * NW;
            if (p < PIECES) glds16(rowp[j] ? rowp[j] + ks * GK : zp, tile + 256 * p);
        }
    }
};

template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_glds(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m, int tiles_n) {
    constexpr int NW = WAVES_M * WAVES_N;
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(AL::ROWS == BM && BL::ROWS == BN, "");
    constexpr int A_FL = BM * GK, B_FL = BN * GK, BUF = A_FL + B_FL;
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int gx = tiles_m, gy = tiles_n;
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % gy, tm = (L / gy) % gx, tz = L / (gx * gy);
    const int m0 = tm * BM, n0 = tn * BN;
    const int ks0 = tz * ksteps_per_split;
    int ks1 = ks0 + ksteps_per_split;
    if (ks1 > ksteps_total) ks1 = ksteps_total;
    al.setup(m0, wave, lane);
    bl.setup(n0, wave, lane);
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ks0 < ks1) {
        al.issue(ks0, lds, wave);
        bl.issue(ks0, lds + A_FL, wave);
    }
    __syncthreads();
    int cur = 0;
    for (int ks = ks0; ks < ks1; ++ks) {
        if (ks + 1 < ks1) {
            al.issue(ks + 1, lds + (cur ^ 1) * BUF, wave);
            bl.issue(ks + 1, lds + (cur ^ 1) * BUF + A_FL, wave);
        }
        const float* A = lds + cur * BUF;
        const float* B = A + A_FL;
        f32x4 af[FM], bf[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = read_frag<true, BM>(A, wm * 16 * FM + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = read_frag<true, BN>(B, wn * 16 * FN + 16 * j, lane);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
        __syncthreads();
        cur ^= 1;
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
