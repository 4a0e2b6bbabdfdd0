// PerformantNet1: conv1's weight gradient fused into conv2's data-gradient GEMM (models.py:14,29).
//
// conv2's data gradient produces dz1 = (dZ2 * W2^T) * (a1 > 0) over the 34 x 34 grid of conv1's
// output, 48 channels per pixel, and conv1's weight gradient is the only reader of dz1:
//     dW1[co][tap, ci] = sum over pixels p of dz1[p][co] * x0[p + tap][ci],  db1[co] = sum dz1[p][co]
// Written out, dz1 is 3.6 GB per 16,384-sample chunk, written by the data gradient and read back by
// the weight gradient.  Here each block keeps conv1's partial dW1 / db1 in MFMA
// accumulators instead: after a tile's dz1 rows are masked in LDS, the block multiplies them by the
// tile's conv1 input columns (27 taps x channels, a ones column for the bias), and at the end writes
// the sum of its tiles into its own row of conv1's weight / bias slabs.  dz1 never leaves the CU.
//
// The grid is persistent: one block per resident slot, each over a contiguous range of M-tiles (so
// a block's partial covers whole tiles and every slab row is written by one block).  The data
// gradient's main loop is gemm_direct_kernel's (gemm_direct.h), unchanged.  The fused product is an
// fp32 MFMA GEMM (16x16x4) of [48 channels] x [32 columns] over each tile's rows: 64 MFMAs per wave
// and tile on six of the eight waves, beside the data gradient's 648.
#pragma once
#include "net_kernels.h"

namespace flsim {

struct C1Fuse {
    const float* a1h;   // HM part of a1 (split.h, channel-slice-major): the ReLU mask of dz1
    const float* x0;    // conv1's input [S][32][32][4]
    float* slab;        // conv1's weight slab [Z][48][KP]
    float* bslab;       // conv1's bias slab [Z][48]
    int M;              // rows = S * 34 * 34
    int KP;             // conv1's packed row length: column (kh * 3 + kw) * 4 + ci
    int zinit;          // slab rows below this accumulate (+=), the rest are overwritten
    int tiles, tpb;     // M-tiles; tiles per block
};

// Waves 0-5 each own one 16 x 16 block of conv1's [48 channels] x [32 columns] partial (4
// accumulator registers; a partial spread over all 8 waves took 24 and cost the main loop its
// occupancy or spilled its address registers into scratch).
template <int FM, int FN, int WAVES, int KB, int DEPTH, class AD, class BL>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_dgrad2_wgrad1(AD ad, BL bl, C1Fuse c, int ksteps) {
    constexpr int BM = 16 * FM * WAVES;
    constexpr int BN = 16 * FN;
    static_assert(BN == 48 && BL::ROWS == BN && BL::KC, "conv1's 48 output channels in one tile");
    constexpr int NT = 64 * WAVES;
    constexpr int BFL = BL::FLOATS;
    constexpr int STG = KB * BFL;
    constexpr int WROWS = 16 * FM;
    constexpr int PR = 128;                     // rows per epilogue pass
    static_assert(BM % PR == 0 && PR % WROWS == 0, "whole waves per pass");
    constexpr int WM_PASS = PR / WROWS;
    constexpr int PASSES = BM / PR;
    constexpr int TLD = BN + 4;                 // dz1 tile row stride (floats)
    constexpr int XLD = 48;                     // x0-column tile row stride: 4 rows on 4 bank quarters
    constexpr int T_OFF = 0, X_OFF = PR * TLD, EPI_FL = X_OFF + PR * XLD;
    constexpr int LDS_FL = 2 * STG > EPI_FL ? 2 * STG : EPI_FL;
    static_assert(WAVES >= 6, "six partial blocks, one per wave");
    static_assert(LDS_FL * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int t0 = (int)blockIdx.x * c.tpb;
    const int t1 = t0 + c.tpb < c.tiles ? t0 + c.tpb : c.tiles;

    bl.setup(0, tid);
    const int pi = wave >> 1, pj = wave & 1;    // this wave's partial block (waves 0-5)
    f32x4 cacc = zero4();
    if constexpr (WAVES == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }

    constexpr int R = DEPTH + 1;
    static_assert(KB % R == 0, "the A register ring index must be static");
    const int nst = ksteps / KB;
    for (int t = t0; t < t1; ++t) {
        const int m0 = t * BM;
        ad.setup(m0 + wave * WROWS, lane);
        f32x4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = zero4();
        // ---- conv2's data gradient: gemm_direct_kernel's main loop ----
        f32x4 ra[R][FM];
        f32x4 rb[BL::UNITS];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) ad.load(d, ra[d]);
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            bl.load(kk, rb);
            bl.store(lds + kk * BFL, rb);
        }
        __syncthreads();
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
                f32x4 bf[FN];
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    bf[j] = read_frag<true, BN>(Bs + kk * BFL, 16 * j, lane);
#pragma unroll
                for (int kq = 0; kq < 4; ++kq)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = mfma16(ra[kk % R][i][kq], bf[j][kq], acc[i][j]);
                __builtin_amdgcn_sched_barrier(0);
            }
            bl.store(Bn + (KB - 1) * BFL, rb);
            __syncthreads();
        }
        // ---- epilogue: dz1 rows masked in LDS, times conv1's input columns ----
        // Per pass: the pass's global loads (mask h parts, x0 values) go out first, under the
        // accumulator writes and the barrier; the main loop's last barrier already freed the LDS
        // for pass 0.  The partial product runs as four independent MFMA chains (16 x 16 x 4 f32:
        // a dependent chain waits out each MFMA's latency), summed into cacc at the pass end.
#pragma unroll 1
        for (int pass = 0; pass < PASSES; ++pass) {
            float* T = lds + T_OFF;
            float* X = lds + X_OFF;
            const int mp = m0 + pass * PR;
            constexpr int MU = PR * 12 / NT, XU = PR * 32 / NT;
            static_assert(PR * 12 % NT == 0 && PR * 32 % NT == 0, "whole units per thread");
            f32x2 hv[MU];
            float xv[XU];
#pragma unroll
            for (int it = 0; it < MU; ++it) {
                const int q = tid + it * NT, r = q / 12, cu = q - r * 12;
                hv[it] = mp + r < c.M ? reinterpret_cast<const f32x2*>(c.a1h)[
                                            2 * xs_unit<48, 1156, true>((unsigned)(mp + r), cu)]
                                      : f32x2{0.f, 0.f};
            }
#pragma unroll
            for (int it = 0; it < XU; ++it) {
                const int q = tid + it * NT, r = q >> 5, k = q & 31;
                const int m = mp + r;
                float v = 0.f;
                if (m < c.M) {
                    if (k < 27) {
                        const int n = m / 1156, rem = m - n * 1156;
                        const int oh = rem / 34, ow = rem - oh * 34;
                        const int tap = k / 3, ci = k - 3 * tap;
                        const int ih = oh + tap / 3 - 2, iw = ow + tap % 3 - 2;
                        if ((unsigned)ih < 32u && (unsigned)iw < 32u)
                            v = c.x0[((long)n * 1024 + ih * 32 + iw) * 4 + ci];
                    } else if (k == 27) {
                        v = 1.f;                     // the bias column
                    }
                }
                xv[it] = v;
            }
            if (pass > 0) __syncthreads();           // the previous pass's MFMAs read T, X
            if (wave / WM_PASS == pass) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        const int ml = (wave - pass * WM_PASS) * WROWS + 16 * i + 4 * (lane >> 4);
                        const int nl = 16 * j + (lane & 15);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) T[(ml + rr) * TLD + nl] = acc[i][j][rr];
                    }
            }
#pragma unroll
            for (int it = 0; it < XU; ++it) {
                const int q = tid + it * NT;
                X[(q >> 5) * XLD + (q & 31)] = xv[it];
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it < MU; ++it) {
                const int q = tid + it * NT, r = q / 12, cu = q - r * 12;
                f32x4* p = reinterpret_cast<f32x4*>(T + r * TLD + 4 * cu);
                *p = mask4(*p, xs_pos4(hv[it]));     // rows past M: h = 0, masked to zero
            }
            __syncthreads();
            // channels [16 pi, +16) x columns [16 pj, +16) over the pass's rows, 4 rows per MFMA
            if (wave < 6) {
                f32x4 ch[4] = {zero4(), zero4(), zero4(), zero4()};
#pragma unroll
                for (int s = 0; s < PR / 4; ++s) {
                    const int r = 4 * s + (lane >> 4);
                    ch[s & 3] = mfma16(T[r * TLD + 16 * pi + (lane & 15)],
                                       X[r * XLD + 16 * pj + (lane & 15)], ch[s & 3]);
                }
                cacc += (ch[0] + ch[1]) + (ch[2] + ch[3]);
            }
        }
        __syncthreads();                         // the next tile's B stage reuses this LDS
    }
    // ---- the block's partial: one slab row, each wave its block (column 27: the bias) ----
    if (wave < 6) {
        const int z = (int)blockIdx.x;
        const int k = 16 * pj + (lane & 15);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int co = 16 * pi + 4 * (lane >> 4) + rr;
            float* dst = k < 27 ? c.slab + ((long)z * 48 + co) * c.KP + (k / 3) * 4 + k % 3
                                : c.bslab + (long)z * 48 + co;
            if (k > 27) continue;
            if (z < c.zinit) *dst += cacc[rr];
            else *dst = cacc[rr];
        }
    }
}

// conv2's data gradient (dZ2 over conv2's 36 x 36 input grid, flipped packed weights [48][KP2])
// with conv1's weight / bias gradient into their slabs; FM / FMS: rows per wave of the large- /
// small-chunk tiles (bit-identical data-gradient sums either way).  *zused = the slab rows written.
template <int FM, int FMS, int FN, int WAVES, int KB, int DEPTH>
static int conv2_dgrad_conv1_wgrad(const float* dz2, int S, const float* Wpk, int KP2,
                                   const float* a1h, const float* x0, float* slab, float* bslab,
                                   int Z, int KP1, int zinit, int* zused, hipStream_t st, int kid) {
    if constexpr (FMS != FM) {
        if (S <= small_chunk_samples())
            return conv2_dgrad_conv1_wgrad<FMS, FMS, FN, WAVES, KB, DEPTH>(
                dz2, S, Wpk, KP2, a1h, x0, slab, bslab, Z, KP1, zinit, zused, st, kid);
    }
    using AD = Im2colDirect<36, 36, 48, 0, FM, false, 0>;
    using BL = RowsKCStage<16 * FN, 64 * WAVES>;
    constexpr int BM = 16 * FM * WAVES;
    FLSIM_REQUIRE((KP2 / GK) % KB == 0, "direct GEMM: %d k-steps not a multiple of %d", KP2 / GK,
                  KB);
    FLSIM_REQUIRE(KP1 >= 36, "conv1 packed row of %d columns", KP1);
    AD ad;
    ad.X = dz2;
    ad.M = S * AD::ROWS_PER_IMG;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP2;
    bl.NR = 48;
    auto kfn = k_dgrad2_wgrad1<FM, FN, WAVES, KB, DEPTH, AD, BL>;
    static const int cap = resident_blocks((const void*)kfn, 64 * WAVES);
    const int tiles = ceil_div(ad.M, BM);
    int nb = cap > 0 ? cap : 1024;
    if (nb > Z) nb = Z;
    const int tpb = ceil_div(tiles, nb);
    const int nblk = ceil_div(tiles, tpb);
    C1Fuse c{a1h, x0, slab, bslab, ad.M, KP1, zinit, tiles, tpb};
    if (zused) *zused = nblk;
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL(kfn, dim3(nblk), dim3(64 * WAVES), 0, st, ps.start, ps.stop, 0, ad, bl, c,
                          KP2 / GK);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, kid, 2.0 * ad.M * 48 * KP2 + 2.0 * ad.M * 48 * 27);
}

}  // namespace flsim
