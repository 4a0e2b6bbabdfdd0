// fp32 MFMA GEMM core for gfx950 (v_mfma_f32_16x16x4_f32), LDS-tiled, register-staged
// double buffer (loads issued a full k-step ahead of their LDS write), one barrier per 16-deep
// K step.
//
// C[m][n] = sum_k A[m][k] * B[k][n]; each operand is produced by a Loader that knows the
// implicit-GEMM address math (im2col for convolutions, plain rows for the linear layers) and
// which LDS orientation it uses:
//   KC ("k-contiguous"): LDS tile [rows][16] (64-B rows, 16-B chunks XOR-swizzled so that the
//       ds_read_b128 fragment reads of 16 distinct rows are bank-conflict free)
//   KM ("k-major"):      LDS tile [16][rows + 4] (row stride = 4 mod 8 floats: the two 16-lane
//       halves of a ds_read_b32 land on disjoint banks)
//
// MFMA operand mapping (16x16x4 f32): lane l holds A[i = l&15][kslot = l>>4] and
// B[kslot = l>>4][j = l&15]. For one 16-deep K step a lane owns k = 4*(l>>4) + j, j = 0..3, and
// MFMA j consumes element j of that 4-vector, so A and B agree on which k each slot holds.
// C/D: col = l&15, row = 4*(l>>4) + reg.
#pragma once
#include <type_traits>

#include "common.h"

namespace flsim {

constexpr int GK = 16;  // K depth per LDS stage

__device__ __forceinline__ int kc_swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// byte-free helpers for LDS addressing (float units)
template <int ROWS>
struct KCTile {
    static constexpr int FLOATS = ROWS * GK;
    __device__ static inline int chunk_off(int row, int chunk) {
        return row * GK + 4 * (chunk ^ kc_swz(row));
    }
};
template <int ROWS>
struct KMTile {
    static constexpr int STRIDE = ROWS + 4;
    // one spare 16-B chunk after the tile: k-major loaders whose unit count does not divide the
    // block store their surplus units there instead of branching around the store (weight
    // gradients +0.5-1 %; the same for the k-contiguous tiles measured 1-5 % slower, r02f)
    static constexpr int DUMMY = GK * STRIDE;
    static constexpr int FLOATS = GK * STRIDE + 4;
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Read one operand fragment (16 rows x 4 k per lane) for rows [r0, r0+16).
template <bool KC, int ROWS>
__device__ __forceinline__ f32x4 read_frag(const float* lds, int r0, int lane) {
    if constexpr (KC) {
        const int row = r0 + (lane & 15);
        return *reinterpret_cast<const f32x4*>(lds + KCTile<ROWS>::chunk_off(row, lane >> 4));
    } else {
        constexpr int S = KMTile<ROWS>::STRIDE;
        const int col = r0 + (lane & 15);
        const int k0 = 4 * (lane >> 4);
        f32x4 v;
        v.x = lds[(k0 + 0) * S + col];
        v.y = lds[(k0 + 1) * S + col];
        v.z = lds[(k0 + 2) * S + col];
        v.w = lds[(k0 + 3) * S + col];
        return v;
    }
}

// Store a staged vec4 unit into the LDS tile.
//   KC: unit = (row, chunk) holding k = 4*chunk..4*chunk+3 of that row
//   KM: unit = (krow, col4) holding rows krow, cols 4*col4..4*col4+3
template <bool KC, int ROWS>
__device__ __forceinline__ void store_unit(float* lds, int a, int b, f32x4 v) {
    if constexpr (KC) {
        *reinterpret_cast<f32x4*>(lds + KCTile<ROWS>::chunk_off(a, b)) = v;
    } else {
        *reinterpret_cast<f32x4*>(lds + a * KMTile<ROWS>::STRIDE + 4 * b) = v;
    }
}

// k-major store of a unit that may be surplus (valid = false: the tile's spare chunk)
template <int ROWS>
__device__ __forceinline__ void store_km_or_spare(float* lds, bool valid, int a, int b, f32x4 v) {
    const int off = valid ? a * KMTile<ROWS>::STRIDE + 4 * b : KMTile<ROWS>::DUMMY;
    *reinterpret_cast<f32x4*>(lds + off) = v;
}

template <bool KC, int ROWS>
constexpr int tile_floats() {
    if constexpr (KC) return KCTile<ROWS>::FLOATS;
    else return KMTile<ROWS>::FLOATS;
}

// Loader concept (all device functions):
//   static constexpr bool KC; static constexpr int ROWS; static constexpr int UNITS;
//   void setup(int tile_row0, int tid)           -- per-thread precompute (rows fixed per tile)
//   void load(int kstep, f32x4 (&r)[UNITS])      -- global loads of the K step into registers
//   void store(float* lds, const f32x4 (&r)[UNITS])
//
// Epilogue concept:  void operator()(int m, int n, float v)   (m, n global; bounds checked inside)
//                    or apply4(m0, n, f32x4) for 4 consecutive rows of one column.

// Epilogues with STAGED = true write the block's whole BM x BN tile through LDS: the tile is
// BN = the full output row width, so its rows are one contiguous range of the output and the
// epilogue stores it with coalesced float4 writes instead of 64-byte column pieces.
template <class E, class = void>
struct IsStaged : std::false_type {};
template <class E>
struct IsStaged<E, std::void_t<decltype(E::STAGED)>> : std::bool_constant<E::STAGED> {};

// Staged epilogues with PARTIAL = true take a tile narrower than the output row: the kernels call
// store_rows(tile, ld, m0, bm, n0, bn, tid, nt) with the tile's columns [n0, n0 + bn)
template <class E, class = void>
struct IsPartial : std::false_type {};
template <class E>
struct IsPartial<E, std::void_t<decltype(E::PARTIAL)>> : std::bool_constant<E::PARTIAL> {};

// store the staged tile's rows through the epilogue (full rows, or the PARTIAL column range)
template <class EPI>
__device__ __forceinline__ void staged_store(const EPI& epi, const float* tile, int ld, int m0,
                                             int bm, int n0, int bn, int tid, int nt) {
    if constexpr (IsPartial<EPI>::value)
        epi.store_rows(tile, ld, m0, bm, n0, bn, tid, nt);
    else
        epi.store_rows(tile, ld, m0, bm, tid, nt);
}

// Epilogues with PRE = true load the per-fragment inputs of a fragment row first
// (pre4(m, n, z) -> f32x4), then store its fragments (apply4p(m, n, z, acc, pre))
template <class E, class = void>
struct HasPre : std::false_type {};
template <class E>
struct HasPre<E, std::void_t<decltype(E::PRE)>> : std::bool_constant<E::PRE> {};

// Blocks of one or two waves keep a single LDS buffer: their barriers span at most two waves, so
// the store -> barrier -> read order costs little, and half the LDS lifts the LDS-bound ones
// (PerformantNet1's conv2 / conv3 weight gradients, 48 x 48 of 1 wave, 96 x 48 of 2) from 3 to 5 and
// 4 to 5 waves per SIMD: conv2 7.37 -> 6.85 ms, conv3 4.43 -> 4.25 ms, the same arithmetic (A B A B,
// profiles/r06/ab_single_buf; vgg11 unchanged, 1238.6-1242.2 against 1240.6-1242.8).
// FLSIM_SINGLE_BUF = the largest block (waves) that runs single-buffered; lab override 0 / 1.
#ifndef FLSIM_SINGLE_BUF
#define FLSIM_SINGLE_BUF 2
#endif

template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_kernel(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
            int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(AL::ROWS == BM, "A loader rows != BM");
    static_assert(BL::ROWS == BN, "B loader rows != BN");
    constexpr int A_FL = tile_floats<AL::KC, BM>();
    constexpr int B_FL = tile_floats<BL::KC, BN>();
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int STAGE_LD = BN + 4;   // row stride 4 (mod 64) banks: the 4 row groups of a
                                       // wave's accumulator writes land on disjoint banks
    // the staged tile goes out in passes of WM_PASS wave-rows (16 FM rows each) that fit the
    // pipeline's own LDS footprint or 32 KB, whichever is larger (conv1: one pass in 26.6 KB,
    // 1.23 vs 1.33 ms for two; conv2 data-grad: two passes in the pipeline's 38 KB)
    constexpr bool SB = WAVES_M * WAVES_N <= FLSIM_SINGLE_BUF && !STAGED;
    constexpr int BASE_FL = (SB ? 1 : 2) * (A_FL + B_FL);
    constexpr int STAGE_BUDGET = BASE_FL > 8192 ? BASE_FL : 8192;
    constexpr int WROWS = 16 * FM;
    constexpr int WM_FIT = STAGE_BUDGET / (WROWS * STAGE_LD);
    constexpr int WM_PASS = WM_FIT < 1 ? 1 : (WM_FIT > WAVES_M ? WAVES_M : WM_FIT);
    constexpr int LDS_FL = STAGED && WM_PASS * WROWS * STAGE_LD > BASE_FL
                               ? WM_PASS * WROWS * STAGE_LD : BASE_FL;
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WAVES_N;
    const int wn = wave % WAVES_N;
    // 1-D grid.  Hardware deals block b to XCD (b % 8); remap so that each XCD gets a contiguous
    // range of logical tiles, ordered n-tile fastest, then m-tile, then split: the tiles that
    // share an operand panel (all n-tiles of an m-tile; all tiles of a K split) share one L2.
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
    f32x4 ra[AL::UNITS];
    f32x4 rb[BL::UNITS];
    constexpr int BUF = A_FL + B_FL;

    // Staging pipeline: the registers hold the NEXT tile's loads for a whole k-step.  At the top
    // of step ks (after the barrier that ended step ks-1, so nobody still reads that buffer) the
    // tile ks+1 loaded during step ks-1 is written to the other LDS buffer and the loads of tile
    // ks+2 are issued at once; the MFMAs of step ks then hide their latency.
    if (ks0 < ks1) {
        al.load(ks0, ra);
        bl.load(ks0, rb);
        if constexpr (!SB) {
            al.store(lds, ra);
            bl.store(lds + A_FL, rb);
            if (ks0 + 1 < ks1) {
                al.load(ks0 + 1, ra);
                bl.load(ks0 + 1, rb);
            }
        }
    }
    __syncthreads();
    // 8-wave blocks put waves w and w + 4 on one SIMD; the second-dispatched half loses every
    // issue arbitration, so it gets static priority (MI355X_MICROARCH.md "Two waves per SIMD",
    // item 4)
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    int cur = 0;
    // (the staging interleaved with the MFMAs in a branch-free body, as gemm_x6.h's X6_PP does
    // for the split forwards, made conv3's data gradient 3 % slower here and left VGG-11's fp32
    // data gradients unchanged, profiles/r05/ab/core_interleave.txt: removed)
    for (int ks = ks0; ks < ks1; ++ks) {
        if constexpr (SB) {
            al.store(lds, ra);
            bl.store(lds + A_FL, rb);
            if (ks + 1 < ks1) {
                al.load(ks + 1, ra);
                bl.load(ks + 1, rb);
            }
            __syncthreads();
        } else if (ks + 1 < ks1) {
            al.store(lds + (cur ^ 1) * BUF, ra);
            bl.store(lds + (cur ^ 1) * BUF + A_FL, rb);
            if (ks + 2 < ks1) {
                al.load(ks + 2, ra);
                bl.load(ks + 2, rb);
            }
        }
        const float* A = lds + (SB ? 0 : cur * BUF);
        const float* B = A + A_FL;
        if constexpr (EPI::ASUM) {
            // bias gradient fused into the weight gradient: column sums of the KM dZ tile
            // (rows = reduction index), accumulated by the n-tile-0 blocks in K order
            static_assert(!AL::KC, "ASUM needs a k-major A tile");
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
        __syncthreads();
        cur ^= 1;
    }

    if constexpr (EPI::ASUM) {
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
                        for (int r = 0; r < 4; ++r)
                            lds[(ml + r) * STAGE_LD + nl] = epi.value(nl, acc[i][j][r]);
                    }
            }
            __syncthreads();
            const int wm_hi = (pass + 1) * WM_PASS < WAVES_M ? (pass + 1) * WM_PASS : WAVES_M;
            staged_store(epi, lds, STAGE_LD, m0 + pass * WM_PASS * WROWS,
                         (wm_hi - pass * WM_PASS) * WROWS, n0, BN, tid, 64 * WAVES_M * WAVES_N);
        }
    } else if constexpr (HasPre<EPI>::value) {
        // one fragment row at a time: its FN fragments' inputs are loaded before any is stored
        // (FN round trips become one; FN * 4 extra registers, not FM * FN * 4)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
            const int nb = n0 + wn * 16 * FN + (lane & 15);
            f32x4 pre[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) pre[j] = epi.pre4(m, nb + 16 * j, tz);
#pragma unroll
            for (int j = 0; j < FN; ++j) epi.apply4p(m, nb + 16 * j, tz, acc[i][j], pre[j]);
        }
    } else {
        // epilogue: lane holds rows 4*(lane>>4)+r, col lane&15 of each 16x16 tile
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
