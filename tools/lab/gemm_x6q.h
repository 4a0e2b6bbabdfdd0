// Split-bf16 GEMM with planar LDS tiles ("x6q") for k-contiguous operand pairs (gfx950).
//
// gemm_x6_kernel (gemm_x6.h) feeds each bf16 MFMA two split terms of 4 k (its 32 k slots are
// (term, k) pairs), so its LDS tiles hold the combination planes [h|m], [h|l] / [l|h]: 8 B per
// operand element are written and read per k.  Here each MFMA takes 8 consecutive k of ONE term:
// a stage is 32 k deep (two of the loaders' 16-deep k-steps), each operand tile keeps three plain
// planes h, m, l (6 B per element), laid out like the fp32 KC tile (64-B rows, 16-B chunks
// XOR-swizzled), and every fragment is one ds_read_b128 of one plane.  A staged 4-k unit goes in
// as three 8-B stores (h4, m4, l4).  Per stage and 16x16 output tile the six products are six
// MFMAs, smallest terms first (hl, lh, hm, mh, mm, hh), accumulated into the running sum.
#pragma once
#include <type_traits>

#include "gemm_x6.h"

namespace flsim {

// one operand tile of a 32-k stage: planes h, m, l of KCTile<ROWS> geometry (ROWS x 64 B each)
template <int ROWS>
struct X6QTile {
    static constexpr int PLANE = KCTile<ROWS>::FLOATS;
    static constexpr int FL = 3 * PLANE;
    // unit (row, 4-k quad kq = 0..7 of the stage) -> byte offset inside a plane: chunk kq / 2
    // (swizzled like the fp32 KC tile), half kq % 2
    __device__ static int off_bytes(int row, int kq) {
        return 4 * KCTile<ROWS>::chunk_off(row, kq >> 1) + 8 * (kq & 1);
    }
    __device__ static void store(float* s, int row, int kq, const XsUnit& v, bool = true) {
        char* b = reinterpret_cast<char*>(s) + off_bytes(row, kq);
        *reinterpret_cast<f32x2*>(b) = f32x2{v.hm.x, v.hm.y};                       // h4
        *reinterpret_cast<f32x2*>(b + 4 * PLANE) = f32x2{v.hm.z, v.hm.w};           // m4
        *reinterpret_cast<f32x2*>(b + 8 * PLANE) = v.l;                              // l4
    }
    __device__ static void store(float* s, int row, int kq, f32x4 v, bool = true) {
        store(s, row, kq, xs_of(v));
    }
    struct Frag {
        f32x4 h, m, l;
    };
    __device__ static Frag frag(const float* s, int r0, int lane) {
        return Frag{read_frag<true, ROWS>(s, r0, lane), read_frag<true, ROWS>(s + PLANE, r0, lane),
                    read_frag<true, ROWS>(s + 2 * PLANE, r0, lane)};
    }
};

// k-major operand tile of a 32-k stage (the weight gradients: the pixel is the reduction index of
// both dZ and im2col): planes h, m, l as [32 k][LD] bf16, LD = ROWS + 8 (as X6Tile's), one spare
// 8-B slot after each for surplus units; a unit (k row, 4 columns) is three 8-B stores, a
// fragment (8 consecutive k of 16 columns) two transposing reads per plane
template <int ROWS>
struct X6QTileKM {
    static constexpr int LD = ROWS + 8;
    static constexpr int PLANE = (2 * GK * LD + 4) / 2;       // floats
    static constexpr int FL = 3 * PLANE;
    static constexpr int SPARE = 2 * GK * LD;                 // bf16 units
    __device__ static void store(float* s, int krow, int c4, const XsUnit& v, bool valid) {
        const int off = valid ? krow * LD + 4 * c4 : SPARE;
        __bf16* base = reinterpret_cast<__bf16*>(s) + off;
        *reinterpret_cast<f32x2*>(base) = f32x2{v.hm.x, v.hm.y};
        *reinterpret_cast<f32x2*>(base + 2 * PLANE) = f32x2{v.hm.z, v.hm.w};
        *reinterpret_cast<f32x2*>(base + 4 * PLANE) = v.l;
    }
    __device__ static void store(float* s, int krow, int c4, f32x4 v, bool valid) {
        store(s, krow, c4, xs_of(v), valid);
    }
    // 8 consecutive k (8g .. 8g + 7 for lane group g) of tile column r0 + (lane & 15)
    __device__ static f32x4 read8(const float* plane, int r0, int lane) {
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const __bf16* base = reinterpret_cast<const __bf16*>(plane) + (8 * g + q) * LD + r0 + 4 * p;
        typedef __attribute__((address_space(3))) s16x4v lds_s16x4;
        const s16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
        const s16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + 4 * LD));
        return cat_bf16(__builtin_bit_cast(bf16x4v, lo), __builtin_bit_cast(bf16x4v, hi));
    }
    struct Frag {
        f32x4 h, m, l;
    };
    __device__ static Frag frag(const float* s, int r0, int lane) {
        return Frag{read8(s, r0, lane), read8(s + PLANE, r0, lane), read8(s + 2 * PLANE, r0, lane)};
    }
    // column sum over the stage's 32 k rows (the bias gradient): h + m + l per element
    __device__ static float colsum(const float* s, int col) {
        const __bf16* ph = reinterpret_cast<const __bf16*>(s);
        const __bf16* pm = reinterpret_cast<const __bf16*>(s + PLANE);
        const __bf16* pl = reinterpret_cast<const __bf16*>(s + 2 * PLANE);
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * GK; ++k)
            a += ((float)ph[k * LD + col] + (float)pm[k * LD + col]) + (float)pl[k * LD + col];
        return a;
    }
};

// the tile type of a loader: KC planes or k-major planes
template <class LD_, int ROWS>
using X6QTileOf = std::conditional_t<LD_::KC, X6QTile<ROWS>, X6QTileKM<ROWS>>;

// one 32-k stage of a 16x16 tile: six single-term MFMAs into the running sum, smallest first
// (straight accumulation: gemm_x6.h FLSIM_X6_FRESH)
__device__ __forceinline__ f32x4 x6q_step(f32x4 acc, const f32x4& ah, const f32x4& am,
                                          const f32x4& al, const f32x4& bh, const f32x4& bm,
                                          const f32x4& bl) {
    acc = mfma_x32(ah, bl, acc);
    acc = mfma_x32(al, bh, acc);
    acc = mfma_x32(ah, bm, acc);
    acc = mfma_x32(am, bh, acc);
    acc = mfma_x32(am, bm, acc);
    return mfma_x32(ah, bh, acc);
}

// Same contract as gemm_x6_kernel for KC loader pairs (each_unit over 16-deep k-steps): the grid
// is XCD-grouped, K is walked in stages of two loader k-steps (kstages = ceil(ksteps / 2); a
// missing second half reads as zeros), registers hold the next stage's units while the current
// stage computes, one barrier per stage.
template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_x6q_kernel(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
                int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(AL::ROWS == BM && BL::ROWS == BN, "loader rows != tile");
    static_assert(!EPI::ASUM || !AL::KC, "ASUM needs a k-major A tile");
    using TA = X6QTileOf<AL, BM>;
    using TB = X6QTileOf<BL, BN>;
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
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % tiles_n;
    const int tm = (L / tiles_n) % tiles_m;
    const int tz = L / (tiles_m * tiles_n);
    const int m0 = tm * BM;
    const int n0 = tn * BN;
    const int ks0 = tz * ksteps_per_split;
    int ks1 = ks0 + ksteps_per_split;
    if (ks1 > ksteps_total) ks1 = ksteps_total;
    const int nst = (ks1 - ks0 + 1) / 2;

    al.setup(m0, tid);
    bl.setup(n0, tid);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float asum = 0.f;
    typename AL::Unit ra[2][AL::UNITS];
    typename BL::Unit rb[2][BL::UNITS];
    // the two loader k-steps of stage s (a second half past ks1 is zeroed: its units are staged
    // as zeros, never read from memory)
    auto load = [&](int s) {
        const int k = ks0 + 2 * s;
        al.load(k, ra[0]);
        bl.load(k, rb[0]);
        if (k + 1 < ks1) {
            al.load(k + 1, ra[1]);
            bl.load(k + 1, rb[1]);
        } else {
#pragma unroll
            for (int j = 0; j < AL::UNITS; ++j) ra[1][j] = typename AL::Unit{};
#pragma unroll
            for (int j = 0; j < BL::UNITS; ++j) rb[1][j] = typename BL::Unit{};
        }
    };
    // a KC unit (row, chunk c of the 16-k step h) is 4-k quad 4h + c of the stage; a KM unit
    // (k row, column chunk) is k row 16h + row
    auto stage = [&](float* s) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            al.each_unit(ra[h], [&](int a, int c, const auto& v, bool ok) {
                if constexpr (AL::KC) TA::store(s, a, 4 * h + c, v, ok);
                else TA::store(s, 16 * h + a, c, v, ok);
            });
            bl.each_unit(rb[h], [&](int a, int c, const auto& v, bool ok) {
                if constexpr (BL::KC) TB::store(s + TA::FL, a, 4 * h + c, v, ok);
                else TB::store(s + TA::FL, 16 * h + a, c, v, ok);
            });
        }
    };

    if (nst > 0) {
        load(0);
        stage(lds);
        if (nst > 1) load(1);
    }
    __syncthreads();
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    int cur = 0;
    for (int s = 0; s < nst; ++s) {
        if (s + 1 < nst) {
            stage(lds + (cur ^ 1) * BUF);
            if (s + 2 < nst) load(s + 2);
        }
        const float* A = lds + cur * BUF;
        const float* B = A + TA::FL;
        if constexpr (EPI::ASUM) {
            if (tn == 0 && tid < BM) asum += TA::colsum(A, tid);
        }
        // A fragments of the wave's FM row blocks first, then one B fragment at a time (12 VGPRs
        // live for B instead of 12 FN)
        typename TA::Frag af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = TA::frag(A, wm * 16 * FM + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const typename TB::Frag bf = TB::frag(B, wn * 16 * FN + 16 * j, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i)
                acc[i][j] = x6q_step(acc[i][j], af[i].h, af[i].m, af[i].l, bf.h, bf.m, bf.l);
        }
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
                        for (int rr = 0; rr < 4; ++rr)
                            lds[(ml + rr) * STAGE_LD + nl] = epi.value(nl, acc[i][j][rr]);
                    }
            }
            __syncthreads();
            const int wm_hi = (pass + 1) * WM_PASS < WAVES_M ? (pass + 1) * WM_PASS : WAVES_M;
            staged_store(epi, lds, STAGE_LD, m0 + pass * WM_PASS * WROWS,
                         (wm_hi - pass * WM_PASS) * WROWS, n0, BN, tid, 64 * WAVES_M * WAVES_N);
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
