// fp32 GEMM on the bf16 matrix cores at fp32 accuracy ("bf16x6").
//
// gfx950's fp32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16 rate.  Each fp32 operand
// x is split into h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (round to nearest even; x - h
// and x - h - m are exact in fp32), so x = h + m + l exactly (split.h).  Operands that their
// producer already wrote in that split form (split.h "xs" tensors: XsSrc loaders) are staged as
// they stand; fp32 operands (BufSrc loaders) are split by the thread that stages them.
// A product a*b is the sum of six exact partial products
//     ah*bh + am*bh  +  ah*bm + am*bm  +  ah*bl + al*bh
// (the three dropped, am*bl + al*bm + al*bl, are below 2^-25 |a b|), accumulated in fp32.
// One v_mfma_f32_16x16x32_bf16 sums 32 products per lane slot, so the two terms of each pair above
// go into ONE instruction over the same 16-deep k-step: its 32 slots are (term, k) pairs.  A lane
// of the 16x16x32 MFMA supplies slots 8g .. 8g+7 (g = lane >> 4) of its row / column; with the
// k-contiguous LDS unit of 4 k values per lane (k = 4g .. 4g+3, gemm_core.h) the A operand is
// the 16-B unit [ah | am] (slots 8g..8g+3 = ah, 8g+4..8g+7 = am) and B is [bh | bm], etc.:
//     MFMA 1: A [h|m] x B [h|m]  = ah bh + am bm
//     MFMA 2: A [h|m] x B [m|h]  = ah bm + am bh
//     MFMA 3: A [h|l] x B [l|h]  = ah bl + al bh
// so the LDS holds two 16-B combination planes of each tile (A: [h|m], [h|l]; B: [h|m], [l|h]),
// each laid out and swizzled exactly like the fp32 KC tile; every fragment is one ds_read_b128,
// and B's [m|h] is its [h|m] fragment with the two halves swapped in registers.
// k-major operands (the weight gradients: the pixel is the reduction index of both dZ and im2col)
// keep three plain planes h, m, l as [16 k][LD] bf16 (LD = km_ld) and read each 4-k half with
// gfx950's transposing ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses k row q,
// columns 4p..4p+3; lane i receives column i's four k), the halves paired in registers.
// Three 16-cycle bf16 MFMAs replace four 32-cycle fp32 ones per k-step (profiles/r03v:
// bf16x6 max error 1.0-3.1 x 2^-24 of sum |a b| against the fp32 MFMA's 1.6-3.3 on the same
// data, K = 1728 and 16384; pre-split operands run the inner loop at 312-316 fp32-equivalent
// TF/s against 148).
#pragma once
#include "gemm_core.h"
#include "split.h"

namespace flsim {

__device__ __forceinline__ f32x4 mfma_x32(f32x4 a, f32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8v, a),
                                                   __builtin_bit_cast(bf16x8v, b), c, 0, 0, 0);
}

// One k-step of a 16x16 output tile: the six partial products of its 16 k, A = ([h|m] a0,
// [h|l] a1), B = ([h|m] b0, [m|h] b1, [l|h] b2), smallest terms first.
//
// How the bf16 MFMA adds (tools/lab/mfma_numerics.hip, profiles/r05/mfma_numerics.txt): it is
// NOT an exact sum rounded once.  Its addends (the accumulator and the 32 products) are aligned
// to the largest of them and bits more than ~3 below that one's last bit are dropped, per addend
// and toward zero (C = 1 plus 32 products of 2^-27 returns 1; 16 x 2^-26 and 16 x -2^-27 on
// C = 1 return 1 + 2 ulp, the negative ones vanish).  Accumulating a k-step's six products
// straight into the running sum (FRESH = false) therefore truncates the small terms against the
// whole sum, a per-MFMA loss of up to ~2^-25 of |C| that leans toward zero: on PerformantNet1's
// data gradients 2.9-6.0e-7 rel-L2 against torch fp32's 1.0-1.7e-7 on the same inputs
// (tools/gemm_diag.py, profiles/r05).  FRESH = true sums the k-step's products from zero (so they
// are truncated against the k-step's own largest product) and adds that to the running sum with
// one fp32 add (round to nearest even): 1.5-2.1e-7.
template <bool FRESH>
__device__ __forceinline__ f32x4 x6_step(f32x4 acc, f32x4 a0, f32x4 a1, f32x4 b0, f32x4 b1,
                                         f32x4 b2) {
    if constexpr (FRESH) {
        f32x4 t = mfma_x32(a1, b2, f32x4{0.f, 0.f, 0.f, 0.f});   // ah bl + al bh
        t = mfma_x32(a0, b1, t);                                   // ah bm + am bh
        t = mfma_x32(a0, b0, t);                                   // ah bh + am bm
        return acc + t;
    } else {
        acc = mfma_x32(a1, b2, acc);
        acc = mfma_x32(a0, b1, acc);
        return mfma_x32(a0, b0, acc);
    }
}

// Which accumulations are fresh (measurement levels, FLSIM_X6_FRESH): 0 none; 1 every x6 main
// accumulator (round 4's experiment); 2 the k-contiguous GEMMs (forward and data gradients:
// gemm_x6 with a KC A tile, gemm_dx6) and the bias column sums; 3 everything; 4 the k-major
// (weight-gradient) GEMMs and the bias column sums; 5 the k-major GEMMs' main accumulation only.
#ifndef FLSIM_X6_FRESH
#define FLSIM_X6_FRESH 0
#endif
constexpr bool x6_fresh(bool kc) {
    return FLSIM_X6_FRESH == 1 || FLSIM_X6_FRESH == 3 || (FLSIM_X6_FRESH == 2 && kc) ||
           ((FLSIM_X6_FRESH == 4 || FLSIM_X6_FRESH == 5) && !kc);
}
constexpr bool x6_fresh_bias() { return FLSIM_X6_FRESH >= 2 && FLSIM_X6_FRESH != 5; }

// The k-major GEMMs (weight gradients: K = the chunk's pixels, up to 3.2M) flush their running
// MFMA sums into an fp32 total every X6_FLUSH k-steps (and restart them from zero), so the bf16
// MFMA's truncation only ever acts against a 16 * X6_FLUSH-pixel partial sum: the bias it leaves
// stays at the short chain's (tools/lab/wg_numerics.hip: 1.5e-7 rel-L2 for 512-pixel chains
// against 1.6e-6 for 16,384-pixel ones) instead of growing with K.  0: no flush.
#ifndef FLSIM_X6_FLUSH
#define FLSIM_X6_FLUSH 0
#endif

// Main-loop schedule of the k-contiguous GEMMs (both tiles KC: the staged forwards): the staging
// of the next k-step interleaved with the current k-step's MFMAs by sched_group_barrier, per MFMA
// V VALU, an LDS store every W MFMAs, a global load every L, in a branch-free loop body.  Lab
// (tools/lab/pp_lab.hip, profiles/r05/lab_x6_interleave.txt): conv5 forward 1.06-1.10x, conv6
// forward 1.01-1.04x, bit-identical; the k-major weight gradients lose up to 6 %, so they keep
// the compiler's order, and so do the GEMMs that split an fp32 operand while staging it (linear1's
// forward +3 %, VGG-11's forwards: configs[4] 1369 -> 1346 worker-steps/s with it,
// profiles/r05/ab/vgg_x6_interleave.txt).  So it runs where both operands arrive split, PN1's
// conv5 / conv6 forwards (A B A B, profiles/r05/ab/x6_interleave_kc.txt): conv6 forward
// 9.22-9.28 -> 9.01-9.07 ms, conv5 unchanged, the headline +0.2 %.  -DFLSIM_X6_PP_V=0: off.
#ifndef FLSIM_X6_PP_V
#define FLSIM_X6_PP_V 3
#define FLSIM_X6_PP_W 2
#define FLSIM_X6_PP_L 4
#endif
constexpr int X6_PP_V = FLSIM_X6_PP_V, X6_PP_W = FLSIM_X6_PP_W, X6_PP_L = FLSIM_X6_PP_L;

typedef short s16x4v __attribute__((ext_vector_type(4)));

// 4 consecutive k of one tile row from a k-major bf16 plane [16][LD] (ds_read_b64_tr_b16)
__device__ __forceinline__ bf16x4v read_km_half(const float* plane, int LD, int r0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const __bf16* base = reinterpret_cast<const __bf16*>(plane) + (4 * g + q) * LD + r0 + 4 * p;
    typedef __attribute__((address_space(3))) s16x4v lds_s16x4;
    const s16x4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base));
    return __builtin_bit_cast(bf16x4v, v);
}

// Row stride (bf16 units) of a k-major plane [16 k][LD].  A transposing read serves 32 lanes per
// LDS cycle: 8 k rows x 32 B, conflict-free when the 8 rows' 32-B pieces cover the 256 B of the
// 64 banks, i.e. when the row stride 2 LD bytes is an odd multiple of 32 (LD = 16 mod 32).  Of
// those strides
// the smallest >= ROWS whose ds_write_b64 unit stores (16 lanes per cycle on 32 banks; TPR lanes
// per k row, so a 16-lane group may span two rows) are conflict-free too, else the smallest.
// (ROWS + 8, used before, cost 2 extra LDS cycles per transposed read: SQ_LDS_BANK_CONFLICT
// 0.4-1.0 G cycles per weight-gradient launch, profiles/r04/prof_r04e.)
constexpr bool km_writes_free(int ld, int tpr) {
    if (tpr >= 16) return true;
    bool used[16] = {};
    for (int l = 0; l < 16; ++l) {
        const int row = l / tpr, c = l % tpr;
        const int chunk = ((row * 2 * ld + 8 * c) % 128) / 8;
        if (used[chunk]) return false;
        used[chunk] = true;
    }
    return true;
}
constexpr int km_ld(int rows, int tpr) {
    for (int ld = rows; ld < rows + 128; ++ld)
        if (ld % 32 == 16 && km_writes_free(ld, tpr)) return ld;
    for (int ld = rows; ld < rows + 32; ++ld)
        if (ld % 32 == 16) return ld;
    return rows + 8;
}

// One operand tile of a stage.  AROLE: the A side ([h|m], [h|l]) or the B side ([h|m], [m|h],
// [l|h]).  KC: combination planes laid out like the fp32 KC tile; KM: planes h, m, l as
// [16][LD] bf16 (LD = km_ld: conflict-free transposed reads), one spare 8-B slot after each for
// surplus units.  TPR: the loader's threads per k row (NT / 16).
template <bool KC, int ROWS, bool AROLE, int TPR = 16>
struct X6Tile {
    static constexpr int LD = km_ld(ROWS, TPR);
    static constexpr int NPL = KC ? 2 : 3;
    static constexpr int PLANE_FL = KC ? KCTile<ROWS>::FLOATS : (GK * LD + 4) / 2;
    static constexpr int FL = NPL * PLANE_FL;
    struct Frag {
        f32x4 x0, x1, x2;
    };
    // a unit already in the split form (split.h: loaders over HM / L tensors): plane stores only
    __device__ static void store(float* s, int a, int b, const XsUnit& v, bool valid) {
        if constexpr (KC) {
            store_unit<true, ROWS>(s, a, b, v.hm);
            store_unit<true, ROWS>(s + PLANE_FL, a, b, AROLE ? xs_hl(v) : xs_lh(v));
        } else {
            const int off = valid ? a * LD + 4 * b : GK * LD;   // bf16 units
            __bf16* base = reinterpret_cast<__bf16*>(s) + off;
            *reinterpret_cast<f32x2*>(base) = f32x2{v.hm.x, v.hm.y};
            *reinterpret_cast<f32x2*>(base + 2 * PLANE_FL) = f32x2{v.hm.z, v.hm.w};
            *reinterpret_cast<f32x2*>(base + 4 * PLANE_FL) = v.l;
        }
    }
    // an fp32 unit: split here, when it is staged
    __device__ static void store(float* s, int a, int b, f32x4 v, bool valid) {
        store(s, a, b, xs_of(v), valid);
    }
    __device__ static Frag frag(const float* s, int r0, int lane) {
        Frag f;
        if constexpr (KC) {
            f.x0 = read_frag<true, ROWS>(s, r0, lane);                        // [h|m]
            if constexpr (AROLE) {
                f.x1 = read_frag<true, ROWS>(s + PLANE_FL, r0, lane);         // [h|l]
            } else {
                f.x1 = f32x4{f.x0.z, f.x0.w, f.x0.x, f.x0.y};                 // [m|h]
                f.x2 = read_frag<true, ROWS>(s + PLANE_FL, r0, lane);         // [l|h]
            }
        } else {
            const bf16x4v h = read_km_half(s, LD, r0, lane);
            const bf16x4v m = read_km_half(s + PLANE_FL, LD, r0, lane);
            const bf16x4v l = read_km_half(s + 2 * PLANE_FL, LD, r0, lane);
            f.x0 = cat_bf16(h, m);
            if constexpr (AROLE) {
                f.x1 = cat_bf16(h, l);
            } else {
                f.x1 = cat_bf16(m, h);
                f.x2 = cat_bf16(l, h);
            }
        }
        return f;
    }
    // column sum of a k-major tile's 16 k rows (the bias gradient, ASUM): h + m + l per element
    __device__ static float colsum(const float* s, int col) {
        const __bf16* ph = reinterpret_cast<const __bf16*>(s);
        const __bf16* pm = reinterpret_cast<const __bf16*>(s + PLANE_FL);
        const __bf16* pl = reinterpret_cast<const __bf16*>(s + 2 * PLANE_FL);
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < GK; ++k)
            a += ((float)ph[k * LD + col] + (float)pm[k * LD + col]) + (float)pl[k * LD + col];
        return a;
    }
};

// Epilogues with ASUM_MFMA = true take the bias column sum (ASUM) on the matrix cores: the wave
// column wn = 0 of the tn = 0 blocks multiplies each A fragment it already holds by a ones operand,
// [h|m] x [1|1] + [h|l] x [0|1] = sum over the k-step of h + m + l per row, two MFMAs per fragment,
// instead of the VALU column sum over the LDS tile (TA::colsum: 3 bf16 reads, a convert and an add
// per element and k, on BM threads while the block waits at the next barrier).
template <class E, class = void>
struct AsumMfma : std::false_type {};
template <class E>
struct AsumMfma<E, std::void_t<decltype(E::ASUM_MFMA)>> : std::bool_constant<E::ASUM_MFMA> {};

// Epilogues with X6_FRESH = true make their GEMM's main accumulation fresh whatever the build's
// FLSIM_X6_FRESH level (x6_step): PerformantNet1's linear1 forward, whose error e1 carries into
// linear2's weight gradient.
template <class E, class = void>
struct X6Fresh : std::false_type {};
template <class E>
struct X6Fresh<E, std::void_t<decltype(E::X6_FRESH)>> : std::bool_constant<E::X6_FRESH> {};

__device__ __forceinline__ f32x4 bf16_ones(bool lo, bool hi) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t a = lo ? 0x3f803f80u : 0u, b = hi ? 0x3f803f80u : 0u;
    return __builtin_bit_cast(f32x4, u32x4{a, a, b, b});
}

// Same contract as gemm_kernel (gemm_core.h: 1-D XCD-aware grid, register-staged double buffer,
// one barrier per 16-deep k-step, STAGED / plain / PRE / ASUM epilogues); loaders expose
// each_unit().  The B side of a KC tile keeps two planes [h|m], [l|h] and pairs
// ah bh + am bm, ah bm + am bh (B [m|h] = [h|m] with its halves swapped in registers),
// ah bl + al bh; a third plane ([h|h], [m|m], [l|h], no swaps) measured 3-24 % slower
// (profiles/r03w/x6_lab2.txt, "BP3"): these kernels are bound by LDS bandwidth.
template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_x6_kernel(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m,
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
    constexpr bool PP_KC = X6_PP_V > 0 && AL::KC && BL::KC && !X6Fresh<EPI>::value &&
                           std::is_same_v<typename AL::Unit, XsUnit> &&
                           std::is_same_v<typename BL::Unit, XsUnit>;
    // (the 192-row k-major weight-gradient tiles of PN1's conv5 / conv6 interleaved too, two
    // VALU per MFMA, a store and a load every third: +2.7 % / +0.8 % in the lab,
    // profiles/r05/lab_x6_interleave_wgrad.txt, but 5-6 % slower in the product,
    // profiles/r05/ab/x6_interleave_km.txt: removed)
    constexpr bool PP = PP_KC;
    constexpr int PV = X6_PP_V, PW = X6_PP_W, PL = X6_PP_L;
    constexpr int FLUSH = AL::KC ? 0 : FLSIM_X6_FLUSH;
    f32x4 tot[FLUSH ? FM : 1][FLUSH ? FN : 1];
    f32x4 btot[FLUSH && AMF ? FM : 1];
    if constexpr (FLUSH > 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
            for (int j = 0; j < FN; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (AMF) btot[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    auto main_loop = [&](auto with_sum) {
        constexpr bool WS = decltype(with_sum)::value;
        for (int ks = ks0; ks < ks1; ++ks) {
            if constexpr (PP) {
                // branch-free (one basic block, so the staging can be interleaved with the
                // MFMAs, below): the last k-step stages into the buffer nobody reads again, and
                // the loads past the split re-read its last k-step
                stage(lds + (cur ^ 1) * BUF);
                const int kl = ks + 2 < ks1 ? ks + 2 : ks1 - 1;
                al.load(kl, ra);
                bl.load(kl, rb);
            } else if (ks + 1 < ks1) {
                stage(lds + (cur ^ 1) * BUF);
                if (ks + 2 < ks1) {
                    al.load(ks + 2, ra);
                    bl.load(ks + 2, rb);
                }
            }
            const float* A = lds + cur * BUF;
            const float* B = A + TA::FL;
            if constexpr (WS && !AMF) {
                if (tid < BM) asum += TA::colsum(A, tid);
            }
            typename TB::Frag bf[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bf[j] = TB::frag(B, wn * 16 * FN + 16 * j, lane);
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const typename TA::Frag af = TA::frag(A, wm * 16 * FM + 16 * i, lane);
                if constexpr (WS && AMF) {
                    if constexpr (x6_fresh_bias()) {
                        f32x4 t = mfma_x32(af.x1, bf16_ones(false, true),
                                           f32x4{0.f, 0.f, 0.f, 0.f});                // l
                        t = mfma_x32(af.x0, bf16_ones(true, true), t);                 // h + m
                        bacc[i] = bacc[i] + t;
                    } else {
                        bacc[i] = mfma_x32(af.x1, bf16_ones(false, true), bacc[i]);   // l
                        bacc[i] = mfma_x32(af.x0, bf16_ones(true, true), bacc[i]);    // h + m
                    }
                }
                constexpr bool FRESH = x6_fresh(AL::KC) || X6Fresh<EPI>::value;
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    acc[i][j] = x6_step<FRESH>(acc[i][j], af.x0, af.x1, bf[j].x0, bf[j].x1,
                                               bf[j].x2);
                }
            }
            if constexpr (PP) {
                // per MFMA X6_PP_V VALU (the staging's split and address arithmetic), an LDS
                // store every X6_PP_W MFMAs and a global load every X6_PP_L
#pragma unroll
                for (int n = 0; n < 3 * FM * FN; ++n) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, PV, 0);
                    if (n % PW == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
                    if (n % PL == 1 % PL) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                }
            }
            if constexpr (FLUSH > 0) {
                if ((ks - ks0) % FLUSH == FLUSH - 1) {        // block-uniform
#pragma unroll
                    for (int i = 0; i < FM; ++i) {
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            tot[i][j] += acc[i][j];
                            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                        }
                        if constexpr (WS && AMF) {
                            btot[i] += bacc[i];
                            bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                        }
                    }
                }
            }
            __syncthreads();
            cur ^= 1;
        }
    };
    // Waves of one block may run different compiled forms of the loop, so they meet their
    // barriers at different call sites.  That is sound on gfx9 (s_barrier counts waves) because
    // every form runs the same block-uniform k range ks0 .. ks1 with exactly one barrier per
    // k-step; keep both invariants when changing the loop.
    bool sum_wave = false;
    if constexpr (AMF) sum_wave = bwave;
    else if constexpr (EPI::ASUM) sum_wave = tn == 0 && wave * 64 < BM;
    if (sum_wave) main_loop(std::true_type{});
    else main_loop(std::false_type{});
    if constexpr (FLUSH > 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j] + acc[i][j];
            if constexpr (AMF) bacc[i] = btot[i] + bacc[i];
        }
    }

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
