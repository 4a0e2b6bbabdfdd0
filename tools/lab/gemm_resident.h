// Resident-B persistent fp32 MFMA GEMM for the narrow convolutions (gfx950).
//
// gemm_direct_kernel (gemm_direct.h) loads the A operand (im2col rows) per wave straight into MFMA
// fragments and stages B (packed weights) through LDS in KB-step stages, one barrier per stage.
// When ALL of B fits in LDS -- conv2's forward and data gradient: N = 48 columns x K = 432, 83 KB --
// the block can load it once and keep it: one block per CU walks a contiguous range of M-tiles,
// each wave streams its A fragments DEPTH k-steps ahead (the ring continues into the next tile, so
// the next tile's first loads are in flight during this tile's last k-steps), and the main loop has
// no barrier and no LDS store at all.  Only a staged epilogue (full output rows through LDS)
// synchronises, once per tile.
//
// The MFMA sequence per accumulator is gemm_kernel's (k ascending, the four k slots of a k-step in
// order), so the results are bit-identical to gemm_kernel / gemm_direct_kernel.
#pragma once
#include "gemm_direct.h"

namespace flsim {

// LDS floats of the staged-epilogue region for a block of WAVES waves of WROWS rows each and BN
// columns, when PASSES passes are used (WAVES / PASSES waves stage their rows per pass)
template <int WAVES, int WROWS, int BN, int PASSES>
constexpr int resident_stage_floats() {
    return (WAVES / PASSES) * WROWS * (BN + 4);
}

// Block = WAVES waves stacked along M (16*FM rows each) x all N = BN = 16*FN columns.
// KS = k-steps (K / 16), compile-time so the k-loop unrolls and the A ring index is static.
// Block b takes tiles [b * T / nb, (b + 1) * T / nb) of the T = tiles_m M-tiles.
template <int FM, int FN, int WAVES, int KS, int DEPTH, int PASSES, class AD, class EPI>
__global__ void __launch_bounds__(64 * WAVES)
gemm_resident_kernel(AD ad, const float* Wpk, int ldw, int NR, EPI epi, int tiles_m) {
    constexpr int BM = 16 * FM * WAVES;
    constexpr int BN = 16 * FN;
    constexpr int NT = 64 * WAVES;
    constexpr int BFL = KCTile<BN>::FLOATS;     // one k-step of B
    constexpr int B_FL = KS * BFL;
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int WROWS = 16 * FM;
    constexpr int STAGE_LD = BN + 4;
    static_assert(WAVES % PASSES == 0, "passes split the waves evenly");
    constexpr int WPP = WAVES / PASSES;         // waves staged per pass
    constexpr int STG_FL = STAGED ? resident_stage_floats<WAVES, WROWS, BN, PASSES>() : 0;
    static_assert((B_FL + STG_FL) * 4 <= 160 * 1024, "B + epilogue staging exceed the CU's LDS");
    constexpr int R = DEPTH + 1;
    static_assert(KS % R == 0, "the A ring must keep its phase across tiles");
    __shared__ __attribute__((aligned(16))) float lds[B_FL + STG_FL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    int tile = (int)((long)b * tiles_m / nb);
    const int t_end = (int)((long)(b + 1) * tiles_m / nb);

    // all of B, once: k-step ks, row r, 16-B chunk q -> the swizzled KCTile slot
    {
        BufSrc wb;
        wb.init(Wpk, (unsigned long)NR * ldw * 4);
        constexpr int UNITS = KS * BN * 4;
        for (int u = tid; u < UNITS; u += NT) {
            const int ks = u / (BN * 4);
            const int rem = u - ks * (BN * 4);
            const int r = rem >> 2, q = rem & 3;
            const unsigned off = r < NR ? (unsigned)((r * ldw + ks * GK + 4 * q) * 4) : BUF_OOB;
            *reinterpret_cast<f32x4*>(lds + ks * BFL + KCTile<BN>::chunk_off(r, q)) = wb.ld(off);
        }
    }
    if (tile >= t_end) return;                  // (only when there are more blocks than tiles)

    AD cur = ad;
    cur.setup(tile * BM + wave * WROWS, lane);
    f32x4 ra[R][FM];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) cur.load(d, ra[d]);
    __syncthreads();
    if constexpr (WAVES == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }

    for (; tile < t_end; ++tile) {
        // the next tile's rows (past the last tile: rows >= M, which load as zeros)
        AD nxt = ad;
        nxt.setup((tile + 1) * BM + wave * WROWS, lane);
        f32x4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + DEPTH < KS) cur.load(ks + DEPTH, ra[(ks + DEPTH) % R]);
            else nxt.load(ks + DEPTH - KS, ra[(ks + DEPTH) % R]);
            __builtin_amdgcn_sched_barrier(0);
            f32x4 bf[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bf[j] = read_frag<true, BN>(lds + ks * BFL, 16 * j, lane);
#pragma unroll
            for (int kq = 0; kq < 4; ++kq)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = mfma16(ra[ks % R][i][kq], bf[j][kq], acc[i][j]);
            __builtin_amdgcn_sched_barrier(0);
        }
        const int m0 = tile * BM;
        if constexpr (STAGED) {
            static_assert(BN == EPI::NCOL, "staged epilogue needs the full row in one block");
            float* stg = lds + B_FL;
#pragma unroll 1
            for (int pass = 0; pass < PASSES; ++pass) {
                __syncthreads();                 // the previous pass's rows are out
                if (wave / WPP == pass) {
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j) {
                            const int ml = (wave - pass * WPP) * WROWS + 16 * i + 4 * (lane >> 4);
                            const int nl = 16 * j + (lane & 15);
#pragma unroll
                            for (int rr = 0; rr < 4; ++rr)
                                stg[(ml + rr) * STAGE_LD + nl] = epi.value(nl, acc[i][j][rr]);
                        }
                }
                __syncthreads();
                epi.store_rows(stg, STAGE_LD, m0 + pass * WPP * WROWS, WPP * WROWS, tid, NT);
            }
        } else {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int m = m0 + wave * WROWS + 16 * i + 4 * (lane >> 4);
                    const int n = 16 * j + (lane & 15);
                    epi.apply4(m, n, 0, acc[i][j]);
                }
        }
        cur = nxt;
    }
}

}  // namespace flsim
