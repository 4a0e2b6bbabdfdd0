// Direct-A fp32 MFMA GEMM for the convolutions' forward and data-gradient passes (gfx950).
//
// gemm_kernel (gemm_core.h) stages BOTH operands through LDS every 16-deep k-step, with one block
// barrier per k-step.  For an implicit-GEMM convolution the A operand (rows = output pixels, k =
// 16 consecutive input channels of one tap) already has the MFMA fragment shape in global memory:
// lane l of a 16x16x4 MFMA holds A[row l&15][k 4(l>>4)..+3], i.e. four consecutive channels of one
// input pixel = one 16-B load.  So here each wave owns 16*FM rows of the block tile and loads its
// A fragments straight into registers (DEPTH k-steps ahead), with no LDS store, no LDS read and no
// barrier for A.  Only the B operand (packed weights, the block's BN columns) goes through LDS, in
// stages of KB k-steps: one barrier per stage instead of one per k-step, and the next stage's B is
// loaded and stored one k-step at a time under the current stage's MFMAs.
//
// The MFMA sequence per accumulator (k ascending; within a k-step the four k slots in order) is the
// one gemm_kernel issues, so the results are bit-identical to it.
#pragma once
#include "loaders.h"

namespace flsim {

// Scheduling fences around each k-step's MFMAs (measurement override -DFLSIM_DIRECT_FENCES=<0|1>)
#ifndef FLSIM_DIRECT_FENCES
#define FLSIM_DIRECT_FENCES 1
#endif
constexpr bool DIRECT_FENCES = FLSIM_DIRECT_FENCES;

// A operand of a 3x3 / stride-1 convolution (forward, or data gradient as a valid convolution of
// dZ with the flipped weights) loaded per wave into MFMA fragments.  Same K order and the same
// geometry options (WIN: pool-window row order; OHX: explicit output size) as Im2colKC with
// CI % 16 == 0: k-step ks = 9 * (ci0 / 16) + tap.
template <int IH, int IW, int CI, int PAD, int FM, bool WIN = false, int OHX = 0,
          class SRC = BufSrc>
struct Im2colDirect {
    using Unit = typename SRC::Unit;
    // floats between neighbouring pixels / between channel slices (SRC::SM: slice-major input)
    static constexpr int PIX = SRC::SM ? GK : CI;
    static constexpr int SLICE = SRC::SM ? IH * IW * GK : GK;
    static constexpr int OH = OHX > 0 ? OHX : IH + 2 * PAD - 2;
    static constexpr int OW = OHX > 0 ? OHX : IW + 2 * PAD - 2;
    static constexpr int PH = OH / 2, PW = OW / 2;
    static constexpr int ROWS_PER_IMG = WIN ? 4 * PH * PW : OH * OW;
    static_assert(CI % 16 == 0, "direct A needs whole 16-channel slices");

    const float* X;
    const float* XL = nullptr;   // SRC = XsSrc: X is the HM part, XL the L part (split.h)
    int M;
    unsigned vb[FM];          // byte offset of input pixel (oh - PAD, ow - PAD), channel 4 (lane >> 4)
    unsigned short tapmask[FM];
    SRC buf;

    // r0: the wave's first row; fragment f covers rows r0 + 16 f + (lane & 15)
    __device__ void setup(int r0, int lane) {
        const int q = lane >> 4;
        buf.init(X, XL, (unsigned long)((M + ROWS_PER_IMG - 1) / ROWS_PER_IMG) * IH * IW * CI * 4);
#pragma unroll
        for (int f = 0; f < FM; ++f) {
            const int m = r0 + 16 * f + (lane & 15);
            long base = 0;
            int msk = 0;
            if (m < M) {
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
                base = (long)nimg * IH * IW * CI + ((long)(oh - PAD) * IW + (ow - PAD)) * PIX +
                       4 * q;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int ih = oh + t / 3 - PAD, iw = ow + t % 3 - PAD;
                    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) msk |= 1 << t;
                }
            }
            vb[f] = (unsigned)base * 4u;
            tapmask[f] = (unsigned short)msk;
        }
    }
    __device__ void load(int ks, Unit (&r)[FM]) const {
        const int cs = ks / 9;                  // uniform
        const int khkw = ks - 9 * cs;
        const int kh = khkw / 3;
        const unsigned off = (unsigned)(((kh * IW + (khkw - 3 * kh)) * PIX + cs * SLICE) * 4);
#pragma unroll
        for (int f = 0; f < FM; ++f) r[f] = buf.ld_or0(vb[f] + off, (tapmask[f] >> khkw) & 1);
    }
};

// B operand staging for gemm_direct_kernel: rows [n0, n0 + ROWS) of a row-major [NR][ld] matrix
// (packed weights), one 16-deep k-step per load/store, k-contiguous swizzled LDS tile (KCTile)
// followed by one spare 16-B chunk.  Every thread loads and stores every one of its units: a unit
// past the tile re-reads a valid chunk and stores it into the spare chunk, and rows >= NR read as
// zeros through the buffer bound, so neither the load nor the store sits under a branch (a load
// whose only use is a predicated store is sunk next to it and waited for at once).
template <int TR, int NT>
struct RowsKCStage {
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    static constexpr int FLOATS = KCTile<ROWS>::FLOATS + 4;   // tile + spare chunk
    const float* P;
    long ld;
    int NR;
    unsigned rowb[UNITS];
    int dst[UNITS];            // LDS float offset of the unit (the spare chunk for a surplus unit)
    BufSrc buf;
    __device__ void setup(int r0, int tid) {
        buf.init(P, (unsigned long)NR * ld * 4);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u0 = tid + j * NT;
            const bool real = u0 < TOTAL;
            const int u = real ? u0 : u0 % TOTAL;
            const int r = u >> 2, q = u & 3;
            rowb[j] = r0 + r < NR ? (unsigned)(((long)(r0 + r) * ld + 4 * q) * 4) : BUF_OOB;
            dst[j] = real ? KCTile<ROWS>::chunk_off(r, q) : KCTile<ROWS>::FLOATS;
        }
    }
    __device__ void load(int ks, f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            r[j] = buf.ld(rowb[j] == BUF_OOB ? BUF_OOB : rowb[j] + (unsigned)(ks * GK * 4));
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) *reinterpret_cast<f32x4*>(lds + dst[j]) = r[j];
    }
};

// Block = WAVES waves stacked along M (each 16*FM rows) x all BN = 16*FN columns of its n-tile.
template <int FM, int FN, int WAVES, int KB, int DEPTH, class AD, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES)
gemm_direct_kernel(AD ad, BL bl, EPI epi, int ksteps, int tiles_m, int tiles_n) {
    constexpr int BM = 16 * FM * WAVES;
    constexpr int BN = 16 * FN;
    static_assert(BL::ROWS == BN && BL::KC, "B loader: k-contiguous tile of BN rows");
    constexpr int BFL = BL::FLOATS;             // one k-step of B (+ the stager's spare chunk)
    constexpr int STG = KB * BFL;               // one stage
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int STAGE_LD = BN + 4;
    constexpr int BASE_FL = 2 * STG;
    constexpr int WROWS = 16 * FM;
    constexpr int WM_FIT = (BASE_FL > 8192 ? BASE_FL : 8192) / (WROWS * STAGE_LD);
    constexpr int WM_PASS = WM_FIT < 1 ? 1 : (WM_FIT > WAVES ? WAVES : WM_FIT);
    constexpr int LDS_FL = STAGED && WM_PASS * WROWS * STAGE_LD > BASE_FL
                               ? WM_PASS * WROWS * STAGE_LD : BASE_FL;
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

    // Loads are unconditional: a conditional load into a register that is also live from an
    // earlier load makes the compiler copy it (phi) and wait for vmcnt(0) there, serialising the
    // prefetch.  Past the end of K the loads read in-buffer garbage or out-of-range zeros that
    // nothing consumes (the last stage's "next" B buffer is free; the A ring is not read again).
    // The host guarantees ksteps % KB == 0.
    // A ring of R = DEPTH + 1 register slots: k-step ks reads slot ks % R while the load of
    // ks + DEPTH goes into another slot, issued BEFORE the step's MFMAs.  Scheduling fences keep
    // the compiler from sinking the loads next to their use (it otherwise groups them at the end
    // of the stage, where their latency is exposed at the next stage's first k-step).
    constexpr int R = DEPTH + 1;
    static_assert(KB % R == 0, "the A register ring index must be static");
    f32x4 ra[R][FM];
    f32x4 rb[BL::UNITS];
    const int nst = ksteps / KB;
    // prologue: B stage 0 and the first DEPTH k-steps of A
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
        const int kn = (s + 1) * KB;           // first k-step of the next stage
#pragma unroll
        for (int kk = 0; kk < KB; ++kk) {
            const int ks = s * KB + kk;
            // next stage's B: store the k-step loaded one step ago, load the next one; A of
            // k-step ks + DEPTH into the ring slot this step does not read
            if (kk > 0) bl.store(Bn + (kk - 1) * BFL, rb);
            bl.load(kn + kk, rb);
            ad.load(ks + DEPTH, ra[(kk + DEPTH) % R]);
            if constexpr (DIRECT_FENCES) __builtin_amdgcn_sched_barrier(0);
            f32x4 bf[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) bf[j] = read_frag<true, BN>(Bs + kk * BFL, 16 * j, lane);
#pragma unroll
            for (int kq = 0; kq < 4; ++kq)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = mfma16(ra[kk % R][i][kq], bf[j][kq], acc[i][j]);
            if constexpr (DIRECT_FENCES) __builtin_amdgcn_sched_barrier(0);
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
