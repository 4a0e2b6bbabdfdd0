// Halo-staged direct split-bf16 GEMM (lab, development tool, not part of libflsim.so): the
// gemm_dx6_kernel form of a 3x3 / stride-1 convolution's forward pass, with the A operand served
// from an LDS patch instead of per-tap vector loads.
//
// gemm_dx6_kernel loads every A fragment from memory at every tap, so each input element passes
// the texture path 9 times (TD busy 0.87-0.90 on conv2-4's forwards).  Here a block
// stages, per 16-channel slice, the input rows its output rows need -- the rows of a contiguous
// range of "global input rows" g = img * IH + ih, all IW pixels, the slice's 16 channels in the
// split form (HM 16 B + L 8 B per 4 channels) -- into LDS once, and the nine taps of that slice
// read their fragments from the patch.  The next slice's patch is loaded into registers during
// the current slice and stored after its last barrier.  B (the packed weights) is staged one
// k-step at a time, double-buffered.
//
// The k order (ks = 9 * slice + tap) and the MFMA sequence per accumulator are gemm_dx6_kernel's,
// so the outputs are bit-identical to it.  Input: split, channel-slice-major (XsSrcSM layout).
#pragma once
#include "gemm_dx6.h"

namespace flsim {

template <int IH, int IW, int CI, int PAD, int FM, bool WIN, int NRP>
struct HaloA {
    static constexpr int OH = IH + 2 * PAD - 2, OW = IW + 2 * PAD - 2;
    static constexpr int PH = OH / 2, PW = OW / 2;
    static constexpr int ROWS_PER_IMG = WIN ? 4 * PH * PW : OH * OW;
    static constexpr int CS = CI / 16;
    static constexpr int ROW_UNITS = IW * 4;                // one patch row: IW pixels x 4 units
    static constexpr int UNITS = NRP * ROW_UNITS;
    static constexpr int HM_FL = UNITS * 4;                 // 16 B per unit
    static constexpr int FL = HM_FL + UNITS * 2;            // + 8 B per unit (L)
    static_assert(CI % 16 == 0, "whole 16-channel slices");

    const float* X;     // HM part, [img][CS][IH][IW][16]
    const float* XL;    // L part
    int M;
    XsSrc buf;
    int g_lo, nr;                 // block-uniform: first global input row, rows in the patch
    int ubase[FM];                // patch unit of tap (0, 0) for the lane's row of fragment f
    unsigned short tapmask[FM];

    __device__ static void rowpos(int m, int& img, int& oh, int& ow) {
        img = m / ROWS_PER_IMG;
        const int rem = m - img * ROWS_PER_IMG;
        if constexpr (WIN) {
            const int qq = rem >> 2;
            const int ph = qq / PW;
            oh = 2 * ph + ((rem >> 1) & 1);
            ow = 2 * (qq - ph * PW) + (rem & 1);
        } else {
            oh = rem / OW;
            ow = rem - oh * OW;
        }
    }
    // the output-row range of a row's pooled window (WIN) or the row itself
    __device__ static void ohrange(int m, int& img, int& lo, int& hi) {
        int oh, ow;
        rowpos(m, img, oh, ow);
        lo = WIN ? (oh & ~1) : oh;
        hi = WIN ? (oh | 1) : oh;
    }
    // patch rows of the block's rows [m0, m1] (m1 < M)
    __device__ void setup_block(int m0, int m1) {
        int i0, lo0, hi0, i1, lo1, hi1;
        ohrange(m0, i0, lo0, hi0);
        ohrange(m1, i1, lo1, hi1);
        const int a = lo0 - PAD, b = hi1 - PAD + 2;
        g_lo = i0 * IH + (a > 0 ? a : 0);
        const int g_hi = i1 * IH + (b < IH - 1 ? b : IH - 1);
        nr = g_hi - g_lo + 1;
        if (nr > NRP) nr = NRP;       // (the host checks NRP covers every block)
        buf.init(X, XL, (unsigned long)((M + ROWS_PER_IMG - 1) / ROWS_PER_IMG) * IH * IW * CI * 4);
    }
    // r0: the wave's first row; fragment f covers rows r0 + 16 f + (lane & 15)
    __device__ void setup_lane(int r0, int lane) {
        const int q = lane >> 4;
#pragma unroll
        for (int f = 0; f < FM; ++f) {
            const int m = r0 + 16 * f + (lane & 15);
            int msk = 0, ub = 0;
            if (m < M) {
                int img, oh, ow;
                rowpos(m, img, oh, ow);
                ub = ((img * IH + oh - PAD - g_lo) * IW + (ow - PAD)) * 4 + q;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int ih = oh + t / 3 - PAD, iw = ow + t % 3 - PAD;
                    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) msk |= 1 << t;
                }
            }
            ubase[f] = ub;
            tapmask[f] = (unsigned short)msk;
        }
    }
    // the patch of slice cs: unit u = (row r, pixel iw, quad) of global row g_lo + r
    template <int UPT, int NT>
    __device__ void load_patch(int cs, XsUnit (&pr)[UPT], int tid) const {
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
            const int u = tid + j * NT;
            unsigned off = BUF_OOB;
            if (u < nr * ROW_UNITS) {
                const int r = u / ROW_UNITS, w4 = u - r * ROW_UNITS;
                const int g = g_lo + r;
                const int img = g / IH, ih = g - img * IH;
                off = (unsigned)((((img * CS + cs) * IH + ih) * ROW_UNITS + w4) * 16);
            }
            pr[j] = buf.ld(off);
        }
    }
    template <int UPT, int NT>
    __device__ static void store_patch(float* lds, const XsUnit (&pr)[UPT], int tid) {
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
            const int u = tid + j * NT;
            if (UPT * NT <= UNITS || u < UNITS) {
                *reinterpret_cast<f32x4*>(lds + 4 * u) = pr[j].hm;
                *reinterpret_cast<f32x2*>(lds + HM_FL + 2 * u) = pr[j].l;
            }
        }
    }
    __device__ XsUnit frag(const float* lds, int tap, int f) const {
        const bool ok = (tapmask[f] >> tap) & 1;
        const int u = ok ? ubase[f] + ((tap / 3) * IW + tap % 3) * 4 : 0;
        XsUnit x;
        x.hm = *reinterpret_cast<const f32x4*>(lds + 4 * u);
        x.l = *reinterpret_cast<const f32x2*>(lds + HM_FL + 2 * u);
        if (!ok) {
            x.hm = f32x4{0.f, 0.f, 0.f, 0.f};
            x.l = f32x2{0.f, 0.f};
        }
        return x;
    }
};

// Block = WAVES waves stacked along M (each 16*FM rows) x all BN = 16*FN columns of its n-tile.
// ksteps = 9 * CS.
template <int FM, int FN, int WAVES, class HA, class BL, class EPI, int MINW = 1>
__global__ void __launch_bounds__(64 * WAVES, MINW)
gemm_hx6_kernel(HA ha, BL bl, EPI epi, int tiles_m, int tiles_n) {
    constexpr int NT = 64 * WAVES;
    constexpr int BM = 16 * FM * WAVES;
    constexpr int BN = 16 * FN;
    static_assert(BL::ROWS == BN && BL::KC, "B loader: k-contiguous tile of BN rows");
    constexpr int BFL = BL::FLOATS;
    constexpr int PLANE = BL::PLANE;
    constexpr int UPT = (HA::UNITS + NT - 1) / NT;
    constexpr bool STAGED = IsStaged<EPI>::value;
    constexpr int STAGE_LD = BN + 4;
    constexpr int BASE_FL = HA::FL + 2 * BFL;
    constexpr int WROWS = 16 * FM;
    constexpr int WM_FIT = BASE_FL / (WROWS * STAGE_LD);
    constexpr int WM_PASS = WM_FIT < 1 ? 1 : (WM_FIT > WAVES ? WAVES : WM_FIT);
    constexpr int LDS_FL = STAGED && WM_PASS * WROWS * STAGE_LD > BASE_FL
                               ? WM_PASS * WROWS * STAGE_LD : BASE_FL;
    static_assert(LDS_FL * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[LDS_FL];
    float* const Bbuf = lds + HA::FL;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % tiles_n;
    const int tm = L / tiles_n;
    const int m0 = tm * BM;
    const int n0 = tn * BN;
    const int m1 = (m0 + BM < ha.M ? m0 + BM : ha.M) - 1;

    ha.setup_block(m0, m1);
    ha.setup_lane(m0 + wave * WROWS, lane);
    bl.setup(n0, tid);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    XsUnit pr[UPT];
    typename BL::Unit rb[BL::UNITS];
    ha.template load_patch<UPT, NT>(0, pr, tid);
    bl.load(0, rb);
    HA::template store_patch<UPT, NT>(lds, pr, tid);
    bl.store(Bbuf, rb);
    if (HA::CS > 1) ha.template load_patch<UPT, NT>(1, pr, tid);
    bl.load(1, rb);
    __syncthreads();
    if constexpr (WAVES == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
#pragma unroll 1
    for (int cs = 0; cs < HA::CS; ++cs) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ks = 9 * cs + tap;
            const float* Bs = Bbuf + (ks & 1) * BFL;
            float* Bn = Bbuf + ((ks + 1) & 1) * BFL;
            bl.store(Bn, rb);          // k-step ks + 1 (loaded one step ago)
            bl.load(ks + 2, rb);       // past the end: out-of-range zeros, never stored for use
            __builtin_amdgcn_sched_barrier(0);
            f32x4 a0[FM], a1[FM];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const XsUnit x = ha.frag(lds, tap, i);
                a0[i] = x.hm;           // [h|m]
                a1[i] = xs_hl(x);       // [h|l]
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const f32x4 x0 = read_frag<true, BN>(Bs, 16 * j, lane);              // [h|m]
                const f32x4 x2 = read_frag<true, BN>(Bs + PLANE, 16 * j, lane);      // [l|h]
                const f32x4 x1 = f32x4{x0.z, x0.w, x0.x, x0.y};                      // [m|h]
#pragma unroll
                for (int i = 0; i < FM; ++i)
                    acc[i][j] = x6_step<false>(acc[i][j], a0[i], a1[i], x0, x1, x2);
            }
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
        }
        if (cs + 1 < HA::CS) {       // every wave is past the slice's last read of the patch
            HA::template store_patch<UPT, NT>(lds, pr, tid);
            if (cs + 2 < HA::CS) ha.template load_patch<UPT, NT>(cs + 2, pr, tid);
            __syncthreads();
        }
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
                         (w_hi - pass * WM_PASS) * WROWS, n0, BN, tid, NT);
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
