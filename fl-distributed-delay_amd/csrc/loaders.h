// Operand loaders and epilogues for gemm_kernel (gemm_core.h).
#pragma once
#include "gemm_core.h"
#include "pn1.h"

namespace flsim {

__device__ __forceinline__ f32x4 ldg4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------------------------------------
// A operand of a 3x3 / stride-1 convolution run as implicit GEMM (forward, or data-gradient as
// a "valid" convolution of dZ with the flipped weights).  Rows = output pixels m = (n, oh, ow);
// k = (ci / 16) * 144 + (kh*3 + kw) * 16 + ci % 16 for CI a multiple of 16 (channel-slice-major),
// k = (kh*3 + kw) * 4 + ci for CI == 4 (the padded input).
// Input X is NHWC.  Output spatial OH = IH + 2*PAD - 2.
// ---------------------------------------------------------------------------------------------
// WIN = true: output rows in max-pool window order, m = ((n * PH + ph) * PW + pw) * 4 + 2 dy + dx
// with (oh, ow) = (2 ph + dy, 2 pw + dx); the floor-mode border rows/columns a 2x2 pool drops
// are not computed at all (PerformantNet1 discards them: models.py:31,35,39).
template <int IH, int IW, int CI, int PAD, int TR, int NT, bool WIN = false>
struct Im2colKC {
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int OH = IH + 2 * PAD - 2;
    static constexpr int OW = IW + 2 * PAD - 2;
    static constexpr int PH = OH / 2, PW = OW / 2;
    static constexpr int ROWS_PER_IMG = WIN ? 4 * PH * PW : OH * OW;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    // CI % 16 == 0: a 16-deep k step lies inside one filter tap, so the tap and the channel base
    // are block-uniform (scalar) and each unit needs one add and one mask test per step
    static constexpr bool TAP_UNIFORM = CI % 16 == 0;
    static_assert(NT % 4 == 0, "");
    static_assert(CI == 4 || CI % 16 == 0, "");

    const float* X;
    int M;
    long base[UNITS];       // element offset of input pixel (oh - PAD, ow - PAD), channel 4q
    short tapmask[UNITS];   // bit kh*3+kw set iff that tap of this output pixel is inside X
    short row[UNITS];
    int q;

    __device__ void setup(int m0, int tid) {
        q = tid & 3;
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            const int r = u >> 2;
            row[j] = (short)r;
            const int m = m0 + r;
            base[j] = 0;
            tapmask[j] = 0;
            if (u < TOTAL && m < M) {
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
                base[j] = ((long)nimg * IH * IW + (long)(oh - PAD) * IW + (ow - PAD)) * CI + 4 * q;
                int msk = 0;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int ih = oh + t / 3 - PAD, iw = ow + t % 3 - PAD;
                    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) msk |= 1 << t;
                }
                tapmask[j] = (short)msk;
            }
        }
    }
    __device__ void load(int ks, f32x4 (&r)[UNITS]) const {
        if constexpr (TAP_UNIFORM) {
            // channel-slice-major K order: k-step ks = 9 * (ci0 / 16) + tap, so the nine taps of
            // one 16-channel slice of the input window are read in nine consecutive k-steps and
            // their re-reads hit L1/L2 (conv6 forward: 15.7 -> 3.3 GB fetched per launch,
            // profiles/r02d/lab_order.txt).  The packed weights follow (k_pack_fwd/_dgrad).
            const int cs = ks / 9;                  // uniform
            const int khkw = ks - 9 * cs;
            const int ci0 = cs * GK;
            const int kh = khkw / 3;
            const long off = (long)(kh * IW + (khkw - 3 * kh)) * CI + ci0;
#pragma unroll
            for (int j = 0; j < UNITS; ++j) {
                const bool ok = khkw < 9 && ((tapmask[j] >> khkw) & 1);
                r[j] = ok ? ldg4(X + base[j] + off) : zero4();
            }
        } else {
            const int k = ks * GK + 4 * q;          // CI == 4: one tap per lane quad
            const int khkw = k / CI;
            const int kh = khkw / 3;
            const long off = (long)(kh * IW + (khkw - 3 * kh)) * CI - 4 * q + (k - khkw * CI);
#pragma unroll
            for (int j = 0; j < UNITS; ++j) {
                const bool ok = khkw < 9 && ((tapmask[j] >> khkw) & 1);
                r[j] = ok ? ldg4(X + base[j] + off) : zero4();
            }
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) store_unit<true, ROWS>(lds, row[j], q, r[j]);
    }
};

// ---------------------------------------------------------------------------------------------
// Row-major matrix whose rows are the tile rows and whose reduction index is contiguous (KC):
// element (row, k) at P[row * ld + k].  Rows >= NR read as zero.  K must be a multiple of 16.
// ---------------------------------------------------------------------------------------------
template <int TR, int NT>
struct RowsKC {
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    static_assert(NT % 4 == 0, "");
    const float* P;
    long ld;
    int NR;
    const float* rowp[UNITS];
    short row[UNITS];
    int q;
    __device__ void setup(int r0, int tid) {
        q = tid & 3;
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            const int r = u >> 2;
            row[j] = (short)r;
            rowp[j] = (u < TOTAL && r0 + r < NR) ? P + (long)(r0 + r) * ld + 4 * q : nullptr;
        }
    }
    __device__ void load(int ks, f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) r[j] = rowp[j] ? ldg4(rowp[j] + ks * GK) : zero4();
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) store_unit<true, ROWS>(lds, row[j], q, r[j]);
    }
};

// ---------------------------------------------------------------------------------------------
// Row-major matrix whose ROWS are the reduction index (KM): element (k, col) at P[k * ld + col];
// the tile spans columns [c0, c0 + ROWS).  k >= NK or col >= NC read as zero (NC % 4 == 0).
// PO > 0: the rows are the pixels of PO x PO images and k walks only the top-left PV x PV
// window of each (k -> row img*PO*PO + oh*PO + ow): conv6's weight gradient skips the pixels
// the floor-mode pool never reads (their dZ is zero).
// ---------------------------------------------------------------------------------------------
template <int TR, int NT, int PO = 0, int PV = 0>
struct RowsKM {
    static constexpr int ROWS = TR;
    static constexpr bool KC = false;
    static constexpr int C4 = ROWS / 4;
    static constexpr int TOTAL = GK * C4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    const float* P;
    long ld;
    int NK;
    int NC;
    int c_off[UNITS];
    short krow[UNITS], c4[UNITS];
    __device__ void setup(int c0, int tid) {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            krow[j] = (short)(u / C4);
            c4[j] = (short)(u % C4);
            const int col = c0 + 4 * (u % C4);
            c_off[j] = (u < TOTAL && col < NC) ? col : -1;
        }
    }
    __device__ void load(int ks, f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int k = ks * GK + krow[j];
            long row = k;
            if constexpr (PO > 0) {
                const unsigned img = (unsigned)k / (unsigned)(PV * PV);
                const unsigned rem = (unsigned)k - img * (PV * PV);
                const unsigned oh = rem / (unsigned)PV;
                row = (long)img * (PO * PO) + oh * PO + (rem - oh * PV);
            }
            r[j] = (c_off[j] >= 0 && k < NK) ? ldg4(P + row * ld + c_off[j]) : zero4();
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || krow[j] < GK) store_unit<false, ROWS>(lds, krow[j], c4[j], r[j]);
    }
};

// ---------------------------------------------------------------------------------------------
// B operand of the weight gradient: im2col(X) with the pixel as the reduction index (KM).
// Tile columns = kk = (kh*3 + kw) * CI + ci in [c0, c0 + ROWS); reduction rows = pixels p.
// VO > 0: p walks only the top-left VO x VO output window of each image (pairs with RowsKM's
// PV window).
// ---------------------------------------------------------------------------------------------
template <int IH, int IW, int CI, int PAD, int TR, int NT, int VO = 0>
struct Im2colKM {
    static constexpr int ROWS = TR;
    static constexpr bool KC = false;
    static constexpr int OH = VO > 0 ? VO : IH + 2 * PAD - 2;
    static constexpr int OW = VO > 0 ? VO : IW + 2 * PAD - 2;
    static constexpr int C4 = ROWS / 4;
    static constexpr int TOTAL = GK * C4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    const float* X;
    int M;  // total pixels
    int coff[UNITS];   // ci, or -1 when the column is padding / out of range
    short kh[UNITS], kw[UNITS];
    short krow[UNITS], c4[UNITS];
    __device__ void setup(int c0, int tid) {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            krow[j] = (short)(u / C4);
            c4[j] = (short)(u % C4);
            const int kk = c0 + 4 * (u % C4);
            const int khkw = kk / CI;
            const int ci = kk - khkw * CI;
            kh[j] = (short)(khkw / 3);
            kw[j] = (short)(khkw % 3);
            coff[j] = (u < TOTAL && khkw < 9) ? ci : -1;
        }
    }
    __device__ void load(int ks, f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int p = ks * GK + krow[j];
            f32x4 v = zero4();
            if (coff[j] >= 0 && p < M) {
                const int nimg = p / (OH * OW);
                const int rem = p - nimg * (OH * OW);
                const int oh = rem / OW;
                const int ow = rem - oh * OW;
                const int ih = oh + kh[j] - PAD;
                const int iw = ow + kw[j] - PAD;
                if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW)
                    v = ldg4(X + ((long)nimg * IH * IW + ih * IW + iw) * CI + coff[j]);
            }
            r[j] = v;
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || krow[j] < GK) store_unit<false, ROWS>(lds, krow[j], c4[j], r[j]);
    }
};

// ---------------------------------------------------------------------------------------------
// Epilogues
// ---------------------------------------------------------------------------------------------
// conv forward without activation: Y[m][n] = acc + bias[n]  (vgg11_bn: the BatchNorm input)
struct EpiBias {
    static constexpr bool ASUM = false;
    float* Y;
    const float* bias;
    int M, N;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
        const float b = bias[n];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) Y[(long)(m + r) * N + n] = v[r] + b;
    }
};

// conv forward: Y[m][n] = relu(acc + bias[n])  (NHWC, row length N)
struct EpiBiasRelu {
    static constexpr bool ASUM = false;
    float* Y;
    const float* bias;
    int M, N;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
        const float b = bias[n];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) Y[(long)(m + r) * N + n] = fmaxf(v[r] + b, 0.f);
    }
};

// bias + ReLU staged through LDS (gemm_core.h STAGED): the block covers all NC output columns,
// so its BM rows are one contiguous piece of Y written with float4 stores
template <int NC>
struct EpiBiasReluRows {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr int NCOL = NC;
    static_assert(NC % 4 == 0, "float4 rows");
    float* Y;
    const float* bias;
    int M;
    __device__ float value(int n, float v) const { return fmaxf(v + bias[n], 0.f); }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int N4 = NC / 4;
        f32x4* dst = reinterpret_cast<f32x4*>(Y + (long)m0 * NC);
        for (int q = tid; q < rows * N4; q += nt) {
            const int r = q / N4, c = q - r * N4;
            dst[q] = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
        }
    }
};

// conv forward + bias + ReLU + 2x2 max-pool + dropout (models.py:30-32 / 34-36 / 38-40), rows in
// pool-window order (Im2colKC<..., WIN>): a lane's 4 accumulator rows are one pooling window of
// one channel.  Writes the pooled, dropped output d (NHWC, or torch flatten order for NCHW_OUT)
// and the argmax (first max in row-major window order, as torch CPU) for the backward pass.
template <int PH, int PW, int C, bool NCHW_OUT>
struct EpiPoolDrop {
    static constexpr bool ASUM = false;
    float* d;
    uint8_t* idx;
    const float* bias;
    const WorkerRec* workers;
    uint64_t seed;
    uint32_t site, thr;
    float scale;
    int dropout;
    int M;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= C || m >= M) return;
        const float b = bias[n];
        float mv = fmaxf(v[0] + b, 0.f);
        int mi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
            const float x = fmaxf(v[r] + b, 0.f);
            if (x > mv) { mv = x; mi = r; }
        }
        const int q = m >> 2;                       // pooled pixel (s, ph, pw)
        const int pw = q % PW;
        const int ph = (q / PW) % PH;
        const int s = q / (PW * PH);
        const int w = s / SAMPLES_PER_WORKER;
        const int nl = s - w * SAMPLES_PER_WORKER;
        float out = mv;
        if (dropout) {
            const WorkerRec wr = workers[w];
            const uint32_t en = (uint32_t)(((nl * C + n) * PH + ph) * PW + pw);
            out = philox_word(seed, wr.t, wr.i, site, en) >= thr ? mv * scale : 0.f;
        }
        const long e = (long)q * C + n;
        idx[e] = (uint8_t)mi;
        if (NCHW_OUT)
            d[(long)s * (C * PH * PW) + (n * PH + ph) * PW + pw] = out;
        else
            d[e] = out;
    }
};

// data gradient: Y[m][n] = acc * (act[m][n] > 0)  (MASK) or acc
template <bool MASK>
struct EpiMask {
    static constexpr bool ASUM = false;
    float* Y;
    const float* act;
    int M, N;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) {
                const long o = (long)(m + r) * N + n;
                float x = v[r];
                if (MASK) x = act[o] > 0.f ? x : 0.f;
                Y[o] = x;
            }
    }
};

// EpiMask<true> staged through LDS (gemm_core.h STAGED): float4 rows of the ReLU mask source
// and of the output
template <int NC>
struct EpiMaskRows {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr int NCOL = NC;
    static_assert(NC % 4 == 0, "float4 rows");
    float* Y;
    const float* act;
    int M;
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int N4 = NC / 4;
        f32x4* dst = reinterpret_cast<f32x4*>(Y + (long)m0 * NC);
        const f32x4* a4 = reinterpret_cast<const f32x4*>(act + (long)m0 * NC);
        for (int q = tid; q < rows * N4; q += nt) {
            const int r = q / N4, c = q - r * N4;
            const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
            const f32x4 a = a4[q];
            f32x4 o;
            o.x = a.x > 0.f ? t.x : 0.f;
            o.y = a.y > 0.f ? t.y : 0.f;
            o.z = a.z > 0.f ? t.z : 0.f;
            o.w = a.w > 0.f ? t.w : 0.f;
            dst[q] = o;
        }
    }
};

// gradient of a dropout(relu(.)) output: Y = acc * scale * (act > 0)  (act = dropped output)
struct EpiDropMask {
    static constexpr bool ASUM = false;
    float* Y;
    const float* act;
    float scale;
    int M, N;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) {
                const long o = (long)(m + r) * N + n;
                Y[o] = act[o] > 0.f ? v[r] * scale : 0.f;
            }
    }
};

// split-K partial slab, accumulated across chunks: S[z][m][n] += acc   (one owner per element);
// with Bsl != nullptr also the bias gradient Bsl[z][m] += column sum of the dZ tile (ASUM)
struct EpiSlabAcc {
    static constexpr bool ASUM = true;
    float* S;
    int M, N;
    long zstride;
    float* Bsl;
    __device__ void asum(int m, int z, float v) const {
        if (Bsl && m < M) Bsl[(long)z * M + m] += v;
    }
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
        float* base = S + z * zstride;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) base[(long)(m + r) * N + n] += v[r];
    }
};

// split-K partial, overwritten: S[z][m][n] = acc
struct EpiSlabStore {
    static constexpr bool ASUM = false;
    float* S;
    int M, N;
    long zstride;
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
        float* base = S + z * zstride;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) base[(long)(m + r) * N + n] = v[r];
    }
};

}  // namespace flsim
