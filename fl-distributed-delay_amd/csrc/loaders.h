// Operand loaders and epilogues for gemm_kernel (gemm_core.h).
#pragma once
#include "gemm_core.h"
#include "pn1.h"
#include "split.h"

namespace flsim {

__device__ __forceinline__ f32x4 ldg4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
// streaming store (non-temporal): activations and gradients written once per chunk, far larger
// than L2 + MALL.  Plain stores of them reach ~3.8 TB/s, these ~5.4 (profiles/r02d/lab_conv1.txt)
__device__ __forceinline__ void st_nt4(float* p, f32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}

// Predicated operand load: lanes whose unit is padding or out of range issue no memory request
// (exec-masked).  A branch-free form that loads from a fixed valid address and selects zero was
// 6-12 % slower on every conv GEMM (all masked lanes hit one line; profiles/r02d/lab_ablation.txt).
__device__ __forceinline__ f32x4 ldg4_or0(const float* p, const float* /*safe*/, bool ok) {
    return ok ? ldg4(p) : zero4();
}

// Buffer-resource loads (FLSIM_BUFLOAD, default on): the operand tensor is one buffer of `bytes`
// bytes (< 4 GB, every activation at the 16,384-sample chunk is), addressed by 32-bit byte offsets.
// A masked unit (padding tap, row or column past the matrix) passes the out-of-range offset
// BUF_OOB and the hardware returns zeros: no exec-mask branch around the load, no zeroing of the
// destination registers, no 64-bit address arithmetic per unit.
#ifndef FLSIM_BUFLOAD
#define FLSIM_BUFLOAD 1
#endif
constexpr unsigned BUF_OOB = 0xfffffff0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, unsigned long bytes) {
    // raw buffer (stride 0): num_records in bytes; dword 3 = the gfx9 raw-buffer format word
    const unsigned n = bytes < (unsigned long)BUF_OOB ? (unsigned)bytes : BUF_OOB;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}
struct BufSrc {
    using Unit = f32x4;
    static constexpr bool SPLIT = false;
    static constexpr bool SM = false;
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ void init(const float* base, unsigned long bytes) {
        r = raw_rsrc(base, bytes);
    }
    __device__ __forceinline__ void init(const float* base, const float*, unsigned long bytes) {
        init(base, bytes);
    }
    __device__ __forceinline__ f32x4 ld(unsigned byte_off) const {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
    }
    __device__ __forceinline__ f32x4 ld_or0(unsigned byte_off, bool ok) const {
        return ld(ok ? byte_off : BUF_OOB);
    }
};
// fp32, channel-slice-major ([img][C/16][H][W][16]; split.h xs_store_f's copies of a1, d1, a3)
struct BufSrcSM : BufSrc {
    static constexpr bool SM = true;
};
// The same over a tensor in the split-bf16 form (split.h): byte offsets are the fp32 tensor's; the
// HM unit is read at that offset and the L unit at half of it.  A masked unit's BUF_OOB halves to
// 0x7ffffff8, still past the end of the L buffer (< 2 GB: every split tensor here is; the fp32
// equivalent is < 4 GB), so both reads return zeros.
struct XsSrc {
    using Unit = XsUnit;
    static constexpr bool SPLIT = true;
    static constexpr bool SM = false;
    __amdgpu_buffer_rsrc_t rhm, rl;
    __device__ __forceinline__ void init(const float* hm, const float* l, unsigned long bytes) {
        rhm = raw_rsrc(hm, bytes);
        rl = raw_rsrc(l, bytes / 2);
    }
    __device__ __forceinline__ XsUnit ld(unsigned byte_off) const {
        XsUnit u;
        u.hm = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rhm, byte_off, 0, 0));
        u.l = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rl, byte_off >> 1, 0, 0));
        return u;
    }
    __device__ __forceinline__ XsUnit ld_or0(unsigned byte_off, bool ok) const {
        return ld(ok ? byte_off : BUF_OOB);
    }
};

// A split tensor of C channels stored channel-slice-major, [img][C/16][H][W][16]: the 16 channels of
// one slice of neighbouring pixels are contiguous, so the 16 rows of a direct-A fragment (16
// neighbouring output pixels, one tap, one slice) read whole cache lines.  Only the loaders that
// read conv inputs (Im2colDirect, Im2colKM) accept it; the others assert pixel-major sources.
struct XsSrcSM : XsSrc {
    static constexpr bool SM = true;
};

// A split tensor read back as fp32 for the fp32 GEMM (gemm_core.h): each unit's HM and L parts
// loaded as by XsSrc and put back together, (h + m) + l, which is the fp32 value exactly
// (split.h).  The PerformantNet1 conv2-6 weight gradients run on the fp32 MFMA this way over the
// layer inputs their producers wrote split (summed over a 16,384-sample chunk, the
// bf16 MFMA's truncating accumulation leaves a relative bias of 5e-7 .. 1e-6 in them, above
// SURVEY 8(c)'s bound; the fp32 MFMA is an fmaf chain).
struct XsF32Src : XsSrc {
    using Unit = f32x4;
    static constexpr bool SPLIT = false;
    __device__ __forceinline__ f32x4 ld(unsigned byte_off) const {
        return xs_value(XsSrc::ld(byte_off));
    }
    __device__ __forceinline__ f32x4 ld_or0(unsigned byte_off, bool ok) const {
        return ld(ok ? byte_off : BUF_OOB);
    }
};
struct XsF32SrcSM : XsF32Src {
    static constexpr bool SM = true;
};

// r / D for 0 <= r < R by one 24-bit multiply and a shift (exact on that range, checked at
// compile time): the per-unit pixel -> (row, column) split of the k-major loaders
template <unsigned D, unsigned R>
struct SmallDiv {
    static constexpr unsigned find(bool want_shift) {
        for (unsigned sh = 4; sh < 24; ++sh) {
            const unsigned m = ((1u << sh) + D - 1) / D;
            if ((unsigned long long)(R - 1) * m >= (1ull << 24) * 256ull) break;
            bool ok = true;
            for (unsigned r = 0; r < R && ok; ++r) ok = ((r * m) >> sh) == r / D;
            if (ok) return want_shift ? sh : m;
        }
        return 0;
    }
    static constexpr unsigned M = find(false), SH = find(true);
    static_assert(M != 0 && R * M < (1u << 31) && R < (1u << 24), "no 24-bit magic for this range");
    __device__ static unsigned div(unsigned r) { return __umul24(r, M) >> SH; }
};

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
// OHX > 0: output OHX x OHX instead of IH + 2 PAD - 2, i.e. taps past the bottom/right edge of X
// read as zero (conv6's data gradient over the compact 14x14 dZ, whose 15th row/column would be
// zero: the floor-mode pool never reads conv6's row/column 14).
template <int IH, int IW, int CI, int PAD, int TR, int NT, bool WIN = false, int OHX = 0,
          class SRC = BufSrc>
struct Im2colKC {
    using Unit = typename SRC::Unit;
    static_assert(!SRC::SM, "pixel-major operand");
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int OH = OHX > 0 ? OHX : IH + 2 * PAD - 2;
    static constexpr int OW = OHX > 0 ? OHX : IW + 2 * PAD - 2;
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
    const float* XL = nullptr;   // SRC = XsSrc: X is the HM part, XL the L part (split.h)
    int M;
    long base[UNITS];       // element offset of input pixel (oh - PAD, ow - PAD), channel 4q
    unsigned vb[UNITS];     // the same in bytes, mod 2^32 (buffer loads)
    short tapmask[UNITS];   // bit kh*3+kw set iff that tap of this output pixel is inside X
    short row[UNITS];
    int q;
    SRC buf;
    static_assert(FLSIM_BUFLOAD || !SRC::SPLIT, "split operands use buffer loads");

    __device__ void setup(int m0, int tid) {
        q = tid & 3;
        if constexpr (FLSIM_BUFLOAD)
            buf.init(X, XL, (unsigned long)((M + ROWS_PER_IMG - 1) / ROWS_PER_IMG) * IH * IW * CI * 4);
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
            vb[j] = (unsigned)base[j] * 4u;
        }
    }
    __device__ void load(int ks, Unit (&r)[UNITS]) const {
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
                const bool ok = (tapmask[j] >> khkw) & 1;
                if constexpr (FLSIM_BUFLOAD)
                    r[j] = buf.ld_or0(vb[j] + (unsigned)off * 4u, ok);
                else
                    r[j] = ldg4_or0(X + base[j] + off, X, ok);
            }
        } else {
            const int k = ks * GK + 4 * q;          // CI == 4: one tap per lane quad
            const int khkw = k / CI;
            const int kh = khkw / 3;
            const long off = (long)(kh * IW + (khkw - 3 * kh)) * CI - 4 * q + (k - khkw * CI);
#pragma unroll
            for (int j = 0; j < UNITS; ++j) {
                const bool ok = khkw < 9 && ((tapmask[j] >> khkw) & 1);
                if constexpr (FLSIM_BUFLOAD)
                    r[j] = buf.ld_or0(vb[j] + (unsigned)off * 4u, ok);
                else
                    r[j] = ldg4_or0(X + base[j] + off, X, ok);
            }
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) store_unit<true, ROWS>(lds, row[j], q, r[j]);
    }
    // f(row, chunk, value, valid) for each staged unit (the split-bf16 kernel's plane stores)
    template <class F>
    __device__ void each_unit(const Unit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) f(row[j], q, r[j], true);
    }
};

// ---------------------------------------------------------------------------------------------
// Row-major matrix whose rows are the tile rows and whose reduction index is contiguous (KC):
// element (row, k) at P[row * ld + k].  Rows >= NR read as zero.  K must be a multiple of 16.
// ---------------------------------------------------------------------------------------------
template <int TR, int NT, class SRC = BufSrc>
struct RowsKC {
    using Unit = typename SRC::Unit;
    static_assert(!SRC::SM, "pixel-major operand");
    static constexpr int ROWS = TR;
    static constexpr bool KC = true;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    static_assert(NT % 4 == 0, "");
    static_assert(FLSIM_BUFLOAD || !SRC::SPLIT, "split operands use buffer loads");
    const float* P;
    const float* PL = nullptr;   // SRC = XsSrc: P is the HM part, PL the L part (split.h)
    long ld;
    int NR;
    const float* rowp[UNITS];
    unsigned rowb[UNITS];   // byte offset of the unit's row chunk, BUF_OOB past the matrix
    short row[UNITS];
    int q;
    SRC buf;
    __device__ void setup(int r0, int tid) {
        q = tid & 3;
        if constexpr (FLSIM_BUFLOAD) buf.init(P, PL, (unsigned long)NR * ld * 4);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            const int r = u >> 2;
            row[j] = (short)r;
            const bool ok = u < TOTAL && r0 + r < NR;
            rowp[j] = ok ? P + (long)(r0 + r) * ld + 4 * q : nullptr;
            rowb[j] = ok ? (unsigned)(((long)(r0 + r) * ld + 4 * q) * 4) : BUF_OOB;
        }
    }
    __device__ void load(int ks, Unit (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            if constexpr (FLSIM_BUFLOAD)
                r[j] = buf.ld(rowb[j] == BUF_OOB ? BUF_OOB : rowb[j] + (unsigned)(ks * GK * 4));
            else
                r[j] = ldg4_or0(rowp[j] + ks * GK, P, rowp[j] != nullptr);
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) store_unit<true, ROWS>(lds, row[j], q, r[j]);
    }
    // f(row, chunk, value, valid) for each staged unit (the split-bf16 kernel's plane stores)
    template <class F>
    __device__ void each_unit(const Unit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) f(row[j], q, r[j], true);
    }
};

// ---------------------------------------------------------------------------------------------
// k-major tile row of thread tid when TPR threads share a row.  ds_write_b128 is serviced in
// groups of 8 lanes on 32 banks (MI355X_MICROARCH.md, LDS table); with TPR = 4 (one-wave blocks)
// a group holds two rows, and rows a, a + 1 (stride STRIDE = 4 mod 8) overlap on 4 banks: a
// 2-way conflict on every store (conv2 weight gradient: SQ_LDS_BANK_CONFLICT 569 M cycles per
// launch, profiles/r03a/pmc).  Rows a and a + 4 sit 4 * STRIDE = 16 (mod 32) banks apart, so the
// two halves of each group take rows 4 apart.  The tile contents are unchanged.
// ---------------------------------------------------------------------------------------------
template <int TPR>
__device__ __forceinline__ int km_row(int tid) {
    if constexpr (TPR == 4) {
        const int g = tid >> 3;
        return (g & 3) + 4 * ((tid >> 2) & 1) + 8 * (g >> 2);
    } else {
        return tid / TPR;
    }
}

// ---------------------------------------------------------------------------------------------
// Row-major matrix whose ROWS are the reduction index (KM): element (k, col) at P[k * ld + col];
// the tile spans columns [c0, c0 + ROWS).  k >= NK or col >= NC read as zero (NC % 4 == 0).
// PO > 0: the rows are the pixels of PO x PO images and k walks only the top-left PV x PV
// window of each (k -> row img*PO*PO + oh*PO + ow): conv6's weight gradient skips the pixels
// the floor-mode pool never reads (their dZ is zero).
// ---------------------------------------------------------------------------------------------
template <int TR, int NT, int PO = 0, int PV = 0, class SRC = BufSrc>
struct RowsKM {
    using Unit = typename SRC::Unit;
    static_assert(!SRC::SM, "pixel-major operand");
    static constexpr int ROWS = TR;
    static constexpr bool KC = false;
    static constexpr int C4 = ROWS / 4;
    // thread -> (one k row, UNITS column chunks): the row's address (and for PO > 0 its window
    // split) is computed once per thread and k-step, not once per unit
    static constexpr int TPR = NT / GK;
    static_assert(NT % GK == 0, "");
    static constexpr int UNITS = (C4 + TPR - 1) / TPR;
    static_assert(FLSIM_BUFLOAD || !SRC::SPLIT, "split operands use buffer loads");
    const float* P;
    const float* PL = nullptr;   // SRC = XsSrc: P is the HM part, PL the L part (split.h)
    long ld;
    int NK;
    int NC;
    int krow;
    int c_off[UNITS];
    short c4[UNITS];
    SRC buf;
    __device__ void setup(int c0, int tid) {
        krow = km_row<TPR>(tid);
        if constexpr (FLSIM_BUFLOAD) {
            long rows = NK;
            if constexpr (PO > 0) rows = (long)((NK + PV * PV - 1) / (PV * PV)) * PO * PO;
            buf.init(P, PL, (unsigned long)rows * ld * 4);
        }
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int c = tid % TPR + TPR * j;
            c4[j] = (short)c;
            const int col = c0 + 4 * c;
            c_off[j] = (c < C4 && col < NC) ? col : -1;
        }
    }
    __device__ void load(int ks, Unit (&r)[UNITS]) const {
        const int k = ks * GK + krow;
        long row = k;
        if constexpr (PO > 0) {
            // window split: block-uniform base once (scalar), the thread's row by a carry and a
            // small division
            const unsigned img0 = (unsigned)(ks * GK) / (unsigned)(PV * PV);
            unsigned rem = (unsigned)(ks * GK) - img0 * (PV * PV) + krow, img = img0;
            static_assert(PV * PV >= GK, "window split assumes one image carry at most");
            if (rem >= (unsigned)(PV * PV)) { rem -= PV * PV; ++img; }
            const unsigned oh = SmallDiv<PV, PV * PV + GK>::div(rem);
            row = (long)img * (PO * PO) + oh * PO + (rem - oh * PV);
        }
        const bool rok = k < NK;
        if constexpr (FLSIM_BUFLOAD) {
            const unsigned rb = (unsigned)row * ((unsigned)ld * 4u);
#pragma unroll
            for (int j = 0; j < UNITS; ++j)
                r[j] = buf.ld_or0(rb + (unsigned)c_off[j] * 4u, rok && c_off[j] >= 0);
        } else {
            const float* rp = P + row * ld;
#pragma unroll
            for (int j = 0; j < UNITS; ++j) r[j] = ldg4_or0(rp + c_off[j], P, rok && c_off[j] >= 0);
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            store_km_or_spare<ROWS>(lds, C4 % TPR == 0 || c4[j] < C4, krow, c4[j], r[j]);
    }
    // f(k row, column chunk, value, valid) for each staged unit (split-bf16 plane stores; a
    // surplus unit has valid = false and goes to the plane's spare slot)
    template <class F>
    __device__ void each_unit(const Unit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) f(krow, c4[j], r[j], C4 % TPR == 0 || c4[j] < C4);
    }
};

// ---------------------------------------------------------------------------------------------
// B operand of the weight gradient: im2col(X) with the pixel as the reduction index (KM).
// Tile columns = kk = (kh*3 + kw) * CI + ci in [c0, c0 + ROWS); reduction rows = pixels p.
// VO > 0: p walks only the top-left VO x VO output window of each image (pairs with RowsKM's
// PV window).
// ---------------------------------------------------------------------------------------------
template <int IH, int IW, int CI, int PAD, int TR, int NT, int VO = 0, class SRC = BufSrc>
struct Im2colKM {
    using Unit = typename SRC::Unit;
    static constexpr int ROWS = TR;
    static constexpr bool KC = false;
    static constexpr int OH = VO > 0 ? VO : IH + 2 * PAD - 2;
    static constexpr int OW = VO > 0 ? VO : IW + 2 * PAD - 2;
    static constexpr int C4 = ROWS / 4;
    // thread -> (one pixel row of the tile, UNITS column chunks): the pixel split is done once
    // per thread and k-step, each unit only adds its tap
    static constexpr int TPR = NT / GK;
    static_assert(NT % GK == 0, "");
    static constexpr int UNITS = (C4 + TPR - 1) / TPR;
    static_assert(FLSIM_BUFLOAD || !SRC::SPLIT, "split operands use buffer loads");
    // floats between neighbouring pixels / from channel slice 0 to slice ci / 16 (SRC::SM)
    static constexpr int PIX = SRC::SM ? GK : CI;
    static constexpr int SLICE = SRC::SM ? IH * IW * GK : GK;
    static_assert(!SRC::SM || CI % GK == 0, "slice-major maps have whole 16-channel slices");
    const float* X;
    const float* XL = nullptr;   // SRC = XsSrc: X is the HM part, XL the L part (split.h)
    int M;  // total pixels
    int krow;
    int coff[UNITS];   // ((kh - PAD) * IW + kw - PAD) * PIX + channel offset: from pixel (oh, ow)
    short kh[UNITS], kw[UNITS];   // tap of the column; kh = -64 when it is padding
    short c4[UNITS];
    SRC buf;
    __device__ void setup(int c0, int tid) {
        krow = km_row<TPR>(tid);
        if constexpr (FLSIM_BUFLOAD)
            buf.init(X, XL, (unsigned long)((M + OH * OW - 1) / (OH * OW)) * IH * IW * CI * 4);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int c = tid % TPR + TPR * j;
            c4[j] = (short)c;
            const int kk = c0 + 4 * c;
            const int khkw = kk / CI;
            const int ci = kk - khkw * CI;
            const bool real = c < C4 && khkw < 9;
            kh[j] = (short)(real ? khkw / 3 : -64);
            kw[j] = (short)(khkw % 3);
            coff[j] = real ? ((khkw / 3 - PAD) * IW + (khkw % 3 - PAD)) * PIX + (ci / GK) * SLICE +
                                 ci % GK
                           : 0;
        }
    }
    __device__ void load(int ks, Unit (&r)[UNITS]) const {
        const int p = ks * GK + krow;
        const unsigned img0 = (unsigned)(ks * GK) / (unsigned)(OH * OW);   // block-uniform
        unsigned rem = (unsigned)(ks * GK) - img0 * (OH * OW) + krow, img = img0;
        if constexpr (OH * OW >= GK) {        // the thread's pixel is at most one image further
            if (rem >= (unsigned)(OH * OW)) { rem -= OH * OW; ++img; }
        } else {                              // tiny maps (VGG's 2x2): several images per k-step
            const unsigned q = SmallDiv<OH * OW, OH * OW + GK>::div(rem);
            img += q;
            rem -= q * (OH * OW);
        }
        const int oh = (int)SmallDiv<OW, OH * OW + GK>::div(rem);
        const int ow = (int)rem - oh * OW;
        const bool pok = p < M;
        if constexpr (FLSIM_BUFLOAD) {
            const unsigned xb = img * (unsigned)(IH * IW * CI * 4) + (unsigned)(oh * IW + ow) * (PIX * 4u);
#pragma unroll
            for (int j = 0; j < UNITS; ++j) {
                const int ih = oh + kh[j] - PAD, iw = ow + kw[j] - PAD;
                const bool ok = pok && (unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW;
                r[j] = buf.ld_or0(xb + (unsigned)coff[j] * 4u, ok);
            }
        } else {
            static_assert(!SRC::SM, "slice-major maps use buffer loads");
            const long xo = ((long)img * IH * IW + oh * IW + ow) * CI;
#pragma unroll
            for (int j = 0; j < UNITS; ++j) {
                const int ih = oh + kh[j] - PAD, iw = ow + kw[j] - PAD;
                const bool ok = pok && (unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW;
                r[j] = ldg4_or0(X + xo + coff[j], X, ok);
            }
        }
    }
    __device__ void store(float* lds, const f32x4 (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            store_km_or_spare<ROWS>(lds, C4 % TPR == 0 || c4[j] < C4, krow, c4[j], r[j]);
    }
    // f(k row, column chunk, value, valid) for each staged unit (split-bf16 plane stores; a
    // surplus unit has valid = false and goes to the plane's spare slot)
    template <class F>
    __device__ void each_unit(const Unit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j) f(krow, c4[j], r[j], C4 % TPR == 0 || c4[j] < C4);
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
            st_nt4(reinterpret_cast<float*>(dst + q), *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c));
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
    // the pass's mask operand is loaded for BATCH of a thread's units before any is used (one
    // HBM round trip per pass; profiles/r03s: conv2's data gradient 6.15 -> 6.00 ms)
    static constexpr int BATCH = 8;
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int N4 = NC / 4;
        f32x4* dst = reinterpret_cast<f32x4*>(Y + (long)m0 * NC);
        const f32x4* a4 = reinterpret_cast<const f32x4*>(act + (long)m0 * NC);
        const int total = rows * N4;
        auto unit = [&](int q, f32x4 a) {
            const int r = q / N4, c = q - r * N4;
            const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
            f32x4 o;
            o.x = a.x > 0.f ? t.x : 0.f;
            o.y = a.y > 0.f ? t.y : 0.f;
            o.z = a.z > 0.f ? t.z : 0.f;
            o.w = a.w > 0.f ? t.w : 0.f;
            st_nt4(reinterpret_cast<float*>(dst + q), o);
        };
        f32x4 av[BATCH];
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) av[it] = a4[q];
        }
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) unit(q, av[it]);
        }
        for (int q = tid + BATCH * nt; q < total; q += nt) unit(q, a4[q]);
    }
};

// gradient of a dropout(relu(.)) output: Y = acc * scale * (act > 0)  (act = dropped output)
struct EpiDropMask {
    static constexpr bool ASUM = false;
    float* Y;
    const float* act;
    float scale;
    int M, N;
    __device__ f32x4 pre4(int m, int n, int) const {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        if (n < N) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (m + r < M) a[r] = act[(long)(m + r) * N + n];
        }
        return a;
    }
    __device__ void apply4p(int m, int n, int z, f32x4 v, f32x4 a) const {
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (m + r < M) Y[(long)(m + r) * N + n] = a[r] > 0.f ? v[r] * scale : 0.f;
    }
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

// EpiDropMask with PRE: the GEMM kernels load the mask values of a whole fragment row (pre4)
// before storing any of it (apply4p) -- a store to Y may alias act for the compiler, which
// otherwise keeps each fragment's loads behind the previous fragment's stores.  profiles/r03s:
// linear1's data gradient 1.33 -> 1.23 ms; the same for EpiMask (conv4/conv6 data gradients) and
// EpiSlabAcc (conv5 weight gradient) measured 2-7 % slower, their larger tiles lose occupancy to
// the extra VGPRs, so only the linear data gradients use it
struct EpiDropMaskPre : EpiDropMask {
    static constexpr bool PRE = true;
};

// EpiDropMask fused with the 2x2 max-pool backward of the layer below (PerformantNet1 pool1 and
// pool2, models.py:31-32,35-36): the masked gradient g of pooled element (m, n) goes straight to
// the full-resolution dZ at the position the forward's argmax recorded (idx, 2 dy + dx), zeros to
// the other three, instead of being written as gy and scattered by k_pool_scatter.  The values
// are the same floats; the pooled gradient never goes through HBM.  m = (img * PH + ph) * PW + pw;
// dZ is [img][2 PH][2 PW][NC] (no floor-mode border: both maps are even).  The tile is staged
// through LDS (gemm_core.h STAGED, the block covers all NC channels): a thread takes (pooled pixel,
// 4 channels) and writes the four positions of its 2x2 window as float4 pieces of whole dZ pixel
// rows (profiles/r02j: 16 scalar stores per lane from the accumulator layout were 10 % slower on
// conv3's data gradient).  BATCH: how many of a thread's units have their pooled activations and
// argmax bytes loaded before any is used (one HBM round trip per pass, not one per unit); 0 keeps
// one unit at a time (profiles/r03s: batching is 2 % faster on conv3's data gradient, 2 % slower
// on conv5's, whose 96-column tile has more VGPRs live at this point)
template <int PH, int PW, int NC, int BATCH = 8>
struct EpiDropScatterRows {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr int NCOL = NC;
    static_assert(NC % 4 == 0, "float4 rows");
    float* dZ;
    const float* act;
    const uint8_t* idx;
    float scale;
    int M;
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int N4 = NC / 4;
        const f32x4* a4 = reinterpret_cast<const f32x4*>(act + (long)m0 * NC);
        const uint32_t* i4 = reinterpret_cast<const uint32_t*>(idx + (long)m0 * NC);
        const int total = rows * N4;
        int q0 = tid;
        if constexpr (BATCH > 0) {
            f32x4 av[BATCH];
            uint32_t iv[BATCH];
#pragma unroll
            for (int it = 0; it < BATCH; ++it) {
                const int q = tid + it * nt;
                if (q < total) {
                    av[it] = a4[q];
                    iv[it] = i4[q];
                }
            }
#pragma unroll
            for (int it = 0; it < BATCH; ++it) {
                const int q = tid + it * nt;
                if (q < total) unit(tile, ld, m0, q, av[it], iv[it]);
            }
            q0 = tid + BATCH * nt;
        }
        for (int q = q0; q < total; q += nt) unit(tile, ld, m0, q, a4[q], i4[q]);
    }
    __device__ void unit(const float* tile, int ld, int m0, int q, f32x4 a, uint32_t id) const {
        constexpr int N4 = NC / 4;
        {
            const int r = q / N4, c = q - r * N4;
            const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
            f32x4 g;
            g.x = a.x > 0.f ? t.x * scale : 0.f;
            g.y = a.y > 0.f ? t.y * scale : 0.f;
            g.z = a.z > 0.f ? t.z * scale : 0.f;
            g.w = a.w > 0.f ? t.w * scale : 0.f;
            const unsigned mm = (unsigned)(m0 + r);
            const unsigned img = mm / (PH * PW);
            const unsigned rem = mm - img * (PH * PW);
            const unsigned ph = rem / PW, pw = rem - ph * PW;
            float* base = dZ + (((long)img * (2 * PH) + 2 * ph) * (2 * PW) + 2 * pw) * NC + 4 * c;
#pragma unroll
            for (int pos = 0; pos < 4; ++pos) {
                f32x4 o;
                o.x = (id & 0xffu) == (uint32_t)pos ? g.x : 0.f;
                o.y = ((id >> 8) & 0xffu) == (uint32_t)pos ? g.y : 0.f;
                o.z = ((id >> 16) & 0xffu) == (uint32_t)pos ? g.z : 0.f;
                o.w = (id >> 24) == (uint32_t)pos ? g.w : 0.f;
                st_nt4(base + ((pos >> 1) * (2 * PW) + (pos & 1)) * (long)NC, o);
            }
        }
    }
};

// split-K partial slab, accumulated across chunks: S[z][m][n] += acc   (one owner per element);
// with Bsl != nullptr also the bias gradient Bsl[z][m] += column sum of the dZ tile (ASUM)
// zinit: slab rows z >= zinit have not been written yet this epoch (begin_epoch does not clear
// the slabs): those blocks store instead of accumulating
struct EpiSlabAcc {
    static constexpr bool ASUM = true;
    static constexpr bool ASUM_MFMA = true;     // split-bf16 kernels: the column sum on the MFMA
    float* S;
    int M, N;
    long zstride;
    float* Bsl;
    int zinit = 0x7fffffff;
    __device__ void asum(int m, int z, float v) const {
        if (!Bsl || m >= M) return;
        if (z < zinit) Bsl[(long)z * M + m] += v;
        else Bsl[(long)z * M + m] = v;
    }
    __device__ void apply4(int m, int n, int z, f32x4 v) const {
        if (n >= N) return;
        float* base = S + z * zstride;
        if (z < zinit) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (m + r < M) base[(long)(m + r) * N + n] += v[r];
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (m + r < M) base[(long)(m + r) * N + n] = v[r];
        }
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

// EpiSlabStore whose x6 GEMM accumulates each k-step fresh (gemm_x6.h X6Fresh)
struct EpiSlabStoreFresh : EpiSlabStore {
    static constexpr bool X6_FRESH = true;
};

}  // namespace flsim
