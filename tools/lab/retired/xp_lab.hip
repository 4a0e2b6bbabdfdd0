// Planar split-bf16 GEMM lab (development tool, not part of libflsim.so).
//
// gemm_x6_kernel pairs two split terms in each bf16 MFMA (k slots = 4 k x 2 terms), so its LDS
// holds [h|m] / [h|l] / [l|h] combination planes: 8 B per operand element written and read.  Here
// every MFMA takes 8 consecutive k of ONE term (k slots = 8 k): the LDS holds the three parts as
// three planes h, m, l (6 B per element), a stage is 32 k deep, and the six products of a 16x16
// tile are six MFMAs per stage (the same count per k), accumulated fresh and added once.  The
// operands come from planar split tensors (H, M, L: three bf16 copies of the fp32 layout), so a
// staged unit is 8 consecutive k of one row = three 16-B loads and three 16-B LDS stores.
// Compared against gemm_x6_kernel over the same data in the HM + L form (xs) on PerformantNet1's
// conv shapes at 16,384 samples: time, fp32-equivalent TF/s, max |difference| / max |y|.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//         -I fl-distributed-delay_amd/csrc tools/lab/xp_lab.hip -o tools/lab/xp_lab
#include <cmath>

#include "gemm_x6.h"
#include "lab_common.h"

struct Planes {
    __bf16* h;
    __bf16* m;
    __bf16* l;
};

struct XpUnit {
    f32x4 h, m, l;
};

struct PlaneSrc {
    __amdgpu_buffer_rsrc_t rh, rm, rl;
    __device__ void init(const Planes& p, unsigned long elems) {
        rh = raw_rsrc(p.h, elems * 2);
        rm = raw_rsrc(p.m, elems * 2);
        rl = raw_rsrc(p.l, elems * 2);
    }
    __device__ XpUnit ld(unsigned byte_off) const {
        XpUnit u;
        u.h = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rh, byte_off, 0, 0));
        u.m = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rm, byte_off, 0, 0));
        u.l = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, byte_off, 0, 0));
        return u;
    }
};

// im2col rows (output pixels) x 32-k stages; k in 16-blocks b = (ci / 16) * 9 + tap (the
// product's channel-slice-major order), a stage = blocks 2 ks and 2 ks + 1, a unit = 8 channels
template <int IH, int IW, int CI, int PAD, int TR, int NT, int OHX = 0>
struct Im2colP {
    static constexpr int ROWS = TR;
    static constexpr int OH = OHX > 0 ? OHX : IH + 2 * PAD - 2;
    static constexpr int OW = OHX > 0 ? OHX : IW + 2 * PAD - 2;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    static constexpr int NB = 9 * CI / 16;
    static_assert(CI % 16 == 0, "");
    Planes X;
    int M;
    unsigned vb[UNITS];
    short tapmask[UNITS];
    short row[UNITS];
    int q;
    PlaneSrc src;
    __device__ void setup(int m0, int tid) {
        q = tid & 3;
        src.init(X, (unsigned long)((M + OH * OW - 1) / (OH * OW)) * IH * IW * CI);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            const int r = u >> 2;
            row[j] = (short)r;
            const int m = m0 + r;
            long base = 0;
            int msk = 0;
            if (u < TOTAL && m < M) {
                const int nimg = m / (OH * OW);
                const int rem = m - nimg * (OH * OW);
                const int oh = rem / OW, ow = rem - oh * OW;
                base = ((long)nimg * IH * IW + (long)(oh - PAD) * IW + (ow - PAD)) * CI + 8 * (q & 1);
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int ih = oh + t / 3 - PAD, iw = ow + t % 3 - PAD;
                    if ((unsigned)ih < (unsigned)IH && (unsigned)iw < (unsigned)IW) msk |= 1 << t;
                }
            }
            vb[j] = (unsigned)base * 2u;
            tapmask[j] = (short)msk;
        }
    }
    __device__ void load(int ks, XpUnit (&r)[UNITS]) const {
        const int b = 2 * ks + (q >> 1);
        const int cs = b / 9, tap = b - 9 * cs;
        const int kh = tap / 3;
        const unsigned off = (unsigned)(((kh * IW + (tap - 3 * kh)) * CI + 16 * cs) * 2);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const bool ok = b < NB && ((tapmask[j] >> tap) & 1);
            r[j] = src.ld(ok ? vb[j] + off : BUF_OOB);
        }
    }
    template <class F>
    __device__ void each_unit(const XpUnit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) f(row[j], q, r[j]);
    }
};

// packed weights [NR][KP32] planar, KP32 = the K blocks rounded to whole stages (zero padded)
template <int TR, int NT>
struct RowsP {
    static constexpr int ROWS = TR;
    static constexpr int TOTAL = ROWS * 4;
    static constexpr int UNITS = (TOTAL + NT - 1) / NT;
    Planes P;
    int ld, NR;
    unsigned rowb[UNITS];
    short row[UNITS];
    int q;
    PlaneSrc src;
    __device__ void setup(int r0, int tid) {
        q = tid & 3;
        src.init(P, (unsigned long)NR * ld);
#pragma unroll
        for (int j = 0; j < UNITS; ++j) {
            const int u = tid + j * NT;
            const int r = u >> 2;
            row[j] = (short)r;
            rowb[j] = (u < TOTAL && r0 + r < NR) ? (unsigned)(((long)(r0 + r) * ld + 8 * q) * 2)
                                                 : BUF_OOB;
        }
    }
    __device__ void load(int ks, XpUnit (&r)[UNITS]) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            r[j] = src.ld(rowb[j] == BUF_OOB ? BUF_OOB : rowb[j] + (unsigned)(ks * 64));
    }
    template <class F>
    __device__ void each_unit(const XpUnit (&r)[UNITS], F&& f) const {
#pragma unroll
        for (int j = 0; j < UNITS; ++j)
            if (TOTAL % NT == 0 || row[j] < ROWS) f(row[j], q, r[j]);
    }
};

template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_xp_kernel(AL al, BL bl, EPI epi, int nks, int tiles_m, int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    constexpr int PA = KCTile<BM>::FLOATS, PB = KCTile<BN>::FLOATS;   // one plane (64 B rows)
    constexpr int BUF = 3 * (PA + PB);
    static_assert(2 * BUF * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int nb = gridDim.x, b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % tiles_n, tm = L / tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    al.setup(m0, tid);
    bl.setup(n0, tid);
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    XpUnit ra[AL::UNITS], rb[BL::UNITS];
    auto stage = [&](float* s) {
        al.each_unit(ra, [&](int row, int c, const XpUnit& v) {
            store_unit<true, BM>(s, row, c, v.h);
            store_unit<true, BM>(s + PA, row, c, v.m);
            store_unit<true, BM>(s + 2 * PA, row, c, v.l);
        });
        float* sb = s + 3 * PA;
        bl.each_unit(rb, [&](int row, int c, const XpUnit& v) {
            store_unit<true, BN>(sb, row, c, v.h);
            store_unit<true, BN>(sb + PB, row, c, v.m);
            store_unit<true, BN>(sb + 2 * PB, row, c, v.l);
        });
    };
    al.load(0, ra);
    bl.load(0, rb);
    stage(lds);
    if (nks > 1) {
        al.load(1, ra);
        bl.load(1, rb);
    }
    __syncthreads();
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    int cur = 0;
    for (int ks = 0; ks < nks; ++ks) {
        if (ks + 1 < nks) {
            stage(lds + (cur ^ 1) * BUF);
            if (ks + 2 < nks) {
                al.load(ks + 2, ra);
                bl.load(ks + 2, rb);
            }
        }
        const float* A = lds + cur * BUF;
        const float* B = A + 3 * PA;
        f32x4 bh[FN], bm[FN], bll[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int r0 = wn * 16 * FN + 16 * j;
            bh[j] = read_frag<true, BN>(B, r0, lane);
            bm[j] = read_frag<true, BN>(B + PB, r0, lane);
            bll[j] = read_frag<true, BN>(B + 2 * PB, r0, lane);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int r0 = wm * 16 * FM + 16 * i;
            const f32x4 ah = read_frag<true, BM>(A, r0, lane);
            const f32x4 am = read_frag<true, BM>(A + PA, r0, lane);
            const f32x4 al_ = read_frag<true, BM>(A + 2 * PA, r0, lane);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                f32x4 t = mfma_x32(ah, bll[j], f32x4{0.f, 0.f, 0.f, 0.f});
                t = mfma_x32(al_, bh[j], t);
                t = mfma_x32(ah, bm[j], t);
                t = mfma_x32(am, bh[j], t);
                t = mfma_x32(am, bm[j], t);
                t = mfma_x32(ah, bh[j], t);
                acc[i][j] = acc[i][j] + t;
            }
        }
        __syncthreads();
        cur ^= 1;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
            const int n = n0 + wn * 16 * FN + 16 * j + (lane & 15);
            epi.apply4(m, n, 0, acc[i][j]);
        }
}

static __global__ void k_to_xs(const float* x, float* hm, float* l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(x)[u]);
}
static __global__ void k_to_planes(const float* x, __bf16* h, __bf16* m, __bf16* l, long n) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const __bf16 hh = (__bf16)x[e];
    const float r1 = x[e] - (float)hh;
    const __bf16 mm = (__bf16)r1;
    h[e] = hh;
    m[e] = mm;
    l[e] = (__bf16)(r1 - (float)mm);
}
// weights [NR][K] fp32 -> planar [NR][KP32] (zero padded)
static __global__ void k_w_planes(const float* w, int NR, int K, int KP32, __bf16* h, __bf16* m,
                                  __bf16* l) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)NR * KP32) return;
    const int r = (int)(e / KP32), k = (int)(e - (long)r * KP32);
    const float x = k < K ? w[(long)r * K + k] : 0.f;
    const __bf16 hh = (__bf16)x;
    const float r1 = x - (float)hh;
    const __bf16 mm = (__bf16)r1;
    h[e] = hh;
    m[e] = mm;
    l[e] = (__bf16)(r1 - (float)mm);
}

static Planes planes(size_t n) {
    Planes p;
    CK(hipMalloc(&p.h, n * 2));
    CK(hipMalloc(&p.m, n * 2));
    CK(hipMalloc(&p.l, n * 2));
    return p;
}

template <class K, class... Args>
static double timeit(K kern, dim3 g, int nt, Args... args) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = getenv("LAB_ITERS") ? atoi(getenv("LAB_ITERS")) : 5;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, g, dim3(nt), 0, 0, args...);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, g, dim3(nt), 0, 0, args...);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / it;
}

static double maxrel(const float* a, const float* b, size_t n) {
    std::vector<float> h0(n), h1(n);
    CK(hipMemcpy(h0.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), b, n * 4, hipMemcpyDeviceToHost));
    double d = 0, y = 0;
    for (size_t i = 0; i < n; ++i) {
        d = std::max(d, fabs((double)h0[i] - h1[i]));
        y = std::max(y, (double)fabs(h0[i]));
    }
    return d / (y > 0 ? y : 1);
}

struct Bufs {
    float* X;
    float *Xhm, *Xl;
    Planes Xp;
    float* W;
    float *Whm, *Wl;
    Planes Wp;
    float* b;
    float *Y0, *Y1;
};

template <int IH, int CI, int PAD, int OHX, int CO, int FM, int FN, int WM, int WN, int PFM,
          int PFN, int PWM, int PWN>
static void conv(const char* tag, const Bufs& B, int S) {
    const int KP = 9 * CI;
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using ALs = Im2colKC<IH, IH, CI, PAD, BM, NT, false, OHX, XsSrc>;
    using BLs = RowsKC<BN, NT, XsSrc>;
    ALs als;
    als.X = B.Xhm;
    als.XL = B.Xl;
    als.M = S * ALs::OH * ALs::OW;
    const int M = als.M;
    BLs bls;
    bls.P = B.Whm;
    bls.PL = B.Wl;
    bls.ld = KP;
    bls.NR = CO;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const double t0 = timeit(gemm_x6_kernel<FM, FN, WM, WN, ALs, BLs, EpiBiasRelu>, dim3(tm * tn),
                             NT, als, bls, EpiBiasRelu{B.Y0, B.b, M, CO}, KP / GK, KP / GK, tm, tn);
    // planar
    constexpr int PNT = 64 * PWM * PWN, PBM = 16 * PFM * PWM, PBN = 16 * PFN * PWN;
    constexpr int NB = 9 * CI / 16;
    const int nks = (NB + 1) / 2, KP32 = 32 * nks;
    // weights re-packed planar with the stage padding (the lab's W is [CO][KP] fp32)
    hipLaunchKernelGGL(k_w_planes, dim3(ceil_div((long)CO * KP32, 256)), dim3(256), 0, 0, B.W, CO,
                       KP, KP32, B.Wp.h, B.Wp.m, B.Wp.l);
    using ALp = Im2colP<IH, IH, CI, PAD, PBM, PNT, OHX>;
    using BLp = RowsP<PBN, PNT>;
    ALp alp;
    alp.X = B.Xp;
    alp.M = M;
    BLp blp;
    blp.P = B.Wp;
    blp.ld = KP32;
    blp.NR = CO;
    const int ptm = ceil_div(M, PBM), ptn = ceil_div(CO, PBN);
    const double t1 = timeit(gemm_xp_kernel<PFM, PFN, PWM, PWN, ALp, BLp, EpiBiasRelu>,
                             dim3(ptm * ptn), PNT, alp, blp, EpiBiasRelu{B.Y1, B.b, M, CO}, nks,
                             ptm, ptn);
    const double flops = 2.0 * M * CO * KP;
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    printf("%-10s xs %3dx%3d %7.3f ms %6.1f | xp %3dx%3d %7.3f ms %6.1f TF/s (x%.2f) | "
           "max|d|/max|y| %.2e\n", tag, BM, BN, t0, tf(t0), PBM, PBN, t1, tf(t1), t0 / t1,
           maxrel(B.Y0, B.Y1, (size_t)M * CO));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 22 * 22 * 96;       // the largest input used below (dg4)
    Bufs B;
    B.X = dalloc(big, 1.f);
    CK(hipMalloc(&B.Xhm, big * 4));
    CK(hipMalloc(&B.Xl, big * 2));
    hipLaunchKernelGGL(k_to_xs, dim3(ceil_div((long)big / 4, 256)), dim3(256), 0, 0, B.X, B.Xhm,
                       B.Xl, (long)big / 4);
    B.Xp = planes(big);
    hipLaunchKernelGGL(k_to_planes, dim3(ceil_div((long)big, 256)), dim3(256), 0, 0, B.X, B.Xp.h,
                       B.Xp.m, B.Xp.l, (long)big);
    const size_t wn = 192 * 1728;
    B.W = dalloc(wn, 0.05f);
    CK(hipMalloc(&B.Whm, wn * 4));
    CK(hipMalloc(&B.Wl, wn * 2));
    hipLaunchKernelGGL(k_to_xs, dim3(ceil_div((long)wn / 4, 256)), dim3(256), 0, 0, B.W, B.Whm,
                       B.Wl, (long)wn / 4);
    B.Wp = planes(192 * 1760);
    B.b = dalloc(256, 0.01f);
    const size_t ybig = big;             // S * 22 * 22 * 96: the largest output (fwd4)
    B.Y0 = dalloc(ybig, 0.f);
    B.Y1 = dalloc(ybig, 0.f);
    CK(hipDeviceSynchronize());
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define C(tag, IH, CI, PAD, OHX, CO, FM, FN, WM, WN, PFM, PFN, PWM, PWN) \
    if (want(tag)) conv<IH, CI, PAD, OHX, CO, FM, FN, WM, WN, PFM, PFN, PWM, PWN>(tag, B, S);
    C("fwd6 a", 13, 192, 2, 0, 192, 4, 6, 4, 2, 4, 4, 4, 2)
    C("fwd6 b", 13, 192, 2, 0, 192, 4, 6, 4, 2, 3, 6, 4, 2)
    C("fwd6 c", 13, 192, 2, 0, 192, 4, 6, 4, 2, 2, 6, 4, 2)
    C("fwd6 d", 13, 192, 2, 0, 192, 4, 6, 4, 2, 4, 6, 2, 2)
    C("dg6 a", 14, 192, 0, 13, 192, 4, 6, 4, 2, 4, 4, 4, 2)
    C("dg6 b", 14, 192, 0, 13, 192, 4, 6, 4, 2, 3, 6, 4, 2)
    C("fwd4 a", 20, 96, 2, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    C("fwd4 b", 20, 96, 2, 0, 96, 4, 3, 4, 2, 4, 6, 4, 1)
    C("dg4 a", 22, 96, 0, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    C("dg3 a", 20, 96, 0, 0, 48, 8, 3, 4, 1, 4, 3, 4, 1)
    C("dg3 b", 20, 96, 0, 0, 48, 8, 3, 4, 1, 2, 3, 8, 1)
    return 0;
}
