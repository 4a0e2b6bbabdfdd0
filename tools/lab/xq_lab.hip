// Planar-LDS split-bf16 GEMM lab (development tool, not part of libflsim.so): gemm_x6q_kernel
// (gemm_x6q.h: three plain planes per operand tile, 32-k stages, single-term MFMAs) against
// gemm_x6_kernel (combination planes, 16-k steps), both over split operands (HM + L tensors, the
// product's form), on PerformantNet1's conv forward / data-gradient shapes at 16,384 samples.
// The two sum in different orders: the line prints max |difference| / max |y|.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//         -I fl-distributed-delay_amd/csrc tools/lab/xq_lab.hip -o tools/lab/xq_lab
#include <cmath>

#include "gemm_x6q.h"
#include "lab_common.h"

static __global__ void k_to_xs(const float* x, float* hm, float* l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(x)[u]);
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
    float *Xhm, *Xl, *Whm, *Wl, *b, *Y0, *Y1;
};

template <int IH, int CI, int PAD, int OHX, int CO, int FM, int FN, int WM, int WN, int QFM,
          int QFN, int QWM, int QWN>
static void conv(const char* tag, const Bufs& B, int S) {
    const int KP = 9 * CI;
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT, false, OHX, XsSrc>;
    using BL = RowsKC<BN, NT, XsSrc>;
    AL al;
    al.X = B.Xhm;
    al.XL = B.Xl;
    al.M = S * AL::OH * AL::OW;
    const int M = al.M;
    BL bl;
    bl.P = B.Whm;
    bl.PL = B.Wl;
    bl.ld = KP;
    bl.NR = CO;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const double t0 = timeit(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>, dim3(tm * tn),
                             NT, al, bl, EpiBiasRelu{B.Y0, B.b, M, CO}, KP / GK, KP / GK, tm, tn);
    constexpr int QNT = 64 * QWM * QWN, QBM = 16 * QFM * QWM, QBN = 16 * QFN * QWN;
    using ALq = Im2colKC<IH, IH, CI, PAD, QBM, QNT, false, OHX, XsSrc>;
    using BLq = RowsKC<QBN, QNT, XsSrc>;
    ALq alq;
    alq.X = B.Xhm;
    alq.XL = B.Xl;
    alq.M = M;
    BLq blq;
    blq.P = B.Whm;
    blq.PL = B.Wl;
    blq.ld = KP;
    blq.NR = CO;
    const int qtm = ceil_div(M, QBM), qtn = ceil_div(CO, QBN);
    const double t1 = timeit(gemm_x6q_kernel<QFM, QFN, QWM, QWN, ALq, BLq, EpiBiasRelu>,
                             dim3(qtm * qtn), QNT, alq, blq, EpiBiasRelu{B.Y1, B.b, M, CO},
                             KP / GK, KP / GK, qtm, qtn);
    const double flops = 2.0 * M * CO * KP;
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    printf("%-10s x6 %3dx%3d %7.3f ms %6.1f | x6q %3dx%3d %7.3f ms %6.1f TF/s (x%.2f) | "
           "max|d|/max|y| %.2e\n", tag, BM, BN, t0, tf(t0), QBM, QBN, t1, tf(t1), t0 / t1,
           maxrel(B.Y0, B.Y1, (size_t)M * CO));
    fflush(stdout);
}

// weight gradient (pad 1 convolution of X): slab[z][co][kk] = sum over the split's pixels of
// dz[p][co] im2col(X)[p][kk], both operands split (RowsKM / Im2colKM over HM + L)
template <int IH, int CI, int CO, int Z, int FM, int FN, int WM, int WN, int QFM, int QFN, int QWM,
          int QWN>
static void wgrad(const char* tag, const Bufs& B, float* S0, float* S1, float* B0, float* B1,
                  int S) {
    constexpr int PAD = 1;
    const int KP = 9 * CI;
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = RowsKM<BM, NT, 0, 0, XsSrc>;
    using BL = Im2colKM<IH, IH, CI, PAD, BN, NT, 0, XsSrc>;
    const int M = S * BL::OH * BL::OW;
    AL al;
    al.P = B.Xhm;
    al.PL = B.Xl;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = B.Xhm;
    bl.XL = B.Xl;
    bl.M = M;
    const int ks = ceil_div(M, GK);
    const int per = ceil_div(ks, Z);
    const int tm = ceil_div(CO, BM), tn = ceil_div(KP, BN);
    EpiSlabAcc e0{S0, CO, KP, (long)CO * KP, B0, 0};
    const double t0 = timeit(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>,
                             dim3(tm * tn * Z), NT, al, bl, e0, ks, per, tm, tn);
    constexpr int QNT = 64 * QWM * QWN, QBM = 16 * QFM * QWM, QBN = 16 * QFN * QWN;
    using ALq = RowsKM<QBM, QNT, 0, 0, XsSrc>;
    using BLq = Im2colKM<IH, IH, CI, PAD, QBN, QNT, 0, XsSrc>;
    ALq alq;
    alq.P = B.Xhm;
    alq.PL = B.Xl;
    alq.ld = CO;
    alq.NK = M;
    alq.NC = CO;
    BLq blq;
    blq.X = B.Xhm;
    blq.XL = B.Xl;
    blq.M = M;
    const int qtm = ceil_div(CO, QBM), qtn = ceil_div(KP, QBN);
    const int qper = 2 * ceil_div(ks, 2 * Z);             // whole 32-k stages per split
    EpiSlabAcc e1{S1, CO, KP, (long)CO * KP, B1, 0};
    const double t1 = timeit(gemm_x6q_kernel<QFM, QFN, QWM, QWN, ALq, BLq, EpiSlabAcc>,
                             dim3(qtm * qtn * Z), QNT, alq, blq, e1, ks, qper, qtm, qtn);
    // per-split slabs differ in their split boundaries; compare the slab sums over z
    auto zsum = [&](const float* sl, long n, int zz) {
        std::vector<float> h((size_t)zz * n);
        CK(hipMemcpy(h.data(), sl, h.size() * 4, hipMemcpyDeviceToHost));
        std::vector<double> o(n, 0.0);
        for (int z = 0; z < zz; ++z)
            for (long i = 0; i < n; ++i) o[i] += h[(size_t)z * n + i];
        return o;
    };
    const long n = (long)CO * KP;
    const std::vector<double> a = zsum(S0, n, Z), b = zsum(S1, n, Z);
    double d = 0, y = 0;
    for (long i = 0; i < n; ++i) {
        d = std::max(d, fabs(a[i] - b[i]));
        y = std::max(y, fabs(a[i]));
    }
    const double flops = 2.0 * M * CO * KP;
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    printf("%-10s x6 %3dx%3d %7.3f ms %6.1f | x6q %3dx%3d %7.3f ms %6.1f TF/s (x%.2f) | "
           "slab sum max|d|/max %.2e\n", tag, BM, BN, t0, tf(t0), QBM, QBN, t1, tf(t1), t0 / t1,
           d / (y > 0 ? y : 1));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 22 * 22 * 96;
    Bufs B;
    float* X = dalloc(big, 1.f);
    CK(hipMalloc(&B.Xhm, big * 4));
    CK(hipMalloc(&B.Xl, big * 2));
    hipLaunchKernelGGL(k_to_xs, dim3(ceil_div((long)big / 4, 256)), dim3(256), 0, 0, X, B.Xhm,
                       B.Xl, (long)big / 4);
    const size_t wn = 192 * 1728;
    float* W = dalloc(wn, 0.05f);
    CK(hipMalloc(&B.Whm, wn * 4));
    CK(hipMalloc(&B.Wl, wn * 2));
    hipLaunchKernelGGL(k_to_xs, dim3(ceil_div((long)wn / 4, 256)), dim3(256), 0, 0, W, B.Whm,
                       B.Wl, (long)wn / 4);
    B.b = dalloc(256, 0.01f);
    const size_t ybig = big;             // S * 22 * 22 * 96: the largest output (fwd4)
    B.Y0 = dalloc(ybig, 0.f);
    B.Y1 = dalloc(ybig, 0.f);
    CK(hipDeviceSynchronize());
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define C(tag, IH, CI, PAD, OHX, CO, FM, FN, WM, WN, QFM, QFN, QWM, QWN) \
    if (want(tag)) conv<IH, CI, PAD, OHX, CO, FM, FN, WM, WN, QFM, QFN, QWM, QWN>(tag, B, S);
    C("fwd6 a", 13, 192, 2, 0, 192, 4, 6, 4, 2, 4, 4, 4, 2)       // 256x128 8w
    C("fwd6 b", 13, 192, 2, 0, 192, 4, 6, 4, 2, 3, 6, 4, 2)       // 192x192 8w
    C("fwd6 c", 13, 192, 2, 0, 192, 4, 6, 4, 2, 4, 6, 2, 2)       // 128x192 4w
    C("fwd6 d", 13, 192, 2, 0, 192, 4, 6, 4, 2, 4, 3, 4, 2)       // 256x96 8w
    C("dg6 a", 14, 192, 0, 13, 192, 4, 6, 4, 2, 4, 4, 4, 2)
    C("dg6 b", 14, 192, 0, 13, 192, 4, 6, 4, 2, 3, 6, 4, 2)
    C("fwd5 a", 11, 96, 2, 0, 192, 4, 6, 4, 2, 4, 4, 4, 2)
    C("dg5 a", 13, 192, 0, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    C("fwd4 a", 20, 96, 2, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    C("dg4 a", 22, 96, 0, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    C("fwd3 a", 18, 48, 2, 0, 96, 4, 3, 4, 2, 4, 3, 4, 2)
    const size_t slabn = (size_t)256 * 192 * 1728;
    float* S0 = dalloc(slabn, 0.f);
    float* S1 = dalloc(slabn, 0.f);
    float* B0 = dalloc(1024 * 192, 0.f);
    float* B1 = dalloc(1024 * 192, 0.f);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN, QFM, QFN, QWM, QWN) \
    if (want(tag)) wgrad<IH, CI, CO, Z, FM, FN, WM, WN, QFM, QFN, QWM, QWN>(tag, B, S0, S1, B0, \
                                                                           B1, S);
    G("wg6 a", 13, 192, 192, 256, 6, 3, 2, 2, 6, 3, 2, 2)
    G("wg6 b", 13, 192, 192, 256, 6, 3, 2, 2, 3, 3, 2, 2)
    G("wg5 a", 11, 96, 192, 512, 6, 3, 2, 2, 6, 3, 2, 2)
    G("wg5 b", 11, 96, 192, 512, 6, 3, 2, 2, 3, 3, 2, 2)
    G("wg4 a", 20, 96, 96, 1024, 3, 3, 2, 2, 3, 3, 2, 2)
    return 0;
}
