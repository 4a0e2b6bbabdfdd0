// GEMM tile-configuration lab (development tool, not part of libflsim.so): times the worker-
// batched conv GEMMs of PerformantNet1 at chunk size S = 4096 samples for several tile shapes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/gemm_lab.hip -o tools/lab/gemm_lab
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "gemm_variants.h"
#include "gemm_glds.h"

using namespace flsim;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float* dalloc(size_t n, float scale) {
    float* p;
    CK(hipMalloc(&p, n * 4));
    std::vector<float> h(n < (1u << 24) ? n : (1u << 24));
    for (size_t i = 0; i < h.size(); ++i) h[i] = scale * ((float)((i * 2654435761u) % 1000) / 500.f - 1.f);
    for (size_t o = 0; o < n; o += h.size())
        CK(hipMemcpy(p + o, h.data(), 4 * std::min(h.size(), n - o), hipMemcpyHostToDevice));
    return p;
}

template <int FM, int FN, int WM, int WN, class AL, class BL, class EPI>
static double time_gemm(const char* tag, const AL& al, const BL& bl, const EPI& epi, int M, int N,
                        int ksteps, int Z, double flops) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * Z);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm_kernel<FM, FN, WM, WN, AL, BL, EPI>;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipDeviceSynchronize());
    const int iters = 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-34s FM%d FN%d W%dx%d tile %3dx%3d Z%4d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, FM, FN,
           WM, WN, BM, BN, Z, grid.x, ms, flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return ms;
}

// forward conv: out[m][n] m < S*OH*OW, n < CO, k = 9*CI
template <int IH, int CI, int PAD, int FM, int FN, int WM, int WN>
static void conv_fwd(const char* tag, const float* X, const float* W, const float* b, float* Y,
                     int S, int CO, int kreal) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    const int KP = (9 * CI + 15) / 16 * 16;
    bl.ld = KP;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, al.M, CO};
    time_gemm<FM, FN, WM, WN>(tag, al, bl, epi, al.M, CO, KP / GK, 1, 2.0 * al.M * CO * kreal);
}

template <int IH, int CI, int FM, int FN, int WM, int WN>
static void conv_wgrad(const char* tag, const float* dz, const float* X, float* slab, float* bslab,
                       int S, int CO, int Z, int kreal) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = RowsKM<BM, NT>;
    using BL = Im2colKM<IH, IH, CI, 2, BN, NT>;
    const int M = S * BL::OH * BL::OW;
    const int KP = (9 * CI + 15) / 16 * 16;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    time_gemm<FM, FN, WM, WN>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * kreal);
}


// conv6-style weight gradient over the top-left VO x VO output window (product: conv_wgrad VO)
template <int IH, int CI, int FM, int FN, int WM, int WN, int VO>
static void conv_wgrad_vo(const char* tag, const float* dz, const float* X, float* slab,
                          float* bslab, int S, int CO, int Z, int kreal) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2;
    using AL = RowsKM<BM, NT, OFULL, VO>;
    using BL = Im2colKM<IH, IH, CI, 2, BN, NT, VO>;
    const int M = S * VO * VO;
    const int KP = (9 * CI + 15) / 16 * 16;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    time_gemm<FM, FN, WM, WN>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * kreal);
}

template <int FM, int FN, int WM, int WN, int KSUB, int PRIO, int MINW, int MODE = 0, class AL, class BL, class EPI>
static double time_gemm_v(const char* tag, const AL& al, const BL& bl, const EPI& epi, int M, int N,
                          int ksteps, int Z, double flops) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * Z);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm_kernel_v<FM, FN, WM, WN, KSUB, PRIO, MINW, AL, BL, EPI, MODE>;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipDeviceSynchronize());
    const int iters = 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-34s FM%d FN%d W%dx%d KSUB%d PRIO%d MINW%d tile %3dx%3d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, FM, FN,
           WM, WN, KSUB, PRIO, MINW, BM, BN, grid.x, ms, flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return ms;
}

template <int IH, int CI, int PAD, int FM, int FN, int WM, int WN, int KSUB, int PRIO, int MINW, int MODE = 0>
static void conv_fwd_v(const char* tag, const float* X, const float* W, const float* b, float* Y,
                       int S, int CO, int kreal) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    const int KP = (9 * CI + 15) / 16 * 16;
    bl.ld = KP;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, al.M, CO};
    time_gemm_v<FM, FN, WM, WN, KSUB, PRIO, MINW, MODE>(tag, al, bl, epi, al.M, CO, KP / GK, 1, 2.0 * al.M * CO * kreal);
}

template <int IH, int CI, int FM, int FN, int WM, int WN, int KSUB, int PRIO, int MINW>
static void conv_wgrad_v(const char* tag, const float* dz, const float* X, float* slab, float* bslab,
                         int S, int CO, int Z, int kreal) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = RowsKM<BM, NT>;
    using BL = Im2colKM<IH, IH, CI, 2, BN, NT>;
    const int M = S * BL::OH * BL::OW;
    const int KP = (9 * CI + 15) / 16 * 16;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    time_gemm_v<FM, FN, WM, WN, KSUB, PRIO, MINW>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * kreal);
}

template <int IH, int CI, int PAD, int FM, int FN, int WM, int WN>
static void conv_fwd_glds(const char* tag, const float* X, const float* W, const float* b, float* Y,
                          int S, int CO, int kreal, const float* zp) {
    constexpr int NW = WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colGlds<IH, IH, CI, PAD, BM, NW>;
    using BL = RowsGlds<BN, NW>;
    AL al;
    al.X = X;
    al.zp = zp;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    bl.zp = zp;
    const int KP = (9 * CI + 15) / 16 * 16;
    bl.ld = KP;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, al.M, CO};
    const int M = al.M, N = CO, ksteps = KP / GK;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm_glds<FM, FN, WM, WN, AL, BL, EpiBiasRelu>;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * NW), 0, 0, al, bl, epi, ksteps, ksteps, tm, tn);
    CK(hipDeviceSynchronize());
    const int iters = 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, grid, dim3(64 * NW), 0, 0, al, bl, epi, ksteps, ksteps, tm, tn);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-34s FM%d FN%d W%dx%d GLDS tile %3dx%3d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, FM, FN, WM, WN,
           BM, BN, grid.x, ms, 2.0 * M * N * kreal / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

// copy of Y after the reference kernel, to check the glds kernel's output
static void check_same(const float* Y, const float* Yref, size_t n, const char* tag) {
    std::vector<float> a(n), b(n);
    CK(hipMemcpy(a.data(), Y, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Yref, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("  check %s: %zu of %zu differ\n", tag, bad, n);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 4096;   // samples per chunk
    const size_t big = (size_t)S * 36 * 36 * 48;   // largest activation
    float* X = dalloc(big, 1.f);
    float* Y = dalloc(big, 0.f);
    float* W = dalloc(192 * 1728 + 64, 0.05f);
    float* b = dalloc(256, 0.01f);
    float* slab = dalloc((size_t)8192 * 48 * 432 > (size_t)512 * 192 * 1728 ? (size_t)8192 * 48 * 432 : (size_t)512 * 192 * 1728, 0.f);
    float* bsl = dalloc(8192 * 192, 0.f);
    float* zp = dalloc(64, 0.f);
    float* Y2 = dalloc(big, 0.f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define F(tag, IH, CI, PAD, CO, K, FM, FN, WM, WN) \
    if (want(tag)) conv_fwd<IH, CI, PAD, FM, FN, WM, WN>(tag, X, W, b, Y, S, CO, K);
#define FV(tag, IH, CI, PAD, CO, K, FM, FN, WM, WN, KS, PR, MW) \
    if (want(tag)) conv_fwd_v<IH, CI, PAD, FM, FN, WM, WN, KS, PR, MW>(tag, X, W, b, Y, S, CO, K);
#define G(tag, IH, CI, CO, Z, K, FM, FN, WM, WN) \
    if (want(tag)) conv_wgrad<IH, CI, FM, FN, WM, WN>(tag, Y, X, slab, bsl, S, CO, Z, K);
#define GV(tag, IH, CI, CO, Z, K, FM, FN, WM, WN, KS, PR, MW) \
    if (want(tag)) conv_wgrad_v<IH, CI, FM, FN, WM, WN, KS, PR, MW>(tag, Y, X, slab, bsl, S, CO, Z, K);
#define FM_(tag, IH, CI, PAD, CO, K, FM, FN, WM, WN, MODE) \
    if (want(tag)) conv_fwd_v<IH, CI, PAD, FM, FN, WM, WN, 1, 0, 1, MODE>(tag, X, W, b, Y, S, CO, K);
#define FG(tag, IH, CI, PAD, CO, K, FM, FN, WM, WN) \
    if (want(tag)) { conv_fwd_glds<IH, CI, PAD, FM, FN, WM, WN>(tag, X, W, b, Y2, S, CO, K, zp); \
                     conv_fwd<IH, CI, PAD, FM, FN, WM, WN>(tag, X, W, b, Y, S, CO, K); \
                     check_same(Y2, Y, (size_t)S * (IH + 2 * PAD - 2) * (IH + 2 * PAD - 2) * CO, tag); }
#define G14(tag, Z, FM, FN, WM, WN) \
    if (want(tag)) conv_wgrad_vo<13, 192, FM, FN, WM, WN, 14>(tag, Y, X, slab, bsl, S, 192, Z, 1728);
    // conv6 weight gradient (14x14 window): tile sweep
    G14("wg6 192x96 4w z128 (current)", 128, 6, 3, 2, 2)
    G14("wg6 192x96 4w z64", 64, 6, 3, 2, 2)
    G14("wg6 192x96 4w z256", 256, 6, 3, 2, 2)
    G14("wg6 192x96 8w 48x48", 128, 3, 3, 4, 2)
    G14("wg6 192x96 4w 48x96", 128, 3, 6, 4, 1)
    G14("wg6 192x96 6w 64x48", 128, 4, 3, 3, 2)
    G14("wg6 192x48 2w", 128, 6, 3, 2, 1)
    G14("wg6 96x96 4w", 128, 3, 3, 2, 2)
    G14("wg6 192x192 8w 96x48", 128, 6, 3, 2, 4)
    G14("wg6 192x144 6w", 128, 6, 3, 2, 3)
    // conv2 / conv3 weight gradients: deeper LDS stages (KSUB), issue priority, occupancy hint
    G("wgv2 base 48x144 z2048", 34, 48, 48, 2048, 432, 3, 3, 1, 3)
    GV("wgv2 ks2", 34, 48, 48, 2048, 432, 3, 3, 1, 3, 2, 0, 1)
    GV("wgv2 ks2 prio", 34, 48, 48, 2048, 432, 3, 3, 1, 3, 2, 1, 1)
    GV("wgv2 ks1 prio", 34, 48, 48, 2048, 432, 3, 3, 1, 3, 1, 1, 1)
    GV("wgv2 ks4", 34, 48, 48, 2048, 432, 3, 3, 1, 3, 4, 0, 1)
    GV("wgv2 ks2 z1024", 34, 48, 48, 1024, 432, 3, 3, 1, 3, 2, 0, 1)
    GV("wgv2 ks2 6w 96x144", 34, 48, 48, 2048, 432, 3, 3, 2, 3, 2, 0, 1)
    G("wgv3 base 96x96 z1024", 18, 48, 96, 1024, 432, 3, 3, 2, 2)
    GV("wgv3 ks2", 18, 48, 96, 1024, 432, 3, 3, 2, 2, 2, 0, 1)
    GV("wgv3 ks2 prio", 18, 48, 96, 1024, 432, 3, 3, 2, 2, 2, 1, 1)
    GV("wgv3 ks4", 18, 48, 96, 1024, 432, 3, 3, 2, 2, 4, 0, 1)
    // split counts at the 128-worker chunk (FLSIM_LAB_S=16384): ZW is fixed per layer, so the
    // K range per block grew 4x with the chunk
    G("zs wg2 z2048", 34, 48, 48, 2048, 432, 3, 3, 1, 3)
    G("zs wg2 z4096", 34, 48, 48, 4096, 432, 3, 3, 1, 3)
    G("zs wg2 z8192", 34, 48, 48, 8192, 432, 3, 3, 1, 3)
    G("zs wg3 z1024", 18, 48, 96, 1024, 432, 3, 3, 2, 2)
    G("zs wg3 z2048", 18, 48, 96, 2048, 432, 3, 3, 2, 2)
    G("zs wg3 z4096", 18, 48, 96, 4096, 432, 3, 3, 2, 2)
    G("zs wg4 z512", 20, 96, 96, 512, 864, 3, 3, 2, 2)
    G("zs wg4 z1024", 20, 96, 96, 1024, 864, 3, 3, 2, 2)
    G("zs wg4 z2048", 20, 96, 96, 2048, 864, 3, 3, 2, 2)
    G("zs wg5 z256", 11, 96, 192, 256, 864, 6, 3, 2, 2)
    G("zs wg5 z512", 11, 96, 192, 512, 864, 6, 3, 2, 2)
    G("zs wg5 z1024", 11, 96, 192, 1024, 864, 6, 3, 2, 2)
    G14("zs wg6 z128", 128, 6, 3, 2, 2)
    G14("zs wg6 z256", 256, 6, 3, 2, 2)
    G14("zs wg6 z512", 512, 6, 3, 2, 2)
    return 0;
}
