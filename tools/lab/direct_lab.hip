// Direct-A lab (development tool, not part of libflsim.so): the product's gemm_kernel against
// gemm_direct_kernel (csrc/gemm_direct.h) on PerformantNet1's forward / data-gradient conv shapes
// at S = 16,384 samples, EpiBiasRelu epilogue; outputs compared bit for bit.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/direct_lab.hip -o tools/lab/direct_lab
#include "lab_common.h"
#include "gemm_direct.h"
#include "gemm_resident.h"

static int g_iters = 5;

template <class F>
static float time_it(F launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < g_iters; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / g_iters;
}

static void compare(const char* tag, const float* a, const float* b, size_t n) {
    std::vector<float> ha(n), hb(n);
    CK(hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), b, n * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    double nz = 0;
    for (size_t i = 0; i < n; ++i) {
        if (memcmp(&ha[i], &hb[i], 4)) ++diff;
        nz += ha[i] != 0.f;
    }
    printf("  check %-28s %zu of %zu words differ (nonzero frac %.3f)\n", tag, diff, n, nz / n);
}

// product: gemm_kernel<FM, FN, WM, WN> with Im2colKC + RowsKC
template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN, int OHX = 0>
static void prod(const char* tag, const float* X, const float* W, const float* b, float* Y, int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT, false, OHX>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    const int KP = 9 * CI;
    bl.ld = KP;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, al.M, CO};
    const int tm = ceil_div(al.M, BM), tn = ceil_div(CO, BN);
    const int ks = KP / GK;
    auto k = gemm_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>;
    const float ms = time_it([&] {
        hipLaunchKernelGGL(k, dim3(tm * tn), dim3(NT), 0, 0, al, bl, epi, ks, ks, tm, tn);
    });
    const double fl = 2.0 * al.M * CO * KP;
    printf("%-30s prod   tile %3dx%3d %dw      %8.3f ms  %6.1f TF/s\n", tag, BM, BN, WM * WN, ms,
           fl / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WAVES, int KB, int DEPTH, int OHX = 0>
static void direct(const char* tag, const float* X, const float* W, const float* b, float* Y,
                   int S) {
    constexpr int NT = 64 * WAVES, BM = 16 * FM * WAVES, BN = 16 * FN;
    using AD = Im2colDirect<IH, IH, CI, PAD, FM, false, OHX>;
    using BL = RowsKCStage<BN, NT>;
    AD ad;
    ad.X = X;
    ad.M = S * AD::OH * AD::OW;
    BL bl;
    bl.P = W;
    const int KP = 9 * CI;
    bl.ld = KP;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, ad.M, CO};
    const int tm = ceil_div(ad.M, BM), tn = ceil_div(CO, BN);
    const int ks = KP / GK;
    auto k = gemm_direct_kernel<FM, FN, WAVES, KB, DEPTH, AD, BL, EpiBiasRelu>;
    if (ks % KB) { printf("ksteps %% KB\n"); return; }
    const float ms = time_it([&] {
        hipLaunchKernelGGL(k, dim3(tm * tn), dim3(NT), 0, 0, ad, bl, epi, ks, tm, tn);
    });
    const double fl = 2.0 * ad.M * CO * KP;
    printf("%-30s direct tile %3dx%3d %dw KB%d D%d %8.3f ms  %6.1f TF/s\n", tag, BM, BN, WAVES, KB,
           DEPTH, ms, fl / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

// resident-B persistent kernel (gemm_resident.h): grid = NB blocks (one per CU by default)
template <int IH, int CI, int PAD, int CO, int FM, int FN, int WAVES, int DEPTH, int OHX = 0>
static void resident(const char* tag, const float* X, const float* W, const float* b, float* Y,
                     int S, int NB) {
    constexpr int BM = 16 * FM * WAVES;
    constexpr int KS = 9 * CI / GK;
    using AD = Im2colDirect<IH, IH, CI, PAD, FM, false, OHX>;
    AD ad;
    ad.X = X;
    ad.M = S * AD::OH * AD::OW;
    EpiBiasRelu epi{Y, b, ad.M, CO};
    const int tm = ceil_div(ad.M, BM);
    auto k = gemm_resident_kernel<FM, FN, WAVES, KS, DEPTH, 1, AD, EpiBiasRelu>;
    const float ms = time_it([&] {
        hipLaunchKernelGGL(k, dim3(NB), dim3(64 * WAVES), 0, 0, ad, W, 9 * CI, CO, epi, tm);
    });
    const double fl = 2.0 * ad.M * CO * 9 * CI;
    printf("%-30s resid  tile %3dx%3d %dw D%d nb%d %8.3f ms  %6.1f TF/s\n", tag, BM, 16 * FN, WAVES,
           DEPTH, NB, ms, fl / (ms * 1e-3) / 1e12);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    if (getenv("LAB_ITERS")) g_iters = atoi(getenv("LAB_ITERS"));
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y0 = dalloc(big, 0.f);
    float* Y1 = dalloc(big, 0.f);
    float* W = dalloc(192 * 1728 + 64, 0.05f);
    float* b = dalloc(256, 0.01f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
    // out elements of each shape (for the bitwise check)
#define P(tag, IH, CI, PAD, CO, FM, FN, WM, WN, OHX) \
    if (want(tag)) prod<IH, CI, PAD, CO, FM, FN, WM, WN, OHX>(tag, X, W, b, Y0, S);
#define D(tag, IH, CI, PAD, CO, FM, FN, WV, KB, DP, OHX, OUT)                           \
    if (want(tag)) {                                                                     \
        CK(hipMemset(Y1, 0, (size_t)(OUT) * 4));                                         \
        direct<IH, CI, PAD, CO, FM, FN, WV, KB, DP, OHX>(tag, X, W, b, Y1, S);           \
        compare(tag, Y0, Y1, (size_t)(OUT));                                             \
    }
    const size_t o6 = (size_t)S * 15 * 15 * 192, o6d = (size_t)S * 13 * 13 * 192;
    const size_t o4 = (size_t)S * 22 * 22 * 96, o4d = (size_t)S * 20 * 20 * 96;
    const size_t o2 = (size_t)S * 36 * 36 * 48;
    const size_t o3d = (size_t)S * 18 * 18 * 48;
    const size_t o5 = (size_t)S * 13 * 13 * 192;
    const size_t o5d = (size_t)S * 11 * 11 * 96, o3 = (size_t)S * 20 * 20 * 96;
    const size_t o2d = (size_t)S * 34 * 34 * 48;
    // round-3 sweep: per layer the product tile, then direct-A variants (FM, FN, waves, KB, DEPTH)
#define SWEEP(tag, IH, CI, PAD, CO, OHX, OUT, FNF)                                      \
    D(tag, IH, CI, PAD, CO, 2, FNF, 8, 3, 2, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 2, FNF, 8, 6, 2, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 2, FNF, 8, 9, 2, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 2, FNF, 8, 6, 5, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 4, FNF, 8, 3, 2, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 1, FNF, 8, 3, 2, OHX, OUT)                                   \
    D(tag, IH, CI, PAD, CO, 2, FNF, 6, 3, 2, OHX, OUT)
    P("fwd6", 13, 192, 2, 192, 2, 3, 4, 2, 0)
    SWEEP("fwd6", 13, 192, 2, 192, 0, o6, 6)
    P("dg6", 14, 192, 0, 192, 4, 3, 4, 2, 13)
    SWEEP("dg6", 14, 192, 0, 192, 13, o6d, 6)
    P("fwd5", 11, 96, 2, 192, 2, 3, 4, 2, 0)
    SWEEP("fwd5", 11, 96, 2, 192, 0, o5, 6)
    P("dg5", 13, 192, 0, 96, 4, 3, 2, 2, 0)
    SWEEP("dg5", 13, 192, 0, 96, 0, o5d, 6)
    P("fwd4", 20, 96, 2, 96, 4, 3, 2, 2, 0)
    SWEEP("fwd4", 20, 96, 2, 96, 0, o4, 6)
    P("dg4", 22, 96, 0, 96, 4, 3, 2, 2, 0)
    SWEEP("dg4", 22, 96, 0, 96, 0, o4d, 6)
    P("fwd3", 18, 48, 2, 96, 2, 3, 4, 2, 0)
    SWEEP("fwd3", 18, 48, 2, 96, 0, o3, 6)
    P("dg3", 20, 96, 0, 48, 4, 3, 4, 1, 0)
    SWEEP("dg3", 20, 96, 0, 48, 0, o3d, 3)
#define RS(tag, IH, CI, PAD, CO, FM, FN, WV, DP, OHX, OUT, NB)                          \
    if (want(tag)) {                                                                     \
        CK(hipMemset(Y1, 0, (size_t)(OUT) * 4));                                         \
        resident<IH, CI, PAD, CO, FM, FN, WV, DP, OHX>(tag, X, W, b, Y1, S, NB);          \
        compare(tag, Y0, Y1, (size_t)(OUT));                                             \
    }
    // round 3: resident-B persistent kernel on conv2's forward and data gradient (B = 83 KB)
    P("rfwd2", 34, 48, 2, 48, 2, 3, 4, 1, 0)
    D("rfwd2", 34, 48, 2, 48, 2, 3, 8, 3, 2, 0, o2)
    RS("rfwd2", 34, 48, 2, 48, 2, 3, 8, 2, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 2, 3, 8, 8, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 2, 3, 4, 2, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 4, 3, 4, 2, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 4, 3, 8, 2, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 1, 3, 8, 2, 0, o2, 256)
    RS("rfwd2", 34, 48, 2, 48, 2, 3, 8, 2, 0, o2, 512)
    P("rdg2", 36, 48, 0, 48, 2, 3, 4, 1, 0)
    D("rdg2", 36, 48, 0, 48, 2, 3, 8, 3, 2, 0, o2d)
    RS("rdg2", 36, 48, 0, 48, 2, 3, 8, 2, 0, o2d, 256)
    RS("rdg2", 36, 48, 0, 48, 2, 3, 8, 8, 0, o2d, 256)
    RS("rdg2", 36, 48, 0, 48, 4, 3, 4, 2, 0, o2d, 256)
    RS("rdg2", 36, 48, 0, 48, 4, 3, 8, 2, 0, o2d, 256)
    P("fwd2", 34, 48, 2, 48, 2, 3, 4, 1, 0)
    SWEEP("fwd2", 34, 48, 2, 48, 0, o2, 3)
    P("dg2", 36, 48, 0, 48, 2, 3, 4, 1, 0)
    SWEEP("dg2", 36, 48, 0, 48, 0, o2d, 3)
    return 0;
}
