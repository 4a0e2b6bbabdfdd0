// Direct-A lab (development tool, not part of libflsim.so): the product's gemm_kernel against
// gemm_direct_kernel (csrc/gemm_direct.h) on PerformantNet1's forward / data-gradient conv shapes
// at S = 16,384 samples, EpiBiasRelu epilogue; outputs compared bit for bit.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/direct_lab.hip -o tools/lab/direct_lab
#include "lab_common.h"
#include "gemm_direct.h"

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
    // conv6 forward (13x13x192 -> 15x15x192)
    P("fwd6", 13, 192, 2, 192, 2, 3, 4, 2, 0)
    D("fwd6", 13, 192, 2, 192, 2, 6, 8, 9, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 2, 6, 4, 9, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 4, 6, 4, 9, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 2, 12, 8, 3, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 4, 3, 8, 9, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 2, 6, 8, 3, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 2, 6, 4, 3, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 4, 6, 4, 3, 2, 0, o6)
    D("fwd6", 13, 192, 2, 192, 4, 3, 4, 3, 2, 0, o6)
    // conv6 data gradient (14x14 dZ, pad 0 -> 13x13)
    P("dg6", 14, 192, 0, 192, 4, 3, 4, 2, 13)
    D("dg6", 14, 192, 0, 192, 2, 6, 8, 9, 2, 13, o6d)
    D("dg6", 14, 192, 0, 192, 4, 3, 8, 9, 2, 13, o6d)
    D("dg6", 14, 192, 0, 192, 2, 6, 8, 3, 2, 13, o6d)
    D("dg6", 14, 192, 0, 192, 4, 6, 4, 3, 2, 13, o6d)
    // conv4 data gradient (22x22x96 -> 20x20x96)
    P("dg4", 22, 96, 0, 96, 4, 3, 2, 2, 0)
    D("dg4", 22, 96, 0, 96, 2, 6, 8, 9, 2, 0, o4d)
    D("dg4", 22, 96, 0, 96, 4, 6, 4, 9, 2, 0, o4d)
    D("dg4", 22, 96, 0, 96, 2, 6, 4, 9, 2, 0, o4d)
    D("dg4", 22, 96, 0, 96, 2, 6, 8, 3, 2, 0, o4d)
    D("dg4", 22, 96, 0, 96, 4, 6, 4, 3, 2, 0, o4d)
    D("dg4", 22, 96, 0, 96, 2, 6, 4, 3, 2, 0, o4d)
    // conv4 forward (20x20x96 -> 22x22x96)
    P("fwd4", 20, 96, 2, 96, 4, 3, 2, 2, 0)
    D("fwd4", 20, 96, 2, 96, 2, 6, 8, 9, 2, 0, o4)
    D("fwd4", 20, 96, 2, 96, 4, 6, 4, 9, 2, 0, o4)
    D("fwd4", 20, 96, 2, 96, 2, 6, 8, 3, 2, 0, o4)
    D("fwd4", 20, 96, 2, 96, 2, 6, 4, 3, 2, 0, o4)
    // conv5 forward (11x11x96 -> 13x13x192)
    P("fwd5", 11, 96, 2, 192, 2, 3, 4, 2, 0)
    D("fwd5", 11, 96, 2, 192, 2, 6, 8, 9, 2, 0, o5)
    D("fwd5", 11, 96, 2, 192, 4, 6, 4, 9, 2, 0, o5)
    // conv2 forward (34x34x48 -> 36x36x48)
    P("fwd2", 34, 48, 2, 48, 2, 3, 4, 1, 0)
    D("fwd2", 34, 48, 2, 48, 2, 3, 8, 9, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 4, 3, 4, 9, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 2, 3, 4, 9, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 4, 3, 8, 9, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 2, 3, 8, 3, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 4, 3, 4, 3, 2, 0, o2)
    D("fwd2", 34, 48, 2, 48, 2, 3, 4, 3, 2, 0, o2)
    // conv3 data gradient (20x20x96 dZ -> 18x18x48)
    P("dg3", 20, 96, 0, 48, 4, 3, 4, 1, 0)
    D("dg3", 20, 96, 0, 48, 2, 3, 8, 9, 2, 0, o3d)
    D("dg3", 20, 96, 0, 48, 4, 3, 4, 9, 2, 0, o3d)
    D("dg3", 20, 96, 0, 48, 4, 3, 8, 9, 2, 0, o3d)
    D("dg3", 20, 96, 0, 48, 2, 3, 8, 3, 2, 0, o3d)
    D("dg3", 20, 96, 0, 48, 4, 3, 4, 3, 2, 0, o3d)
    return 0;
}
