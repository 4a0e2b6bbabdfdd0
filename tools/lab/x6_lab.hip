// Split-bf16 GEMM lab (development tool, not part of libflsim.so): gemm_x6_kernel (gemm_x6.h)
// against the fp32 gemm_kernel on PerformantNet1's conv shapes (implicit-GEMM forward / data
// gradient: im2col rows x packed weights, both k-contiguous), same loaders and epilogue.
// Prints time, fp32-equivalent TF/s and the largest difference between the two outputs
// relative to the output's largest magnitude.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I fl-distributed-delay_amd/csrc
//         tools/lab/x6_lab.hip -o tools/lab/x6_lab
#include <cmath>

#include "gemm_x6.h"
#include "lab_common.h"

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN>
static void conv(const char* tag, const float* X, const float* W, const float* b, float* Y0,
                 float* Y1, int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    const int KP = 9 * CI;
    bl.ld = KP;
    bl.NR = CO;
    const int M = al.M;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const double flops = 2.0 * M * CO * KP;
    dim3 g1(tm * tn);
    auto run = [&](auto kern, float* Y) {
        EpiBiasRelu epi{Y, b, M, CO};
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < 2; ++i)
            hipLaunchKernelGGL(kern, g1, dim3(NT), 0, 0, al, bl, epi, KP / GK, KP / GK, tm, tn);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 5; ++i)
            hipLaunchKernelGGL(kern, g1, dim3(NT), 0, 0, al, bl, epi, KP / GK, KP / GK, tm, tn);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / 5;
    };
    const double t0 = run(gemm_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>, Y0);
    const double t1 = run(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>, Y1);
    const size_t n = (size_t)M * CO;
    std::vector<float> h0(n), h1(n);
    CK(hipMemcpy(h0.data(), Y0, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), Y1, n * 4, hipMemcpyDeviceToHost));
    double dmax = 0, ymax = 0;
    size_t nd = 0;
    for (size_t i = 0; i < n; ++i) {
        const double d = fabs((double)h0[i] - (double)h1[i]);
        dmax = d > dmax ? d : dmax;
        ymax = fabs(h0[i]) > ymax ? fabs(h0[i]) : ymax;
        nd += h0[i] != h1[i];
    }
    printf("%-22s tile %3dx%3d  fp32 %7.3f ms %6.1f TF/s | x6 %7.3f ms %6.1f TF/s (x%.2f) | "
           "max|d| / max|y| %.2e, %.1f %% differ\n",
           tag, BM, BN, t0, flops / (t0 * 1e-3) / 1e12, t1, flops / (t1 * 1e-3) / 1e12, t0 / t1,
           dmax / (ymax > 0 ? ymax : 1), 100.0 * nd / n);
    fflush(stdout);
}


// weight gradient: slab[z][co][kk] = sum over the split's pixels of dz[p][co] im2col(X)[p][kk]
// (k-major operands) with the bias column sums (ASUM); dz = the forward's output buffer
template <int IH, int CI, int CO, int FM, int FN, int WM, int WN>
static void wgrad(const char* tag, const float* dz, const float* X, float* S0, float* S1,
                  float* B0, float* B1, int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int PAD = 1;
    using AL = RowsKM<BM, NT>;
    using BL = Im2colKM<IH, IH, CI, PAD, BN, NT>;
    const int M = S * BL::OH * BL::OW;
    const int KP = 9 * CI;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    const int ks = ceil_div(M, GK);
    const int per = ceil_div(ks, Z);
    const int tm = ceil_div(CO, BM), tn = ceil_div(KP, BN);
    const double flops = 2.0 * M * CO * KP;
    dim3 g1(tm * tn * Z);
    auto run = [&](auto kern, float* sl, float* bs) {
        EpiSlabAcc epi{sl, CO, KP, (long)CO * KP, bs, 0};   // zinit 0: every split stores
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < 2; ++i)
            hipLaunchKernelGGL(kern, g1, dim3(NT), 0, 0, al, bl, epi, ks, per, tm, tn);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 5; ++i)
            hipLaunchKernelGGL(kern, g1, dim3(NT), 0, 0, al, bl, epi, ks, per, tm, tn);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / 5;
    };
    const double t0 = run(gemm_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>, S0, B0);
    const double t1 = run(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>, S1, B1);
    auto cmp = [&](const float* d0, const float* d1, size_t n, double& rel) {
        std::vector<float> h0(n), h1(n);
        CK(hipMemcpy(h0.data(), d0, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h1.data(), d1, n * 4, hipMemcpyDeviceToHost));
        double dmax = 0, ymax = 0;
        for (size_t i = 0; i < n; ++i) {
            dmax = std::max(dmax, fabs((double)h0[i] - (double)h1[i]));
            ymax = std::max(ymax, (double)fabs(h0[i]));
        }
        rel = dmax / (ymax > 0 ? ymax : 1);
    };
    double rw, rb;
    cmp(S0, S1, (size_t)Z * CO * KP, rw);
    cmp(B0, B1, (size_t)Z * CO, rb);
    printf("%-22s tile %3dx%3d Z %4d  fp32 %7.3f ms %6.1f TF/s | x6 %7.3f ms %6.1f TF/s (x%.2f) | "
           "slab max|d|/max %.2e, bias %.2e\n",
           tag, BM, BN, Z, t0, flops / (t0 * 1e-3) / 1e12, t1, flops / (t1 * 1e-3) / 1e12, t0 / t1,
           rw, rb);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y0 = dalloc(big, 0.f);
    float* Y1 = dalloc(big, 0.f);
    float* W = dalloc(512 * 4608 + 64, 0.05f);
    float* b = dalloc(256, 0.01f);
    const size_t slabn = (size_t)8192 * 48 * 432;
    float* S0 = dalloc(slabn, 0.f);
    float* S1 = dalloc(slabn, 0.f);
    float* B0 = dalloc(4096 * 192, 0.f);
    float* B1 = dalloc(4096 * 192, 0.f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define C(tag, IH, CI, PAD, CO, FM, FN, WM, WN) \
    if (want(tag)) conv<IH, CI, PAD, CO, FM, FN, WM, WN>(tag, X, W, b, Y0, Y1, S);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN) \
    if (want(tag)) wgrad<IH, CI, CO, FM, FN, WM, WN>(tag, X, X, S0, S1, B0, B1, S, Z);
    // weight gradients (pixel split Z as the product: >= 32 k-steps per split)
    G("wg6 192x192 8w", 13, 192, 192, 256, 6, 6, 2, 4)
    G("wg6 192x96 4w", 13, 192, 192, 256, 6, 3, 2, 2)
    G("wg6 96x192 4w", 13, 192, 192, 256, 3, 6, 2, 2)
    G("wg4 96x96 4w", 20, 96, 96, 1024, 3, 3, 2, 2)
    G("wg4 96x192 4w", 20, 96, 96, 1024, 3, 6, 2, 2)
    G("wg2 48x144 3w", 34, 48, 48, 4096, 3, 3, 1, 3)
    G("wg2 48x48 1w", 34, 48, 48, 4096, 3, 3, 1, 1)
    G("wg2 48x144 1w", 34, 48, 48, 4096, 3, 9, 1, 1)
    // conv6-like: 13x13x192 -> 192 (K 1728)
    C("c6 128x96 4w", 13, 192, 1, 192, 4, 3, 2, 2)
    C("c6 256x96 8w", 13, 192, 1, 192, 4, 3, 4, 2)
    C("c6 128x192 4w", 13, 192, 1, 192, 4, 6, 2, 2)
    C("c6 256x192 8w", 13, 192, 1, 192, 4, 6, 4, 2)
    C("c6 128x192 8w", 13, 192, 1, 192, 2, 6, 4, 2)
    C("c6 256x64 8w", 13, 192, 1, 192, 4, 2, 4, 2)
    // conv4-like: 20x20x96 -> 96 (K 864)
    C("c4 256x96 8w", 20, 96, 1, 96, 4, 3, 4, 2)
    C("c4 256x96 4w", 20, 96, 1, 96, 8, 3, 2, 2)
    // conv2-like: 34x34x48 -> 48 (K 432)
    C("c2 512x48 8w", 34, 48, 1, 48, 4, 3, 8, 1)
    C("c2 256x48 4w", 34, 48, 1, 48, 4, 3, 4, 1)
    return 0;
}
