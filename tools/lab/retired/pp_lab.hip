// Main-loop order lab (development tool, not part of libflsim.so): gemm_x6_kernel (the product)
// against gemm_x6pp_kernel (tools/lab/gemm_x6pp.h: the next k-step's LDS stores and global loads
// moved behind the first / half of the current k-step's MFMAs) on PerformantNet1's staged
// split-bf16 shapes at 16,384 samples: conv5 / conv6 forward (split input and weights) and the
// conv4-6 weight gradients (fp32 dZ split while staged, split layer input), with the product's
// tiles.  Every variant must equal the product bit for bit (same MFMA order per accumulator); the
// line prints the count of differing outputs.  A B A B per shape.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//         -I fl-distributed-delay_amd/csrc -I tools/lab tools/lab/pp_lab.hip -o tools/lab/pp_lab
#include <string>

#include "gemm_x6pp.h"
#include "lab_common.h"

static __global__ void k_to_xs(const float* x, float* hm, float* l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(x)[u]);
}

struct Xs {
    float* hm;
    float* l;
};

static Xs to_xs(const float* x, size_t n) {
    Xs s;
    CK(hipMalloc(&s.hm, n * 4));
    CK(hipMalloc(&s.l, n * 2));
    const long units = (long)(n / 4);
    hipLaunchKernelGGL(k_to_xs, dim3((units + 255) / 256), dim3(256), 0, 0, x, s.hm, s.l, units);
    CK(hipDeviceSynchronize());
    return s;
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

static size_t ndiff(const float* a, const float* b, size_t n) {
    std::vector<float> h0(n), h1(n);
    CK(hipMemcpy(h0.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), b, n * 4, hipMemcpyDeviceToHost));
    size_t d = 0;
    for (size_t i = 0; i < n; ++i) d += memcmp(&h0[i], &h1[i], 4) != 0;
    return d;
}

// conv forward on the staged kernel: Y = relu(im2col(X) W^T + b), split X and W
template <int IH, int CI, int CO, int FM, int FN, int WM, int WN>
static void conv(const char* tag, const Xs& Xx, const Xs& Wx, const float* b, float* Y0, float* Y1,
                 int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int PAD = 2;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT, false, 0, XsSrc>;
    using BL = RowsKC<BN, NT, XsSrc>;
    const int KP = 9 * CI;
    AL al;
    al.X = Xx.hm;
    al.XL = Xx.l;
    al.M = S * AL::OH * AL::OW;
    const int M = al.M;
    BL bl;
    bl.P = Wx.hm;
    bl.PL = Wx.l;
    bl.ld = KP;
    bl.NR = CO;
    const double flops = 2.0 * M * CO * KP;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const dim3 g(tm * tn);
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    auto prod = gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>;
    const size_t n = (size_t)M * CO;
    EpiBiasRelu e0{Y0, b, M, CO}, e1{Y1, b, M, CO};
    auto run = [&](auto k, const EpiBiasRelu& e) {
        return timeit(k, g, NT, al, bl, e, KP / GK, KP / GK, tm, tn);
    };
    std::vector<void*> ks = {
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 3, 2, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 4, 2, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 2, 3, 3, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 3, 2, 2, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 3, 1, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiBiasRelu, 3, 2, 4, 2>};
    const char* names[] = {"V3W2L4", "V4W2L4", "V2W3L3", "V3W2L2", "V3W1L4", "V3W2L4R2"};
    double tp[2];
    for (int r = 0; r < 2; ++r) tp[r] = run(prod, e0);
    printf("%-6s %3dx%3d product %7.3f %7.3f ms %6.1f TF/s\n", tag, BM, BN, tp[0], tp[1], tf(tp[1]));
    for (size_t v = 0; v < ks.size(); ++v) {
        using KT = decltype(prod);
        const KT kv = reinterpret_cast<KT>(ks[v]);
        const double a = run(kv, e1);
        const size_t d = ndiff(Y0, Y1, n);
        const double p = run(prod, e0), c = run(kv, e1);
        printf("%-6s   %-9s %7.3f %7.3f ms %6.1f TF/s (x%.3f against the product's %7.3f %7.3f) "
               "differ %zu\n", tag, names[v], a, c, tf(c), (tp[1] + p) / (a + c), tp[1], p, d);
        tp[1] = p;
    }
    fflush(stdout);
}

// weight gradient: slab[z][co][kk] = sum over the split's pixels of dz[p][co] im2col(X)[p][kk];
// dz fp32 (split while staged), X split, the product's bias column sum on the MFMA
template <int IH, int CI, int CO, int FM, int FN, int WM, int WN>
static void wgrad(const char* tag, const float* dz, const Xs& Xx, float* S0, float* S1, float* B0,
                  float* B1, int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int PAD = 2;
    using AL = RowsKM<BM, NT, 0, 0, BufSrc>;
    using BL = Im2colKM<IH, IH, CI, PAD, BN, NT, 0, XsSrc>;
    const int M = S * BL::OH * BL::OW;
    const int KP = 9 * CI;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = Xx.hm;
    bl.XL = Xx.l;
    bl.M = M;
    const int ks = ceil_div(M, GK);
    const int per = ceil_div(ks, Z);
    const int tm = ceil_div(CO, BM), tn = ceil_div(KP, BN);
    const dim3 g(tm * tn * Z);
    const double flops = 2.0 * M * CO * KP;
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    EpiSlabAcc e0{S0, CO, KP, (long)CO * KP, B0, 0}, e1{S1, CO, KP, (long)CO * KP, B1, 0};
    auto prod = gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>;
    const size_t n = (size_t)Z * CO * KP, nb = (size_t)Z * CO;
    auto run = [&](auto k, const EpiSlabAcc& e) { return timeit(k, g, NT, al, bl, e, ks, per, tm, tn); };
    std::vector<void*> kv_ = {
        (void*)gemm_x6pp_kernel<3, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 3, 2, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 1, 3, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 2, 3, 3, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 2, 4, 6, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 6, 3, 4, 0>,
        (void*)gemm_x6pp_kernel<5, FM, FN, WM, WN, AL, BL, EpiSlabAcc, 2, 3, 3, 3>};
    const char* names[] = {"branchfree", "V1W3L4", "V2W3L3", "V2W4L6", "V6W3L4", "V2W3L3R3"};
    double tp[2];
    for (int r = 0; r < 2; ++r) tp[r] = run(prod, e0);
    printf("%-6s %3dx%3d Z %4d product %7.3f %7.3f ms %6.1f TF/s\n", tag, BM, BN, Z, tp[0], tp[1],
           tf(tp[1]));
    for (size_t v = 0; v < kv_.size(); ++v) {
        using KT = decltype(prod);
        const KT kv = reinterpret_cast<KT>(kv_[v]);
        const double a = run(kv, e1);
        const size_t d = ndiff(S0, S1, n) + ndiff(B0, B1, nb);
        const double p = run(prod, e0), c = run(kv, e1);
        printf("%-6s   %-9s %7.3f %7.3f ms %6.1f TF/s (x%.3f against the product's %7.3f %7.3f) "
               "differ %zu\n", tag, names[v], a, c, tf(c), (tp[1] + p) / (a + c), tp[1], p, d);
        tp[1] = p;
    }
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 22 * 22 * 96;      // the largest input / dZ below
    float* X = dalloc(big, 1.f);
    const Xs Xx = to_xs(X, big);
    float* Y0 = dalloc(big, 0.f);
    float* Y1 = dalloc(big, 0.f);
    const size_t wn = 192 * 1728;
    float* W = dalloc(wn, 0.05f);
    const Xs Wx = to_xs(W, wn);
    float* b = dalloc(256, 0.01f);
    const size_t slabn = (size_t)1024 * 96 * 864;
    float* S0 = dalloc(slabn, 0.f);
    float* S1 = dalloc(slabn, 0.f);
    float* B0 = dalloc(1024 * 192, 0.f);
    float* B1 = dalloc(1024 * 192, 0.f);
    const std::string only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return only.empty() || only.find(t) != std::string::npos; };
    // the product's tiles (pn1_net.hip): forward 256x192 8 waves; weight gradients 192x96 /
    // 96x96 4 waves
    if (want("fwd6")) conv<13, 192, 192, 4, 6, 4, 2>("fwd6", Xx, Wx, b, Y0, Y1, S);
    if (want("fwd5")) conv<11, 96, 192, 4, 6, 4, 2>("fwd5", Xx, Wx, b, Y0, Y1, S);
    if (want("wg6")) wgrad<13, 192, 192, 6, 3, 2, 2>("wg6", X, Xx, S0, S1, B0, B1, S, 256);
    if (want("wg5")) wgrad<11, 96, 192, 6, 3, 2, 2>("wg5", X, Xx, S0, S1, B0, B1, S, 512);
    if (want("wg4")) wgrad<20, 96, 96, 3, 3, 2, 2>("wg4", X, Xx, S0, S1, B0, B1, S, 1024);
    return 0;
}
