// Halo lab (development tool, not part of libflsim.so): the product's direct split-bf16 forward
// (gemm_dx6_kernel, A fragments loaded per tap) against gemm_hx6_kernel (tools/lab/gemm_hx6.h, A
// served from a per-slice LDS patch) on PerformantNet1's conv2 / conv3 / conv4 forward shapes at
// 16,384 samples, with the product's tiles; input split and channel-slice-major as in the product.
// The outputs must agree bit for bit (same k order and MFMA sequence); A B A B timing.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//         -I fl-distributed-delay_amd/csrc -I tools/lab tools/lab/halo_lab.hip -o tools/lab/halo_lab
#include <string>

#include "gemm_hx6.h"
#include "gemm_dx6pp.h"
#include "lab_common.h"

static __global__ void k_to_xs(const float* x, float* hm, float* l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(x)[u]);
}
// [img][pix][CI] split -> channel-slice-major [img][CI/16][pix][16]
static __global__ void k_to_sm(const f32x4* hm, const f32x2* l, f32x4* hm_o, f32x2* l_o, long units,
                               int hw, int ci4) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u >= units) return;
    const int c4 = (int)(u % ci4);
    const long pix = u / ci4;
    const long img = pix / hw, p = pix - img * hw;
    const long o = ((img * (ci4 / 4) + c4 / 4) * hw + p) * 4 + (c4 & 3);
    hm_o[o] = hm[u];
    l_o[o] = l[u];
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

// the patch rows a block needs, computed as HaloA::setup_block does (host copy)
template <int IH, int PAD, bool WIN, int OHW>
static int max_patch_rows(int M, int BM) {
    constexpr int PW = OHW / 2;
    constexpr int RPI = WIN ? 4 * PW * PW : OHW * OHW;
    auto range = [&](int m, int& img, int& lo, int& hi) {
        img = m / RPI;
        const int rem = m - img * RPI;
        int oh;
        if (WIN) {
            const int qq = rem >> 2;
            oh = 2 * (qq / PW) + ((rem >> 1) & 1);
        } else {
            oh = rem / OHW;
        }
        lo = WIN ? (oh & ~1) : oh;
        hi = WIN ? (oh | 1) : oh;
    };
    int mx = 0;
    for (int m0 = 0; m0 < M; m0 += BM) {
        const int m1 = std::min(m0 + BM, M) - 1;
        int i0, lo0, hi0, i1, lo1, hi1;
        range(m0, i0, lo0, hi0);
        range(m1, i1, lo1, hi1);
        const int g_lo = i0 * IH + std::max(0, lo0 - PAD);
        const int g_hi = i1 * IH + std::min(IH - 1, hi1 - PAD + 2);
        mx = std::max(mx, g_hi - g_lo + 1);
    }
    return mx;
}

template <int IH, int CI, int CO, bool WIN, int FM, int FN, int WAVES, int KB, int NRP, int MINW = 1>
static void shape(const char* tag, const Xs& Xsm, const Xs& Wx, const float* b, float* Y0,
                  float* Y1, int S) {
    constexpr int PAD = 2, NT = 64 * WAVES, BM = 16 * FM * WAVES, BN = 16 * FN;
    constexpr int OHW = IH + 2 * PAD - 2;
    const int KP = 9 * CI;
    const int M = S * (WIN ? 4 * (OHW / 2) * (OHW / 2) : OHW * OHW);
    const int need = max_patch_rows<IH, PAD, WIN, OHW>(M, BM);
    if (need > NRP) {
        printf("%-6s NRP %d < %d patch rows needed: skipped\n", tag, NRP, need);
        return;
    }
    using AD = Im2colDirect<IH, IH, CI, PAD, FM, WIN, 0, XsSrcSM>;
    using BD = RowsKCStageXs<BN, NT, 2>;
    using HA = HaloA<IH, IH, CI, PAD, FM, WIN, NRP>;
    AD ad;
    ad.X = Xsm.hm;
    ad.XL = Xsm.l;
    ad.M = M;
    BD bd;
    bd.P = Wx.hm;
    bd.PL = Wx.l;
    bd.ld = KP;
    bd.NR = CO;
    HA ha;
    ha.X = Xsm.hm;
    ha.XL = Xsm.l;
    ha.M = M;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const dim3 g(tm * tn);
    const double flops = 2.0 * M * CO * KP;
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    auto kd = gemm_dx6_kernel<FM, FN, WAVES, KB, 2, AD, BD, EpiBiasRelu>;
    auto kh = gemm_hx6_kernel<FM, FN, WAVES, HA, BD, EpiBiasRelu, MINW>;
    double t[2][2];
    for (int r = 0; r < 2; ++r) {
        t[r][0] = timeit(kd, g, NT, ad, bd, EpiBiasRelu{Y0, b, M, CO}, KP / GK, tm, tn);
        t[r][1] = timeit(kh, g, NT, ha, bd, EpiBiasRelu{Y1, b, M, CO}, tm, tn);
    }
    const size_t d = ndiff(Y0, Y1, (size_t)M * CO);
    printf("[waves per EU >= %d] ", MINW);
    if (getenv("LAB_DX6PP") && MINW == 1) {       // the direct kernel's scheduling variants
        auto k1 = gemm_dx6pp_kernel<1, FM, FN, WAVES, KB, 2, AD, BD, EpiBiasRelu>;
        auto k2 = gemm_dx6pp_kernel<2, FM, FN, WAVES, KB, 2, AD, BD, EpiBiasRelu>;
        auto k3 = gemm_dx6pp_kernel<3, FM, FN, WAVES, KB, 2, AD, BD, EpiBiasRelu>;
        double u[2][4];
        size_t dd[3];
        for (int r = 0; r < 2; ++r) {
            u[r][0] = timeit(kd, g, NT, ad, bd, EpiBiasRelu{Y0, b, M, CO}, KP / GK, tm, tn);
            u[r][1] = timeit(k1, g, NT, ad, bd, EpiBiasRelu{Y1, b, M, CO}, KP / GK, tm, tn);
            if (r == 0) dd[0] = ndiff(Y0, Y1, (size_t)M * CO);
            u[r][2] = timeit(k2, g, NT, ad, bd, EpiBiasRelu{Y1, b, M, CO}, KP / GK, tm, tn);
            if (r == 0) dd[1] = ndiff(Y0, Y1, (size_t)M * CO);
            u[r][3] = timeit(k3, g, NT, ad, bd, EpiBiasRelu{Y1, b, M, CO}, KP / GK, tm, tn);
            if (r == 0) dd[2] = ndiff(Y0, Y1, (size_t)M * CO);
        }
        printf("\n%-6s dx6 product %7.3f %7.3f | no fences %7.3f %7.3f | interleave2 %7.3f %7.3f | "
               "interleave3 %7.3f %7.3f ms | differ %zu %zu %zu\n", tag, u[0][0], u[1][0], u[0][1],
               u[1][1], u[0][2], u[1][2], u[0][3], u[1][3], dd[0], dd[1], dd[2]);
    }
    printf("%-6s %3dx%3d %d waves  product dx6 %7.3f %7.3f ms %6.1f TF/s | halo (patch %d rows, "
           "%.1f KB) %7.3f %7.3f ms %6.1f TF/s (x%.3f) | differ %zu of %zu\n",
           tag, BM, BN, WAVES, t[0][0], t[1][0], tf(t[1][0]), need,
           HA::FL * 4 / 1024.0, t[0][1], t[1][1], tf(t[1][1]),
           (t[0][0] + t[1][0]) / (t[0][1] + t[1][1]), d, (size_t)M * CO);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const std::string only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return only.empty() || only.find(t) != std::string::npos; };
    const size_t big = (size_t)S * 36 * 36 * 96;     // largest output (conv4: 20x20x96 in -> 20^2x96)
    float* X = dalloc((size_t)S * 34 * 34 * 48, 1.f);
    const size_t w = 96 * 864;
    float* W = dalloc(w, 0.05f);
    const Xs Wx = to_xs(W, w);
    float* b = dalloc(256, 0.01f);
    float* Y0 = dalloc(big / 2, 0.f);
    float* Y1 = dalloc(big / 2, 0.f);
    auto sm = [&](int hw, int ci) {        // X[0 : S*hw*ci] split, slice-major
        const size_t n = (size_t)S * hw * ci;
        Xs x = to_xs(X, n), o;
        CK(hipMalloc(&o.hm, n * 4));
        CK(hipMalloc(&o.l, n * 2));
        const long units = (long)(n / 4);
        hipLaunchKernelGGL(k_to_sm, dim3((units + 255) / 256), dim3(256), 0, 0,
                           reinterpret_cast<const f32x4*>(x.hm), reinterpret_cast<const f32x2*>(x.l),
                           reinterpret_cast<f32x4*>(o.hm), reinterpret_cast<f32x2*>(o.l), units, hw,
                           ci / 4);
        CK(hipDeviceSynchronize());
        CK(hipFree(x.hm));
        CK(hipFree(x.l));
        return o;
    };
    // the product's tiles (pn1_net.hip): conv2 4 waves of 64 rows, conv3 / conv4 8 waves of 32
    if (want("fwd2")) {
        const Xs x = sm(34 * 34, 48);
        shape<34, 48, 48, true, 4, 3, 4, 3, 14>("fwd2", x, Wx, b, Y0, Y1, S);
        shape<34, 48, 48, true, 4, 3, 4, 3, 14, 2>("fwd2", x, Wx, b, Y0, Y1, S);
        shape<34, 48, 48, true, 4, 3, 8, 3, 22, 2>("fwd2", x, Wx, b, Y0, Y1, S);
        shape<34, 48, 48, true, 2, 3, 8, 3, 14, 2>("fwd2", x, Wx, b, Y0, Y1, S);
        shape<34, 48, 48, true, 2, 3, 8, 3, 14, 3>("fwd2", x, Wx, b, Y0, Y1, S);
        CK(hipFree(x.hm));
        CK(hipFree(x.l));
    }
    if (want("fwd3")) {
        const Xs x = sm(18 * 18, 48);
        shape<18, 48, 96, false, 2, 6, 8, 3, 18>("fwd3", x, Wx, b, Y0, Y1, S);
        shape<18, 48, 96, false, 4, 6, 4, 3, 18, 2>("fwd3", x, Wx, b, Y0, Y1, S);
        CK(hipFree(x.hm));
        CK(hipFree(x.l));
    }
    if (want("fwd4")) {
        const Xs x = sm(20 * 20, 96);
        shape<20, 96, 96, true, 2, 6, 8, 3, 20>("fwd4", x, Wx, b, Y0, Y1, S);
        shape<20, 96, 96, true, 2, 6, 8, 3, 20, 3>("fwd4", x, Wx, b, Y0, Y1, S);
        shape<20, 96, 96, true, 4, 6, 4, 3, 20, 2>("fwd4", x, Wx, b, Y0, Y1, S);
        CK(hipFree(x.hm));
        CK(hipFree(x.l));
    }
    return 0;
}
