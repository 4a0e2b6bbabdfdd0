// Split-form operand lab (development tool, not part of libflsim.so): the split-bf16 GEMMs over
// operands that arrive already split (split.h: HM + L tensors written by their producers) against
// gemm_x6_kernel over fp32 operands (split while staged), on PerformantNet1's shapes at 16,384
// samples.  Three kernels per conv forward / data-gradient shape:
//   x6   gemm_x6_kernel, fp32 operands (the round-3 product)
//   xs   gemm_x6_kernel, split operands (plane stores only)
//   dx6  gemm_dx6_kernel, split operands, A straight into registers, B staged KB k-steps a time
// and x6 / xs for the weight gradients.  Every split variant must equal x6 bit for bit (same RNE
// split, same MFMA order per accumulator); the line prints the count of differing outputs.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include \
//         -I fl-distributed-delay_amd/csrc tools/lab/xs_lab.hip -o tools/lab/xs_lab
#include <cmath>
#include <string>

#include "gemm_dx6.h"
#include "lab_common.h"

static __global__ void k_to_xs(const float* x, float* hm, float* l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(x)[u]);
}

struct Xs {
    float* hm;
    float* l;
};

// [img][pix][CI] split tensor -> channel-slice-major [img][CI/16][pix][16] (whole 16-B HM / 8-B L units)
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

// conv forward / data gradient: Y = relu(im2col(X) W^T + b), fp32 out
template <int IH, int CI, int PAD, int OHX, int CO, int FM, int FN, int WM, int WN, int DFM,
          int DFN, int DW, int KB, int DEPTH, int NPL>
static void conv(const char* tag, const float* X, const Xs& Xx, const float* W, const Xs& Wx,
                 const float* b, float* Y0, float* Y1, float* Y2, int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT, false, OHX>;
    using BL = RowsKC<BN, NT>;
    using ALs = Im2colKC<IH, IH, CI, PAD, BM, NT, false, OHX, XsSrc>;
    using BLs = RowsKC<BN, NT, XsSrc>;
    const int KP = 9 * CI;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    const int M = al.M;
    BL bl;
    bl.P = W;
    bl.ld = KP;
    bl.NR = CO;
    ALs als;
    als.X = Xx.hm;
    als.XL = Xx.l;
    als.M = M;
    BLs bls;
    bls.P = Wx.hm;
    bls.PL = Wx.l;
    bls.ld = KP;
    bls.NR = CO;
    const double flops = 2.0 * M * CO * KP;
    const int tm = ceil_div(M, BM), tn = ceil_div(CO, BN);
    const double t0 = timeit(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiBiasRelu>, dim3(tm * tn),
                             NT, al, bl, EpiBiasRelu{Y0, b, M, CO}, KP / GK, KP / GK, tm, tn);
    const double t1 = timeit(gemm_x6_kernel<FM, FN, WM, WN, ALs, BLs, EpiBiasRelu>, dim3(tm * tn),
                             NT, als, bls, EpiBiasRelu{Y1, b, M, CO}, KP / GK, KP / GK, tm, tn);
    // direct: DW waves of 16*DFM rows, all 16*DFN columns of an n-tile
    using AD = Im2colDirect<IH, IH, CI, PAD, DFM, false, OHX, XsSrc>;
    using BD = RowsKCStageXs<16 * DFN, 64 * DW, NPL>;
    AD ad;
    ad.X = Xx.hm;
    ad.XL = Xx.l;
    ad.M = M;
    BD bd;
    bd.P = Wx.hm;
    bd.PL = Wx.l;
    bd.ld = KP;
    bd.NR = CO;
    const int dtm = ceil_div(M, 16 * DFM * DW), dtn = ceil_div(CO, 16 * DFN);
    const double t2 = timeit(gemm_dx6_kernel<DFM, DFN, DW, KB, DEPTH, AD, BD, EpiBiasRelu>,
                             dim3(dtm * dtn), 64 * DW, ad, bd, EpiBiasRelu{Y2, b, M, CO}, KP / GK,
                             dtm, dtn);
    const size_t n = (size_t)M * CO;
    const size_t d1 = ndiff(Y0, Y1, n), d2 = ndiff(Y0, Y2, n);
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    printf("%-16s x6 %3dx%3d %7.3f ms %6.1f | xs %7.3f ms %6.1f | dx6 %3dx%3d kb%d d%d p%d %7.3f ms "
           "%6.1f TF/s | differ xs %zu dx6 %zu\n",
           tag, BM, BN, t0, tf(t0), t1, tf(t1), 16 * DFM * DW, 16 * DFN, KB, DEPTH, NPL, t2, tf(t2),
           d1, d2);
    if (getenv("LAB_SM")) {
        // the same direct kernel over a channel-slice-major copy of X (A B A B on one box)
        const long units = (long)S * IH * IH * CI / 4;
        Xs sm;
        CK(hipMalloc(&sm.hm, units * 16));
        CK(hipMalloc(&sm.l, units * 8));
        hipLaunchKernelGGL(k_to_sm, dim3((units + 255) / 256), dim3(256), 0, 0,
                           reinterpret_cast<const f32x4*>(Xx.hm), reinterpret_cast<const f32x2*>(Xx.l),
                           reinterpret_cast<f32x4*>(sm.hm), reinterpret_cast<f32x2*>(sm.l), units,
                           IH * IH, CI / 4);
        CK(hipDeviceSynchronize());
        using AS = Im2colDirect<IH, IH, CI, PAD, DFM, false, OHX, XsSrcSM>;
        AS as;
        as.X = sm.hm;
        as.XL = sm.l;
        as.M = M;
        auto kd = gemm_dx6_kernel<DFM, DFN, DW, KB, DEPTH, AD, BD, EpiBiasRelu>;
        auto ks = gemm_dx6_kernel<DFM, DFN, DW, KB, DEPTH, AS, BD, EpiBiasRelu>;
        const dim3 g(dtm * dtn);
        const double s0 = timeit(ks, g, 64 * DW, as, bd, EpiBiasRelu{Y1, b, M, CO}, KP / GK, dtm, dtn);
        const size_t d3 = ndiff(Y2, Y1, n);
        const double p1 = timeit(kd, g, 64 * DW, ad, bd, EpiBiasRelu{Y2, b, M, CO}, KP / GK, dtm, dtn);
        const double s1 = timeit(ks, g, 64 * DW, as, bd, EpiBiasRelu{Y1, b, M, CO}, KP / GK, dtm, dtn);
        printf("%-16s dx6 %7.3f %7.3f ms | dx6 slice-major %7.3f %7.3f ms %6.1f TF/s (x%.3f) | "
               "differs from dx6 in %zu\n", tag, t2, p1, s0, s1, tf(0.5 * (s0 + s1)),
               (t2 + p1) / (s0 + s1), d3);
        CK(hipFree(sm.hm));
        CK(hipFree(sm.l));
    }
    fflush(stdout);
}

// the same slab epilogue without the in-loop bias column sum (what the ASUM colsum costs)
struct EpiSlabAccNA : EpiSlabAcc {
    static constexpr bool ASUM = false;
};
// ... with the column sum on the vector unit (the round-3 form), and on the matrix cores (the
// product's EpiSlabAcc, gemm_x6.h AsumMfma)
struct EpiSlabAccValu : EpiSlabAcc {
    static constexpr bool ASUM_MFMA = false;
};
struct EpiSlabAccMF : EpiSlabAcc {
    static constexpr bool ASUM_MFMA = true;
};

// weight gradient: slab[z][co][kk] = sum over the split's pixels of dz[p][co] im2col(X)[p][kk]
template <int IH, int CI, int CO, int FM, int FN, int WM, int WN>
static void wgrad(const char* tag, const float* dz, const Xs& dzx, const float* X, const Xs& Xx,
                  float* S0, float* S1, float* B0, float* B1, int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int PAD = 1;
    using AL = RowsKM<BM, NT>;
    using BL = Im2colKM<IH, IH, CI, PAD, BN, NT>;
    using ALs = RowsKM<BM, NT, 0, 0, XsSrc>;
    using BLs = Im2colKM<IH, IH, CI, PAD, BN, NT, 0, XsSrc>;
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
    ALs als;
    als.P = dzx.hm;
    als.PL = dzx.l;
    als.ld = CO;
    als.NK = M;
    als.NC = CO;
    BLs bls;
    bls.X = Xx.hm;
    bls.XL = Xx.l;
    bls.M = M;
    const int ks = ceil_div(M, GK);
    const int per = ceil_div(ks, Z);
    const int tm = ceil_div(CO, BM), tn = ceil_div(KP, BN);
    const double flops = 2.0 * M * CO * KP;
    EpiSlabAcc e0{S0, CO, KP, (long)CO * KP, B0, 0}, e1{S1, CO, KP, (long)CO * KP, B1, 0};
    EpiSlabAccValu v0, v1;
    static_cast<EpiSlabAcc&>(v0) = e0;
    static_cast<EpiSlabAcc&>(v1) = e1;
    const double t0 = timeit(gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAccValu>,
                             dim3(tm * tn * Z), NT, al, bl, v0, ks, per, tm, tn);
    const double t1 = timeit(gemm_x6_kernel<FM, FN, WM, WN, ALs, BLs, EpiSlabAccValu>,
                             dim3(tm * tn * Z), NT, als, bls, v1, ks, per, tm, tn);
    const size_t d = ndiff(S0, S1, (size_t)Z * CO * KP), db = ndiff(B0, B1, (size_t)Z * CO);
    EpiSlabAccNA e2;
    static_cast<EpiSlabAcc&>(e2) = e1;
    const double t2 = timeit(gemm_x6_kernel<FM, FN, WM, WN, ALs, BLs, EpiSlabAccNA>,
                             dim3(tm * tn * Z), NT, als, bls, e2, ks, per, tm, tn);
    std::vector<float> hb1((size_t)Z * CO);
    hipMemcpy(hb1.data(), B1, hb1.size() * 4, hipMemcpyDeviceToHost);
    EpiSlabAccMF e3;
    static_cast<EpiSlabAcc&>(e3) = e1;
    e3.Bsl = B0;
    const double t3 = timeit(gemm_x6_kernel<FM, FN, WM, WN, ALs, BLs, EpiSlabAccMF>,
                             dim3(tm * tn * Z), NT, als, bls, e3, ks, per, tm, tn);
    std::vector<float> hb3((size_t)Z * CO);
    hipMemcpy(hb3.data(), B0, hb3.size() * 4, hipMemcpyDeviceToHost);
    double num = 0, den = 0;
    for (size_t i = 0; i < hb1.size(); ++i) {
        num += ((double)hb3[i] - hb1[i]) * ((double)hb3[i] - hb1[i]);
        den += (double)hb1[i] * hb1[i];
    }
    auto tf = [&](double t) { return flops / (t * 1e-3) / 1e12; };
    printf("%-16s x6 %3dx%3d Z %4d %7.3f ms %6.1f | xs (valu bias sum) %7.3f ms %6.1f | xs no-bias-sum "
           "%7.3f ms %6.1f | xs mfma-bias-sum %7.3f ms %6.1f TF/s | differ slab %zu bias %zu | mfma bias "
           "rel-L2 vs valu %.2e\n",
           tag, BM, BN, Z, t0, tf(t0), t1, tf(t1), t2, tf(t2), t3, tf(t3), d, db,
           std::sqrt(num / (den > 0 ? den : 1)));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    const Xs Xx = to_xs(X, big);
    float* Y0 = dalloc(big, 0.f);
    float* Y1 = dalloc(big, 0.f);
    float* Y2 = dalloc(big, 0.f);
    const size_t wn = 512 * 4608;
    float* W = dalloc(wn, 0.05f);
    const Xs Wx = to_xs(W, wn);
    float* b = dalloc(256, 0.01f);
    const size_t slabn = (size_t)4096 * 48 * 432;
    float* S0 = dalloc(slabn, 0.f);
    float* S1 = dalloc(slabn, 0.f);
    float* B0 = dalloc(4096 * 192, 0.f);
    float* B1 = dalloc(4096 * 192, 0.f);
    // argv[1]: a tag substring, or a comma-separated list of exact tags ("fwd6,dg4,wg6")
    const std::string only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) {
        if (only.empty()) return true;
        if (only.find(',') == std::string::npos) return strstr(t, only.c_str()) != nullptr;
        size_t p0 = 0;
        while (p0 <= only.size()) {
            const size_t p1 = std::min(only.find(',', p0), only.size());
            if (only.compare(p0, p1 - p0, t) == 0 && strlen(t) == p1 - p0) return true;
            p0 = p1 + 1;
        }
        return false;
    };
    // C(tag, IH, CI, PAD, OHX, CO, x6 tile FM FN WM WN, direct DFM DFN WAVES KB DEPTH NPL)
#define C(tag, IH, CI, PAD, OHX, CO, FM, FN, WM, WN, DFM, DFN, DW, KB, DEP, NPL) \
    if (want(tag)) conv<IH, CI, PAD, OHX, CO, FM, FN, WM, WN, DFM, DFN, DW, KB, DEP, NPL>( \
        tag, X, Xx, W, Wx, b, Y0, Y1, Y2, S);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN) \
    if (want(tag)) wgrad<IH, CI, CO, FM, FN, WM, WN>(tag, X, Xx, X, Xx, S0, S1, B0, B1, S, Z);
    C("fwd6", 13, 192, 2, 0, 192, 4, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd6 p3", 13, 192, 2, 0, 192, 4, 6, 4, 2, 2, 6, 8, 3, 2, 3)
    C("fwd6 n192", 13, 192, 2, 0, 192, 4, 6, 4, 2, 2, 12, 8, 2, 1, 2)
    C("fwd6 kb1", 13, 192, 2, 0, 192, 4, 6, 4, 2, 2, 6, 8, 2, 1, 2)
    C("fwd5", 11, 96, 2, 0, 192, 4, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd4", 20, 96, 2, 0, 96, 4, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd3", 18, 48, 2, 0, 96, 4, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd2", 34, 48, 2, 0, 48, 4, 3, 8, 1, 2, 3, 8, 3, 2, 2)
    C("dg6", 14, 192, 0, 13, 192, 4, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg5", 13, 192, 0, 0, 96, 4, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg4", 22, 96, 0, 0, 96, 4, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg3", 20, 96, 0, 0, 48, 8, 3, 4, 1, 2, 3, 8, 3, 2, 2)
    C("dg2", 36, 48, 0, 0, 48, 4, 3, 8, 1, 2, 3, 8, 3, 2, 2)
    // conv2 forward: direct-kernel variants (DFM DFN waves KB DEPTH NPL) beside round 4's 2 3 8 3 2 2
    // (KB must divide the 27 / 54 k-steps: r04j's KB 6 / 4 / 2 variants skipped k-steps)
    C("fwd2v a", 34, 48, 2, 0, 48, 4, 3, 8, 1, 4, 3, 8, 3, 2, 2)
    C("fwd2v b", 34, 48, 2, 0, 48, 4, 3, 8, 1, 2, 3, 4, 3, 2, 2)
    C("fwd2v e", 34, 48, 2, 0, 48, 4, 3, 8, 1, 4, 3, 4, 3, 2, 2)
    C("fwd2v g", 34, 48, 2, 0, 48, 4, 3, 8, 1, 3, 3, 8, 3, 2, 2)
    C("fwd2v h", 34, 48, 2, 0, 48, 4, 3, 8, 1, 4, 3, 4, 9, 2, 2)
    C("fwd2v i", 34, 48, 2, 0, 48, 4, 3, 8, 1, 2, 3, 8, 9, 2, 2)
    C("fwd2v k", 34, 48, 2, 0, 48, 4, 3, 8, 1, 8, 3, 2, 3, 2, 2)
    C("fwd2v l", 34, 48, 2, 0, 48, 4, 3, 8, 1, 4, 3, 2, 3, 2, 2)
    // conv3 / conv4 forward (product: DFM 2, 8 waves, KB 3)
    C("fwd3v a", 18, 48, 2, 0, 96, 4, 3, 4, 2, 4, 6, 4, 3, 2, 2)
    C("fwd4v a", 20, 96, 2, 0, 96, 4, 3, 4, 2, 4, 6, 4, 3, 2, 2)
    C("fwd4v b", 20, 96, 2, 0, 96, 4, 3, 4, 2, 2, 6, 8, 6, 2, 2)
    // weight-gradient tile variants for conv3 / conv2 (product: wg3 3 3 2 2 since r04j, wg2 3 3 1 3)
    G("wg3v 96x96x4", 18, 48, 96, 1024, 3, 3, 2, 2)
    G("wg3v 96x144x2", 18, 48, 96, 1024, 3, 9, 2, 1)
    G("wg3v 96x144x6", 18, 48, 96, 1024, 3, 3, 2, 3)
    G("wg3v 48x48x1", 18, 48, 96, 1024, 3, 3, 1, 1)
    G("wg2v 48x144x1", 34, 48, 48, 4096, 3, 9, 1, 1)
    G("wg2v 48x48x1", 34, 48, 48, 4096, 3, 3, 1, 1)
    G("wg2v 48x96x2", 34, 48, 48, 4096, 3, 3, 1, 2)
    // staged (xs) tile variants for the N = 192 / 96 forward and data-gradient GEMMs
    // (product: fwd5/fwd6/dg6 4 6 4 2, dg4/dg5 4 3 4 2)
    C("fwd6v a", 13, 192, 2, 0, 192, 3, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd6v b", 13, 192, 2, 0, 192, 2, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg6v a", 14, 192, 0, 13, 192, 3, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg6v b", 14, 192, 0, 13, 192, 2, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("fwd5v a", 11, 96, 2, 0, 192, 3, 6, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg5v a", 13, 192, 0, 0, 96, 4, 6, 4, 1, 2, 6, 8, 3, 2, 2)
    C("dg5v b", 13, 192, 0, 0, 96, 2, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    C("dg4v a", 22, 96, 0, 0, 96, 4, 6, 4, 1, 2, 6, 8, 3, 2, 2)
    C("dg4v b", 22, 96, 0, 0, 96, 2, 3, 4, 2, 2, 6, 8, 3, 2, 2)
    // weight-gradient tile variants for conv4 / conv5 / conv6 (product: 3 3 2 2 / 6 3 2 2 / 6 3 2 2)
    G("wg4v 96x144x2", 20, 96, 96, 1024, 3, 9, 2, 1)
    G("wg4v 96x144x6", 20, 96, 96, 1024, 3, 3, 2, 3)
    G("wg4v 96x96x2", 20, 96, 96, 1024, 3, 6, 2, 1)
    G("wg5v 192x144x6", 11, 96, 192, 512, 6, 3, 2, 3)
    G("wg5v 192x96x8", 11, 96, 192, 512, 3, 3, 4, 2)
    G("wg6v 192x192x4", 13, 192, 192, 256, 6, 6, 2, 2)
    G("wg6v 192x144x6", 13, 192, 192, 256, 6, 3, 2, 3)
    G("wg6v 192x96x8", 13, 192, 192, 256, 3, 3, 4, 2)
    G("wg6v 192x192x8", 13, 192, 192, 256, 3, 6, 4, 2)
    // round 5: larger per-wave fragments at fewer waves
    C("fwd6wa", 13, 192, 2, 0, 192, 8, 6, 2, 2, 2, 6, 8, 3, 2, 2)
    C("fwd6wb", 13, 192, 2, 0, 192, 4, 12, 4, 1, 2, 6, 8, 3, 2, 2)
    C("fwd6wc", 13, 192, 2, 0, 192, 8, 12, 2, 1, 2, 6, 8, 3, 2, 2)
    C("fwd6wd", 13, 192, 2, 0, 192, 6, 6, 2, 2, 2, 6, 8, 3, 2, 2)
    G("wg6wa", 13, 192, 192, 256, 6, 6, 2, 1)
    G("wg6wb", 13, 192, 192, 256, 6, 12, 2, 1)
    G("wg6wc", 13, 192, 192, 256, 12, 3, 1, 3)
    // weight gradients (product tiles and splits: >= 32 k-steps per split)
    G("wg6", 13, 192, 192, 256, 6, 3, 2, 2)
    G("wg5", 11, 96, 192, 512, 6, 3, 2, 2)
    G("wg4", 20, 96, 96, 1024, 3, 3, 2, 2)
    G("wg3", 18, 48, 96, 1024, 3, 3, 2, 1)
    G("wg2", 34, 48, 48, 4096, 3, 3, 1, 3)
    return 0;
}
