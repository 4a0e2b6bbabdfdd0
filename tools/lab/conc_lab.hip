// Concurrency lab (development tool, not part of libflsim.so): do two independent GEMM launches of
// one layer's backward (the data gradient and the weight gradient both read dZ) gain from running on
// two streams at once, i.e. how much do the launch tails cost?  PerformantNet1 conv6 / conv4 / conv2
// shapes at S = 16384 samples, the product's gemm_kernel and tiles.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/conc_lab.hip -o tools/lab/conc_lab
#include <functional>

#include "lab_common.h"

using Launch = std::function<void(hipStream_t)>;

template <int FM, int FN, int WM, int WN, class AL, class BL, class EPI>
static Launch make(const AL& al, const BL& bl, const EPI& epi, int M, int N, int ksteps, int Z) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    return [=](hipStream_t st) {
        hipLaunchKernelGGL((gemm_kernel<FM, FN, WM, WN, AL, BL, EPI>), dim3(tm * tn * Z),
                           dim3(64 * WM * WN), 0, st, al, bl, epi, ksteps, per, tm, tn);
    };
}

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN>
static Launch conv(const float* X, const float* W, const float* b, float* Y, int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IH, CI, PAD, BM, NT>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = W;
    bl.ld = 9 * CI;
    bl.NR = CO;
    EpiBiasRelu epi{Y, b, al.M, CO};
    return make<FM, FN, WM, WN>(al, bl, epi, al.M, CO, 9 * CI / GK, 1);
}

template <int IH, int CI, int CO, int FM, int FN, int WM, int WN, int VO = 0>
static Launch wgrad(const float* dz, const float* X, float* slab, float* bsl, int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2;
    using AL = RowsKM<BM, NT, (VO > 0 ? OFULL : 0), VO>;
    using BL = Im2colKM<IH, IH, CI, 2, BN, NT, VO>;
    const int M = S * BL::OH * BL::OW;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, 9 * CI, (long)CO * 9 * CI, bsl};
    return make<FM, FN, WM, WN>(al, bl, epi, CO, 9 * CI, ceil_div(M, GK), Z);
}

static float time_pair(const Launch& a, const Launch& b, hipStream_t s1, hipStream_t s2, bool conc,
                       int iters) {
    hipEvent_t e0, e1, j;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&j));
    a(s1);
    b(s1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s1));
    CK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) {
        a(s1);
        b(conc ? s2 : s1);
    }
    CK(hipEventRecord(j, s2));
    CK(hipStreamWaitEvent(s1, j, 0));
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

int main() {
    const int S = 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y = dalloc(big, 0.5f);
    float* Y2 = dalloc(big, 0.f);
    float* W = dalloc(192 * 1728 + 64, 0.05f);
    float* b = dalloc(256, 0.01f);
    float* slab = dalloc((size_t)4096 * 48 * 432, 0.f);
    float* bsl = dalloc(4096 * 192, 0.f);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    struct Case { const char* tag; Launch a, b; };
    Case cases[] = {
        {"conv6 dgrad + wgrad", conv<15, 192, 0, 192, 2, 6, 4, 2>(Y, W, b, Y2, S),
         wgrad<13, 192, 192, 6, 3, 2, 2, 14>(Y, X, slab, bsl, S, 256)},
        {"conv4 dgrad + wgrad", conv<22, 96, 0, 96, 4, 3, 4, 2>(Y, W, b, Y2, S),
         wgrad<20, 96, 96, 3, 3, 2, 2>(Y, X, slab, bsl, S, 1024)},
        {"conv2 dgrad + wgrad", conv<36, 48, 0, 48, 2, 3, 8, 1>(Y, W, b, Y2, S),
         wgrad<34, 48, 48, 3, 3, 1, 3>(Y, X, slab, bsl, S, 4096)},
    };
    for (auto& c : cases) {
        const float ta = time_pair(c.a, [](hipStream_t) {}, s1, s2, false, 5);
        const float tb = time_pair([](hipStream_t) {}, c.b, s1, s2, false, 5);
        const float ser = time_pair(c.a, c.b, s1, s2, false, 5);
        const float con = time_pair(c.a, c.b, s1, s2, true, 5);
        printf("%-22s A %7.3f  B %7.3f  serial %7.3f  concurrent %7.3f ms  (%.1f %% saved)\n", c.tag,
               ta, tb, ser, con, 100.f * (ser - con) / ser);
        fflush(stdout);
    }
    return 0;
}
