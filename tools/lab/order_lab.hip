// K-order lab (development tool, not part of libflsim.so): the conv GEMMs of PerformantNet1 at the
// 128-worker chunk (S = 16384 samples) with the reduction index in the product's tap-major order
// (k = tap * CI + ci) against a channel-slice-major order (k = (ci / 16) * 144 + tap * 16 + ci % 16):
// the nine taps of one 16-channel slice of the input window are then read in nine consecutive
// k-steps (forward / data gradient) or by one block (weight-gradient columns), so the re-reads hit
// L1/L2 instead of going back out past L2.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/order_lab.hip -o tools/lab/order_lab
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>

#include "loaders.h"

using namespace flsim;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// Im2colKC with the k-step -> (tap, channel slice) map selectable (CI % 16 == 0 only)
template <int IH, int IW, int CI, int PAD, int TR, int NT, int ORD>
struct Im2colKCo : Im2colKC<IH, IW, CI, PAD, TR, NT> {
    using Base = Im2colKC<IH, IW, CI, PAD, TR, NT>;
    static_assert(CI % 16 == 0, "");
    __device__ void load(int ks, f32x4 (&r)[Base::UNITS]) const {
        int khkw, ci0;
        if constexpr (ORD == 0) {
            khkw = ks * GK / CI;
            ci0 = ks * GK - khkw * CI;
        } else {
            const int cs = ks / 9;
            khkw = ks - 9 * cs;
            ci0 = cs * GK;
        }
        const int kh = khkw / 3;
        const long off = (long)(kh * IW + (khkw - 3 * kh)) * CI + ci0;
#pragma unroll
        for (int j = 0; j < Base::UNITS; ++j) {
            const bool ok = khkw < 9 && ((this->tapmask[j] >> khkw) & 1);
            r[j] = ok ? ldg4(this->X + this->base[j] + off) : zero4();
        }
    }
};

template <int IH, int IW, int CI, int PAD, int TR, int NT, int ORD, int VO = 0>
struct Im2colKMo : Im2colKM<IH, IW, CI, PAD, TR, NT, VO> {
    using Base = Im2colKM<IH, IW, CI, PAD, TR, NT, VO>;
    __device__ void setup(int c0, int tid) {
        Base::setup(c0, tid);
        if constexpr (ORD == 1) {
#pragma unroll
            for (int j = 0; j < Base::UNITS; ++j) {
                const int u = tid + j * NT;
                const int kk = c0 + 4 * (u % Base::C4);
                const int cs = kk / 144, rem = kk - 144 * cs;
                const int tap = rem >> 4;
                this->kh[j] = (short)(tap / 3);
                this->kw[j] = (short)(tap % 3);
                this->coff[j] = (u < Base::TOTAL && cs < CI / 16) ? cs * 16 + (rem & 15) : -1;
            }
        }
    }
};

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
    for (int i = 0; i < 2; ++i)
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipDeviceSynchronize());
    const int iters = getenv("LAB_ITERS") ? atoi(getenv("LAB_ITERS")) : 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-30s tile %3dx%3d Z%5d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, BM, BN, Z, grid.x, ms,
           flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return ms;
}

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN, int ORD>
static void conv_fwd(const char* tag, const float* X, const float* W, const float* b, float* Y,
                     int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKCo<IH, IH, CI, PAD, BM, NT, ORD>;
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
    time_gemm<FM, FN, WM, WN>(tag, al, bl, epi, al.M, CO, KP / GK, 1, 2.0 * al.M * CO * KP);
}

template <int IH, int CI, int CO, int FM, int FN, int WM, int WN, int ORD, int VO = 0>
static void conv_wgrad(const char* tag, const float* dz, const float* X, float* slab, float* bslab,
                       int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2;
    using AL = RowsKM<BM, NT, (VO > 0 ? OFULL : 0), VO>;
    using BL = Im2colKMo<IH, IH, CI, 2, BN, NT, ORD, VO>;
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
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    time_gemm<FM, FN, WM, WN>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * KP);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y = dalloc(big, 0.f);
    float* W = dalloc(192 * 1728 + 64, 0.05f);
    float* b = dalloc(256, 0.01f);
    const size_t slabn = (size_t)4096 * 48 * 432;
    float* slab = dalloc(slabn, 0.f);
    float* bsl = dalloc(4096 * 192, 0.f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define F(tag, IH, CI, PAD, CO, FM, FN, WM, WN, ORD) \
    if (want(tag)) conv_fwd<IH, CI, PAD, CO, FM, FN, WM, WN, ORD>(tag, X, W, b, Y, S);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN, ORD, VO) \
    if (want(tag)) conv_wgrad<IH, CI, CO, FM, FN, WM, WN, ORD, VO>(tag, Y, X, slab, bsl, S, Z);
    // forward / data-gradient shapes (product tiles)
    F("fwd6 ord0", 13, 192, 2, 192, 2, 6, 4, 2, 0)
    F("fwd6 ord1", 13, 192, 2, 192, 2, 6, 4, 2, 1)
    F("dg6 ord0", 15, 192, 0, 192, 2, 6, 4, 2, 0)
    F("dg6 ord1", 15, 192, 0, 192, 2, 6, 4, 2, 1)
    F("fwd5 ord0", 11, 96, 2, 192, 2, 6, 4, 2, 0)
    F("fwd5 ord1", 11, 96, 2, 192, 2, 6, 4, 2, 1)
    F("dg5 ord0", 13, 192, 0, 96, 4, 3, 4, 2, 0)
    F("dg5 ord1", 13, 192, 0, 96, 4, 3, 4, 2, 1)
    F("fwd4 ord0", 20, 96, 2, 96, 4, 3, 4, 2, 0)
    F("fwd4 ord1", 20, 96, 2, 96, 4, 3, 4, 2, 1)
    F("dg4 ord0", 22, 96, 0, 96, 4, 3, 4, 2, 0)
    F("dg4 ord1", 22, 96, 0, 96, 4, 3, 4, 2, 1)
    F("fwd3 ord0", 18, 48, 2, 96, 4, 3, 4, 2, 0)
    F("fwd3 ord1", 18, 48, 2, 96, 4, 3, 4, 2, 1)
    F("dg3 ord0", 20, 96, 0, 48, 2, 3, 8, 1, 0)
    F("dg3 ord1", 20, 96, 0, 48, 2, 3, 8, 1, 1)
    F("fwd2 ord0", 34, 48, 2, 48, 2, 3, 8, 1, 0)
    F("fwd2 ord1", 34, 48, 2, 48, 2, 3, 8, 1, 1)
    F("dg2 ord0", 36, 48, 0, 48, 2, 3, 8, 1, 0)
    F("dg2 ord1", 36, 48, 0, 48, 2, 3, 8, 1, 1)
    // weight gradients (product tiles and split counts)
    G("wg6 ord0", 13, 192, 192, 256, 6, 3, 2, 2, 0, 14)
    G("wg6 ord1", 13, 192, 192, 256, 6, 3, 2, 2, 1, 14)
    G("wg5 ord0", 11, 96, 192, 512, 6, 3, 2, 2, 0, 0)
    G("wg5 ord1", 11, 96, 192, 512, 6, 3, 2, 2, 1, 0)
    G("wg4 ord0", 20, 96, 96, 1024, 3, 3, 2, 2, 0, 0)
    G("wg4 ord1", 20, 96, 96, 1024, 3, 3, 2, 2, 1, 0)
    G("wg3 ord0", 18, 48, 96, 2048, 3, 3, 2, 2, 0, 0)
    G("wg3 ord1", 18, 48, 96, 2048, 3, 3, 2, 2, 1, 0)
    G("wg2 ord0", 34, 48, 48, 4096, 3, 3, 1, 3, 0, 0)
    G("wg2 ord1", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 0)
    return 0;
}
