// Tile sweep (from the ablation lab).  Ablation lab: 0 full, 1 no barrier, 2 no LDS stores, 3 no global loads, 4 no staging, 5 no staging
// and no barrier, 6 A operand not loaded, 7 B operand not loaded (timing only: 1-5 compute wrong sums).  From the pipeline lab (development tool, not part of libflsim.so): the product's GEMM pipeline with
// KSUB 16-deep sub-steps per LDS stage and barrier (fewer barriers per MFMA), and PIN = keep the
// k-step's MFMAs ahead of the barrier (sched_barrier; the compiler otherwise hoists the barrier
// above them).  Conv shapes of PerformantNet1 at S = 16384 samples, channel-slice-major K order.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/ks_lab.hip -o tools/lab/ks_lab
#include "lab_common.h"

template <int FM, int FN, int WAVES_M, int WAVES_N, int KSUB, int PIN, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_ks(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m, int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    constexpr int A_FL = tile_floats<AL::KC, BM>();
    constexpr int B_FL = tile_floats<BL::KC, BN>();
    constexpr int SUB = A_FL + B_FL;
    constexpr int BUF = KSUB * SUB;
    __shared__ __attribute__((aligned(16))) float lds[2 * BUF];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WAVES_N;
    const int wn = wave % WAVES_N;
    const int gx = tiles_m, gy = tiles_n;
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int q = nb / 8, r = nb % 8, xcd = b % 8;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
    const int tn = L % gy;
    const int tm = (L / gy) % gx;
    const int tz = L / (gx * gy);
    const int m0 = tm * BM;
    const int n0 = tn * BN;
    const int ks0 = tz * ksteps_per_split;
    int ks1 = ks0 + ksteps_per_split;
    if (ks1 > ksteps_total) ks1 = ksteps_total;
    al.setup(m0, tid);
    bl.setup(n0, tid);
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float asum = 0.f;
    f32x4 ra[KSUB][AL::UNITS];
    f32x4 rb[KSUB][BL::UNITS];
    auto load_stage = [&](int ks) {
#pragma unroll
        for (int s = 0; s < KSUB; ++s)
            if (ks + s < ks1) {
                if constexpr (PIN == 3) {     // no global loads: stage register constants
#pragma unroll
                    for (int u = 0; u < AL::UNITS; ++u) ra[s][u] = f32x4{(float)ks, 1.f, 2.f, 3.f};
#pragma unroll
                    for (int u = 0; u < BL::UNITS; ++u) rb[s][u] = f32x4{(float)ks, 1.f, 2.f, 3.f};
                } else if constexpr (PIN == 6) {   // A constant, B loaded
#pragma unroll
                    for (int u = 0; u < AL::UNITS; ++u) ra[s][u] = f32x4{(float)ks, 1.f, 2.f, 3.f};
                    bl.load(ks + s, rb[s]);
                } else if constexpr (PIN == 7) {   // A loaded, B constant
                    al.load(ks + s, ra[s]);
#pragma unroll
                    for (int u = 0; u < BL::UNITS; ++u) rb[s][u] = f32x4{(float)ks, 1.f, 2.f, 3.f};
                } else {
                    al.load(ks + s, ra[s]);
                    bl.load(ks + s, rb[s]);
                }
            }
    };
    auto store_stage = [&](float* base, int ks) {
#pragma unroll
        for (int s = 0; s < KSUB; ++s)
            if (ks + s < ks1) {
                if constexpr (PIN == 2) {     // keep the loads alive, skip the LDS stores
                    float t = 0.f;
#pragma unroll
                    for (int u = 0; u < AL::UNITS; ++u) t += ra[s][u].x;
#pragma unroll
                    for (int u = 0; u < BL::UNITS; ++u) t += rb[s][u].x;
                    if (t == 1234.5f) base[tid] = t;
                } else {
                    al.store(base + s * SUB, ra[s]);
                    bl.store(base + s * SUB + A_FL, rb[s]);
                }
            }
    };
    if (ks0 < ks1) {
        load_stage(ks0);
        store_stage(lds, ks0);
        if (ks0 + KSUB < ks1) load_stage(ks0 + KSUB);
    }
    __syncthreads();
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    int cur = 0;
    for (int ks = ks0; ks < ks1; ks += KSUB) {
        if (PIN != 4 && PIN != 5 && ks + KSUB < ks1) {
            store_stage(lds + (cur ^ 1) * BUF, ks + KSUB);
            if (ks + 2 * KSUB < ks1) load_stage(ks + 2 * KSUB);
        }
#pragma unroll
        for (int s = 0; s < KSUB; ++s) {
            if (KSUB == 1 || ks + s < ks1) {
                const float* A = lds + cur * BUF + s * SUB;
                const float* B = A + A_FL;
                if constexpr (EPI::ASUM) {
                    if (tn == 0 && tid < BM) {
#pragma unroll
                        for (int k = 0; k < GK; ++k) asum += A[k * KMTile<BM>::STRIDE + tid];
                    }
                }
                f32x4 af[FM], bf[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) af[i] = read_frag<AL::KC, BM>(A, wm * 16 * FM + 16 * i, lane);
#pragma unroll
                for (int j = 0; j < FN; ++j) bf[j] = read_frag<BL::KC, BN>(B, wn * 16 * FN + 16 * j, lane);
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
            }
        }
        if constexpr (PIN != 1 && PIN != 5) __syncthreads();
        cur ^= 1;
    }
    if constexpr (EPI::ASUM) {
        if (tn == 0 && tid < BM) epi.asum(m0 + tid, tz, asum);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int m = m0 + wm * 16 * FM + 16 * i + 4 * (lane >> 4);
            const int n = n0 + wn * 16 * FN + 16 * j + (lane & 15);
            epi.apply4(m, n, tz, acc[i][j]);
        }
}

template <int FM, int FN, int WM, int WN, int KSUB, int PIN, class AL, class BL, class EPI>
static double time_ks(const char* tag, const AL& al, const BL& bl, const EPI& epi, int M, int N,
                      int ksteps, int Z, double flops) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = ((ksteps + Z - 1) / Z + KSUB - 1) / KSUB * KSUB;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * ceil_div(ksteps, per));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm_ks<FM, FN, WM, WN, KSUB, PIN, AL, BL, EPI>;
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
    printf("%-24s KSUB%d ABL%d tile %3dx%3d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, KSUB, PIN, BM, BN,
           grid.x, ms, flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return ms;
}

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN, int KSUB, int PIN>
static void conv_fwd(const char* tag, const float* X, const float* W, const float* b, float* Y,
                     int S) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKCo<IH, IH, CI, PAD, BM, NT, 1>;
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
    time_ks<FM, FN, WM, WN, KSUB, PIN>(tag, al, bl, epi, al.M, CO, KP / GK, 1, 2.0 * al.M * CO * KP);
}

template <int IH, int CI, int CO, int FM, int FN, int WM, int WN, int KSUB, int PIN, int VO = 0,
          int PAD = 2>
static void conv_wgrad(const char* tag, const float* dz, const float* X, float* slab, float* bslab,
                       int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2 * PAD - 2;
    using AL = RowsKM<BM, NT, (VO > 0 ? OFULL : 0), VO>;
    using BL = Im2colKMo<IH, IH, CI, PAD, BN, NT, 0, VO>;
    const int M = S * BL::OH * BL::OW;
    const int KP = 9 * CI;
    if ((size_t)Z * CO * KP > (size_t)8192 * 48 * 432 || (size_t)Z * CO > (size_t)4096 * 192) {
        printf("%-24s skipped: Z * CO * KP exceeds the lab's slab capacity\n", tag);
        return;
    }
    if (Z == 0) {   // the product's split for this chunk (net_kernels.h wsplit: >= 32 k-steps
                    // per split, >= 1024 blocks)
        const int tiles = ceil_div(CO, BM) * ceil_div(KP, BN);
        const int ks = ceil_div(M, GK);
        Z = (ks + 31) / 32;
        if (Z < (1024 + tiles - 1) / tiles) Z = (1024 + tiles - 1) / tiles;
    }
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    time_ks<FM, FN, WM, WN, KSUB, PIN>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * KP);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y = dalloc(big, 0.f);
    float* W = dalloc(512 * 4608 + 64, 0.05f);    // up to vgg11's 512 x 4608
    float* b = dalloc(256, 0.01f);
    const size_t slabn = (size_t)8192 * 48 * 432;
    float* slab = dalloc(slabn, 0.f);
    float* bsl = dalloc(4096 * 192, 0.f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define F(tag, IH, CI, PAD, CO, FM, FN, WM, WN, KS, PIN) \
    if (want(tag)) conv_fwd<IH, CI, PAD, CO, FM, FN, WM, WN, KS, PIN>(tag, X, W, b, Y, S);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN, KS, PIN, VO) \
    if (want(tag)) conv_wgrad<IH, CI, CO, FM, FN, WM, WN, KS, PIN, VO>(tag, Y, X, slab, bsl, S, Z);
#define GV(tag, IH, CI, CO, Z, FM, FN, WM, WN) \
    if (want(tag)) conv_wgrad<IH, CI, CO, FM, FN, WM, WN, 1, 0, 0, 1>(tag, Y, X, slab, bsl, S, Z);
    F("fwd2 256x48 8w", 34, 48, 2, 48, 2, 3, 8, 1, 1, 0)
    F("fwd2 256x48 4w", 34, 48, 2, 48, 4, 3, 4, 1, 1, 0)
    F("fwd2 512x48 8w", 34, 48, 2, 48, 4, 3, 8, 1, 1, 0)
    F("fwd2 128x48 4w", 34, 48, 2, 48, 2, 3, 4, 1, 1, 0)
    F("fwd2 192x48 4w", 34, 48, 2, 48, 3, 3, 4, 1, 1, 0)
    F("dg2 256x48 8w", 36, 48, 0, 48, 2, 3, 8, 1, 1, 0)
    F("dg2 256x48 4w", 36, 48, 0, 48, 4, 3, 4, 1, 1, 0)
    F("dg2 512x48 8w", 36, 48, 0, 48, 4, 3, 8, 1, 1, 0)
    G("wg3 96x96 4w", 18, 48, 96, 2048, 3, 3, 2, 2, 1, 0, 0)
    G("wg3 96x48 2w", 18, 48, 96, 2048, 3, 3, 2, 1, 1, 0, 0)
    G("wg3 96x144 3w", 18, 48, 96, 2048, 6, 3, 1, 3, 1, 0, 0)
    G("wg3 48x144 3w", 18, 48, 96, 2048, 3, 3, 1, 3, 1, 0, 0)
    G("wg3 96x48 4w", 18, 48, 96, 2048, 3, 3, 2, 1, 1, 0, 0)
    G("wg2 48x144 3w", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 0, 0)
    G("wg2 48x48 1w", 34, 48, 48, 4096, 3, 3, 1, 1, 1, 0, 0)
    G("wg2 48x144 1w", 34, 48, 48, 4096, 3, 9, 1, 1, 1, 0, 0)
    G("wg2 48x96 2w", 34, 48, 48, 4096, 3, 3, 1, 2, 1, 0, 0)
    // round 2, after the buffer-resource loads: the largest weight gradients and forwards
    G("wg6 192x96 4w", 13, 192, 192, 256, 6, 3, 2, 2, 1, 0, 0)
    G("wg6 192x192 8w", 13, 192, 192, 256, 6, 3, 2, 4, 1, 0, 0)
    G("wg6 96x192 4w", 13, 192, 192, 256, 3, 6, 2, 2, 1, 0, 0)
    G("wg6 192x96 4w m4", 13, 192, 192, 256, 3, 6, 4, 1, 1, 0, 0)
    G("wg6 192x144 6w", 13, 192, 192, 256, 6, 3, 2, 3, 1, 0, 0)
    G("wg5 192x96 4w", 11, 96, 192, 512, 6, 3, 2, 2, 1, 0, 0)
    G("wg5 192x192 8w", 11, 96, 192, 512, 6, 3, 2, 4, 1, 0, 0)
    G("wg4 96x96 4w", 20, 96, 96, 1024, 3, 3, 2, 2, 1, 0, 0)
    G("wg4 96x192 8w", 20, 96, 96, 1024, 3, 3, 2, 4, 1, 0, 0)
    G("wg4 96x144 6w", 20, 96, 96, 1024, 3, 3, 2, 3, 1, 0, 0)
    G("wg3b 96x48 2w", 18, 48, 96, 2048, 3, 3, 2, 1, 1, 0, 0)
    G("wg3b 96x144 6w", 18, 48, 96, 2048, 3, 3, 2, 3, 1, 0, 0)
    G("wg2b 48x144 3w", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 0, 0)
    G("wg2b 48x144 6w", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 0, 0)
    F("fwd6 128x192 8w", 13, 192, 2, 192, 2, 6, 4, 2, 1, 0)
    F("fwd6 256x192 8w", 13, 192, 2, 192, 4, 6, 4, 2, 1, 0)
    F("fwd6 128x192 4w", 13, 192, 2, 192, 4, 6, 2, 2, 1, 0)
    F("fwd6 256x96 8w", 13, 192, 2, 192, 4, 3, 4, 2, 1, 0)
    F("fwd6 128x96 4w", 13, 192, 2, 192, 2, 3, 4, 2, 1, 0)
    F("dg6 128x192 8w", 15, 192, 0, 192, 2, 6, 4, 2, 1, 0)
    F("dg6 256x192 8w", 15, 192, 0, 192, 4, 6, 4, 2, 1, 0)
    F("dg6 256x96 8w", 15, 192, 0, 192, 4, 3, 4, 2, 1, 0)
    F("fwd4 256x96 8w", 20, 96, 2, 96, 4, 3, 4, 2, 1, 0)
    F("fwd4 128x96 4w", 20, 96, 2, 96, 4, 3, 2, 2, 1, 0)
    F("fwd4 256x96 4w", 20, 96, 2, 96, 8, 3, 2, 2, 1, 0)
    F("dg4 256x96 8w", 22, 96, 0, 96, 4, 3, 4, 2, 1, 0)
    F("dg4 128x96 4w", 22, 96, 0, 96, 4, 3, 2, 2, 1, 0)
    F("fwd5 128x192 8w", 11, 96, 2, 192, 2, 6, 4, 2, 1, 0)
    F("fwd5 256x192 8w", 11, 96, 2, 192, 4, 6, 4, 2, 1, 0)
    F("dg5 256x96 8w", 13, 192, 0, 96, 4, 3, 4, 2, 1, 0)
    F("dg5 128x96 4w", 13, 192, 0, 96, 4, 3, 2, 2, 1, 0)
    F("fwd5b 128x96 8w", 11, 96, 2, 192, 2, 3, 4, 2, 1, 0)
    F("fwd5b 128x192 8w", 11, 96, 2, 192, 2, 6, 4, 2, 1, 0)
    F("fwd3 256x96 8w", 18, 48, 2, 96, 4, 3, 4, 2, 1, 0)
    F("fwd3 128x96 4w", 18, 48, 2, 96, 4, 3, 2, 2, 1, 0)
    F("fwd3 128x96 8w", 18, 48, 2, 96, 2, 3, 4, 2, 1, 0)
    F("dg3 256x48 8w", 20, 96, 0, 48, 2, 3, 8, 1, 1, 0)
    F("dg3 128x48 4w", 20, 96, 0, 48, 2, 3, 4, 1, 1, 0)
    F("dg3 256x48 4w", 20, 96, 0, 48, 4, 3, 4, 1, 1, 0)
    F("dg2b 256x48 8w", 36, 48, 0, 48, 2, 3, 8, 1, 1, 0)
    F("dg2b 128x48 4w", 36, 48, 0, 48, 2, 3, 4, 1, 1, 0)
    F("fwd2b 128x48 4w", 34, 48, 2, 48, 2, 3, 4, 1, 1, 0)
    F("fwd2b 128x48 2w", 34, 48, 2, 48, 4, 3, 2, 1, 1, 0)
    F("fwd2c 256x48 4w", 34, 48, 2, 48, 4, 3, 4, 1, 1, 0)
    F("fwd2c 192x48 4w", 34, 48, 2, 48, 3, 3, 4, 1, 1, 0)
    F("fwd2c 128x48 4w", 34, 48, 2, 48, 2, 3, 4, 1, 1, 0)
    F("fwd2c 256x48 8w", 34, 48, 2, 48, 2, 3, 8, 1, 1, 0)
    F("fwd2c 192x48 6w", 34, 48, 2, 48, 2, 3, 6, 1, 1, 0)
    F("dg2c 256x48 4w", 36, 48, 0, 48, 4, 3, 4, 1, 1, 0)
    F("dg2c 192x48 4w", 36, 48, 0, 48, 3, 3, 4, 1, 1, 0)
    F("dg2c 128x48 4w", 36, 48, 0, 48, 2, 3, 4, 1, 1, 0)
    F("dg2c 192x48 6w", 36, 48, 0, 48, 2, 3, 6, 1, 1, 0)
    // round 3: weight-gradient blocks covering several / all taps (the 9 tap n-tiles of a split
    // re-read the split's input window from other blocks today: L2 hit 36 % on conv2's)
    G("wgx2 48x48 1w", 34, 48, 48, 4096, 3, 3, 1, 1, 1, 0, 0)
    G("wgx2 48x432 9w", 34, 48, 48, 4096, 3, 3, 1, 9, 1, 0, 0)
    G("wgx2 48x432 3w", 34, 48, 48, 4096, 3, 9, 1, 3, 1, 0, 0)
    G("wgx2 48x144 3w", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 0, 0)
    G("wgx2 48x432 9w z2k", 34, 48, 48, 2048, 3, 3, 1, 9, 1, 0, 0)
    G("wgx2 48x432 9w z8k", 34, 48, 48, 8192, 3, 3, 1, 9, 1, 0, 0)
    G("wgx3 96x48 2w", 18, 48, 96, 2048, 3, 3, 2, 1, 1, 0, 0)
    G("wgx3 96x432 9w", 18, 48, 96, 2048, 6, 3, 1, 9, 1, 0, 0)
    G("wgx3 48x432 9w", 18, 48, 96, 2048, 3, 3, 1, 9, 1, 0, 0)
    G("wgx4 96x96 4w", 20, 96, 96, 1024, 3, 3, 2, 2, 1, 0, 0)
    G("wgx4 96x288 6w", 20, 96, 96, 1024, 3, 3, 2, 6, 1, 0, 0)
    G("wgx4 48x288 6w", 20, 96, 96, 1024, 3, 3, 1, 6, 1, 0, 0)
    // round 3: small chunks (FLSIM_LAB_S=640, configs[1]), product splits (Z = 0)
    G("s6 wg2 48x48 1w", 34, 48, 48, 0, 3, 3, 1, 1, 1, 0, 0)
    G("s6 wg2 48x96 2w", 34, 48, 48, 0, 3, 3, 1, 2, 1, 0, 0)
    G("s6 wg2 48x144 3w", 34, 48, 48, 0, 3, 3, 1, 3, 1, 0, 0)
    G("s6 wg2 48x144 1w", 34, 48, 48, 0, 3, 9, 1, 1, 1, 0, 0)
    G("s6 wg3 96x48 2w", 18, 48, 96, 0, 3, 3, 2, 1, 1, 0, 0)
    G("s6 wg3 96x96 4w", 18, 48, 96, 0, 3, 3, 2, 2, 1, 0, 0)
    G("s6 wg3 48x48 1w", 18, 48, 96, 0, 3, 3, 1, 1, 1, 0, 0)
    G("s6 wg3 48x144 3w", 18, 48, 96, 0, 3, 3, 1, 3, 1, 0, 0)
    G("s6 wg4 96x96 4w", 20, 96, 96, 0, 3, 3, 2, 2, 1, 0, 0)
    G("s6 wg4 96x48 2w", 20, 96, 96, 0, 3, 3, 2, 1, 1, 0, 0)
    G("s6 wg4 48x96 2w", 20, 96, 96, 0, 3, 3, 1, 2, 1, 0, 0)
    G("s6 wg5 192x96 4w", 11, 96, 192, 0, 6, 3, 2, 2, 1, 0, 0)
    G("s6 wg5 96x96 4w", 11, 96, 192, 0, 3, 3, 2, 2, 1, 0, 0)
    G("s6 wg5 192x48 2w", 11, 96, 192, 0, 6, 3, 2, 1, 1, 0, 0)
    G("s6 wg6 192x192 8w", 13, 192, 192, 0, 6, 3, 2, 4, 1, 0, 0)
    G("s6 wg6 192x96 4w", 13, 192, 192, 0, 6, 3, 2, 2, 1, 0, 0)
    G("s6 wg6 96x96 4w", 13, 192, 192, 0, 3, 3, 2, 2, 1, 0, 0)
    // vgg11 (padding 1), the product's 128x128 4-wave tile against others
    F("vfwd2 128x128 4w", 16, 64, 1, 128, 4, 4, 2, 2, 1, 0)
    F("vfwd2 128x128 8w", 16, 64, 1, 128, 2, 4, 4, 2, 1, 0)
    F("vfwd2 256x128 8w", 16, 64, 1, 128, 4, 4, 4, 2, 1, 0)
    F("vfwd2 128x64 4w", 16, 64, 1, 128, 4, 2, 2, 2, 1, 0)
    F("vfwd4 128x128 4w", 8, 256, 1, 256, 4, 4, 2, 2, 1, 0)
    F("vfwd4 128x128 8w", 8, 256, 1, 256, 2, 4, 4, 2, 1, 0)
    F("vfwd4 256x128 8w", 8, 256, 1, 256, 4, 4, 4, 2, 1, 0)
    F("vfwd4 128x256 8w", 8, 256, 1, 256, 4, 4, 2, 4, 1, 0)
    F("vfwd4 128x64 4w", 8, 256, 1, 256, 4, 2, 2, 2, 1, 0)
    F("vfwd6 128x128 4w", 4, 512, 1, 512, 4, 4, 2, 2, 1, 0)
    F("vfwd6 128x128 8w", 4, 512, 1, 512, 2, 4, 4, 2, 1, 0)
    F("vfwd6 256x128 8w", 4, 512, 1, 512, 4, 4, 4, 2, 1, 0)
    F("vfwd6 128x256 8w", 4, 512, 1, 512, 4, 4, 2, 4, 1, 0)
    F("vfwd6 128x64 4w", 4, 512, 1, 512, 4, 2, 2, 2, 1, 0)
    // vgg11 weight gradients (ZW from vgg_net.hip VG[])
    GV("vwg2 128x128 4w", 16, 64, 128, 512, 4, 4, 2, 2)
    GV("vwg2 128x192 6w", 16, 64, 128, 512, 4, 4, 2, 3)
    GV("vwg2 128x64 2w", 16, 64, 128, 512, 4, 4, 2, 1)
    GV("vwg2 128x128 8w", 16, 64, 128, 512, 2, 4, 4, 2)
    GV("vwg4 128x128 4w", 8, 256, 256, 128, 4, 4, 2, 2)
    GV("vwg4 128x256 8w", 8, 256, 256, 128, 4, 4, 2, 4)
    GV("vwg4 256x128 8w", 8, 256, 256, 128, 4, 4, 4, 2)
    GV("vwg6 128x128 4w", 4, 512, 512, 32, 4, 4, 2, 2)
    GV("vwg6 128x256 8w", 4, 512, 512, 32, 4, 4, 2, 4)
    GV("vwg6 256x128 8w", 4, 512, 512, 32, 4, 4, 4, 2)
    return 0;
}
