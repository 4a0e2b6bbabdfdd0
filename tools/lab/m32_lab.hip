// 32x32x2 MFMA lab (from the pipeline lab; development tool, not part of libflsim.so): the product's GEMM pipeline with
// KSUB 16-deep sub-steps per LDS stage and barrier (fewer barriers per MFMA), and PIN = keep the
// k-step's MFMAs ahead of the barrier (sched_barrier; the compiler otherwise hoists the barrier
// above them).  Conv shapes of PerformantNet1 at S = 16384 samples, channel-slice-major K order.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/ks_lab.hip -o tools/lab/ks_lab
#include <cmath>
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
                al.load(ks + s, ra[s]);
                bl.load(ks + s, rb[s]);
            }
    };
    auto store_stage = [&](float* base, int ks) {
#pragma unroll
        for (int s = 0; s < KSUB; ++s)
            if (ks + s < ks1) {
                al.store(base + s * SUB, ra[s]);
                bl.store(base + s * SUB + A_FL, rb[s]);
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
        if (ks + KSUB < ks1) {
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
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
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

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 32x32x2 f32 MFMA version for k-contiguous operands: FM / FN = 32-row tiles per wave.  Lane l
// (row l & 31, half h = l >> 5) reads k = 8h .. 8h+7 of its row (two ds_read_b128) and MFMA s
// consumes element s, so lane half h supplies k = 8h + s (A and B agree).
template <int FM, int FN, int WAVES_M, int WAVES_N, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm32(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m, int tiles_n) {
    constexpr int BM = 32 * FM * WAVES_M;
    constexpr int BN = 32 * FN * WAVES_N;
    static_assert(AL::KC && BL::KC, "k-contiguous operands");
    constexpr int A_FL = tile_floats<true, BM>();
    constexpr int B_FL = tile_floats<true, BN>();
    constexpr int BUF = A_FL + B_FL;
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
    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    f32x4 ra[AL::UNITS];
    f32x4 rb[BL::UNITS];
    if (ks0 < ks1) {
        al.load(ks0, ra);
        bl.load(ks0, rb);
        al.store(lds, ra);
        bl.store(lds + A_FL, rb);
        if (ks0 + 1 < ks1) {
            al.load(ks0 + 1, ra);
            bl.load(ks0 + 1, rb);
        }
    }
    __syncthreads();
    if constexpr (WAVES_M * WAVES_N == 8) {
        if (wave >= 4) __builtin_amdgcn_s_setprio(1);
    }
    const int h = lane >> 5;
    int cur = 0;
    for (int ks = ks0; ks < ks1; ++ks) {
        if (ks + 1 < ks1) {
            al.store(lds + (cur ^ 1) * BUF, ra);
            bl.store(lds + (cur ^ 1) * BUF + A_FL, rb);
            if (ks + 2 < ks1) {
                al.load(ks + 2, ra);
                bl.load(ks + 2, rb);
            }
        }
        const float* A = lds + cur * BUF;
        const float* B = A + A_FL;
        f32x4 af[FM][2], bf[FN][2];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int row = wm * 32 * FM + 32 * i + (lane & 31);
            af[i][0] = *reinterpret_cast<const f32x4*>(A + KCTile<BM>::chunk_off(row, 2 * h));
            af[i][1] = *reinterpret_cast<const f32x4*>(A + KCTile<BM>::chunk_off(row, 2 * h + 1));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int row = wn * 32 * FN + 32 * j + (lane & 31);
            bf[j][0] = *reinterpret_cast<const f32x4*>(B + KCTile<BN>::chunk_off(row, 2 * h));
            bf[j][1] = *reinterpret_cast<const f32x4*>(B + KCTile<BN>::chunk_off(row, 2 * h + 1));
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s >> 2][s & 3],
                                                                     bf[j][s >> 2][s & 3],
                                                                     acc[i][j], 0, 0, 0);
        __syncthreads();
        cur ^= 1;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = m0 + wm * 32 * FM + 32 * i + 8 * g + 4 * h;
                const int n = n0 + wn * 32 * FN + 32 * j + (lane & 31);
                epi.apply4(m, n, tz, f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1],
                                           acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]});
            }
}

template <int FM, int FN, int WM, int WN, class AL, class BL, class EPI>
static double time_32(const char* tag, const AL& al, const BL& bl, const EPI& epi, int M, int N,
                      int ksteps, double flops) {
    constexpr int BM = 32 * FM * WM, BN = 32 * FN * WN;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm32<FM, FN, WM, WN, AL, BL, EPI>;
    for (int i = 0; i < 2; ++i)
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, ksteps, tm, tn);
    CK(hipDeviceSynchronize());
    const int iters = getenv("LAB_ITERS") ? atoi(getenv("LAB_ITERS")) : 5;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, ksteps, tm, tn);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%-24s MFMA32 tile %3dx%3d (%dx%d waves) grid %7d  %8.3f ms  %6.1f TF/s\n", tag, BM, BN, WM,
           WN, grid.x, ms, flops / (ms * 1e-3) / 1e12);
    fflush(stdout);
    return ms;
}

static void compare(const float* a, const float* b, size_t n, const char* tag) {
    std::vector<float> x(n), y(n);
    CK(hipMemcpy(x.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(y.data(), b, n * 4, hipMemcpyDeviceToHost));
    double num = 0, den = 0, mx = 0;
    for (size_t i = 0; i < n; ++i) {
        const double d = (double)x[i] - y[i];
        num += d * d;
        den += (double)y[i] * y[i];
        mx = std::max(mx, std::fabs(d));
    }
    printf("  check %s: rel_l2 %.3e  max_abs %.3e\n", tag, std::sqrt(num / std::max(den, 1e-300)), mx);
}

template <int IH, int CI, int PAD, int CO, int FM, int FN, int WM, int WN>
static void conv_fwd32(const char* tag, const float* X, const float* W, const float* b, float* Y,
                       float* Yref, int S) {
    constexpr int NT = 64 * WM * WN, BM = 32 * FM * WM, BN = 32 * FN * WN;
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
    time_32<FM, FN, WM, WN>(tag, al, bl, epi, al.M, CO, KP / GK, 2.0 * al.M * CO * KP);
    if (Yref) compare(Y, Yref, (size_t)al.M * CO, tag);
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
    printf("%-24s KSUB%d PIN%d tile %3dx%3d grid %7d  %8.3f ms  %6.1f TF/s\n", tag, KSUB, PIN, BM, BN,
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

template <int IH, int CI, int CO, int FM, int FN, int WM, int WN, int KSUB, int PIN, int VO = 0>
static void conv_wgrad(const char* tag, const float* dz, const float* X, float* slab, float* bslab,
                       int S, int Z) {
    constexpr int NT = 64 * WM * WN, BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2;
    using AL = RowsKM<BM, NT, (VO > 0 ? OFULL : 0), VO>;
    using BL = Im2colKMo<IH, IH, CI, 2, BN, NT, 0, VO>;
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
    time_ks<FM, FN, WM, WN, KSUB, PIN>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z, 2.0 * M * CO * KP);
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
#define F(tag, IH, CI, PAD, CO, FM, FN, WM, WN, KS, PIN) \
    if (want(tag)) conv_fwd<IH, CI, PAD, CO, FM, FN, WM, WN, KS, PIN>(tag, X, W, b, Y, S);
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN, KS, PIN, VO) \
    if (want(tag)) conv_wgrad<IH, CI, CO, FM, FN, WM, WN, KS, PIN, VO>(tag, Y, X, slab, bsl, S, Z);
    float* Y2 = dalloc(big, 0.f);
#define F32(tag, IH, CI, PAD, CO, FM, FN, WM, WN) \
    if (want(tag)) conv_fwd32<IH, CI, PAD, CO, FM, FN, WM, WN>(tag, X, W, b, Y2, Y, S);
    F("fwd6", 13, 192, 2, 192, 2, 6, 4, 2, 1, 0)
    F32("fwd6 w1x3", 13, 192, 2, 192, 1, 3, 4, 2)
    F32("fwd6 w1x3 4w", 13, 192, 2, 192, 1, 3, 4, 1)   // tile 128x96
    F32("fwd6 w2x3 4w", 13, 192, 2, 192, 2, 3, 2, 2)   // 128x192
    F("dg4", 22, 96, 0, 96, 4, 3, 4, 2, 1, 0)
    F32("dg4 w2x3 4w", 22, 96, 0, 96, 2, 3, 4, 1)       // 256x96
    F32("dg4 w1x3 8w", 22, 96, 0, 96, 1, 3, 8, 1)       // 256x96
    return 0;
}
