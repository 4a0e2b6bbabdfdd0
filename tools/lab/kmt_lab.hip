// Grouped k-major fragment lab (development tool, not part of libflsim.so): weight-gradient GEMMs
// (both operands k-major) whose wave tiles are read from LDS as G consecutive rows per lane
// (ds_read_b128 / _b64 for G = 4 / 2) instead of one ds_read_b32 per 16-row tile and k, with the
// MFMA row tiles interleaved to match (PA / PB per operand).  Checked bitwise against the
// ungrouped kernel.  Conv shapes of PerformantNet1 at S = 16384 samples.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/kmt_lab.hip -o tools/lab/kmt_lab
#include "lab_common.h"

// Row-tile groups of a wave's FM (or FN) 16-row tiles: greedy 4, 2, 1.  Tile i of a group of G
// holds rows rowbase + G * ii + t (ii = 0..15, t = i's index in the group): one ds_read_b(32 G)
// per k gives a lane the operands of all G tiles (k-major tile, G consecutive rows).
template <int F>
struct Groups {
    static constexpr int N4 = F / 4, N2 = (F % 4) / 2, N1 = F % 2;
    static constexpr int NG = N4 + N2 + N1;
    __host__ __device__ static constexpr int gsize(int g) { return g < N4 ? 4 : (g < N4 + N2 ? 2 : 1); }
    __host__ __device__ static constexpr int gtile0(int g) { return g < N4 ? 4 * g : (g < N4 + N2 ? 4 * N4 + 2 * (g - N4) : 4 * N4 + 2 * N2); }
    __host__ __device__ static constexpr int growbase(int g) { return 16 * gtile0(g); }
    __host__ __device__ static constexpr int gof(int i) { return i < 4 * N4 ? i / 4 : (i < 4 * N4 + 2 * N2 ? N4 + (i - 4 * N4) / 2 : N4 + N2); }
    // row (within the wave tile) of MFMA-local row ii of tile i
    __host__ __device__ static constexpr int row(int i, int ii) {
        return growbase(gof(i)) + gsize(gof(i)) * ii + (i - gtile0(gof(i)));
    }
};

template <int G>
__device__ __forceinline__ void read_grp(const float* p, float* out) {
    if constexpr (G == 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(p);
        out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
    } else if constexpr (G == 2) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 v = *reinterpret_cast<const f32x2*>(p);
        out[0] = v.x; out[1] = v.y;
    } else {
        out[0] = *p;
    }
}

// frag[i][kk] for the wave's F tiles of a k-major LDS tile (stride S floats per k row)
template <int F, int S>
__device__ __forceinline__ void read_km_grouped(const float* lds, int w0, int lane, float (&fr)[F][4]) {
    using GR = Groups<F>;
    const int ii = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int g = 0; g < GR::NG; ++g) {
        constexpr int dummy = 0; (void)dummy;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            float tmp[4];
            const float* p = lds + (4 * kq + kk) * S + w0 + GR::growbase(g) + GR::gsize(g) * ii;
            if (GR::gsize(g) == 4) read_grp<4>(p, tmp);
            else if (GR::gsize(g) == 2) read_grp<2>(p, tmp);
            else read_grp<1>(p, tmp);
#pragma unroll
            for (int t = 0; t < GR::gsize(g); ++t) fr[GR::gtile0(g) + t][kk] = tmp[t];
        }
    }
}

template <int FM, int FN, int WAVES_M, int WAVES_N, int PA, int PB, class AL, class BL, class EPI>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N)
gemm_kmt(AL al, BL bl, EPI epi, int ksteps_total, int ksteps_per_split, int tiles_m, int tiles_n) {
    constexpr int BM = 16 * FM * WAVES_M;
    constexpr int BN = 16 * FN * WAVES_N;
    static_assert(!AL::KC && !BL::KC, "k-major operands");
    constexpr int A_FL = tile_floats<AL::KC, BM>();
    constexpr int B_FL = tile_floats<BL::KC, BN>();
    constexpr int BUF = A_FL + B_FL;
    constexpr int SA = KMTile<BM>::STRIDE, SB = KMTile<BN>::STRIDE;
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
        if constexpr (EPI::ASUM) {
            if (tn == 0 && tid < BM) {
#pragma unroll
                for (int k = 0; k < GK; ++k) asum += A[k * SA + tid];
            }
        }
        float af[FM][4], bf[FN][4];
        if constexpr (PA) {
            read_km_grouped<FM, SA>(A, wm * 16 * FM, lane, af);
        } else {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const f32x4 v = read_frag<false, BM>(A, wm * 16 * FM + 16 * i, lane);
                af[i][0] = v.x; af[i][1] = v.y; af[i][2] = v.z; af[i][3] = v.w;
            }
        }
        if constexpr (PB) {
            read_km_grouped<FN, SB>(B, wn * 16 * FN, lane, bf);
        } else {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const f32x4 v = read_frag<false, BN>(B, wn * 16 * FN + 16 * j, lane);
                bf[j][0] = v.x; bf[j][1] = v.y; bf[j][2] = v.z; bf[j][3] = v.w;
            }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
        __syncthreads();
        cur ^= 1;
    }
    if constexpr (EPI::ASUM) {
        if (tn == 0 && tid < BM) epi.asum(m0 + tid, tz, asum);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int ii = 4 * (lane >> 4) + rr, jj = lane & 15;
                const int m = m0 + wm * 16 * FM + (PA ? Groups<FM>::row(i, ii) : 16 * i + ii);
                const int n = n0 + wn * 16 * FN + (PB ? Groups<FN>::row(j, jj) : 16 * j + jj);
                epi.apply1(m, n, tz, acc[i][j][rr]);
            }
}

struct EpiSlabAcc1 : EpiSlabAcc {
    __device__ void apply1(int m, int n, int z, float v) const {
        if (n < N && m < M) S[z * zstride + (long)m * N + n] += v;
    }
};

static float* g_ref = nullptr;   // slab of the unpermuted run, for the bitwise check

template <int FM, int FN, int WM, int WN, int PA, int PB, class AL, class BL, class EPI>
static double time_kmt(const char* tag, const AL& al, const BL& bl, const EPI& epi, int M, int N,
                       int ksteps, int Z, double flops, size_t nslab) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * Z);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto k = gemm_kmt<FM, FN, WM, WN, PA, PB, AL, BL, EPI>;
    // one launch from a zero slab for the check
    CK(hipMemset(epi.S, 0, nslab * 4));
    if (epi.Bsl) CK(hipMemset(epi.Bsl, 0, (size_t)Z * M * 4));
    hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), 0, 0, al, bl, epi, ksteps, per, tm, tn);
    CK(hipDeviceSynchronize());
    size_t bad = 0;
    if (!PA && !PB) {
        CK(hipMemcpy(g_ref, epi.S, nslab * 4, hipMemcpyDeviceToDevice));
    } else {
        std::vector<float> a(nslab), r(nslab);
        CK(hipMemcpy(a.data(), epi.S, nslab * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), g_ref, nslab * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < nslab; ++i) bad += a[i] != r[i];
    }
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
    printf("%-16s PA%d PB%d tile %3dx%3d (%dx%d waves) grid %7d  %8.3f ms  %6.1f TF/s  mismatches %zu\n",
           tag, PA, PB, BM, BN, WM, WN, grid.x, ms, flops / (ms * 1e-3) / 1e12, bad);
    fflush(stdout);
    return ms;
}

template <int IH, int CI, int CO, int FM, int FN, int WM, int WN, int PA, int PB, int VO = 0>
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
    EpiSlabAcc1 epi;
    epi.S = slab; epi.M = CO; epi.N = KP; epi.zstride = (long)CO * KP; epi.Bsl = bslab;
    time_kmt<FM, FN, WM, WN, PA, PB>(tag, al, bl, epi, CO, KP, ceil_div(M, GK), Z,
                                     2.0 * M * CO * KP, (size_t)Z * CO * KP);
}

int main(int argc, char** argv) {
    const int S = getenv("FLSIM_LAB_S") ? atoi(getenv("FLSIM_LAB_S")) : 16384;
    const size_t big = (size_t)S * 36 * 36 * 48;
    float* X = dalloc(big, 1.f);
    float* Y = dalloc(big, 0.5f);
    const size_t slabn = (size_t)4096 * 48 * 432;
    float* slab = dalloc(slabn, 0.f);
    CK(hipMalloc(&g_ref, slabn * 4));
    float* bsl = dalloc(4096 * 192, 0.f);
    const char* only = argc > 1 ? argv[1] : "";
    auto want = [&](const char* t) { return !*only || strstr(t, only); };
#define G(tag, IH, CI, CO, Z, FM, FN, WM, WN, PA, PB, VO) \
    if (want(tag)) conv_wgrad<IH, CI, CO, FM, FN, WM, WN, PA, PB, VO>(tag, Y, X, slab, bsl, S, Z);
    G("wg6", 13, 192, 192, 256, 6, 3, 2, 2, 0, 0, 14)
    G("wg6", 13, 192, 192, 256, 6, 3, 2, 2, 1, 0, 14)
    G("wg6", 13, 192, 192, 256, 6, 3, 2, 2, 1, 1, 14)
    G("wg6 t64", 13, 192, 192, 256, 4, 4, 3, 1, 0, 0, 14)
    G("wg6 t64", 13, 192, 192, 256, 4, 4, 3, 1, 1, 1, 14)
    G("wg6 t64x128", 13, 192, 192, 256, 4, 4, 3, 2, 1, 1, 14)
    G("wg5", 11, 96, 192, 512, 6, 3, 2, 2, 0, 0, 0)
    G("wg5", 11, 96, 192, 512, 6, 3, 2, 2, 1, 1, 0)
    G("wg4", 20, 96, 96, 1024, 3, 3, 2, 2, 0, 0, 0)
    G("wg4", 20, 96, 96, 1024, 3, 3, 2, 2, 1, 1, 0)
    G("wg4 6x6", 20, 96, 96, 1024, 6, 6, 1, 1, 1, 1, 0)
    G("wg4 6x3", 20, 96, 96, 1024, 6, 3, 1, 2, 1, 1, 0)
    G("wg3", 18, 48, 96, 2048, 3, 3, 2, 2, 0, 0, 0)
    G("wg3", 18, 48, 96, 2048, 3, 3, 2, 2, 1, 1, 0)
    G("wg2", 34, 48, 48, 4096, 3, 3, 1, 3, 0, 0, 0)
    G("wg2", 34, 48, 48, 4096, 3, 3, 1, 3, 1, 1, 0)
    G("wg2 3x9", 34, 48, 48, 4096, 3, 9, 1, 1, 1, 1, 0)
    return 0;
}
