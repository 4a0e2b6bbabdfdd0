// PerformantNet1 (reference FL/models.py:11-47) forward + backward for a chunk of simulated
// workers, as hand-written gfx950 kernels.  All workers of an epoch run on the same central
// model theta_t (main.py:154,159,169), so a chunk of W workers is ONE batch of W*128 samples;
// their gradients are summed (agents.py:35 accumulates into the shared .grad), which the weight
// gradient GEMMs do along their reduction (pixel / sample) dimension.
//
// Layout in HBM: activations NHWC fp32 (channels innermost); the flatten before linear1 is
// written in torch's NCHW order so linear1 uses the torch weight layout unchanged.
// Conv weights are re-packed once per epoch: Wf[co][(kh*3+kw)*CI + ci] (forward) and
// Wd[ci][(kh'*3+kw')*CO + co] = W[co][ci][2-kh'][2-kw'] (data gradient).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "loaders.h"
#include "pn1.h"
#include "probe.h"

namespace flsim {

// =============================================================================================
// error plumbing
// =============================================================================================
static thread_local char g_err[512];
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
const char* last_error() { return g_err; }

// =============================================================================================
// batch assembly: main.py:138-142 (k-th dataset, 128 samples with replacement, ToTensor +
// Normalize) -> x0 NHWC [S][32][32][4] (4th channel zero), y [S]
// =============================================================================================
__global__ void __launch_bounds__(256)
k_fill_batch(const uint8_t* __restrict__ pool, const int32_t* __restrict__ labels,
             const int32_t* __restrict__ list_a, int len_a, const int32_t* __restrict__ list_b,
             int len_b, const WorkerRec* __restrict__ workers, int n_workers_total, uint64_t seed,
             const float* __restrict__ lut, float* __restrict__ x0, int32_t* __restrict__ y) {
    const int s = blockIdx.x;  // sample within chunk
    const int w = s / SAMPLES_PER_WORKER;
    const int j = s - w * SAMPLES_PER_WORKER;
    const WorkerRec wr = workers[w];
    const bool use_b = (int)wr.k == n_workers_total - 1;   // main.py:78-80: last dataset = {1,9}
    const int len = use_b ? len_b : len_a;
    const uint32_t u = philox_word(seed, wr.t, wr.i, SITE_DATA, (uint32_t)j);
    const int idx = use_b ? list_b[u % (uint32_t)len] : list_a[u % (uint32_t)len];
    if (threadIdx.x == 0) y[s] = labels[idx];
    const uint8_t* img = pool + (long)idx * 3072;
    float* out = x0 + (long)s * 4096;
    for (int p = threadIdx.x; p < 1024; p += 256) {
        f32x4 v;
        v.x = lut[img[p]];
        v.y = lut[img[1024 + p]];
        v.z = lut[img[2048 + p]];
        v.w = 0.f;
        *reinterpret_cast<f32x4*>(out + 4 * p) = v;
    }
}

// evaluation batches (util.py:31-45 testloader, shuffle=False): sample s of the chunk is pool
// image first + s (samples past n_images repeat the last image; their predictions are dropped)
__global__ void __launch_bounds__(256)
k_fill_seq(const uint8_t* __restrict__ pool, int first, int n_images, const float* __restrict__ lut,
           float* __restrict__ x0, int32_t* __restrict__ y) {
    const int s = blockIdx.x;
    const int idx = first + (s < n_images ? s : n_images - 1);
    if (threadIdx.x == 0) y[s] = 0;
    const uint8_t* img = pool + (long)idx * 3072;
    float* out = x0 + (long)s * 4096;
    for (int p = threadIdx.x; p < 1024; p += 256) {
        f32x4 v;
        v.x = lut[img[p]];
        v.y = lut[img[1024 + p]];
        v.z = lut[img[2048 + p]];
        v.w = 0.f;
        *reinterpret_cast<f32x4*>(out + 4 * p) = v;
    }
}

// explicit input (Worker.fwd_bkwd(inp, outp) facade): x NCHW fp32 [S][3][32][32], y int64
__global__ void __launch_bounds__(256)
k_load_input(const float* __restrict__ x, const int64_t* __restrict__ yin, float* __restrict__ x0,
             int32_t* __restrict__ y) {
    const int s = blockIdx.x;
    if (threadIdx.x == 0) y[s] = (int32_t)yin[s];
    const float* img = x + (long)s * 3072;
    float* out = x0 + (long)s * 4096;
    for (int p = threadIdx.x; p < 1024; p += 256) {
        f32x4 v;
        v.x = img[p];
        v.y = img[1024 + p];
        v.z = img[2048 + p];
        v.w = 0.f;
        *reinterpret_cast<f32x4*>(out + 4 * p) = v;
    }
}

// =============================================================================================
// gradient through dropout + max_pool2d: dz[n][h][w][c] = gy[n][h/2][w/2][c] at the window's
// argmax, 0 elsewhere and on the floor-mode border (models.py:31,35,39 backward).  One thread
// per (window, 4 channels): one gy float4 (or 4 NCHW scalars), one idx word, four float4 stores.
// gy is already masked / scaled by the consumer's epilogue.
// =============================================================================================
template <int H, int W, int C, bool NCHW_G>
__global__ void __launch_bounds__(256)
k_pool_scatter(const float* __restrict__ gy, const uint8_t* __restrict__ idx,
               float* __restrict__ dz, long total) {
    constexpr int PH = H / 2, PW = W / 2;
    constexpr int CH = (H + 1) / 2, CW = (W + 1) / 2;   // cells incl. the border
    constexpr int C4 = C / 4;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= total) return;
    const int c = 4 * (int)(e % C4);
    const long cell = e / C4;
    const int cw = (int)(cell % CW);
    const int ch = (int)((cell / CW) % CH);
    const int n = (int)(cell / (CW * CH));
    f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
    uint32_t id = 0xffffffffu;
    if (ch < PH && cw < PW) {
        const long pe = (((long)n * PH + ch) * PW + cw) * C + c;
        id = *reinterpret_cast<const uint32_t*>(idx + pe);
        if constexpr (NCHW_G) {
            const float* b = gy + (long)n * (C * PH * PW) + (long)c * (PH * PW) + ch * PW + cw;
            g.x = b[0];
            g.y = b[PH * PW];
            g.z = b[2 * PH * PW];
            g.w = b[3 * PH * PW];
        } else {
            g = *reinterpret_cast<const f32x4*>(gy + pe);
        }
    }
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
        const int h = 2 * ch + (pos >> 1), w = 2 * cw + (pos & 1);
        if (h >= H || w >= W) continue;
        f32x4 v;
        v.x = ((id & 0xff) == (uint32_t)pos) ? g.x : 0.f;
        v.y = (((id >> 8) & 0xff) == (uint32_t)pos) ? g.y : 0.f;
        v.z = (((id >> 16) & 0xff) == (uint32_t)pos) ? g.z : 0.f;
        v.w = ((id >> 24) == (uint32_t)pos) ? g.w : 0.f;
        *reinterpret_cast<f32x4*>(dz + (((long)n * H + h) * W + w) * C + c) = v;
    }
}

template <int H, int W, int C, bool NCHW_G>
static int pool_scatter(const float* gy, const uint8_t* idx, float* dz, int S, hipStream_t st) {
    const long total = (long)S * ((H + 1) / 2) * ((W + 1) / 2) * (C / 4);
    hipLaunchKernelGGL((k_pool_scatter<H, W, C, NCHW_G>), dim3(ceil_div(total, 256)), dim3(256), 0,
                       st, gy, idx, dz, total);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// =============================================================================================
// linear split-K finish: e[m][n] = dropout(relu(sum_z part[z][m][n] + b[n]))   (models.py:42-45)
// =============================================================================================
__global__ void __launch_bounds__(256)
k_linear_finish(const float* __restrict__ part, int Z, const float* __restrict__ bias,
                float* __restrict__ out, int M, int N, const WorkerRec* __restrict__ workers,
                uint64_t seed, uint32_t site, uint32_t thr, float scale, int dropout) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)M * N) return;
    const int n = (int)(e % N);
    const int m = (int)(e / N);
    float acc = part[e];
    for (int z = 1; z < Z; ++z) acc += part[(long)z * M * N + e];
    float v = fmaxf(acc + bias[n], 0.f);
    if (dropout) {
        const int w = m / SAMPLES_PER_WORKER;
        const int nl = m - w * SAMPLES_PER_WORKER;
        const WorkerRec wr = workers[w];
        v = philox_word(seed, wr.t, wr.i, site, (uint32_t)(nl * N + n)) >= thr ? v * scale : 0.f;
    }
    out[e] = v;
}

// =============================================================================================
// head: linear3 + CrossEntropyLoss(mean over the worker's 128) forward and backward
// (models.py:46, main.py:107, agents.py:34-35).  One wave per sample.
//   loss_s[s] = logsumexp(z) - z_y ; dlog[s][j] = (softmax - onehot) / 128
//   dh2[s][k] = (sum_j dlog[s][j] W3[j][k]) * 2 * (e2[s][k] > 0)   (dropout2 + relu backward)
// =============================================================================================
__global__ void __launch_bounds__(256)
k_head(const float* __restrict__ e2, const float* __restrict__ W3, const float* __restrict__ b3,
       const int32_t* __restrict__ y, float* __restrict__ loss_s, float* __restrict__ dlog,
       float* __restrict__ dh2, int S, int backward, float s50,
       int32_t* __restrict__ pred, int n_pred) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (s >= S) return;
    const f32x4 x = *reinterpret_cast<const f32x4*>(e2 + (long)s * 256 + 4 * lane);
    float z[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const f32x4 wv = *reinterpret_cast<const f32x4*>(W3 + j * 256 + 4 * lane);
        float p = x.x * wv.x + x.y * wv.y + x.z * wv.z + x.w * wv.w;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
        z[j] = p + b3[j];
    }
    float mx = z[0];
#pragma unroll
    for (int j = 1; j < 10; ++j) mx = fmaxf(mx, z[j]);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) se += expf(z[j] - mx);
    const int lab = y[s];
    float zy = 0.f;
#pragma unroll
    for (int j = 0; j < 10; ++j) zy = (j == lab) ? z[j] : zy;
    if (lane == 0) loss_s[s] = (mx + logf(se)) - zy;
    if (pred && lane == 0 && s < n_pred) {       // torch.max(outputs, 1): first max wins
        int am = 0;
#pragma unroll
        for (int j = 1; j < 10; ++j) am = z[j] > z[am] ? j : am;
        pred[s] = am;
    }
    if (!backward) return;
    float g[10];
    const float inv = 1.f / se;
#pragma unroll
    for (int j = 0; j < 10; ++j)
        g[j] = (expf(z[j] - mx) * inv - (j == lab ? 1.f : 0.f)) * (1.f / SAMPLES_PER_WORKER);
    if (lane < 10) {
        float gv = 0.f;
#pragma unroll
        for (int j = 0; j < 10; ++j) gv = (j == lane) ? g[j] : gv;
        dlog[(long)s * 16 + lane] = gv;
    }
    f32x4 d = zero4();
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        const f32x4 wv = *reinterpret_cast<const f32x4*>(W3 + j * 256 + 4 * lane);
        d.x += g[j] * wv.x;
        d.y += g[j] * wv.y;
        d.z += g[j] * wv.z;
        d.w += g[j] * wv.w;
    }
    d.x = x.x > 0.f ? d.x * s50 : 0.f;
    d.y = x.y > 0.f ? d.y * s50 : 0.f;
    d.z = x.z > 0.f ? d.z * s50 : 0.f;
    d.w = x.w > 0.f ? d.w * s50 : 0.f;
    *reinterpret_cast<f32x4*>(dh2 + (long)s * 256 + 4 * lane) = d;
}

// per-worker mean loss (fixed-order tree over the worker's 128 samples)
__global__ void __launch_bounds__(128)
k_worker_loss(const float* __restrict__ loss_s, float* __restrict__ out) {
    __shared__ float sh[128];
    const int w = blockIdx.x;
    sh[threadIdx.x] = loss_s[(long)w * 128 + threadIdx.x];
    __syncthreads();
    for (int o = 64; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[w] = sh[0] / 128.f;
}

// linear3 weight/bias gradient, accumulated: slab3[z][j][0..255] += sum_s dlog[s][j] e2[s][k];
// slab3b[z][j] += sum_s dlog[s][j].  Block (j, z) sums a row range of samples.
__global__ void __launch_bounds__(256)
k_head_wgrad(const float* __restrict__ dlog, const float* __restrict__ e2, float* __restrict__ slab,
             float* __restrict__ slab_b, int S, int Z) {
    const int j = blockIdx.x;
    const int z = blockIdx.y;
    const int k = threadIdx.x;
    const int per = (S + Z - 1) / Z;
    const int s0 = z * per;
    const int s1 = min(S, s0 + per);
    float acc = 0.f, accb = 0.f;
    for (int s = s0; s < s1; ++s) {
        const float g = dlog[(long)s * 16 + j];
        acc += g * e2[(long)s * 256 + k];
        accb += g;
    }
    slab[((long)z * 10 + j) * 256 + k] += acc;
    if (k == 0) slab_b[z * 10 + j] += accb;
}

// =============================================================================================
// per-epoch weight packing (theta in torch layout -> kernel layouts)
// =============================================================================================
// forward: Wf[co][khkw*CIP + ci] = W[co][ci][kh][kw]   (ci < CI; zero padding ci in [CI, CIP)
// and k >= 9*CIP up to KP)
__global__ void k_pack_fwd(const float* __restrict__ W, float* __restrict__ Wf, int CO, int CI,
                           int CIP, int KP) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= CO * KP) return;
    const int co = e / KP;
    const int k = e - co * KP;
    const int khkw = k / CIP;
    const int ci = k - khkw * CIP;
    float v = 0.f;
    if (khkw < 9 && ci < CI) v = W[(co * CI + ci) * 9 + khkw];
    Wf[e] = v;
}
// data gradient: Wd[ci][khkw'*CO + co] = W[co][ci][8 - khkw']
__global__ void k_pack_dgrad(const float* __restrict__ W, float* __restrict__ Wd, int CO, int CI) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int KD = 9 * CO;
    if (e >= CI * KD) return;
    const int ci = e / KD;
    const int k = e - ci * KD;
    const int khkw = k / CO;
    const int co = k - khkw * CO;
    Wd[e] = W[(co * CI + ci) * 9 + (8 - khkw)];
}

// =============================================================================================
// epoch-end finalize: S_t (torch layout) = sum_z slab[z]  (fixed z order: deterministic)
// =============================================================================================
// Block = `cols` element columns x `zl` z-lanes: lane tz sums slabs z = tz, tz + zl, ... (V
// consecutive elements, one vector load per slab), then the zl partials are added in z-lane
// order.  The order is fixed, so S_t is deterministic; every slab byte is read once, coalesced.
// CO > 0 remaps the packed conv layout [co][khkw*CIP + ci] to torch's [co][ci][kh][kw].
template <int V>
__global__ void __launch_bounds__(256)
k_fin_sum(const float* __restrict__ slab, int Z, long n, int zl, float* __restrict__ out, int CO,
          int CI, int CIP, int KP) {
    __shared__ float red[256 * V];
    const int cols = 256 / zl;
    const int tx = threadIdx.x % cols, tz = threadIdx.x / cols;
    const long e0 = ((long)blockIdx.x * cols + tx) * V;
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    if (e0 < n) {
        for (int z = tz; z < Z; z += zl) {
            const float* p = slab + (long)z * n + e0;
            if constexpr (V == 4) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(p);
                acc[0] += x.x;
                acc[1] += x.y;
                acc[2] += x.z;
                acc[3] += x.w;
            } else {
                acc[0] += p[0];
            }
        }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) red[threadIdx.x * V + v] = acc[v];
    __syncthreads();
    if (tz != 0 || e0 >= n) return;
    for (int j = 1; j < zl; ++j)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += red[(j * cols + tx) * V + v];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const long s = e0 + v;
        if (CO > 0) {
            const int co = (int)(s / KP);
            const int k = (int)(s - (long)co * KP);
            const int khkw = k / CIP, ci = k - (k / CIP) * CIP;
            if (khkw < 9 && ci < CI) out[((long)co * CI + ci) * 9 + khkw] = acc[v];
        } else {
            out[s] = acc[v];
        }
    }
}

static int fin_sum(const float* slab, int Z, long n, float* out, hipStream_t st, int CO = 0,
                   int CI = 0, int CIP = 1, int KP = 1) {
    int zl = 1;
    while (zl < Z && zl < 16) zl *= 2;
    const int cols = 256 / zl;
    if (n % 4 == 0) {
        hipLaunchKernelGGL(k_fin_sum<4>, dim3(ceil_div(n, 4L * cols)), dim3(256), 0, st, slab, Z, n,
                           zl, out, CO, CI, CIP, KP);
    } else {
        hipLaunchKernelGGL(k_fin_sum<1>, dim3(ceil_div(n, (long)cols)), dim3(256), 0, st, slab, Z,
                           n, zl, out, CO, CI, CIP, KP);
    }
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// =============================================================================================
// GEMM launch helper
// =============================================================================================
template <int FM, int FN, int WM, int WN, class AL, class BL, class EPI>
static int launch_gemm(const AL& al, const BL& bl, const EPI& epi, int M, int N, int ksteps, int Z,
                       hipStream_t st, int kid, double alg_flops) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * Z);
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL((gemm_kernel<FM, FN, WM, WN, AL, BL, EPI>), grid, dim3(64 * WM * WN), 0,
                          st, ps.start, ps.stop, 0, al, bl, epi, ksteps, per, tm, tn);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, kid, alg_flops);
}

// forward conv (also the data-gradient conv): out[m][n] for m < S*OH*OW, n < N
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, class EPI>
static int conv_like(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                     hipStream_t st, int kid, int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IW, CI, PAD, BM, NT>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP;
    bl.NR = N;
    return launch_gemm<FM, FN, WM, WN>(al, bl, epi, al.M, N, KP / GK, 1, st, kid,
                                       2.0 * al.M * N * kreal);
}

// weight gradient: slab[z][co][kk] += sum_p dz[p][co] * im2col(X)[p][kk]
template <int IH, int IW, int CI, int FM, int FN, int WM, int WN>
static int conv_wgrad(const float* dz, const float* X, int S, int CO, int KP, float* slab,
                      float* bslab, int Z, hipStream_t st, int kid, int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = RowsKM<BM, NT>;
    using BL = Im2colKM<IH, IW, CI, 2, BN, NT>;
    const int M = S * BL::OH * BL::OW;
    AL al;
    al.P = dz;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab};
    return launch_gemm<FM, FN, WM, WN>(al, bl, epi, CO, KP, ceil_div(M, GK), Z, st, kid,
                                       2.0 * M * CO * kreal);
}

// forward conv fused with bias + ReLU + 2x2 max-pool + dropout: GEMM rows in pool-window order
template <int IH, int IW, int CI, int CO, int FM, int FN, int WM, int WN, bool NCHW_OUT>
static int conv_pool_fwd(const float* X, int S, const float* Wpk, int KP, float* d, uint8_t* idx,
                         const float* bias, const WorkerRec* workers, uint64_t seed, uint32_t site,
                         int dropout, hipStream_t st, int kid, int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IW, CI, 2, BM, NT, true>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::ROWS_PER_IMG;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP;
    bl.NR = CO;
    EpiPoolDrop<AL::PH, AL::PW, CO, NCHW_OUT> epi{d, idx, bias, workers, seed, site, THR_P25,
                                                  SCALE_P25, dropout, al.M};
    return launch_gemm<FM, FN, WM, WN>(al, bl, epi, al.M, CO, KP / GK, 1, st, kid,
                                       2.0 * al.M * CO * kreal);
}

// =============================================================================================
// Net plan
// =============================================================================================
struct ConvGeo {
    int CI, CIP, CO, H;  // input channels (real / padded), output channels, input spatial size
    int KP;              // packed forward K (9*CIP rounded to 16)
    int ZW;              // wgrad split
};
// ZW (pixel splits of the weight gradient) sized so each wgrad launch has thousands of blocks:
// several rounds of resident blocks on 256 CUs.  Tile shapes per layer were picked with
// tools/lab/gemm_lab.hip on MI355X (4-wave wgrad tiles: a 6-wave block loads two SIMDs twice).
static const ConvGeo GEO[6] = {
    {3, 4, 48, 32, 48, 8192},    {48, 48, 48, 34, 432, 2048},   {48, 48, 96, 18, 432, 1024},
    {96, 96, 96, 20, 864, 512},  {96, 96, 192, 11, 864, 256},  {192, 192, 192, 13, 1728, 128},
};
static const long P_OFF[18] = {0,       1296,    1344,    22080,   22128,   63600,
                               63696,   146640,  146736,  312624,  312816,  644592,
                               644784,  5461680, 5462192, 5593264, 5593520, 5596080};
constexpr long P_TOTAL = 5596090;
constexpr int ZL1F = 4;     // linear1 forward split-K
constexpr int ZL1W = 8;     // linear1 wgrad split
constexpr int ZL2W = 64;    // linear2 wgrad split
constexpr int ZH = 32;      // head wgrad split

// gradient-state layout (floats): packed weights + slabs
struct GradState {
    float* wf[6];
    float* wd[6];  // wd[0] unused
    float* sw[6];  // conv weight slabs [ZW][CO][KP]
    float* sb[6];  // conv bias slabs [ZW][CO] (fused into the weight-gradient GEMM)
    float* l1w;    // [ZL1W][512][9408]
    float* l1b;    // [ZL1W][512]
    float* l2w;    // [ZL2W][256][512]
    float* l2b;    // [ZL2W][256]
    float* l3w;    // [ZH][10][256]
    float* l3b;    // [ZH][10]
    float* slab_begin;
    long slab_floats;
    long total_floats;
};

static GradState gs_layout(float* base) {
    GradState g;
    long o = 0;
    auto take = [&](long n) {
        float* p = base ? base + o : nullptr;
        o += (n + 63) / 64 * 64;
        return p;
    };
    for (int l = 0; l < 6; ++l) {
        g.wf[l] = take((long)GEO[l].CO * GEO[l].KP);
        g.wd[l] = l ? take((long)GEO[l].CI * 9 * GEO[l].CO) : nullptr;
    }
    const long slab0 = o;
    g.slab_begin = base ? base + o : nullptr;
    for (int l = 0; l < 6; ++l) {
        g.sw[l] = take((long)GEO[l].ZW * GEO[l].CO * GEO[l].KP);
        g.sb[l] = take((long)GEO[l].ZW * GEO[l].CO);
    }
    g.l1w = take((long)ZL1W * 512 * 9408);
    g.l1b = take((long)ZL1W * 512);
    g.l2w = take((long)ZL2W * 256 * 512);
    g.l2b = take((long)ZL2W * 256);
    g.l3w = take((long)ZH * 10 * 256);
    g.l3b = take((long)ZH * 10);
    g.slab_floats = o - slab0;
    g.total_floats = o;
    return g;
}

// workspace (per chunk) layout
struct WS {
    float* x0; float* a1; float* a2; float* d1; float* a3; float* a4; float* d2; float* a5;
    float* a6; float* d3; float* e1; float* e2; float* part; float* dh1; float* dh2;
    float* gx; float* gy; float* loss_s; float* dlog; int32_t* y;
    uint8_t* i1; uint8_t* i2; uint8_t* i3;
    long bytes;
};

static WS ws_layout(char* base, int S) {
    WS w;
    long o = 0;
    auto take = [&](long bytes) {
        char* p = base ? base + o : nullptr;
        o += (bytes + 255) / 256 * 256;
        return p;
    };
    auto tf = [&](long per) { return (float*)take(per * (long)S * 4); };
    w.x0 = tf(4096); w.a1 = tf(55488); w.a2 = tf(62208); w.d1 = tf(15552);
    w.a3 = tf(38400); w.a4 = tf(46464); w.d2 = tf(11616); w.a5 = tf(32448);
    w.a6 = tf(43200); w.d3 = tf(9408); w.e1 = tf(512); w.e2 = tf(256);
    w.part = tf(512L * ZL1F); w.dh1 = tf(512); w.dh2 = tf(256);
    w.gx = tf(55488); w.gy = tf(15552); w.loss_s = tf(1); w.dlog = tf(16);
    w.y = (int32_t*)take(4L * S);
    w.i1 = (uint8_t*)take(15552L * S); w.i2 = (uint8_t*)take(11616L * S);
    w.i3 = (uint8_t*)take(9408L * S);
    w.bytes = o;
    return w;
}

static int pack_weights(const GradState& g, const float* theta, hipStream_t st) {
    for (int l = 0; l < 6; ++l) {
        const ConvGeo& c = GEO[l];
        const float* W = theta + P_OFF[2 * l];
        hipLaunchKernelGGL(k_pack_fwd, dim3(ceil_div((long)c.CO * c.KP, 256)), dim3(256), 0, st, W,
                           g.wf[l], c.CO, c.CI, c.CIP, c.KP);
        FLSIM_LAUNCH_CHECK();
        if (l) {
            hipLaunchKernelGGL(k_pack_dgrad, dim3(ceil_div((long)c.CI * 9 * c.CO, 256)), dim3(256),
                               0, st, W, g.wd[l], c.CO, c.CI);
            FLSIM_LAUNCH_CHECK();
        }
    }
    return 0;
}

#define RC(x) do { int _r = (x); if (_r) return _r; } while (0)

static int forward(const GradState& g, const WS& w, const float* theta, int S,
                   const WorkerRec* workers, uint64_t seed, int dropout, hipStream_t st) {
    // conv1, conv2 (+ReLU)  models.py:29-30
    RC((conv_like<32, 32, 4, 2, 2, 3, 4, 1>(w.x0, S, g.wf[0], 48, 48,
        EpiBiasRelu{w.a1, theta + P_OFF[1], S * 34 * 34, 48}, st, K_FWD1, 27)));
    // conv2 + ReLU + pool1 + dropout1 (models.py:30-32), one fused launch
    RC((conv_pool_fwd<34, 34, 48, 48, 2, 3, 8, 1, false>(w.a1, S, g.wf[1], 432, w.d1, w.i1,
        theta + P_OFF[3], workers, seed, SITE_DROP1, dropout, st, K_FWD2, 432)));
    RC((conv_like<18, 18, 48, 2, 4, 3, 4, 2>(w.d1, S, g.wf[2], 96, 432,
        EpiBiasRelu{w.a3, theta + P_OFF[5], S * 20 * 20, 96}, st, K_FWD3, 432)));
    // conv4 + ReLU + pool2 + dropout1 (models.py:34-36)
    RC((conv_pool_fwd<20, 20, 96, 96, 4, 3, 4, 2, false>(w.a3, S, g.wf[3], 864, w.d2, w.i2,
        theta + P_OFF[7], workers, seed, SITE_DROP2, dropout, st, K_FWD4, 864)));
    RC((conv_like<11, 11, 96, 2, 2, 6, 4, 2>(w.d2, S, g.wf[4], 192, 864,
        EpiBiasRelu{w.a5, theta + P_OFF[9], S * 13 * 13, 192}, st, K_FWD5, 864)));
    // conv6 + ReLU + pool3 + dropout1 (models.py:38-40), written in torch's flatten order
    // (models.py:41) so linear1 keeps the torch weight layout; the floor-mode border row/column
    // of the 15x15 output (dropped by the pool) is never computed
    RC((conv_pool_fwd<13, 13, 192, 192, 2, 6, 4, 2, true>(w.a5, S, g.wf[5], 1728, w.d3, w.i3,
        theta + P_OFF[11], workers, seed, SITE_DROP3, dropout, st, K_FWD6, 1728)));
    // linear1 + relu + dropout2 (models.py:41-43), split-K partials then finish
    {
        constexpr int NT = 256;
        RowsKC<128, NT> al{};
        al.P = w.d3; al.ld = 9408; al.NR = S;
        RowsKC<128, NT> bl{};
        bl.P = theta + P_OFF[12]; bl.ld = 9408; bl.NR = 512;
        EpiSlabStore epi{w.part, S, 512, (long)S * 512};
        RC((launch_gemm<4, 4, 2, 2>(al, bl, epi, S, 512, 9408 / GK, ZL1F, st, K_L1F, 2.0 * S * 512 * 9408)));
        const long tot = (long)S * 512;
        hipLaunchKernelGGL(k_linear_finish, dim3(ceil_div(tot, 256)), dim3(256), 0, st, w.part, ZL1F,
                           theta + P_OFF[13], w.e1, S, 512, workers, seed, SITE_DROP4, THR_P50,
                           SCALE_P50, dropout);
        FLSIM_LAUNCH_CHECK();
    }
    {   // linear2 + relu + dropout2 (models.py:44-45)
        constexpr int NT = 256;
        RowsKC<64, NT> al{};
        al.P = w.e1; al.ld = 512; al.NR = S;
        RowsKC<64, NT> bl{};
        bl.P = theta + P_OFF[14]; bl.ld = 512; bl.NR = 256;
        EpiSlabStore epi{w.part, S, 256, (long)S * 256};
        RC((launch_gemm<2, 2, 2, 2>(al, bl, epi, S, 256, 512 / GK, 1, st, K_L2F, 2.0 * S * 256 * 512)));
        const long tot = (long)S * 256;
        hipLaunchKernelGGL(k_linear_finish, dim3(ceil_div(tot, 256)), dim3(256), 0, st, w.part, 1,
                           theta + P_OFF[15], w.e2, S, 256, workers, seed, SITE_DROP5, THR_P50,
                           SCALE_P50, dropout);
        FLSIM_LAUNCH_CHECK();
    }
    return 0;
}

static int backward(const GradState& g, const WS& w, const float* theta, int S, int dropout,
                    hipStream_t st) {
    const float s25 = dropout ? SCALE_P25 : 1.f;
    const float s50 = dropout ? SCALE_P50 : 1.f;
    // ---- linear3 weight/bias (head already produced dlog, dh2) ----
    hipLaunchKernelGGL(k_head_wgrad, dim3(10, ZH), dim3(256), 0, st, w.dlog, w.e2, g.l3w, g.l3b, S, ZH);
    FLSIM_LAUNCH_CHECK();
    // ---- linear2: wgrad, bias, dgrad (-> dh1 through dropout/relu of linear1) ----
    {
        constexpr int NT = 256;
        RowsKM<128, NT> al{};
        al.P = w.dh2; al.ld = 256; al.NK = S; al.NC = 256;
        RowsKM<128, NT> bl{};
        bl.P = w.e1; bl.ld = 512; bl.NK = S; bl.NC = 512;
        EpiSlabAcc epi{g.l2w, 256, 512, 256L * 512, g.l2b};
        RC((launch_gemm<4, 4, 2, 2>(al, bl, epi, 256, 512, ceil_div(S, GK), ZL2W, st, K_L2W, 2.0 * S * 256 * 512)));
        RowsKC<64, NT> dl{};
        dl.P = w.dh2; dl.ld = 256; dl.NR = S;
        RowsKM<64, NT> wl{};
        wl.P = theta + P_OFF[14]; wl.ld = 512; wl.NK = 256; wl.NC = 512;
        EpiDropMask de{w.dh1, w.e1, s50, S, 512};
        RC((launch_gemm<2, 2, 2, 2>(dl, wl, de, S, 512, 256 / GK, 1, st, K_L2D, 2.0 * S * 256 * 512)));
    }
    // ---- linear1: wgrad, bias, dgrad (-> gradient wrt d3 through dropout1 site 3) ----
    {
        constexpr int NT = 256;
        RowsKM<128, NT> al{};
        al.P = w.dh1; al.ld = 512; al.NK = S; al.NC = 512;
        RowsKM<128, NT> bl{};
        bl.P = w.d3; bl.ld = 9408; bl.NK = S; bl.NC = 9408;
        EpiSlabAcc epi{g.l1w, 512, 9408, 512L * 9408, g.l1b};
        RC((launch_gemm<4, 4, 2, 2>(al, bl, epi, 512, 9408, ceil_div(S, GK), ZL1W, st, K_L1W, 2.0 * S * 512 * 9408)));
        RowsKC<128, NT> dl{};
        dl.P = w.dh1; dl.ld = 512; dl.NR = S;
        RowsKM<128, NT> wl{};
        wl.P = theta + P_OFF[12]; wl.ld = 9408; wl.NK = 512; wl.NC = 9408;
        EpiDropMask de{w.gy, w.d3, s25, S, 9408};
        RC((launch_gemm<4, 4, 2, 2>(dl, wl, de, S, 9408, 512 / GK, 1, st, K_L1D, 2.0 * S * 512 * 9408)));
    }
    // ---- pool3 backward -> dz6 (a6 buffer: conv6 fwd no longer writes it) ----
    RC((pool_scatter<15, 15, 192, true>(w.gy, w.i3, w.a6, S, st)));
    float* dz6 = w.a6;
    // ---- conv6: wgrad (input a5), bias, dgrad -> dz5 = . * (a5 > 0) into gx ----
    RC((conv_wgrad<13, 13, 192, 6, 3, 2, 2>(dz6, w.a5, S, 192, 1728, g.sw[5], g.sb[5], GEO[5].ZW, st, K_WG6, 1728)));
    RC((conv_like<15, 15, 192, 0, 2, 6, 4, 2>(dz6, S, g.wd[5], 192, 1728,
        EpiMask<true>{w.gx, w.a5, S * 13 * 13, 192}, st, K_DG6, 1728)));
    float* dz5 = w.gx;
    // ---- conv5: wgrad (input d2), bias, dgrad -> grad wrt d2 (dropout site 2) into gy ----
    RC((conv_wgrad<11, 11, 96, 6, 3, 2, 2>(dz5, w.d2, S, 192, 864, g.sw[4], g.sb[4], GEO[4].ZW, st, K_WG5, 864)));
    RC((conv_like<13, 13, 192, 0, 4, 3, 4, 2>(dz5, S, g.wd[4], 96, 1728,
        EpiDropMask{w.gy, w.d2, s25, S * 11 * 11, 96}, st, K_DG5, 1728)));
    RC((pool_scatter<22, 22, 96, false>(w.gy, w.i2, w.a4, S, st)));
    float* dz4 = w.a4;
    // ---- conv4: wgrad (input a3), bias, dgrad -> dz3 = . * (a3 > 0) into gx ----
    RC((conv_wgrad<20, 20, 96, 3, 3, 2, 2>(dz4, w.a3, S, 96, 864, g.sw[3], g.sb[3], GEO[3].ZW, st, K_WG4, 864)));
    RC((conv_like<22, 22, 96, 0, 4, 3, 4, 2>(dz4, S, g.wd[3], 96, 864,
        EpiMask<true>{w.gx, w.a3, S * 20 * 20, 96}, st, K_DG4, 864)));
    float* dz3 = w.gx;
    // ---- conv3: wgrad (input d1), bias, dgrad -> grad wrt d1 (site 1) into gy ----
    RC((conv_wgrad<18, 18, 48, 3, 3, 2, 2>(dz3, w.d1, S, 96, 432, g.sw[2], g.sb[2], GEO[2].ZW, st, K_WG3, 432)));
    RC((conv_like<20, 20, 96, 0, 2, 3, 8, 1>(dz3, S, g.wd[2], 48, 864,
        EpiDropMask{w.gy, w.d1, s25, S * 18 * 18, 48}, st, K_DG3, 864)));
    RC((pool_scatter<36, 36, 48, false>(w.gy, w.i1, w.a2, S, st)));
    float* dz2 = w.a2;
    // ---- conv2: wgrad (input a1), bias, dgrad -> dz1 = . * (a1 > 0) into gx ----
    RC((conv_wgrad<34, 34, 48, 3, 3, 1, 3>(dz2, w.a1, S, 48, 432, g.sw[1], g.sb[1], GEO[1].ZW, st, K_WG2, 432)));
    RC((conv_like<36, 36, 48, 0, 2, 3, 8, 1>(dz2, S, g.wd[1], 48, 432,
        EpiMask<true>{w.gx, w.a1, S * 34 * 34, 48}, st, K_DG2, 432)));
    float* dz1 = w.gx;
    // ---- conv1: wgrad (input x0), bias ----
    RC((conv_wgrad<32, 32, 4, 3, 3, 1, 1>(dz1, w.x0, S, 48, 48, g.sw[0], g.sb[0], GEO[0].ZW, st, K_WG1, 27)));
    return 0;
}

}  // namespace flsim

using namespace flsim;

// =============================================================================================
// C-ABI (declared in include/flsim.h)
// =============================================================================================
extern "C" {

const char* flsim_last_error(void) { return last_error(); }

long flsim_pn1_param_count(void) { return P_TOTAL; }

long flsim_pn1_gradstate_bytes(void) { return gs_layout(nullptr).total_floats * 4; }

long flsim_pn1_workspace_bytes(int max_samples) { return ws_layout(nullptr, max_samples).bytes; }

int flsim_pn1_workspace_offset(int which, int samples, long* offset_bytes) {
    char* const fake = reinterpret_cast<char*>(4096);   // layout only; never dereferenced
    WS w = ws_layout(fake, samples);
    const void* p[] = {w.x0, w.a1, w.a2, w.d1, w.a3, w.a4, w.d2, w.a5, w.a6, w.d3,
                       w.e1, w.e2, w.dh1, w.dh2, w.gx, w.gy, w.loss_s, w.dlog, w.y,
                       w.i1, w.i2, w.i3};
    FLSIM_REQUIRE(which >= 0 && which < (int)(sizeof(p) / sizeof(p[0])), "bad workspace id %d", which);
    *offset_bytes = (long)((const char*)p[which] - fake);
    return 0;
}

int flsim_pn1_begin_epoch(void* gradstate, const float* theta, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && theta, "null pointer");
    GradState g = gs_layout((float*)gradstate);
    RC(pack_weights(g, theta, stream));
    FLSIM_CHECK_HIP(hipMemsetAsync(g.slab_begin, 0, g.slab_floats * 4, stream));
    return 0;
}

static int run_chunk(void* gradstate, const WS& w, const float* theta, const WorkerRec* workers,
                     int n_chunk_workers, uint64_t seed, int dropout, int backward_pass,
                     float* worker_loss, hipStream_t stream) {
    const int S = n_chunk_workers * SAMPLES_PER_WORKER;
    GradState g = gs_layout((float*)gradstate);
    RC(forward(g, w, theta, S, workers, seed, dropout, stream));
    hipLaunchKernelGGL(k_head, dim3(ceil_div(S, 4)), dim3(256), 0, stream, w.e2, theta + P_OFF[16],
                       theta + P_OFF[17], w.y, w.loss_s, w.dlog, w.dh2, S, backward_pass,
                       dropout ? SCALE_P50 : 1.f, (int32_t*)nullptr, 0);
    FLSIM_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_worker_loss, dim3(n_chunk_workers), dim3(128), 0, stream, w.loss_s,
                       worker_loss);
    FLSIM_LAUNCH_CHECK();
    if (backward_pass) RC(backward(g, w, theta, S, dropout, stream));
    return 0;
}

int flsim_pn1_fwd_bwd_chunk(void* gradstate, void* workspace, int max_samples, const float* theta,
                            const uint8_t* pool, const int32_t* labels, const int32_t* list_a,
                            int len_a, const int32_t* list_b, int len_b, const float* lut,
                            const WorkerRec* workers, int n_chunk_workers, int n_workers_total,
                            uint64_t seed, int dropout, int backward_pass, float* worker_loss,
                            hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && pool && labels && list_a && list_b && lut &&
                  workers && worker_loss, "null pointer");
    FLSIM_REQUIRE(n_chunk_workers > 0, "empty chunk");
    const int S = n_chunk_workers * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE(S <= max_samples, "chunk of %d samples exceeds workspace (%d)", S, max_samples);
    FLSIM_REQUIRE(S <= 16384, "chunk of %d samples exceeds the 32-bit index budget", S);
    FLSIM_REQUIRE(len_a > 0 && len_b > 0, "empty class list");
    WS w = ws_layout((char*)workspace, max_samples);
    hipLaunchKernelGGL(k_fill_batch, dim3(S), dim3(256), 0, stream, pool, labels, list_a, len_a,
                       list_b, len_b, workers, n_workers_total, seed, lut, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    return run_chunk(gradstate, w, theta, workers, n_chunk_workers, seed, dropout, backward_pass,
                     worker_loss, stream);
}

// explicit batch (the Worker.fwd_bkwd(inp, outp) facade): x NCHW fp32, y int64; n_samples is a
// multiple of 128, workers[n_samples/128] give the dropout keys
int flsim_pn1_fwd_bwd_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                            const float* x, const int64_t* y, int n_samples,
                            const WorkerRec* workers, uint64_t seed, int dropout,
                            int backward_pass, float* worker_loss, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && x && y && workers && worker_loss,
                  "null pointer");
    FLSIM_REQUIRE(n_samples > 0 && n_samples % SAMPLES_PER_WORKER == 0,
                  "batch of %d samples: must be a positive multiple of %d", n_samples,
                  SAMPLES_PER_WORKER);
    FLSIM_REQUIRE(n_samples <= max_samples, "batch of %d samples exceeds workspace (%d)", n_samples,
                  max_samples);
    WS w = ws_layout((char*)workspace, max_samples);
    hipLaunchKernelGGL(k_load_input, dim3(n_samples), dim3(256), 0, stream, x, y, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    return run_chunk(gradstate, w, theta, workers, n_samples / SAMPLES_PER_WORKER, seed, dropout,
                     backward_pass, worker_loss, stream);
}

// Evaluation (util.py:31-45 print_test_accuracy; main.py:190 central.model.eval(), so dropout is
// off): forward of pool images [first, first + n_images) in chunks of max_samples, argmax of the
// logits into pred[n_images].  Re-packs theta (the next begin_epoch packs again).
int flsim_pn1_eval_pool(void* gradstate, void* workspace, int max_samples, const float* theta,
                        const uint8_t* pool, int first, int n_images, const float* lut,
                        int32_t* pred, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && pool && lut && pred, "null pointer");
    FLSIM_REQUIRE(n_images > 0 && first >= 0, "bad image range");
    FLSIM_REQUIRE(max_samples >= SAMPLES_PER_WORKER && max_samples % SAMPLES_PER_WORKER == 0,
                  "max_samples must be a positive multiple of %d", SAMPLES_PER_WORKER);
    GradState g = gs_layout((float*)gradstate);
    WS w = ws_layout((char*)workspace, max_samples);
    RC(pack_weights(g, theta, stream));
    for (int c0 = 0; c0 < n_images; c0 += max_samples) {
        const int n = n_images - c0 < max_samples ? n_images - c0 : max_samples;
        const int S = ceil_div(n, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
        hipLaunchKernelGGL(k_fill_seq, dim3(S), dim3(256), 0, stream, pool, first + c0, n, lut,
                           w.x0, w.y);
        FLSIM_LAUNCH_CHECK();
        RC(forward(g, w, theta, S, nullptr, 0, 0, stream));
        hipLaunchKernelGGL(k_head, dim3(ceil_div(S, 4)), dim3(256), 0, stream, w.e2,
                           theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, w.dlog, w.dh2, S,
                           0, 1.f, pred + c0, n);
        FLSIM_LAUNCH_CHECK();
    }
    return 0;
}

// S_t (torch named_parameters layout, P floats) = sum of the epoch's slabs
int flsim_pn1_end_epoch(void* gradstate, float* grad_out, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && grad_out, "null pointer");
    GradState g = gs_layout((float*)gradstate);
    for (int l = 0; l < 6; ++l) {
        const ConvGeo& c = GEO[l];
        RC(fin_sum(g.sw[l], c.ZW, (long)c.CO * c.KP, grad_out + P_OFF[2 * l], stream, c.CO, c.CI,
                   c.CIP, c.KP));
        RC(fin_sum(g.sb[l], c.ZW, c.CO, grad_out + P_OFF[2 * l + 1], stream));
    }
    RC(fin_sum(g.l1w, ZL1W, 512L * 9408, grad_out + P_OFF[12], stream));
    RC(fin_sum(g.l1b, ZL1W, 512, grad_out + P_OFF[13], stream));
    RC(fin_sum(g.l2w, ZL2W, 256L * 512, grad_out + P_OFF[14], stream));
    RC(fin_sum(g.l2b, ZL2W, 256, grad_out + P_OFF[15], stream));
    RC(fin_sum(g.l3w, ZH, 2560, grad_out + P_OFF[16], stream));
    RC(fin_sum(g.l3b, ZH, 10, grad_out + P_OFF[17], stream));
    return 0;
}

}  // extern "C"
