// Kernels and launch helpers shared by the worker-batched networks (pn1_net.hip:
// PerformantNet1, vgg_net.hip: VGG-11).  Non-template kernels are `static` (one copy per
// translation unit); templates are instantiated per use.
//
// Layout conventions (both nets): activations NHWC fp32, one 128-sample block per simulated
// worker (main.py:43-44 batch_size); conv weights re-packed once per epoch into
// Wf[co][k(khkw, ci)] (forward) and Wd[ci][k(khkw', co)] = W[co][ci][2-kh'][2-kw'] (data
// gradient), k in Im2colKC's channel-slice-major order (k_pack_fwd).
#pragma once
#include "epi_xs.h"
#include "gemm_direct.h"
#include "gemm_dx6.h"
#include "gemm_x6.h"
#include "loaders.h"
#include "pn1.h"
#include "probe.h"

namespace flsim {

// =============================================================================================
// batch assembly: main.py:138-142 (k-th dataset, 128 samples with replacement, ToTensor +
// Normalize) -> x0 NHWC [S][32][32][4] (4th channel zero), y [S]
// =============================================================================================
static __global__ void __launch_bounds__(256)
k_fill_batch(const uint8_t* __restrict__ pool, const int32_t* __restrict__ labels,
             const int32_t* __restrict__ list_a, int len_a, const int32_t* __restrict__ list_b,
             int len_b, const WorkerRec* __restrict__ workers, int n_workers_total, uint64_t seed,
             const float* __restrict__ lut, float* __restrict__ x0, int32_t* __restrict__ y) {
    const int s = blockIdx.x;  // sample within chunk
    const int w = s / SAMPLES_PER_WORKER;
    const int j = s - w * SAMPLES_PER_WORKER;
    const WorkerRec wr = workers[w];
    // --batch_size B (main.py:43-44): WorkerRec.pad = B (0 = 128); the B samples of worker i span
    // ceil(B/128) records with i + g * 2^20 (group g); slot j of group g is sample g*128 + j of
    // the worker's batch, drawn with the worker's own key; slots past B are padding (label -1:
    // no loss, no gradient; zero image)
    const uint32_t bsz = wr.pad ? wr.pad : (uint32_t)SAMPLES_PER_WORKER;
    const uint32_t q = (wr.i >> 20) * SAMPLES_PER_WORKER + (uint32_t)j;
    float* out = x0 + (long)s * 4096;
    if (q >= bsz) {
        if (threadIdx.x == 0) y[s] = -1;
        for (int p = threadIdx.x; p < 1024; p += 256)
            *reinterpret_cast<f32x4*>(out + 4 * p) = f32x4{0.f, 0.f, 0.f, 0.f};
        return;
    }
    const bool use_b = (int)wr.k == n_workers_total - 1;   // main.py:78-80: last dataset = {1,9}
    const int len = use_b ? len_b : len_a;
    const uint32_t u = philox_word(seed, wr.t, wr.i & 0xfffffu, SITE_DATA, q);
    const int idx = use_b ? list_b[u % (uint32_t)len] : list_a[u % (uint32_t)len];
    if (threadIdx.x == 0) y[s] = labels[idx];
    const uint8_t* img = pool + (long)idx * 3072;
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
static __global__ void __launch_bounds__(256)
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
static __global__ void __launch_bounds__(256)
k_load_input(const float* __restrict__ x, const int64_t* __restrict__ yin, int n,
             float* __restrict__ x0, int32_t* __restrict__ y) {
    // samples s >= n pad the batch to whole 128-sample groups: zero image, label -1 (the head
    // gives them zero loss and zero gradient)
    const int s = blockIdx.x;
    const bool real = s < n;
    if (threadIdx.x == 0) y[s] = (real && yin) ? (int32_t)yin[s] : -1;
    const float* img = x + (long)s * 3072;
    float* out = x0 + (long)s * 4096;
    for (int p = threadIdx.x; p < 1024; p += 256) {
        f32x4 v = zero4();
        if (real) {
            v.x = img[p];
            v.y = img[1024 + p];
            v.z = img[2048 + p];
        }
        *reinterpret_cast<f32x4*>(out + 4 * p) = v;
    }
}

// =============================================================================================
// gradient through max_pool2d (+ dropout): dz[n][h][w][c] = gy[n][h/2][w/2][c] at the window's
// argmax, 0 elsewhere and on the floor-mode border.  One thread per (window, 4 channels): one gy
// float4 (or 4 NCHW scalars), one idx word, four float4 stores.  gy is already masked / scaled
// by the consumer's epilogue.
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
        st_nt4(dz + (((long)n * H + h) * W + w) * C + c, v);
    }
}

// NCHW gy (the pool feeding linear1 through torch's C,H,W flatten): one block per sample.  The
// sample's gy plane set (C * PH * PW floats, contiguous) is read into LDS with coalesced float4
// loads, then the (window, 4 channels) threads pick their four channels from LDS, so neither
// side of the transpose makes strided global accesses.
template <int H, int W, int C, bool XS = false>
__global__ void __launch_bounds__(256)
k_pool_scatter_nchw(const float* __restrict__ gy, const uint8_t* __restrict__ idx,
                    float* __restrict__ dz, float* __restrict__ dzl = nullptr) {
    constexpr int PH = H / 2, PW = W / 2, PP = PH * PW;
    constexpr int CH = (H + 1) / 2, CW = (W + 1) / 2;
    constexpr int C4 = C / 4;
    static_assert((C * PP) % 4 == 0, "float4 staging");
    __shared__ __attribute__((aligned(16))) float sg[C * PP];
    const int n = blockIdx.x;
    const f32x4* src = reinterpret_cast<const f32x4*>(gy + (long)n * C * PP);
    for (int i = threadIdx.x; i < C * PP / 4; i += 256)
        reinterpret_cast<f32x4*>(sg)[i] = src[i];
    __syncthreads();
    for (int e = threadIdx.x; e < CH * CW * C4; e += 256) {
        const int c = 4 * (e % C4);
        const int cell = e / C4;
        const int cw = cell % CW, ch = cell / CW;
        f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
        uint32_t id = 0xffffffffu;
        if (ch < PH && cw < PW) {
            id = *reinterpret_cast<const uint32_t*>(idx + (((long)n * PH + ch) * PW + cw) * C + c);
            const float* b = sg + c * PP + ch * PW + cw;
            g.x = b[0];
            g.y = b[PP];
            g.z = b[2 * PP];
            g.w = b[3 * PP];
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
            const long o = (((long)n * H + h) * W + w) * C + c;
            if constexpr (XS)
                xs_store(dz, dzl, o / 4, v);     // dZ in the split form (split.h)
            else
                st_nt4(dz + o, v);
        }
    }
}

template <int H, int W, int C, bool NCHW_G>
static int pool_scatter(const float* gy, const uint8_t* idx, float* dz, int S, hipStream_t st) {
    if constexpr (NCHW_G) {
        hipLaunchKernelGGL((k_pool_scatter_nchw<H, W, C, false>), dim3(S), dim3(256), 0, st, gy,
                           idx, dz, nullptr);
    } else {
        const long total = (long)S * ((H + 1) / 2) * ((W + 1) / 2) * (C / 4);
        hipLaunchKernelGGL((k_pool_scatter<H, W, C, false>), dim3(ceil_div(total, 256)), dim3(256),
                           0, st, gy, idx, dz, total);
    }
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// =============================================================================================
// linear split-K finish: e[m][n] = dropout(relu(sum_z part[z][m][n] + b[n]))
// (PerformantNet1 models.py:42-45; VGG classifier models.py:59-63)
// =============================================================================================
static __global__ void __launch_bounds__(256)
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

static int linear_finish(const float* part, int Z, const float* bias, float* out, int M, int N,
                         const WorkerRec* workers, uint64_t seed, uint32_t site, uint32_t thr,
                         float scale, int dropout, hipStream_t st) {
    hipLaunchKernelGGL(k_linear_finish, dim3(ceil_div((long)M * N, 256)), dim3(256), 0, st, part, Z,
                       bias, out, M, N, workers, seed, site, thr, scale, dropout);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// =============================================================================================
// head: last linear (K -> 10) + CrossEntropyLoss(mean over the worker's 128) forward and
// backward (PerformantNet1 models.py:46 / VGG models.py:64, main.py:107, agents.py:34-35).
// One wave per sample; lane l holds features 4l + 256c (c < K/256).
//   loss_s[s] = logsumexp(z) - z_y ; dlog[s][j] = (softmax - onehot) * gscale
// gscale = 1/128 (one worker's mean over its 128 samples) or 1/n for an n-sample facade batch;
// a label < 0 marks a padding sample: zero loss, zero gradient
//   dh[s][k] = (sum_j dlog[s][j] W[j][k]) * sdrop * (e[s][k] > 0)   (dropout / ReLU backward)
// =============================================================================================
template <int K>
__global__ void __launch_bounds__(256)
k_head(const float* __restrict__ e2, const float* __restrict__ W3, const float* __restrict__ b3,
       const int32_t* __restrict__ y, float* __restrict__ loss_s, float* __restrict__ dlog,
       float* __restrict__ dh2, int S, int backward, float sdrop, float gscale,
       int32_t* __restrict__ pred, int n_pred, const WorkerRec* __restrict__ workers) {
    constexpr int NC = K / 256;
    static_assert(K % 256 == 0, "head width must be a multiple of 256");
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (s >= S) return;
    f32x4 x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
        x[c] = *reinterpret_cast<const f32x4*>(e2 + (long)s * K + 4 * lane + 256 * c);
    float z[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
        float p = 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const f32x4 wv = *reinterpret_cast<const f32x4*>(W3 + j * K + 4 * lane + 256 * c);
            p += x[c].x * wv.x + x[c].y * wv.y + x[c].z * wv.z + x[c].w * wv.w;
        }
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
    if (lane == 0) loss_s[s] = lab >= 0 ? (mx + logf(se)) - zy : 0.f;
    if (pred && lane == 0 && s < n_pred) {       // torch.max(outputs, 1): first max wins
        int am = 0;
#pragma unroll
        for (int j = 1; j < 10; ++j) am = z[j] > z[am] ? j : am;
        pred[s] = am;
    }
    if (!backward) return;
    // CrossEntropyLoss's mean over the worker's B samples (WorkerRec.pad = B, 0: gscale)
    if (workers) {
        const uint32_t b = workers[s / SAMPLES_PER_WORKER].pad;
        if (b) gscale = 1.f / (float)b;
    }
    float g[10];
    const float inv = 1.f / se;
#pragma unroll
    for (int j = 0; j < 10; ++j)
        g[j] = lab >= 0 ? (expf(z[j] - mx) * inv - (j == lab ? 1.f : 0.f)) * gscale : 0.f;
    if (lane < 10) {
        float gv = 0.f;
#pragma unroll
        for (int j = 0; j < 10; ++j) gv = (j == lane) ? g[j] : gv;
        dlog[(long)s * 16 + lane] = gv;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        f32x4 d = zero4();
#pragma unroll
        for (int j = 0; j < 10; ++j) {
            const f32x4 wv = *reinterpret_cast<const f32x4*>(W3 + j * K + 4 * lane + 256 * c);
            d.x += g[j] * wv.x;
            d.y += g[j] * wv.y;
            d.z += g[j] * wv.z;
            d.w += g[j] * wv.w;
        }
        d.x = x[c].x > 0.f ? d.x * sdrop : 0.f;
        d.y = x[c].y > 0.f ? d.y * sdrop : 0.f;
        d.z = x[c].z > 0.f ? d.z * sdrop : 0.f;
        d.w = x[c].w > 0.f ? d.w * sdrop : 0.f;
        *reinterpret_cast<f32x4*>(dh2 + (long)s * K + 4 * lane + 256 * c) = d;
    }
}

// per-worker mean loss (fixed-order tree over the worker's 128 samples)
static __global__ void __launch_bounds__(128)
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

// head forward (+ backward) and the per-worker losses of a chunk of S samples
template <int K>
static int head_and_loss(const float* e, const float* W, const float* b, const int32_t* y,
                         float* loss_s, float* dlog, float* dh, int S, int backward, float sdrop,
                         float gscale, float* worker_loss, hipStream_t st,
                         const WorkerRec* workers = nullptr) {
    hipLaunchKernelGGL(k_head<K>, dim3(ceil_div(S, 4)), dim3(256), 0, st, e, W, b, y, loss_s, dlog,
                       dh, S, backward, sdrop, gscale, (int32_t*)nullptr, 0, workers);
    FLSIM_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_worker_loss, dim3(S / SAMPLES_PER_WORKER), dim3(128), 0, st, loss_s,
                       worker_loss);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// head forward only, argmax predictions for the first n_pred samples (evaluation)
template <int K>
static int head_predict(const float* e, const float* W, const float* b, const int32_t* y,
                        float* loss_s, int S, int32_t* pred, int n_pred, hipStream_t st) {
    hipLaunchKernelGGL(k_head<K>, dim3(ceil_div(S, 4)), dim3(256), 0, st, e, W, b, y, loss_s,
                       (float*)nullptr, (float*)nullptr, S, 0, 1.f, 1.f, pred, n_pred,
                       (const WorkerRec*)nullptr);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// last-linear weight/bias gradient, accumulated: slab[z][j][0..K) += sum_s dlog[s][j] e[s][k];
// slab_b[z][j] += sum_s dlog[s][j].  Block (j, z) sums a row range of samples.
template <int K>
__global__ void __launch_bounds__(256)
k_head_wgrad(const float* __restrict__ dlog, const float* __restrict__ e2, float* __restrict__ slab,
             float* __restrict__ slab_b, int S, int Z) {
    constexpr int NC = K / 256;
    const int j = blockIdx.x;
    const int z = blockIdx.y;
    const int k = threadIdx.x;
    const int per = (S + Z - 1) / Z;
    const int s0 = z * per;
    const int s1 = min(S, s0 + per);
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.f;
    float accb = 0.f;
    for (int s = s0; s < s1; ++s) {
        const float g = dlog[(long)s * 16 + j];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += g * e2[(long)s * K + k + 256 * c];
        accb += g;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) slab[((long)z * 10 + j) * K + k + 256 * c] += acc[c];
    if (k == 0) slab_b[z * 10 + j] += accb;
}

template <int K>
static int head_wgrad(const float* dlog, const float* e, float* slab, float* slab_b, int S, int Z,
                      hipStream_t st) {
    hipLaunchKernelGGL(k_head_wgrad<K>, dim3(10, Z), dim3(256), 0, st, dlog, e, slab, slab_b, S, Z);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// =============================================================================================
// per-epoch weight packing (theta in torch layout -> kernel layouts)
// =============================================================================================
// forward: Wf[co][k] = W[co][ci][kh][kw] in Im2colKC's K order (loaders.h):
//   CIP % 16 == 0: k = (ci/16)*144 + khkw*16 + ci%16   (channel-slice-major)
//   otherwise:     k = khkw*CIP + ci  (ci < CI; zero padding ci in [CI, CIP) and k >= 9*CIP up
//                  to KP)
static __global__ void k_pack_fwd(const float* __restrict__ W, float* __restrict__ Wf, int CO,
                                  int CI, int CIP, int KP) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= CO * KP) return;
    const int co = e / KP;
    const int k = e - co * KP;
    int khkw, ci;
    if (CIP % 16 == 0) {
        const int cs = k / 144, r = k - 144 * cs;
        khkw = r >> 4;
        ci = 16 * cs + (r & 15);
    } else {
        khkw = k / CIP;
        ci = k - khkw * CIP;
    }
    float v = 0.f;
    if (khkw < 9 && ci < CI) v = W[(co * CI + ci) * 9 + khkw];
    Wf[e] = v;
}
// data gradient: Wd[ci][k] = W[co][ci][8 - khkw'], k = (co/16)*144 + khkw'*16 + co%16 (the
// channel-slice-major order of Im2colKC over dZ; CO % 16 == 0 for every layer with a data
// gradient)
static __global__ void k_pack_dgrad(const float* __restrict__ W, float* __restrict__ Wd, int CO,
                                    int CI) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int KD = 9 * CO;
    if (e >= CI * KD) return;
    const int ci = e / KD;
    const int k = e - ci * KD;
    const int cs = k / 144, r = k - 144 * cs;
    const int khkw = r >> 4;
    const int co = 16 * cs + (r & 15);
    Wd[e] = W[(co * CI + ci) * 9 + (8 - khkw)];
}

// The same two packings in the split-bf16 form (split.h), one thread per 4-k unit: the forward
// packing of a layer with CIP % 16 == 0 and the data-gradient packing (PerformantNet1 conv2-6,
// whose GEMMs read split operands)
static __global__ void k_pack_fwd_xs(const float* __restrict__ W, float* __restrict__ hm,
                                     float* __restrict__ l, int CO, int CI, int KP) {
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= CO * KP / 4) return;
    const int e0 = 4 * u;
    const int co = e0 / KP;
    const int k0 = e0 - co * KP;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = k0 + j;
        const int cs = k / 144, r = k - 144 * cs;
        const int khkw = r >> 4;
        const int ci = 16 * cs + (r & 15);
        v[j] = (khkw < 9 && ci < CI) ? W[(co * CI + ci) * 9 + khkw] : 0.f;
    }
    xs_store<false>(hm, l, u, v);
}
static __global__ void k_pack_dgrad_xs(const float* __restrict__ W, float* __restrict__ hm,
                                       float* __restrict__ l, int CO, int CI) {
    const int u = blockIdx.x * 256 + threadIdx.x;
    const int KD = 9 * CO;
    if (u >= CI * KD / 4) return;
    const int e0 = 4 * u;
    const int ci = e0 / KD;
    const int k0 = e0 - ci * KD;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = k0 + j;
        const int cs = k / 144, r = k - 144 * cs;
        const int khkw = r >> 4;
        const int co = 16 * cs + (r & 15);
        v[j] = W[(co * CI + ci) * 9 + (8 - khkw)];
    }
    xs_store<false>(hm, l, u, v);
}
// a row-major matrix (linear1's W [512][9408], torch layout) in the split form
static __global__ void k_split_rows(const float* __restrict__ W, float* __restrict__ hm,
                                    float* __restrict__ l, long units) {
    const long u = (long)blockIdx.x * 256 + threadIdx.x;
    if (u < units) xs_store<false>(hm, l, u, reinterpret_cast<const f32x4*>(W)[u]);
}

// split tensor: HM part and L part (split.h)
struct XsT {
    float* hm;
    float* l;
};

static int pack_conv_xs(const float* W, XsT wf, XsT wd, int CO, int CI, int KP, hipStream_t st) {
    if (CI % 16 != 0 || CO % 16 != 0 || KP != 9 * CI) return 1;
    hipLaunchKernelGGL(k_pack_fwd_xs, dim3(ceil_div((long)CO * KP / 4, 256)), dim3(256), 0, st, W,
                       wf.hm, wf.l, CO, CI, KP);
    FLSIM_LAUNCH_CHECK();
    if (wd.hm) {           // (no split data-gradient packing when that GEMM runs on fp32)
        hipLaunchKernelGGL(k_pack_dgrad_xs, dim3(ceil_div((long)CI * 9 * CO / 4, 256)), dim3(256),
                           0, st, W, wd.hm, wd.l, CO, CI);
        FLSIM_LAUNCH_CHECK();
    }
    return 0;
}

static int split_rows(const float* W, XsT out, long n, hipStream_t st) {
    if (n % 4) return 1;
    hipLaunchKernelGGL(k_split_rows, dim3(ceil_div(n / 4, 256)), dim3(256), 0, st, W, out.hm, out.l,
                       n / 4);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// both packings of one conv layer (wd == nullptr: no data gradient needed, first layer)
static int pack_conv(const float* W, float* wf, float* wd, int CO, int CI, int CIP, int KP,
                     hipStream_t st) {
    hipLaunchKernelGGL(k_pack_fwd, dim3(ceil_div((long)CO * KP, 256)), dim3(256), 0, st, W, wf, CO,
                       CI, CIP, KP);
    FLSIM_LAUNCH_CHECK();
    if (wd) {
        if (CO % 16 != 0) return 1;
        hipLaunchKernelGGL(k_pack_dgrad, dim3(ceil_div((long)CI * 9 * CO, 256)), dim3(256), 0, st,
                           W, wd, CO, CI);
        FLSIM_LAUNCH_CHECK();
    }
    return 0;
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

// Large slabs (n % 4 == 0, n >= 64K): one wave per z-lane, so each wave reads 1 KB contiguous
// per slab, and four slabs in flight per thread (partials u = 0..3 take z = tz + (4j + u) * 4,
// added in u order): fixed order, deterministic.  (Template only for one definition per TU.)
template <int V>
__global__ void __launch_bounds__(256)
k_fin_sum_wide(const float* __restrict__ slab, int Z, long n, float* __restrict__ out, int CO,
               int CI, int CIP, int KP) {
    __shared__ f32x4 red[256];
    const int tx = threadIdx.x & 63, tz = threadIdx.x >> 6;
    const long e0 = ((long)blockIdx.x * 64 + tx) * 4;
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = zero4();
    if (e0 < n) {
        const float* p = slab + e0;
        int z = tz;
        for (; z + 12 < Z; z += 16) {
            f32x4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const f32x4*>(p + (long)(z + 4 * u) * n);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc[u].x += x[u].x;
                acc[u].y += x[u].y;
                acc[u].z += x[u].z;
                acc[u].w += x[u].w;
            }
        }
        for (int u = 0; z < Z; z += 4, ++u) {
            const f32x4 x = *reinterpret_cast<const f32x4*>(p + (long)z * n);
            acc[u].x += x.x;
            acc[u].y += x.y;
            acc[u].z += x.z;
            acc[u].w += x.w;
        }
    }
    f32x4 t = acc[0];
#pragma unroll
    for (int u = 1; u < 4; ++u) {
        t.x += acc[u].x;
        t.y += acc[u].y;
        t.z += acc[u].z;
        t.w += acc[u].w;
    }
    red[threadIdx.x] = t;
    __syncthreads();
    if (tz != 0 || e0 >= n) return;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
        const f32x4 y = red[j * 64 + tx];
        t.x += y.x;
        t.y += y.y;
        t.z += y.z;
        t.w += y.w;
    }
    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const long s = e0 + v;
        if (CO > 0) {
            const int co = (int)(s / KP);
            const int k = (int)(s - (long)co * KP);
            const int khkw = k / CIP, ci = k - (k / CIP) * CIP;
            if (khkw < 9 && ci < CI) out[((long)co * CI + ci) * 9 + khkw] = tv[v];
        } else {
            out[s] = tv[v];
        }
    }
}

static int fin_sum(const float* slab, int Z, long n, float* out, hipStream_t st, int CO = 0,
                   int CI = 0, int CIP = 1, int KP = 1) {
    if (n % 4 == 0 && n >= 65536 && Z >= 4) {
        hipLaunchKernelGGL(k_fin_sum_wide<4>, dim3(ceil_div(n, 256L)), dim3(256), 0, st, slab, Z, n,
                           out, CO, CI, CIP, KP);
        FLSIM_LAUNCH_CHECK();
        return 0;
    }
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
// GEMM launch helpers
// =============================================================================================
// X6: the split-bf16 kernel (gemm_x6.h) instead of the fp32 one
template <int FM, int FN, int WM, int WN, bool X6 = false, class AL, class BL, class EPI>
static int launch_gemm(const AL& al, const BL& bl, const EPI& epi, int M, int N, int ksteps, int Z,
                       hipStream_t st, int kid, double alg_flops) {
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    const int per = (ksteps + Z - 1) / Z;
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    dim3 grid(tm * tn * Z);
    const ProbeSlot ps = probe_begin();
    if constexpr (X6)
        hipExtLaunchKernelGGL((gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EPI>), grid,
                              dim3(64 * WM * WN), 0, st, ps.start, ps.stop, 0, al, bl, epi, ksteps,
                              per, tm, tn);
    else
        hipExtLaunchKernelGGL((gemm_kernel<FM, FN, WM, WN, AL, BL, EPI>), grid, dim3(64 * WM * WN),
                              0, st, ps.start, ps.stop, 0, al, bl, epi, ksteps, per, tm, tn);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, kid, alg_flops);
}

// direct-A GEMM (gemm_direct.h): rows = output pixels loaded per wave straight into MFMA
// fragments, B (packed weights) staged through LDS KB k-steps at a time
template <int FM, int FN, int WAVES, int KB, int DEPTH, class AD, class BL, class EPI>
static int launch_direct(const AD& ad, const BL& bl, const EPI& epi, int M, int N, int ksteps,
                         hipStream_t st, int kid, double alg_flops) {
    constexpr int BM = 16 * FM * WAVES, BN = 16 * FN;
    FLSIM_REQUIRE(ksteps % KB == 0, "direct GEMM: %d k-steps not a multiple of %d", ksteps, KB);
    const int tm = ceil_div(M, BM), tn = ceil_div(N, BN);
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL((gemm_direct_kernel<FM, FN, WAVES, KB, DEPTH, AD, BL, EPI>),
                          dim3(tm * tn), dim3(64 * WAVES), 0, st, ps.start, ps.stop, 0, ad, bl,
                          epi, ksteps, tm, tn);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, kid, alg_flops);
}

// forward conv (also the data-gradient conv) on the direct-A kernel: out[m][n], m < S*OH*OW
// (WIN: pool-window row order, see Im2colKC; OHX: explicit output size)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WAVES, int KB, int DEPTH,
          bool WIN, int OHX, class EPI>
static int conv_direct(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                       hipStream_t st, int kid, int kreal) {
    using AD = Im2colDirect<IH, IW, CI, PAD, FM, WIN, OHX>;
    using BL = RowsKCStage<16 * FN, 64 * WAVES>;
    AD ad;
    ad.X = X;
    ad.M = S * AD::ROWS_PER_IMG;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP;
    bl.NR = N;
    return launch_direct<FM, FN, WAVES, KB, DEPTH>(ad, bl, epi, ad.M, N, KP / GK, st, kid,
                                                   2.0 * ad.M * N * kreal);
}

// conv_pool_fwd on the direct-A kernel (rows in pool-window order, EpiPoolDrop)
template <int IH, int IW, int CI, int CO, int PAD, int FM, int FN, int WAVES, int KB, int DEPTH,
          bool NCHW_OUT>
static int conv_pool_direct(const float* X, int S, const float* Wpk, int KP, float* d,
                            uint8_t* idx, const float* bias, const WorkerRec* workers,
                            uint64_t seed, uint32_t site, uint32_t thr, float scale, int dropout,
                            hipStream_t st, int kid, int kreal) {
    using AD = Im2colDirect<IH, IW, CI, PAD, FM, true>;
    EpiPoolDrop<AD::PH, AD::PW, CO, NCHW_OUT> epi{d, idx, bias, workers, seed, site, thr,
                                                  scale, dropout, S * AD::ROWS_PER_IMG};
    return conv_direct<IH, IW, CI, PAD, FM, FN, WAVES, KB, DEPTH, true, 0>(
        X, S, Wpk, CO, KP, epi, st, kid, kreal);
}

// Small chunks (configs[1]: 5 workers = 640 samples per epoch) leave the 256-row direct tiles with
// a few rounds of blocks on 256 CUs; chunks of at most small_chunk_samples() samples can run the
// same GEMMs with half-height tiles (FM halved, and the weight gradients' small tiles).  The k
// order per output is unchanged, so the results are bit-identical.  Round 3 measured them faster
// up to 2048 samples; on round 5's kernels they lose at configs[1]'s 640 samples (993 against 1038
// worker-steps/s, profiles/r05/ab/c1_small_tiles_off.txt) and still win on the facade's 128-sample
// calls (713-722 against 677, ab/facade_small_tiles.txt): threshold 256 samples.  FLSIM_SMALL_S
// sets it.
static int small_chunk_samples() {
    static int s = -1;
    if (s < 0) {
        const char* e = lab_env("FLSIM_SMALL_S");
        s = e ? atoi(e) : 256;
    }
    return s;
}

template <int IH, int IW, int CI, int PAD, int FM, int FMS, int FN, int WAVES, int KB, int DEPTH,
          bool WIN, int OHX, class EPI>
static int conv_direct_sz(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                          hipStream_t st, int kid, int kreal) {
    if (S <= small_chunk_samples())
        return conv_direct<IH, IW, CI, PAD, FMS, FN, WAVES, KB, DEPTH, WIN, OHX>(X, S, Wpk, N, KP,
                                                                              epi, st, kid, kreal);
    return conv_direct<IH, IW, CI, PAD, FM, FN, WAVES, KB, DEPTH, WIN, OHX>(X, S, Wpk, N, KP, epi,
                                                                          st, kid, kreal);
}

template <int IH, int IW, int CI, int CO, int PAD, int FM, int FMS, int FN, int WAVES, int KB,
          int DEPTH, bool NCHW_OUT>
static int conv_pool_direct_sz(const float* X, int S, const float* Wpk, int KP, float* d,
                               uint8_t* idx, const float* bias, const WorkerRec* workers,
                               uint64_t seed, uint32_t site, uint32_t thr, float scale,
                               int dropout, hipStream_t st, int kid, int kreal) {
    if (S <= small_chunk_samples())
        return conv_pool_direct<IH, IW, CI, CO, PAD, FMS, FN, WAVES, KB, DEPTH, NCHW_OUT>(
            X, S, Wpk, KP, d, idx, bias, workers, seed, site, thr, scale, dropout, st, kid, kreal);
    return conv_pool_direct<IH, IW, CI, CO, PAD, FM, FN, WAVES, KB, DEPTH, NCHW_OUT>(
        X, S, Wpk, KP, d, idx, bias, workers, seed, site, thr, scale, dropout, st, kid, kreal);
}

// Splits of a slab-accumulating GEMM (weight gradients: the reduction runs over the chunk's
// pixels or samples).  The slab has Z rows; a small chunk (configs[1]: 5 workers = 640 samples)
// would leave each split a handful of k-steps, so the per-block prologue and the slab
// read-modify-write dominate.  Such launches use only the first max(ceil(ksteps / KMIN),
// ceil(1024 / tiles)) rows (>= 32 k-steps per split, >= 1024 blocks); the other rows keep what
// earlier chunks accumulated, and the epoch's slab sum reads every row.  KMIN = 32 measured on
// n = 10: 617 -> 645 worker-steps/s, headline unchanged (profiles/r02f/wsplit.txt).
// cap > 0 and FLSIM_WSPLIT_FILL=1: cap = the blocks the GPU holds at once for this kernel, and the
// split grows to fill the last round of resident blocks (same rounds, shorter blocks).  Off by
// default: on configs[1] it moved single weight gradients by -2..+5 % and the epoch not at all
// (776.4 vs 777.0 worker-steps/s, profiles/r03e), while the larger KMIN of the sweep in
// profiles/r03d (fewer, longer splits) made the weight gradients slower (conv6 124 -> 107 TF/s).
static int wsplit(int ksteps, int Z, int tiles, int cap = 0) {
    static int kmin = -1;
    if (kmin < 0) {
        const char* e = lab_env("FLSIM_WSPLIT_KMIN");     // measurement override (0: always Z)
        kmin = e ? atoi(e) : 32;
    }
    if (kmin <= 0) return Z;
    int z = (ksteps + kmin - 1) / kmin;
    const int zb = (1024 + tiles - 1) / tiles;
    if (z < zb) z = zb;
    static int fill = -1;
    if (fill < 0) {
        const char* e = lab_env("FLSIM_WSPLIT_FILL");     // measurement override (1: on)
        fill = e ? atoi(e) : 0;
    }
    if (fill && cap > 0 && z < Z) {
        const long rounds = ((long)tiles * z + cap - 1) / cap;
        const long zf = rounds * cap / tiles;
        if (zf > z) z = (int)(zf < ksteps ? zf : ksteps);
    }
    return z < Z ? z : Z;
}

// blocks of kernel f (block size nt, static LDS only) resident on the whole GPU at once
static int resident_blocks(const void* f, int nt) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = -1;
    }
    int per = 0;
    if (cus <= 0 || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, nt, 0) != hipSuccess)
        return 0;
    return per * cus;
}

// forward conv (also the data-gradient conv): out[m][n] for m < S*OH*OW, n < N
// (OHX > 0: explicit output size, see Im2colKC)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, class EPI, int OHX = 0,
          bool X6 = false>
static int conv_like(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                     hipStream_t st, int kid, int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IW, CI, PAD, BM, NT, false, OHX>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::OH * AL::OW;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP;
    bl.NR = N;
    return launch_gemm<FM, FN, WM, WN, X6>(al, bl, epi, al.M, N, KP / GK, 1, st, kid,
                                           2.0 * al.M * N * kreal);
}

// conv_like on the split-bf16 GEMM (gemm_x6.h): the forward and data-gradient convolutions at
// fp32 accuracy on the bf16 matrix cores
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, int OHX = 0, class EPI>
static int conv_x6(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                   hipStream_t st, int kid, int kreal) {
    return conv_like<IH, IW, CI, PAD, FM, FN, WM, WN, EPI, OHX, true>(X, S, Wpk, N, KP, epi, st,
                                                                      kid, kreal);
}

template <int IH, int IW, int CI, int PAD, int FM, int FMS, int FN, int WM, int WN, class EPI>
static int conv_like_sz(const float* X, int S, const float* Wpk, int N, int KP, const EPI& epi,
                        hipStream_t st, int kid, int kreal) {
    if (S <= small_chunk_samples())
        return conv_like<IH, IW, CI, PAD, FMS, FN, WM, WN>(X, S, Wpk, N, KP, epi, st, kid, kreal);
    return conv_like<IH, IW, CI, PAD, FM, FN, WM, WN>(X, S, Wpk, N, KP, epi, st, kid, kreal);
}

// weight gradient: slab[z][co][kk] += sum_p dz[p][co] * im2col(X)[p][kk]  (conv padding PAD)
// VO > 0: only the top-left VO x VO window of the output pixels (dz is zero outside it)
// DZC: dz is already stored compact over that window ([S][VO][VO][CO]), so its rows are the
// reduction index as they stand
// SRC = XsSrc: dz (and X, unless SRCB says otherwise) in the split form (dzl, Xl their L parts;
// X6 only)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, int VO = 0,
          bool DZC = false, bool X6 = false, class SRC = BufSrc, class SRCB = SRC>
static int conv_wgrad(const float* dz, const float* X, int S, int CO, int KP, float* slab,
                      float* bslab, int Z, hipStream_t st, int kid, int kreal,
                      int zinit = 0x7fffffff, int* zused = nullptr, const float* dzl = nullptr,
                      const float* Xl = nullptr) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    constexpr int OFULL = IH + 2 * PAD - 2;
    static_assert(IH == IW && VO <= OFULL, "square maps only");
    static_assert(X6 || (!SRC::SPLIT && !SRCB::SPLIT), "split operands run on the split-bf16 GEMM");
    using AL = RowsKM<BM, NT, (VO > 0 && !DZC ? OFULL : 0), (DZC ? 0 : VO), SRC>;
    using BL = Im2colKM<IH, IW, CI, PAD, BN, NT, VO, SRCB>;
    const int M = S * BL::OH * BL::OW;
    AL al;
    al.P = dz;
    al.PL = dzl;
    al.ld = CO;
    al.NK = M;
    al.NC = CO;
    BL bl;
    bl.X = X;
    bl.XL = Xl;
    bl.M = M;
    EpiSlabAcc epi{slab, CO, KP, (long)CO * KP, bslab, zinit};
    const int tiles = ceil_div(CO, BM) * ceil_div(KP, BN);
    const void* kfn;
    if constexpr (X6)
        kfn = (const void*)gemm_x6_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>;
    else
        kfn = (const void*)gemm_kernel<FM, FN, WM, WN, AL, BL, EpiSlabAcc>;
    static const int cap = resident_blocks(kfn, NT);
    const int zu = wsplit(ceil_div(M, GK), Z, tiles, cap);
    if (zused) *zused = zu;
    return launch_gemm<FM, FN, WM, WN, X6>(al, bl, epi, CO, KP, ceil_div(M, GK), zu, st, kid,
                                           2.0 * M * CO * kreal);
}

// conv_wgrad with a second tile for chunks of at most small_chunk_samples() samples
// (profiles/r03f/lab_s640_wgrad.txt: at 640 samples 96x96 4-wave tiles beat the 128-worker
// chunk's larger ones on conv3/5/6 by 3-10 %, 48x144 beats 48x48 on conv2 by 4 %)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, int FMS, int FNS,
          int WMS, int WNS, int VO = 0, bool DZC = false, bool X6 = false, class SRC = BufSrc,
          class SRCB = SRC>
static int conv_wgrad_sz(const float* dz, const float* X, int S, int CO, int KP, float* slab,
                         float* bslab, int Z, hipStream_t st, int kid, int kreal, int zinit,
                         int* zused, const float* dzl = nullptr, const float* Xl = nullptr) {
    if (S <= small_chunk_samples())
        return conv_wgrad<IH, IW, CI, PAD, FMS, FNS, WMS, WNS, VO, DZC, X6, SRC, SRCB>(
            dz, X, S, CO, KP, slab, bslab, Z, st, kid, kreal, zinit, zused, dzl, Xl);
    return conv_wgrad<IH, IW, CI, PAD, FM, FN, WM, WN, VO, DZC, X6, SRC, SRCB>(
        dz, X, S, CO, KP, slab, bslab, Z, st, kid, kreal, zinit, zused, dzl, Xl);
}

// ---- split-form operands (split.h): the PerformantNet1 conv2-6 forward / data-gradient GEMMs --
// conv (forward, or data gradient as a valid convolution) over a split input X and split packed
// weights W [N][KP] on the direct-A kernel (gemm_dx6.h): WAVES waves of 16*FM rows, 16*FN columns
// per n-tile, B staged KB k-steps a time (NPL planes), A loaded DEPTH k-steps ahead
// (ASRC = XsSrcSM: X channel-slice-major, loaders.h)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WAVES, int KB, int DEPTH, int NPL,
          bool WIN, int OHX, class ASRC = XsSrc, class EPI>
static int conv_dx6(XsT X, int S, XsT W, int N, int KP, const EPI& epi, hipStream_t st, int kid,
                    int kreal) {
    static_assert(ASRC::SPLIT, "split input");
    using AD = Im2colDirect<IH, IW, CI, PAD, FM, WIN, OHX, ASRC>;
    using BL = RowsKCStageXs<16 * FN, 64 * WAVES, NPL>;
    constexpr int BM = 16 * FM * WAVES, BN = 16 * FN;
    FLSIM_REQUIRE((KP / GK) % KB == 0, "direct GEMM: %d k-steps not a multiple of %d", KP / GK, KB);
    AD ad;
    ad.X = X.hm;
    ad.XL = X.l;
    ad.M = S * AD::ROWS_PER_IMG;
    BL bl;
    bl.P = W.hm;
    bl.PL = W.l;
    bl.ld = KP;
    bl.NR = N;
    const int tm = ceil_div(ad.M, BM), tn = ceil_div(N, BN);
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL((gemm_dx6_kernel<FM, FN, WAVES, KB, DEPTH, AD, BL, EPI>),
                          dim3(tm * tn), dim3(64 * WAVES), 0, st, ps.start, ps.stop, 0, ad, bl,
                          epi, KP / GK, tm, tn);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, kid, 2.0 * ad.M * N * kreal);
}

// the same GEMM on gemm_x6_kernel with both operands staged through LDS (bit-identical to
// conv_dx6: same split, same MFMA order per output): the tiles for small chunks
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, bool WIN, int OHX,
          class EPI>
static int conv_xs(XsT X, int S, XsT W, int N, int KP, const EPI& epi, hipStream_t st, int kid,
                   int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IW, CI, PAD, BM, NT, WIN, OHX, XsSrc>;
    using BL = RowsKC<BN, NT, XsSrc>;
    AL al;
    al.X = X.hm;
    al.XL = X.l;
    al.M = S * AL::ROWS_PER_IMG;
    BL bl;
    bl.P = W.hm;
    bl.PL = W.l;
    bl.ld = KP;
    bl.NR = N;
    return launch_gemm<FM, FN, WM, WN, true>(al, bl, epi, al.M, N, KP / GK, 1, st, kid,
                                             2.0 * al.M * N * kreal);
}

// forward conv fused with bias + ReLU + 2x2 max-pool (+ dropout: keep iff philox >= thr, kept
// values * scale): GEMM rows in pool-window order
template <int IH, int IW, int CI, int CO, int PAD, int FM, int FN, int WM, int WN, bool NCHW_OUT,
          bool X6 = false>
static int conv_pool_fwd(const float* X, int S, const float* Wpk, int KP, float* d, uint8_t* idx,
                         const float* bias, const WorkerRec* workers, uint64_t seed, uint32_t site,
                         uint32_t thr, float scale, int dropout, hipStream_t st, int kid,
                         int kreal) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
    using AL = Im2colKC<IH, IW, CI, PAD, BM, NT, true>;
    using BL = RowsKC<BN, NT>;
    AL al;
    al.X = X;
    al.M = S * AL::ROWS_PER_IMG;
    BL bl;
    bl.P = Wpk;
    bl.ld = KP;
    bl.NR = CO;
    EpiPoolDrop<AL::PH, AL::PW, CO, NCHW_OUT> epi{d, idx, bias, workers, seed, site, thr,
                                                  scale, dropout, al.M};
    return launch_gemm<FM, FN, WM, WN, X6>(al, bl, epi, al.M, CO, KP / GK, 1, st, kid,
                                           2.0 * al.M * CO * kreal);
}

// linear layer part[z] = x W^T over the z-th K range (x [M][K] rows, W [N][K] torch layout)
template <int FM, int FN, int WM, int WN, bool X6 = false, class EPI = EpiSlabStore>
static int linear_fwd(const float* x, const float* W, float* part, int M, int N, int K, int Z,
                      hipStream_t st, int kid) {
    constexpr int NT = 64 * WM * WN;
    RowsKC<16 * FM * WM, NT> al{};
    al.P = x; al.ld = K; al.NR = M;
    RowsKC<16 * FN * WN, NT> bl{};
    bl.P = W; bl.ld = K; bl.NR = N;
    EPI epi{};
    static_cast<EpiSlabStore&>(epi) = EpiSlabStore{part, M, N, (long)M * N};
    return launch_gemm<FM, FN, WM, WN, X6>(al, bl, epi, M, N, K / GK, Z, st, kid, 2.0 * M * N * K);
}

// linear weight gradient: slab[z][n][k] += sum_s dy[s][n] x[s][k]; bias slab[z][n] += sum_s dy
template <int FM, int FN, int WM, int WN, bool X6 = false>
static int linear_wgrad(const float* dy, const float* x, float* slab, float* bslab, int S, int N,
                        int K, int Z, hipStream_t st, int kid, int zinit = 0x7fffffff,
                        int* zused = nullptr) {
    constexpr int NT = 64 * WM * WN;
    RowsKM<16 * FM * WM, NT> al{};
    al.P = dy; al.ld = N; al.NK = S; al.NC = N;
    RowsKM<16 * FN * WN, NT> bl{};
    bl.P = x; bl.ld = K; bl.NK = S; bl.NC = K;
    EpiSlabAcc epi{slab, N, K, (long)N * K, bslab, zinit};
    const int tiles = ceil_div(N, 16 * FM * WM) * ceil_div(K, 16 * FN * WN);
    const int zu = wsplit(ceil_div(S, GK), Z, tiles);
    if (zused) *zused = zu;
    return launch_gemm<FM, FN, WM, WN, X6>(al, bl, epi, N, K, ceil_div(S, GK), zu, st, kid,
                                           2.0 * S * N * K);
}

// linear data gradient through the producer's dropout / ReLU:
// dx[s][k] = (sum_n dy[s][n] W[n][k]) * scale * (act[s][k] > 0)
template <int FM, int FN, int WM, int WN, bool X6 = false>
static int linear_dgrad(const float* dy, const float* W, float* dx, const float* act, float scale,
                        int S, int N, int K, hipStream_t st, int kid) {
    constexpr int NT = 64 * WM * WN;
    RowsKC<16 * FM * WM, NT> dl{};
    dl.P = dy; dl.ld = N; dl.NR = S;
    RowsKM<16 * FN * WN, NT> wl{};
    wl.P = W; wl.ld = K; wl.NK = N; wl.NC = K;
    EpiDropMaskPre de{{dx, act, scale, S, K}};
    return launch_gemm<FM, FN, WM, WN, X6>(dl, wl, de, S, K, N / GK, 1, st, kid,
                                           2.0 * S * N * K);
}

}  // namespace flsim
