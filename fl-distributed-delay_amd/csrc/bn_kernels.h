// BatchNorm2d of vgg11_bn (reference FL/models.py:88-89: Conv2d -> BatchNorm2d(v) -> ReLU;
// torch defaults eps 1e-5, momentum 0.1, affine) for the worker-batched engine.
//
// Train mode normalises with the batch statistics of ONE fwd_bkwd call (agents.py:32-40), i.e.
// of one simulated worker's 128 samples: every (worker, channel) pair has its own mean / invstd.
// torch CPU's arithmetic (aten batch_norm_kernel.cpp), restated:
//   forward   var = M2 / N (biased), invstd = 1 / sqrt(var + eps),
//             alpha = invstd * gamma, shift = beta - mean * alpha, y = z * alpha + shift
//   running   r = momentum * stat + (1 - momentum) * r, stat = mean | M2 / (N - 1)  (per call,
//             in worker order: every computing worker runs the central model, main.py:154-169)
//   backward  sdy = sum dy, dotp = sum (z - mean) dy, k = dotp * invstd^2 / N,
//             dz = (dy - sdy / N - (z - mean) k) * invstd * gamma,
//             dgamma += dotp * invstd, dbeta += sdy
// Eval mode (util.py:31-45 after central.model.eval()) uses the running buffers: one
// (mean, invstd) per channel for every sample (per_worker = 0).
//
// Statistics are deterministic: a worker's N = 128*H*W pixels are cut into fixed blocks of
// BN_SPLIT_FLOATS floats; each block reduces its pixels in a fixed order (two passes: mean, then
// M2 about the block mean), and the blocks are merged in order with Chan's pairwise update.
// All kernels stream NHWC rows as float4 (C/4 lanes per pixel row: coalesced).
#pragma once
#include "net_kernels.h"

namespace flsim {

constexpr float BN_EPS = 1e-5f;
constexpr float BN_MOMENTUM = 0.1f;
constexpr int BN_SPLIT_FLOATS = 16384;   // floats of z per partial-statistics block

template <int C>
struct BNShape {
    static_assert(C % 4 == 0 && 256 % (C / 4) == 0, "BatchNorm channel count");
    static constexpr int C4 = C / 4;            // lanes per pixel row
    static constexpr int R = 256 / C4;          // pixel rows in flight per block
    static constexpr int PPB = BN_SPLIT_FLOATS / C;   // pixels per block
};

// ---- forward statistics -----------------------------------------------------------------
// block (s, w): pixels [s*PPB, (s+1)*PPB) of worker w -> block mean, M2 about it (per channel)
template <int C>
__global__ void __launch_bounds__(256)
k_bn_part(const float* __restrict__ z, int NP, float* __restrict__ pmean, float* __restrict__ pm2) {
    using B = BNShape<C>;
    __shared__ f32x4 red[256];
    __shared__ f32x4 bmean[B::C4];
    const int s = blockIdx.x, w = blockIdx.y, NS = gridDim.x;
    const int tc = threadIdx.x % B::C4, tr = threadIdx.x / B::C4;
    const float* base = z + ((long)w * NP + (long)s * B::PPB) * C + 4 * tc;
    f32x4 acc = zero4();
    for (int p = tr; p < B::PPB; p += B::R) acc += *reinterpret_cast<const f32x4*>(base + (long)p * C);
    red[threadIdx.x] = acc;
    __syncthreads();
    if (tr == 0) {
        f32x4 t = red[tc];
        for (int r = 1; r < B::R; ++r) t += red[r * B::C4 + tc];
        bmean[tc] = t / (float)B::PPB;
    }
    __syncthreads();
    const f32x4 mu = bmean[tc];
    f32x4 m2 = zero4();
    for (int p = tr; p < B::PPB; p += B::R) {
        const f32x4 d = *reinterpret_cast<const f32x4*>(base + (long)p * C) - mu;
        m2 += d * d;
    }
    __syncthreads();
    red[threadIdx.x] = m2;
    __syncthreads();
    if (tr == 0) {
        f32x4 t = red[tc];
        for (int r = 1; r < B::R; ++r) t += red[r * B::C4 + tc];
        const long o = ((long)w * NS + s) * C + 4 * tc;
        *reinterpret_cast<f32x4*>(pmean + o) = mu;
        *reinterpret_cast<f32x4*>(pm2 + o) = t;
    }
}

// (worker, channel): Chan-merge the NS blocks in order -> mean, invstd; optionally the per-call
// statistics for the running buffers: stats[w*nstat + off + c] = mean, [.. + C + c] = M2/(N-1)
template <int C>
__global__ void __launch_bounds__(256)
k_bn_final(const float* __restrict__ pmean, const float* __restrict__ pm2, int NS, int NP, int W,
           float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ stats,
           int off, int nstat) {
    using B = BNShape<C>;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= W * C) return;
    const int w = e / C, c = e - (e / C) * C;
    const float* pm = pmean + (long)w * NS * C + c;
    const float* pq = pm2 + (long)w * NS * C + c;
    float na = (float)B::PPB, ma = pm[0], qa = pq[0];
    const float nb = (float)B::PPB;
    for (int s = 1; s < NS; ++s) {
        const float mb = pm[(long)s * C], qb = pq[(long)s * C];
        const float n = na + nb;
        const float delta = mb - ma;
        ma = ma + delta * (nb / n);
        qa = qa + qb + delta * delta * (na * nb / n);
        na = n;
    }
    const float var = qa / (float)NP;
    mean[e] = ma;
    invstd[e] = 1.f / sqrtf(var + BN_EPS);
    if (stats) {
        stats[(long)w * nstat + off + c] = ma;
        stats[(long)w * nstat + off + C + c] = qa / (float)(NP - 1);
    }
}

// eval mode: per-channel (mean, invstd) from the running buffers (rm, rv)
static __global__ void k_bn_eval_coef(const float* __restrict__ rm, const float* __restrict__ rv,
                                      int C, float* __restrict__ mean, float* __restrict__ invstd) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    mean[c] = rm[c];
    invstd[c] = 1.f / sqrtf(rv[c] + BN_EPS);
}

// running buffers after n_workers calls, in worker order (nn.BatchNorm2d.forward, train mode)
static __global__ void k_bn_running(float* __restrict__ running, const float* __restrict__ stats,
                                    int n_workers, int nstat) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= nstat) return;
    float r = running[e];
    for (int w = 0; w < n_workers; ++w)
        r = BN_MOMENTUM * stats[(long)w * nstat + e] + (1.f - BN_MOMENTUM) * r;
    running[e] = r;
}

__device__ inline float bn_relu(float z, float mean, float inv, float g, float b) {
    const float alpha = inv * g;
    const float shift = b - mean * alpha;
    return fmaxf(z * alpha + shift, 0.f);
}

// ---- forward apply: a = relu(bn(z)) (unpooled layers) -------------------------------------
template <int HW, int C>
__global__ void __launch_bounds__(256)
k_bn_apply(const float* __restrict__ z, const float* __restrict__ mean,
           const float* __restrict__ invstd, const float* __restrict__ gamma,
           const float* __restrict__ beta, int per_worker, float* __restrict__ a, long total4) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= total4) return;
    const int c = 4 * (int)(e % (C / 4));
    const long pix = e / (C / 4);
    const int w = per_worker ? (int)(pix / ((long)HW * SAMPLES_PER_WORKER)) : 0;
    const f32x4 x = *reinterpret_cast<const f32x4*>(z + 4 * e);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + w * C + c);
    const f32x4 iv = *reinterpret_cast<const f32x4*>(invstd + w * C + c);
    const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 b = *reinterpret_cast<const f32x4*>(beta + c);
    f32x4 y;
    y.x = bn_relu(x.x, mu.x, iv.x, g.x, b.x);
    y.y = bn_relu(x.y, mu.y, iv.y, g.y, b.y);
    y.z = bn_relu(x.z, mu.z, iv.z, g.z, b.z);
    y.w = bn_relu(x.w, mu.w, iv.w, g.w, b.w);
    *reinterpret_cast<f32x4*>(a + 4 * e) = y;
}

// ---- forward apply + 2x2 max-pool (+ dropout): d, argmax as EpiPoolDrop writes them -------
// One thread per (pooled pixel, 4 channels); window positions in row-major order, first max
// wins (torch CPU); dropout element index in the pooled NCHW order of the worker's batch.
template <int H, int C>
__global__ void __launch_bounds__(256)
k_bn_apply_pool(const float* __restrict__ z, const float* __restrict__ mean,
                const float* __restrict__ invstd, const float* __restrict__ gamma,
                const float* __restrict__ beta, int per_worker, float* __restrict__ d,
                uint8_t* __restrict__ idx, const WorkerRec* __restrict__ workers, uint64_t seed,
                uint32_t site, uint32_t thr, float scale, int dropout, long total4) {
    constexpr int P = H / 2;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= total4) return;
    const int c = 4 * (int)(e % (C / 4));
    const long q = e / (C / 4);                  // pooled pixel (s, ph, pw)
    const int pw = (int)(q % P);
    const int ph = (int)((q / P) % P);
    const int s = (int)(q / (P * P));
    const int wk = s / SAMPLES_PER_WORKER;
    const int w = per_worker ? wk : 0;
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + w * C + c);
    const f32x4 iv = *reinterpret_cast<const f32x4*>(invstd + w * C + c);
    const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 b = *reinterpret_cast<const f32x4*>(beta + c);
    f32x4 mv;
    uint32_t mi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int pos = 0; pos < 4; ++pos) {
        const int h = 2 * ph + (pos >> 1), x = 2 * pw + (pos & 1);
        const f32x4 v = *reinterpret_cast<const f32x4*>(z + (((long)s * H + h) * H + x) * C + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float y = bn_relu(v[j], mu[j], iv[j], g[j], b[j]);
            if (pos == 0) {
                mv[j] = y;
            } else if (y > mv[j]) {
                mv[j] = y;
                mi[j] = pos;
            }
        }
    }
    if (dropout) {
        const WorkerRec wr = workers[wk];
        const int nl = s - wk * SAMPLES_PER_WORKER;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t en = (uint32_t)(((nl * C + c + j) * P + ph) * P + pw);
            mv[j] = philox_word(seed, wr.t, wr.i, site, en) >= thr ? mv[j] * scale : 0.f;
        }
    }
    *reinterpret_cast<f32x4*>(d + 4 * e) = mv;
    *reinterpret_cast<uint32_t*>(idx + 4 * e) = mi[0] | (mi[1] << 8) | (mi[2] << 16) | (mi[3] << 24);
}

// ---- backward ---------------------------------------------------------------------------
// block (s, w): sum dy and sum (z - mean_w) dy over the block's pixels
template <int C>
__global__ void __launch_bounds__(256)
k_bn_bpart(const float* __restrict__ dy, const float* __restrict__ z,
           const float* __restrict__ mean, int NP, float* __restrict__ psum,
           float* __restrict__ pdot) {
    using B = BNShape<C>;
    __shared__ f32x4 r1[256];
    __shared__ f32x4 r2[256];
    const int s = blockIdx.x, w = blockIdx.y, NS = gridDim.x;
    const int tc = threadIdx.x % B::C4, tr = threadIdx.x / B::C4;
    const long base = ((long)w * NP + (long)s * B::PPB) * C + 4 * tc;
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + w * C + 4 * tc);
    f32x4 a1 = zero4(), a2 = zero4();
    for (int p = tr; p < B::PPB; p += B::R) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(dy + base + (long)p * C);
        const f32x4 x = *reinterpret_cast<const f32x4*>(z + base + (long)p * C);
        a1 += g;
        a2 += (x - mu) * g;
    }
    r1[threadIdx.x] = a1;
    r2[threadIdx.x] = a2;
    __syncthreads();
    if (tr == 0) {
        f32x4 t1 = r1[tc], t2 = r2[tc];
        for (int r = 1; r < B::R; ++r) {
            t1 += r1[r * B::C4 + tc];
            t2 += r2[r * B::C4 + tc];
        }
        const long o = ((long)w * NS + s) * C + 4 * tc;
        *reinterpret_cast<f32x4*>(psum + o) = t1;
        *reinterpret_cast<f32x4*>(pdot + o) = t2;
    }
}

// (worker, channel): sums over the blocks in order -> the dz coefficients and the worker's
// gamma / beta gradient terms
template <int C>
__global__ void __launch_bounds__(256)
k_bn_bfinal(const float* __restrict__ psum, const float* __restrict__ pdot, int NS, int NP, int W,
            const float* __restrict__ invstd, float* __restrict__ cm, float* __restrict__ ck,
            float* __restrict__ dg, float* __restrict__ db) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= W * C) return;
    const int w = e / C, c = e - (e / C) * C;
    float sdy = 0.f, dot = 0.f;
    for (int s = 0; s < NS; ++s) {
        sdy += psum[((long)w * NS + s) * C + c];
        dot += pdot[((long)w * NS + s) * C + c];
    }
    const float iv = invstd[e];
    cm[e] = sdy / (float)NP;
    ck[e] = dot * iv * iv / (float)NP;
    dg[e] = dot * iv;
    db[e] = sdy;
}

// gamma / beta gradient of the chunk, accumulated in worker order into the epoch's sums
template <int C>
__global__ void __launch_bounds__(256)
k_bn_gacc(const float* __restrict__ dg, const float* __restrict__ db, int W,
          float* __restrict__ acc) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float g = acc[c], b = acc[C + c];
    for (int w = 0; w < W; ++w) {
        g += dg[w * C + c];
        b += db[w * C + c];
    }
    acc[c] = g;
    acc[C + c] = b;
}

// dz = (dy - cm - (z - mean) ck) * invstd * gamma, in place over dy
template <int HW, int C>
__global__ void __launch_bounds__(256)
k_bn_bapply(float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ mean,
            const float* __restrict__ invstd, const float* __restrict__ cm,
            const float* __restrict__ ck, const float* __restrict__ gamma, long total4) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= total4) return;
    const int c = 4 * (int)(e % (C / 4));
    const int w = (int)((e / (C / 4)) / ((long)HW * SAMPLES_PER_WORKER));
    const int o = w * C + c;
    const f32x4 g = *reinterpret_cast<const f32x4*>(dy + 4 * e);
    const f32x4 x = *reinterpret_cast<const f32x4*>(z + 4 * e);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + o);
    const f32x4 iv = *reinterpret_cast<const f32x4*>(invstd + o);
    const f32x4 a = *reinterpret_cast<const f32x4*>(cm + o);
    const f32x4 k = *reinterpret_cast<const f32x4*>(ck + o);
    const f32x4 gm = *reinterpret_cast<const f32x4*>(gamma + c);
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ((g[j] - a[j]) - (x[j] - mu[j]) * k[j]) * iv[j] * gm[j];
    *reinterpret_cast<f32x4*>(dy + 4 * e) = r;
}

// ---- launch helpers ---------------------------------------------------------------------
// scratch: pa, pb hold W * NS * C floats each (NS * C = 128 * H * H * C^2 / BN_SPLIT_FLOATS)
template <int H, int C>
static int bn_forward_stats(const float* z, int S, float* mean, float* invstd, float* pa,
                            float* pb, float* stats, int off, int nstat, hipStream_t st) {
    constexpr int NP = SAMPLES_PER_WORKER * H * H;
    constexpr int NS = NP / BNShape<C>::PPB;
    static_assert(NP % BNShape<C>::PPB == 0, "pixels per worker must split into whole blocks");
    const int W = S / SAMPLES_PER_WORKER;
    hipLaunchKernelGGL(k_bn_part<C>, dim3(NS, W), dim3(256), 0, st, z, NP, pa, pb);
    FLSIM_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_bn_final<C>, dim3(ceil_div((long)W * C, 256)), dim3(256), 0, st, pa, pb,
                       NS, NP, W, mean, invstd, stats, off, nstat);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

template <int H, int C>
static int bn_apply(const float* z, int S, const float* mean, const float* invstd,
                    const float* gamma, const float* beta, int per_worker, float* a,
                    hipStream_t st) {
    const long total4 = (long)S * H * H * (C / 4);
    hipLaunchKernelGGL((k_bn_apply<H * H, C>), dim3(ceil_div(total4, 256)), dim3(256), 0, st, z,
                       mean, invstd, gamma, beta, per_worker, a, total4);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

template <int H, int C>
static int bn_apply_pool(const float* z, int S, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int per_worker, float* d,
                         uint8_t* idx, const WorkerRec* workers, uint64_t seed, uint32_t site,
                         uint32_t thr, float scale, int dropout, hipStream_t st) {
    const long total4 = (long)S * (H / 2) * (H / 2) * (C / 4);
    hipLaunchKernelGGL((k_bn_apply_pool<H, C>), dim3(ceil_div(total4, 256)), dim3(256), 0, st, z,
                       mean, invstd, gamma, beta, per_worker, d, idx, workers, seed, site, thr,
                       scale, dropout, total4);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// dy (gradient wrt the BatchNorm output, ReLU mask applied) -> dz in place; gamma / beta
// gradients accumulated into acc[0..C) / acc[C..2C).  scratch: pa, pb as bn_forward_stats;
// cm, ck, dg, db hold W * C floats each.
template <int H, int C>
static int bn_backward(float* dy, const float* z, int S, const float* mean, const float* invstd,
                       const float* gamma, float* pa, float* pb, float* cm, float* ck, float* dg,
                       float* db, float* acc, hipStream_t st) {
    constexpr int NP = SAMPLES_PER_WORKER * H * H;
    constexpr int NS = NP / BNShape<C>::PPB;
    const int W = S / SAMPLES_PER_WORKER;
    hipLaunchKernelGGL(k_bn_bpart<C>, dim3(NS, W), dim3(256), 0, st, dy, z, mean, NP, pa, pb);
    FLSIM_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_bn_bfinal<C>, dim3(ceil_div((long)W * C, 256)), dim3(256), 0, st, pa, pb,
                       NS, NP, W, invstd, cm, ck, dg, db);
    FLSIM_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_bn_gacc<C>, dim3(ceil_div(C, 256)), dim3(256), 0, st, dg, db, W, acc);
    FLSIM_LAUNCH_CHECK();
    const long total4 = (long)S * H * H * (C / 4);
    hipLaunchKernelGGL((k_bn_bapply<H * H, C>), dim3(ceil_div(total4, 256)), dim3(256), 0, st, dy,
                       z, mean, invstd, cm, ck, gamma, total4);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

}  // namespace flsim
