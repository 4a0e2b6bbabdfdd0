// PerformantNet1 (reference FL/models.py:11-47) forward + backward for a chunk of simulated
// workers, as hand-written gfx950 kernels.  All workers of an epoch run on the same central
// model theta_t (main.py:154,159,169), so a chunk of W workers is ONE batch of W*128 samples;
// their gradients are summed (agents.py:35 accumulates into the shared .grad), which the weight
// gradient GEMMs do along their reduction (pixel / sample) dimension.
//
// Layout in HBM: activations NHWC (channels innermost); the flatten before linear1 is written in
// torch's NCHW order so linear1 uses the torch weight layout unchanged.  The tensors that feed the
// conv2-6 GEMMs (a1, d1, a3, d2, a5 and the data gradients dz6 .. dz2) and the packed conv2-6
// weights are stored in the split-bf16 form (split.h: HM + L parts, written once by their
// producer), so those GEMMs never split an operand in their inner loops; d3, e1, e2,
// dz1 and the linear layers stay fp32.
// Conv weights are re-packed once per epoch (net_kernels.h, shared with the VGG-11 engine
// vgg_net.hip together with the batch assembly, pool scatter, head, slab reduction and GEMM
// launchers).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <unordered_map>

#include "net_kernels.h"
#include "slabstep.h"

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
// Splits re-swept at the 128-worker chunk (profiles/r01f/lab_wgrad_splits_s16384.txt): twice the
// 4096-sample choice for conv2..6, 1-3 % faster each; the per-epoch slab sum reads 1.7 GB.
static const ConvGeo GEO[6] = {
    {3, 4, 48, 32, 48, 8192},    {48, 48, 48, 34, 432, 4096},   {48, 48, 96, 18, 432, 2048},
    {96, 96, 96, 20, 864, 1024}, {96, 96, 192, 11, 864, 512},  {192, 192, 192, 13, 1728, 256},
};
static const long P_OFF[18] = {0,       1296,    1344,    22080,   22128,   63600,
                               63696,   146640,  146736,  312624,  312816,  644592,
                               644784,  5461680, 5462192, 5593264, 5593520, 5596080};
constexpr long P_TOTAL = 5596090;
// linear1 forward split-K: 16, for the facade's one-call forwards (128 samples: 32 tiles of 32 x
// 64, so the split sets the block count), 0.447 -> 0.406 ms per call and facade 808 -> 834
// worker-steps/s against 4, the batched chunk unchanged (1051.7 / 1054.3), profiles/r06/r06t
#ifndef FLSIM_ZL1F
#define FLSIM_ZL1F 16
#endif
constexpr int ZL1F = FLSIM_ZL1F;
constexpr int ZL1W = 8;     // linear1 wgrad split
constexpr int ZL2W = 64;    // linear2 wgrad split
constexpr int ZH = 32;      // head wgrad split

// gradient-state layout (floats): packed weights + slabs
struct GradState {
    float* wf[6];  // conv1's fp32 packing (wf[1..5] unused)
    float* wd[6];  // fp32 data-gradient packings of conv2-6 (wd[0] unused)
    XsT wfx[6];    // conv2-6 forward packings, split (wfx[0] unused)
    XsT wdx[6];    // split data-gradient packings (unused: every data gradient runs on fp32)
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
    StepPlan plan;  // the fused server step over the slabs (slabstep.h)
    long cnt_off;   // its tile counters (inside the zeroed slab range) and unit partials
    long part_off;
};

// one segment per parameter tensor (named_parameters order), offsets from the gradstate base
static int pn1_segments(const GradState& g, const float* base, SegSpec* s) {
    int i = 0;
    for (int l = 0; l < 6; ++l) {
        const ConvGeo& c = GEO[l];
        s[i++] = SegSpec{g.sw[l] - base, c.ZW, (long)c.CO * c.KP, P_OFF[2 * l],
                         (long)c.CO * c.CI * 9, c.CO, c.CI, c.CIP, c.KP, l};
        s[i++] = SegSpec{g.sb[l] - base, c.ZW, c.CO, P_OFF[2 * l + 1], c.CO, 0, 0, 1, 1, l};
    }
    s[i++] = SegSpec{g.l1w - base, ZL1W, 512L * 9408, P_OFF[12], 512L * 9408, 0, 0, 1, 1, 6};
    s[i++] = SegSpec{g.l1b - base, ZL1W, 512, P_OFF[13], 512, 0, 0, 1, 1, 6};
    s[i++] = SegSpec{g.l2w - base, ZL2W, 256L * 512, P_OFF[14], 256L * 512, 0, 0, 1, 1, 7};
    s[i++] = SegSpec{g.l2b - base, ZL2W, 256, P_OFF[15], 256, 0, 0, 1, 1, 7};
    s[i++] = SegSpec{g.l3w - base, ZH, 2560, P_OFF[16], 2560, 0, 0, 1, 1};
    s[i++] = SegSpec{g.l3b - base, ZH, 10, P_OFF[17], 10, 0, 0, 1, 1};
    return i;
}

static GradState gs_layout(float* base_in) {
    GradState g;
    // offsets only (sizes, plan) when base_in is null: lay out over a fake base, never dereferenced
    float* const base = base_in ? base_in : reinterpret_cast<float*>(4096);
    long o = 0;
    auto take = [&](long n) {
        float* p = base + o;
        o += (n + 63) / 64 * 64;
        return p;
    };
    for (int l = 0; l < 6; ++l) {
        g.wf[l] = l ? nullptr : take((long)GEO[l].CO * GEO[l].KP);
        g.wd[l] = l ? take((long)GEO[l].CI * 9 * GEO[l].CO) : nullptr;
        g.wfx[l] = g.wdx[l] = XsT{nullptr, nullptr};
        if (l) {
            const long nf = (long)GEO[l].CO * GEO[l].KP;
            g.wfx[l].hm = take(nf);
            g.wfx[l].l = take(nf / 2);
        }
    }
    const long slab0 = o;
    g.slab_begin = base + o;
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
    SegSpec specs[STEP_MAX_SEG];
    plan_step(specs, pn1_segments(g, base, specs), &g.plan);
    g.cnt_off = o;
    take(step_counter_floats(g.plan));
    g.slab_floats = o - slab0;
    g.part_off = o;
    take(step_partial_floats(g.plan));
    g.total_floats = o;
    return g;
}

// workspace (per chunk) layout
// (a1 .. gx below are the HM parts of split tensors; a1l .. gxl their L parts, half the size)
struct WS {
    float* x0; float* a1; float* a2; float* d1; float* a3; float* a4; float* d2; float* a5;
    float* a6; float* d3; float* e1; float* e2; float* part; float* dh1; float* dh2;
    float* gx; float* gy; float* loss_s; float* dlog; int32_t* y;
    uint8_t* i1; uint8_t* i2; uint8_t* i3;
    float* a1l; float* d1l; float* a3l; float* d2l; float* a5l;     // forward split tensors
    float* a6l; float* a4l; float* a2l; float* gxl;                  // (unused: dZ is fp32)
    // fp32 copies of the weight gradients' layer inputs (split.h xs_store_f; a1f, d1f, a3f
    // channel-slice-major like their HM parts)
    float* a1f; float* d1f; float* a3f; float* d2f; float* a5f;
    long bytes;
    XsT x(float* hm, float* l) const { return XsT{hm, l}; }
};

// row0 > 0: the same workspace seen from sample row row0 on (every tensor is sample-major,
// [S][...]), so a pass over S' samples at row0 reads and writes rows [row0, row0 + S') of a
// workspace laid out for S samples (the facade's deferred backward, flsim_pn1_fwd_rows)
static WS ws_layout(char* base, int S, int row0 = 0) {
    WS w;
    long o = 0;
    auto take_rows = [&](long per_bytes) {
        char* p = base ? base + o + per_bytes * row0 : nullptr;
        o += (per_bytes * S + 255) / 256 * 256;
        return p;
    };
    auto tf = [&](long per) { return (float*)take_rows(per * 4); };
    w.x0 = tf(4096); w.a1 = tf(55488); w.a2 = tf(62208); w.d1 = tf(15552);
    w.a3 = tf(38400); w.a4 = tf(46464); w.d2 = tf(11616); w.a5 = tf(32448);
    w.a6 = tf(43200); w.d3 = tf(9408); w.e1 = tf(512); w.e2 = tf(256);
    w.part = tf(512L * ZL1F); w.dh1 = tf(512); w.dh2 = tf(256);
    w.gx = tf(55488); w.gy = tf(15552); w.loss_s = tf(1); w.dlog = tf(16);
    w.y = (int32_t*)take_rows(4);
    w.i1 = (uint8_t*)take_rows(15552); w.i2 = (uint8_t*)take_rows(11616);
    w.i3 = (uint8_t*)take_rows(9408);
    w.a1l = tf(55488 / 2); w.d1l = tf(15552 / 2); w.a3l = tf(38400 / 2); w.d2l = tf(11616 / 2);
    w.a5l = tf(32448 / 2);
    w.a6l = tf(0); w.a4l = tf(0); w.a2l = tf(0); w.gxl = tf(0);   // (dZ is fp32: ids kept, no bytes)
    w.a1f = tf(55488); w.d1f = tf(15552); w.a3f = tf(38400); w.d2f = tf(11616); w.a5f = tf(32448);
    w.bytes = o;
    return w;
}

static int pack_weights(const GradState& g, const float* theta, hipStream_t st) {
    RC(pack_conv(theta + P_OFF[0], g.wf[0], nullptr, GEO[0].CO, GEO[0].CI, GEO[0].CIP, GEO[0].KP,
                 st));
    for (int l = 1; l < 6; ++l) {
        const ConvGeo& c = GEO[l];
        RC(pack_conv_xs(theta + P_OFF[2 * l], g.wfx[l], g.wdx[l], c.CO, c.CI, c.KP, st));
        // every data gradient runs on the fp32 MFMA
        hipLaunchKernelGGL(k_pack_dgrad, dim3(ceil_div((long)c.CI * 9 * c.CO, 256)), dim3(256), 0,
                           st, theta + P_OFF[2 * l], g.wd[l], c.CO, c.CI);
        FLSIM_LAUNCH_CHECK();
    }
    return 0;
}

// conv1 + bias + ReLU (models.py:29), direct.  K is only 27 (3 channels x 9 taps), so the GEMM
// pipeline (LDS-staged operands, K padded to 48) spends its time on staging, not on MFMAs, and the
// kernel is bound by writing a1 (S*34*34*48 floats).  Here each wave keeps conv1's weights in
// registers, loads its input pixels straight into MFMA operands and writes a1 through a private
// LDS tile as whole contiguous rows (float4, coalesced).  No block barrier: waves are independent.
//
// 16x16x4 f32 MFMA, lane l: i = l & 15 (output pixel of the row tile / output channel of the
// column tile), g = l >> 4 (k slot).  Taps 0..7 run as two k-steps s of four MFMAs (kk = input
// channel): lane slot g holds tap 4s + g, so one float4 load of x0 (NHWC, channel 3 = 0) feeds the
// four MFMAs.  Tap 8 is one MFMA whose k slot g is the input channel.  27 real MFMA k-values (plus
// the zero 4th channel), 9 MFMAs per 16x16 output tile.
constexpr int C1_ROWS = 32;     // output pixels per wave iteration (two 16-row tiles)
static_assert(C1_ROWS == 32, "the a1 store loop maps 64 lanes to 16 rows x 4 units of a slice");
constexpr int C1_LD = 52;       // staging row stride (floats): 16-B aligned, rows on different banks
__global__ void __launch_bounds__(256)
k_conv1_fwd(const float* __restrict__ x0, const float* __restrict__ W, const float* __restrict__ bias,
            float* __restrict__ a1, float* __restrict__ a1l, float* __restrict__ a1f, long units) {
    __shared__ __attribute__((aligned(16))) float stage[4][C1_ROWS * C1_LD];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    float* st = stage[wv];
    f32x4 wb[3][2];
    float w8[3], bj[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int co = 16 * j + i;
#pragma unroll
        for (int sx = 0; sx < 2; ++sx) {
            const int tap = 4 * sx + g;
            wb[j][sx] = f32x4{W[(co * 3 + 0) * 9 + tap], W[(co * 3 + 1) * 9 + tap],
                              W[(co * 3 + 2) * 9 + tap], 0.f};
        }
        w8[j] = g < 3 ? W[(co * 3 + g) * 9 + 8] : 0.f;
        bj[j] = bias[co];
    }
    // x0 as one buffer (S * 16 KB < 4 GB): 32-bit index math, out-of-range taps read zeros from
    // the hardware's bounds check instead of an exec-masked branch
    BufSrc xb;
    xb.init(x0, (unsigned long)(units * C1_ROWS / 1156) * 4096 * 4);
    auto load = [&](long u, f32x4 (&xa)[2][2], float (&x8)[2]) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const unsigned m = (unsigned)u * C1_ROWS + 16 * t + i;
            const unsigned smp = m / 1156u;
            const int rem = (int)(m - smp * 1156u);
            const int oh = rem / 34, ow = rem - (rem / 34) * 34;
            const unsigned xs = smp * 4096u;
#pragma unroll
            for (int sx = 0; sx < 2; ++sx) {
                const int tap = 4 * sx + g;
                const int ih = oh + tap / 3 - 2, iw = ow + tap % 3 - 2;
                xa[t][sx] = xb.ld_or0((xs + (unsigned)(ih * 32 + iw) * 4u) * 4u,
                                      (unsigned)ih < 32u && (unsigned)iw < 32u);
            }
            x8[t] = (oh < 32 && ow < 32) ? x0[xs + (oh * 32 + ow) * 4 + g] : 0.f;   // tap 8: (ih, iw) = (oh, ow)
        }
    };
    const long nw = (long)gridDim.x * 4;
    long u = (long)blockIdx.x * 4 + wv;
    f32x4 xa[2][2];
    float x8[2];
    if (u < units) load(u, xa, x8);
    for (; u < units; u += nw) {
        f32x4 acc[2][3];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                f32x4 c = zero4();
#pragma unroll
                for (int sx = 0; sx < 2; ++sx)
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) c = mfma16(xa[t][sx][kk], wb[j][sx][kk], c);
                acc[t][j] = mfma16(x8[t], w8[j], c);
            }
        if (u + nw < units) load(u + nw, xa, x8);     // next unit's loads fly during the stores
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(16 * t + 4 * g + r) * C1_LD + 16 * j + i] = fmaxf(acc[t][j][r] + bj[j], 0.f);
        __builtin_amdgcn_wave_barrier();
        // a1 in the split form (split.h), channel-slice-major ([S][3][34*34][16], loaders.h
        // XsSrcSM): each lane splits whole 4-channel units; the 64 lanes of a store take 16 rows of
        // one 16-channel slice, 1 KB of HM (512 B of L) contiguous.  (Two units per lane, their L
        // parts as one 16-B store, measured 2.06 against 1.23 ms: the lanes' HM stores then land
        // 32 B apart, half lines per instruction; profiles/r04/r04l)
#pragma unroll
        for (int q0 = 0; q0 < C1_ROWS * 12; q0 += 64) {
            const int q = q0 + lane, slice = q >> 7, row = (q & 127) >> 2, c4 = 4 * slice + (q & 3);
            xs_store_f(a1, a1l, a1f, xs_unit<48, 1156, true>((unsigned)(u * C1_ROWS + row), c4),
                       *reinterpret_cast<const f32x4*>(st + row * C1_LD + 4 * c4));
        }
        __builtin_amdgcn_wave_barrier();
    }
}

static int conv1_fwd(const float* x0, const float* W, const float* bias, XsT a1, float* a1f,
                     int S, hipStream_t st) {
    const long M = (long)S * 34 * 34;
    if (M % C1_ROWS) return 1;             // S is a multiple of 128 (whole sample groups)
    const long units = M / C1_ROWS;
    // persistent grid of 2048 blocks (1536 / 3072 / 4096 measured the same: 0.978-0.996 ms,
    // profiles/r03i/head_g*.json)
    const int grid = (int)(units / 4 < 2048 ? (units + 3) / 4 : 2048);
    const ProbeSlot ps = probe_begin();
    hipExtLaunchKernelGGL(k_conv1_fwd, dim3(grid), dim3(256), 0, st, ps.start, ps.stop, 0, x0, W,
                          bias, a1.hm, a1.l, a1f, units);
    FLSIM_LAUNCH_CHECK();
    return probe_end(ps, K_FWD1, 2.0 * M * 48 * 27);
}

// The conv2-4 forward GEMMs: split operands on the direct-A kernel (gemm_dx6.h); FM fragments
// of 16 rows per wave (16 FM x WAVES rows per block), B staged DX_KB k-steps at a time.  Chunks of
// at most small_chunk_samples() samples take half-height blocks: the same arithmetic per output
// (bit-identical), twice the blocks.  conv2 (N = 48) runs 64-row waves, 4 per block: 6.67 against
// 7.24 ms for 32-row waves, 8 per block (profiles/r04/r04j/lab_fwd2.txt, "fwd2v e")
// conv3 / conv4 forwards: 64-row waves (FM 4, 512-row blocks) on large chunks, 16-row waves on
// small ones.  FM 4 against round 5's 2: conv4's forward 5.96-5.98 -> 5.72-5.76 ms, the headline
// 1092.4 / 1093.0 -> 1104.8 / 1106.0 worker-steps/s (A B A B, profiles/r06/ab_dx_fm), the same sums
// per output (lab override -DFLSIM_DX_FM)
#ifndef FLSIM_DX_FM
#define FLSIM_DX_FM 4
#endif
constexpr int DX_FM = FLSIM_DX_FM, DX_FMS = 1, DX_KB = 3, DX_DEPTH = 2, DX_NPL = 2;

// (One-call passes, the facade's 128-sample forwards, on quarter-height 64-row blocks: bit-identical
// and 8 % slower on the facade loop, 748 / 746 against 814 / 804 worker-steps/s, E A E A on one box,
// profiles/r06/facade/facade_tiny_ab: more blocks each staging the same B panel.  Not kept.)

template <int IH, int IW, int CI, int PAD, int FN, bool WIN, int OHX, int FM = DX_FM,
          int WAVES = 8, int FMS = (FM == DX_FM ? DX_FMS : FM / 2), class EPI>
static int dx6(XsT X, int S, XsT W, int N, int KP, const EPI& epi, hipStream_t st, int kid,
               int kreal) {
    // the inputs of conv2-4 (a1, d1, a3) are channel-slice-major (XsSrcSM)
    if (S <= small_chunk_samples())
        return conv_dx6<IH, IW, CI, PAD, FMS, FN, WAVES, DX_KB, DX_DEPTH, DX_NPL, WIN, OHX,
                        XsSrcSM>(X, S, W, N, KP, epi, st, kid, kreal);
    return conv_dx6<IH, IW, CI, PAD, FM, FN, WAVES, DX_KB, DX_DEPTH, DX_NPL, WIN, OHX, XsSrcSM>(
        X, S, W, N, KP, epi, st, kid, kreal);
}

// The same GEMMs on gemm_x6_kernel with both operands staged through LDS (conv_xs; bit-identical
// to conv_dx6): WM x WN waves of 16*FM x 16*FN, FM halved for small chunks.  The wide layers
// (N = 192: conv5/6 forward, conv6 data gradient; N = 96 data gradients of conv4/5) run faster
// this way (profiles/r04/lab/lab_xs_r04b.txt: conv6 data gradient 8.8 vs 10.7 ms, forward
// 11.1 vs 12.0)
template <int IH, int IW, int CI, int PAD, int FM, int FN, int WM, int WN, bool WIN, int OHX,
          class EPI>
static int xs(XsT X, int S, XsT W, int N, int KP, const EPI& epi, hipStream_t st, int kid,
              int kreal) {
    if (S <= small_chunk_samples())
        return conv_xs<IH, IW, CI, PAD, FM / 2, FN, WM, WN, WIN, OHX>(X, S, W, N, KP, epi, st, kid,
                                                                     kreal);
    return conv_xs<IH, IW, CI, PAD, FM, FN, WM, WN, WIN, OHX>(X, S, W, N, KP, epi, st, kid, kreal);
}

static int forward(const GradState& g, const WS& w, const float* theta, int S,
                   const WorkerRec* workers, uint64_t seed, int dropout, hipStream_t st) {
    const XsT a1 = w.x(w.a1, w.a1l), d1 = w.x(w.d1, w.d1l), a3 = w.x(w.a3, w.a3l);
    const XsT d2 = w.x(w.d2, w.d2l), a5 = w.x(w.a5, w.a5l);
    // conv1 + ReLU (models.py:29), a1 written split
    RC(conv1_fwd(w.x0, theta + P_OFF[0], theta + P_OFF[1], a1, w.a1f, S, st));
    // conv2 + ReLU + pool1 + dropout1 (models.py:30-32), one fused launch -> d1 (split)
    RC((dx6<34, 34, 48, 2, 3, true, 0, 4, 4, 2>(a1, S, g.wfx[1], 48, 432,
        EpiPoolDropXs<18, 18, 48, true>{d1.hm, d1.l, w.i1, theta + P_OFF[3], workers, seed, SITE_DROP1,
                                  THR_P25, SCALE_P25, dropout, S * 18 * 18 * 4, w.d1f}, st,
        K_FWD2, 432)));
    // conv3 + ReLU (models.py:33) -> a3 (split)
    RC((dx6<18, 18, 48, 2, 6, false, 0>(d1, S, g.wfx[2], 96, 432,
        EpiBiasReluXs<96, true, 400>{a3.hm, a3.l, theta + P_OFF[5], S * 20 * 20, w.a3f}, st, K_FWD3,
        432)));
    // conv4 + ReLU + pool2 + dropout1 (models.py:34-36) -> d2 (split)
    RC((dx6<20, 20, 96, 2, 6, true, 0>(a3, S, g.wfx[3], 96, 864,
        EpiPoolDropXs<11, 11, 96>{d2.hm, d2.l, w.i2, theta + P_OFF[7], workers, seed, SITE_DROP2,
                                  THR_P25, SCALE_P25, dropout, S * 11 * 11 * 4, w.d2f}, st,
        K_FWD4, 864)));
    // conv5 + ReLU (models.py:37) -> a5 (split)
    RC((xs<11, 11, 96, 2, 4, 6, 4, 2, false, 0>(d2, S, g.wfx[4], 192, 864,
        EpiBiasReluXs<192>{a5.hm, a5.l, theta + P_OFF[9], S * 13 * 13, w.a5f}, st, K_FWD5, 864)));
    // conv6 + ReLU + pool3 + dropout1 (models.py:38-40), written fp32 in torch's flatten order
    // (models.py:41) so linear1 keeps the torch weight layout; the floor-mode border row/column
    // of the 15x15 output (dropped by the pool) is never computed
    RC((xs<13, 13, 192, 2, 4, 6, 4, 2, true, 0>(a5, S, g.wfx[5], 192, 1728,
        EpiPoolDrop<7, 7, 192, true>{w.d3, w.i3, theta + P_OFF[11], workers, seed, SITE_DROP3,
                                     THR_P25, SCALE_P25, dropout, S * 7 * 7 * 4}, st, K_FWD6,
        1728)));
    // linear1 + relu + dropout2 (models.py:41-43), split-K partials then finish
    // small chunks (configs[1]: 640 samples = 5 x 4 tiles of 128 x 128, 80 blocks with the split)
    // take 64 x 64 tiles: the same split, hence the same sums, with 4x the blocks
    // (every tile on the split-bf16 kernel: a chunk's losses must not depend on its size, and
    // the two kernels round differently); fresh accumulation (gemm_x6.h x6_step): e1's error
    // reaches linear2's weight gradient, which the truncating MFMA sum left at the SURVEY 8(c)
    // bound
    if (S <= 2048)          // 32 x 64 tiles: 640 blocks at configs[1]'s 640 samples
        RC((linear_fwd<1, 2, 2, 2, true, EpiSlabStoreFresh>(w.d3, theta + P_OFF[12], w.part, S,
                                                            512, 9408, ZL1F, st, K_L1F)));
    else if (S <= 4096)
        RC((linear_fwd<2, 2, 2, 2, true, EpiSlabStoreFresh>(w.d3, theta + P_OFF[12], w.part, S,
                                                            512, 9408, ZL1F, st, K_L1F)));
    else
        RC((linear_fwd<4, 4, 2, 2, true, EpiSlabStoreFresh>(w.d3, theta + P_OFF[12], w.part, S,
                                                            512, 9408, ZL1F, st, K_L1F)));
    RC(linear_finish(w.part, ZL1F, theta + P_OFF[13], w.e1, S, 512, workers, seed, SITE_DROP4,
                     THR_P50, SCALE_P50, dropout, st));
    // linear2 + relu + dropout2 (models.py:44-45)
    RC((linear_fwd<2, 2, 2, 2>(w.e1, theta + P_OFF[14], w.part, S, 256, 512, 1, st, K_L2F)));
    RC(linear_finish(w.part, 1, theta + P_OFF[15], w.e2, S, 256, workers, seed, SITE_DROP5,
                     THR_P50, SCALE_P50, dropout, st));
    return 0;
}

// Slab rows written so far this epoch, per slab group (conv1..6, linear1, linear2), host side.
// begin_epoch does not clear the 1.9 GB of slabs: the weight-gradient GEMMs store into rows not
// yet written this epoch and accumulate into the others (EpiSlabAcc::zinit), and the epoch's
// slab sum reads only the written rows (SlabSeg::zlim).  Small chunks use fewer rows (wsplit), so
// an n = 10 epoch no longer pays a 0.3 ms clear and a full 1.9 GB read.  Keyed by the gradstate
// address; the entry is created by begin_epoch and erased by flsim_pn1_release (engine teardown),
// and a backward pass on a gradstate without one is refused: the slab rows would otherwise be
// read or accumulated without ever having been written.
struct EpochRows {
    int z[8];
};
static std::mutex g_rows_mu;
static std::unordered_map<const void*, EpochRows> g_rows;

static EpochRows* epoch_rows(const void* gradstate) {
    std::lock_guard<std::mutex> lk(g_rows_mu);
    auto it = g_rows.find(gradstate);
    return it == g_rows.end() ? nullptr : &it->second;
}

// Chunk pipelining (flsim_pn1_fwd_bwd_chunk_async): chunk i's forward runs on the caller's stream
// while chunk i-1's backward runs on the gradstate's own backward stream, so the HBM-bound kernels
// (conv1, the batch draw, pool scatter, the head) and every GEMM's last partial round of blocks
// of one pass fill the other's gaps.  Two workspaces alternate: a forward waits for the backward
// that last read its workspace; backwards stay in order on one stream (the slab accumulation
// order is the synchronous path's).  Every other entry point on the gradstate first joins the
// caller's stream to the outstanding backward work (pipe_join), so the packing of the next
// epoch's weights, the slab reduction and the evaluations see a finished epoch.
struct Pipe {
    hipStream_t bs = nullptr;
    hipEvent_t fwd_done = nullptr, bwd_tail = nullptr;
    std::unordered_map<const void*, hipEvent_t> ws_free;   // workspace -> its last backward
    bool pending = false;
};
static std::mutex g_pipe_mu;
static std::unordered_map<const void*, Pipe> g_pipes;

static int pipe_join(const void* gradstate, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    auto it = g_pipes.find(gradstate);
    if (it == g_pipes.end() || !it->second.pending) return 0;
    Pipe& p = it->second;
    FLSIM_CHECK_HIP(hipEventRecord(p.bwd_tail, p.bs));
    FLSIM_CHECK_HIP(hipStreamWaitEvent(st, p.bwd_tail, 0));
    p.pending = false;
    return 0;
}

static void pipe_release(const void* gradstate) {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    auto it = g_pipes.find(gradstate);
    if (it == g_pipes.end()) return;
    Pipe& p = it->second;
    (void)hipStreamSynchronize(p.bs);
    for (auto& kv : p.ws_free) (void)hipEventDestroy(kv.second);
    (void)hipEventDestroy(p.fwd_done);
    (void)hipEventDestroy(p.bwd_tail);
    (void)hipStreamDestroy(p.bs);
    g_pipes.erase(it);
}

// the plan replanned over each tracked segment's rows written this epoch: a small chunk
// (configs[1]: conv1..conv5 write 18-41 % of their Z rows) otherwise leaves most of the units of a
// full-Z plan empty, each still taking part in its tile's partial hand-off.  The replanned units
// and tiles never exceed the full plan's, so the counters and partials laid out for it suffice.
static StepPlan plan_in_use(const GradState& g, const void* gradstate) {
    const EpochRows* er = epoch_rows(gradstate);
    if (!er) return g.plan;
    SegSpec specs[STEP_MAX_SEG];
    const int n = pn1_segments(g, reinterpret_cast<const float*>(gradstate), specs);
    int zin[STEP_MAX_SEG];
    for (int i = 0; i < n; ++i) {
        zin[i] = specs[i].Z;
        if (specs[i].group >= 0) {
            const int z = er->z[specs[i].group];
            zin[i] = z < specs[i].Z ? z : specs[i].Z;
            specs[i].Z = zin[i] > 0 ? zin[i] : 1;
        }
    }
    StepPlan p;
    plan_step(specs, n, &p);
    // plan_step orders the segments by class: match them back by slab offset for zlim
    for (int i = 0; i < p.nseg; ++i)
        for (int j = 0; j < n; ++j)
            if (specs[j].slab_off == p.seg[i].slab_off) p.seg[i].zlim = zin[j];
    return p;
}

// Small chunks run each layer's weight gradient on a second stream beside its data gradient (the
// two read the same dZ and write different outputs): at 640 samples (configs[1]) or a 128-sample
// fwd_bkwd call every GEMM is a few rounds of blocks, and the other one fills the last, partial
// round.  The side stream joins back before a data gradient overwrites a buffer a queued weight
// gradient still reads (gx holds dz5, dz3, dz1 in turn) and at the end of the backward pass.
// One non-blocking side stream and two events per device, created on first use.
// The two events are shared by every backward pass on the device, so a pass holds `mu` from its
// first fork to its last join: two host threads' passes would otherwise record and wait on each
// other's events (a weight gradient could start before its own dZ is written).
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t to_side = nullptr, to_main = nullptr;
    std::mutex* mu = nullptr;
};
static SideStream* side_stream() {
    static std::mutex mu;
    static std::unordered_map<int, SideStream> per_dev;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    SideStream& ss = per_dev[dev];
    if (!ss.s) {
        if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ss.to_side, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ss.to_main, hipEventDisableTiming) != hipSuccess) {
            ss = SideStream{};
            return nullptr;
        }
        ss.mu = new std::mutex();          // lives as long as the process, like the stream
    }
    return &ss;
}
static bool concurrent_backward(int S) {
    static int smax = -1;
    if (smax < 0) {
        // measurement override: the largest chunk (samples) that runs the two streams; 0: off
        const char* e = lab_env("FLSIM_CONCURRENT_BWD");
        smax = e ? atoi(e) : 2048;
    }
    return S <= smax;
}

// fragment rows per wave of the conv4-6 fp32 data gradients on chunks of at most
// small_chunk_samples() samples: 2, the large-chunk tile (configs[1] 984 -> 995 worker-steps/s
// against 1, A B A B, profiles/r05/c1_dg_fms.txt; measurement override -DFLSIM_DG_FMS=<1|2>)
#ifndef FLSIM_DG_FMS
#define FLSIM_DG_FMS 2
#endif
constexpr int DG_FMS = FLSIM_DG_FMS;

// conv2-6 weight gradients on the split-bf16 GEMM (1) or the fp32 one (0); the split form needs
// the flushed accumulation (gemm_x6.h FLSIM_X6_FLUSH) to meet SURVEY 8(c) at the chunk's K
#ifndef FLSIM_WGRAD_X6
#define FLSIM_WGRAD_X6 0
#endif

// debug / measurement: FLSIM_DEBUG_BWD_STOP=6 / 5 / 4 / 3 ends the backward pass after conv6's /
// conv5's / conv4's / conv3's data gradient (dz5 in gx; dz4 in a4, dz5 in gx; dz3 in gx, dz4 in
// a4; dz2 in a2, dz3 in gx; all fp32), so each GEMM can be checked on its own inputs
// (tools/gemm_diag.py, tests/test_gpu_survey_chunk.py); the weight gradients that ran (conv6 ..
// conv<stop>, the linear layers) reach the epoch's slab sum, the others stay zero.  Read per call
// (tests switch it in-process).
static int debug_stop() {
    const char* e = getenv("FLSIM_DEBUG_BWD_STOP");
    return e ? atoi(e) : 0;
}

static int backward(const GradState& g, const WS& w, const float* theta, int S, int dropout,
                    hipStream_t st, EpochRows* er) {
    constexpr int ALL = 0x7fffffff;
    auto zi = [&](int grp) { return er ? er->z[grp] : ALL; };
    int zu[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const float s25 = dropout ? SCALE_P25 : 1.f;
    const float s50 = dropout ? SCALE_P50 : 1.f;
    SideStream* ss = concurrent_backward(S) ? side_stream() : nullptr;
    std::unique_lock<std::mutex> ss_lock;
    if (ss) ss_lock = std::unique_lock<std::mutex>(*ss->mu);   // fork .. last join (SideStream)
    hipStream_t sw = ss ? ss->s : st;              // the weight gradients' stream
    auto fork = [&]() -> int {                     // sw sees everything queued on st so far
        if (!ss) return 0;
        FLSIM_CHECK_HIP(hipEventRecord(ss->to_side, st));
        FLSIM_CHECK_HIP(hipStreamWaitEvent(ss->s, ss->to_side, 0));
        return 0;
    };
    auto join = [&]() -> int {                     // st waits for everything queued on sw
        if (!ss) return 0;
        FLSIM_CHECK_HIP(hipEventRecord(ss->to_main, ss->s));
        FLSIM_CHECK_HIP(hipStreamWaitEvent(st, ss->to_main, 0));
        return 0;
    };
    auto finish = [&]() -> int {                   // the last join; record the slab rows written
        RC(join());
        if (er)
            for (int i = 0; i < 8; ++i)
                if (zu[i] > er->z[i]) er->z[i] = zu[i];
        return 0;
    };
    // ---- linear3 weight/bias (head already produced dlog, dh2) ----
    RC(head_wgrad<256>(w.dlog, w.e2, g.l3w, g.l3b, S, ZH, st));
    // ---- linear2: wgrad, bias, dgrad (-> dh1 through dropout/relu of linear1) ----
    RC(fork());
    RC((linear_wgrad<4, 4, 2, 2>(w.dh2, w.e1, g.l2w, g.l2b, S, 256, 512, ZL2W, sw, K_L2W, zi(7),
                                 &zu[7])));
    RC((linear_dgrad<2, 2, 2, 2>(w.dh2, theta + P_OFF[14], w.dh1, w.e1, s50, S, 256, 512, st,
                                 K_L2D)));
    // ---- linear1: wgrad, bias, dgrad (-> gradient wrt d3 through dropout1 site 3) ----
    RC(fork());
    RC((linear_wgrad<4, 4, 2, 2, true>(w.dh1, w.d3, g.l1w, g.l1b, S, 512, 9408, ZL1W, sw, K_L1W,
                                       zi(6), &zu[6])));
    // (fp32: on the split-bf16 kernel 1.32 vs 1.24 ms, profiles/r03z)
    if (S <= 2048)          // 64 x 128 tiles: twice the blocks of 128 x 128 on a small chunk
        RC((linear_dgrad<2, 4, 2, 2>(w.dh1, theta + P_OFF[12], w.gy, w.d3, s25, S, 512, 9408, st,
                                     K_L1D)));
    else
        RC((linear_dgrad<4, 4, 2, 2>(w.dh1, theta + P_OFF[12], w.gy, w.d3, s25, S, 512, 9408, st,
                                     K_L1D)));
    // ---- pool3 backward -> dz6 (a6 buffer: conv6 fwd no longer writes it), fp32 ----
    // Row/column 14 of conv6's 15x15 output is never pooled (floor mode), so its dz is zero: dz6
    // is stored compact as [S][14][14][192].  The weight gradient then runs over those rows as
    // they stand, and the data gradient reads the missing 15th row/column as zero padding.
    // Every dZ is fp32: the data gradients run on the fp32 MFMA and read each dZ element once per
    // tap (9x), the split-bf16 weight gradients split dZ while staging it (once per block)
    RC((pool_scatter<14, 14, 192, true>(w.gy, w.i3, w.a6, S, st)));
    float* const dz6 = w.a6;
    float* const dz5 = w.gx;
    float* const dz4 = w.a4;
    // ---- conv6: wgrad (input a5), bias, dgrad -> dz5 = . * (a5 > 0) into gx ----
    RC(fork());
    // (192 x 192 tiles of 8 waves ran 9.10-9.13 against 9.41 ms in the lab,
    // profiles/r04/r04l/lab_wg6v.txt, but 9.26-9.29 against 9.10-9.12 in the product, A B A B on
    // one box, profiles/r04/r04s: kept 192 x 96)
#if FLSIM_WGRAD_X6
    RC((conv_wgrad_sz<13, 13, 192, 2, 6, 3, 2, 2, 3, 3, 2, 2, 14, true, true, BufSrc, XsSrc>(
        dz6, w.a5, S, 192, 1728, g.sw[5], g.sb[5], GEO[5].ZW, sw, K_WG6, 1728, zi(5), &zu[5],
        nullptr, w.a5l)));
#else
    RC((conv_wgrad<13, 13, 192, 2, 6, 3, 2, 4, 14, true, false, BufSrc, BufSrc>(
        dz6, w.a5f, S, 192, 1728, g.sw[5], g.sb[5], GEO[5].ZW, sw, K_WG6, 1728, zi(5), &zu[5])));
#endif
    // (every data gradient runs on the fp32 MFMA: the bf16 MFMA truncates small addends toward
    // zero, which biases the per-channel sums of its outputs 30-100x beyond the CPU fp32 port's
    // and failed SURVEY 8(c) on conv1-4, conv6's alone too (tools/gemm_diag.py))
    RC((conv_direct_sz<14, 14, 192, 0, 2, DG_FMS, 6, 8, 6, 2, false, 13>(dz6, S, g.wd[5], 192, 1728,
        EpiMaskXs<192, false>{dz5, nullptr, w.a5, S * 13 * 13}, st, K_DG6, 1728)));
    if (debug_stop() == 6) return finish();       // (debug: dz5 stays in gx)
    // ---- conv5: wgrad (input d2), bias, dgrad -> grad wrt d2 (dropout site 2), scattered through
    //      pool2 straight into dz4 (a4 buffer; no gy round trip) ----
    RC(fork());
#if FLSIM_WGRAD_X6
    RC((conv_wgrad_sz<11, 11, 96, 2, 6, 3, 2, 2, 3, 3, 2, 2, 0, false, true, BufSrc, XsSrc>(
        dz5, w.d2, S, 192, 864, g.sw[4], g.sb[4], GEO[4].ZW, sw, K_WG5, 864, zi(4), &zu[4],
        nullptr, w.d2l)));
#else
    RC((conv_wgrad<11, 11, 96, 2, 6, 3, 2, 2, 0, false, false, BufSrc, BufSrc>(
        dz5, w.d2f, S, 192, 864, g.sw[4], g.sb[4], GEO[4].ZW, sw, K_WG5, 864, zi(4), &zu[4])));
#endif
    RC((conv_direct_sz<13, 13, 192, 0, 2, DG_FMS, 6, 8, 3, 2, false, 0>(dz5, S, g.wd[4], 96, 1728,
        EpiDropScatterXs<11, 11, 96, false>{dz4, nullptr, w.d2, w.i2, s25, S * 11 * 11}, st,
        K_DG5, 1728)));
    if (debug_stop() == 5) return finish();       // (debug: dz4 in a4, dz5 in gx)
    // ---- conv4: wgrad (input a3), bias, dgrad -> dz3 = . * (a3 > 0) into gx (fp32) ----
    // dz3 and dz2 stay fp32: their data gradients have N = 48 columns, where the fp32 MFMA
    // kernels are faster than any split-bf16 form (profiles/r04/lab/lab_xs_r04b.txt: conv3's
    // 3.8 ms fp32 against 4.4 / 4.9 / 5.6 ms for x6 / dx6 / xs), so conv3 / conv2's weight
    // gradients split dZ while staging (split-bf16 kernel over an fp32 dZ and a split layer input)
    RC(join());                                   // conv5's wgrad reads gx = dz5: done first
    RC(fork());
    // (fp32 tiles 96 x 144 of 6 waves: 15.2 against 11.0 ms, profiles/r06/r06r)
#if FLSIM_WGRAD_X6
    RC((conv_wgrad<20, 20, 96, 2, 3, 3, 2, 2, 0, false, true, BufSrc, XsSrcSM>(
        dz4, w.a3, S, 96, 864, g.sw[3], g.sb[3], GEO[3].ZW, sw, K_WG4, 864, zi(3), &zu[3],
        nullptr, w.a3l)));
#else
    RC((conv_wgrad<20, 20, 96, 2, 3, 3, 2, 2, 0, false, false, BufSrc, BufSrcSM>(
        dz4, w.a3f, S, 96, 864, g.sw[3], g.sb[3], GEO[3].ZW, sw, K_WG4, 864, zi(3), &zu[3])));
#endif
    RC((conv_direct_sz<22, 22, 96, 0, 2, DG_FMS, 6, 8, 3, 2, false, 0>(dz4, S, g.wd[3], 96, 864,
        EpiMaskXs<96, false, true, 400>{w.gx, nullptr, w.a3, S * 20 * 20}, st, K_DG4, 864)));
    if (debug_stop() == 4) return finish();       // (debug: dz3 in gx, dz4 in a4)
    float* dz3 = w.gx;
    // ---- conv3: wgrad (input d1), bias, dgrad -> grad wrt d1 (site 1), scattered through pool1
    //      straight into dz2 (a2 buffer, fp32) ----
    RC(fork());
    // (96 x 96 tiles of 4 waves: 2.96 against 3.54 ms for 96 x 48 of 2, profiles/r04/r04j/lab_wg.txt)
#if FLSIM_WGRAD_X6
    RC((conv_wgrad_sz<18, 18, 48, 2, 3, 3, 2, 2, 3, 3, 2, 2, 0, false, true, BufSrc, XsSrcSM>(
        dz3, w.d1, S, 96, 432, g.sw[2], g.sb[2], GEO[2].ZW, sw, K_WG3, 432, zi(2), &zu[2],
        nullptr, w.d1l)));
#else
    RC((conv_wgrad<18, 18, 48, 2, 3, 3, 2, 1, 0, false, false, BufSrc, BufSrcSM>(
        dz3, w.d1f, S, 96, 432, g.sw[2], g.sb[2], GEO[2].ZW, sw, K_WG3, 432, zi(2), &zu[2])));
#endif
    // (gemm_kernel: the direct-A form measured 3.87 vs 3.78 ms with this staged epilogue, r03b)
    // (128 x 48 tiles on large chunks too, FM 2 against 4: 3.68-3.69 against 3.79 ms, the same
    // sums per output, A B A B, profiles/r06/ab_dg3_fm; lab override -DFLSIM_DG3_FM)
#ifndef FLSIM_DG3_FM
#define FLSIM_DG3_FM 2
#endif
    RC((conv_like_sz<20, 20, 96, 0, FLSIM_DG3_FM, 2, 3, 4, 1>(dz3, S, g.wd[2], 48, 864,
        EpiDropScatterXs<18, 18, 48, false, true>{w.a2, nullptr, w.d1, w.i1, s25, S * 18 * 18}, st,
        K_DG3, 864)));
    if (debug_stop() == 3) return finish();       // (debug: dz2 in a2, dz3 in gx)
    float* dz2 = w.a2;
    // ---- conv2: wgrad (input a1), bias, dgrad -> dz1 = . * (a1 > 0) into gx (fp32) ----
    RC(join());                                   // conv3's wgrad reads gx = dz3: done first
    RC(fork());
#if FLSIM_WGRAD_X6
    RC((conv_wgrad_sz<34, 34, 48, 2, 3, 3, 1, 3, 3, 3, 1, 3, 0, false, true, BufSrc, XsSrcSM>(
        dz2, w.a1, S, 48, 432, g.sw[1], g.sb[1], GEO[1].ZW, sw, K_WG2, 432, zi(1), &zu[1],
        nullptr, w.a1l)));
#else
    // (one 48 x 48 wave per block; its tap tiles fetch dZ and the layer input once each, 53 GB
    // per launch, profiles/traffic.json.  Blocks spanning 3 or 9 taps, 48 x 144 of 3 waves /
    // 48 x 432 of 9, ran slower: 9.06 / 14.9 against 8.91 ms, profiles/r06/r06r)
    RC((conv_wgrad<34, 34, 48, 2, 3, 3, 1, 1, 0, false, false, BufSrc, BufSrcSM>(
        dz2, w.a1f, S, 48, 432, g.sw[1], g.sb[1], GEO[1].ZW, sw, K_WG2, 432, zi(1), &zu[1])));
#endif
    RC((conv_direct_sz<36, 36, 48, 0, 2, 1, 3, 8, 3, 2, false, 0>(dz2, S, g.wd[1], 48, 432,
        EpiMaskXs<48, false, true, 1156>{w.gx, nullptr, w.a1, S * 34 * 34}, st, K_DG2, 432)));
    float* dz1 = w.gx;
    // ---- conv1: wgrad (input x0), bias ----
    // (3 waves of 16 rows each: 0.272 vs 0.325 ms for one 48x48 wave, profiles/r01c/lab_conv1.txt;
    // fusing it into conv2's data gradient measured slower: 7.27 ms against 6.14 + 0.87 ms for
    // the two launches, the fused epilogue's registers cost the data gradient a third of its
    // occupancy, profiles/r04/r04n)
    RC((conv_wgrad<32, 32, 4, 2, 1, 3, 3, 1>(dz1, w.x0, S, 48, 48, g.sw[0], g.sb[0], GEO[0].ZW,
                                            st, K_WG1, 27, zi(0), &zu[0])));
    return finish();                              // (the next chunk's forward rewrites a1, a2)
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
                       w.i1, w.i2, w.i3,
                       w.a1l, w.d1l, w.a3l, w.d2l, w.a5l, w.a6l, w.a4l, w.a2l, w.gxl,
                       w.a1f, w.d1f, w.a3f, w.d2f, w.a5f};
    FLSIM_REQUIRE(which >= 0 && which < (int)(sizeof(p) / sizeof(p[0])), "bad workspace id %d", which);
    *offset_bytes = (long)((const char*)p[which] - fake);
    return 0;
}

// a workspace tensor held in the split-bf16 form (split.h): the id of its L part (its HM part is
// `which` itself), or -1 for an fp32 tensor (every dZ: dz6 in a6, dz5 / dz3 / dz1 in gx, dz4 in
// a4, dz2 in a2).
int flsim_pn1_workspace_split_part(int which) {
    switch (which) {
        case 1: return 22;     // a1
        case 3: return 23;     // d1
        case 4: return 24;     // a3
        case 6: return 25;     // d2
        case 7: return 26;     // a5
        default: return -1;
    }
}

int flsim_pn1_workspace_slice_major(int which) {
    return which == 1 || which == 3 || which == 4;    // a1, d1, a3 (XsSrcSM)
}

int flsim_pn1_begin_epoch(void* gradstate, const float* theta, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && theta, "null pointer");
    RC(pipe_join(gradstate, stream));
    GradState g = gs_layout((float*)gradstate);
    RC(pack_weights(g, theta, stream));
    // only the head's slabs (k_head_wgrad accumulates) and the step's tile counters are cleared;
    // the other slabs are overwritten by their first writer this epoch (EpochRows)
    FLSIM_CHECK_HIP(hipMemsetAsync(g.l3w, 0, (g.l3b + ZH * 10 - g.l3w) * 4, stream));
    FLSIM_CHECK_HIP(hipMemsetAsync((float*)gradstate + g.cnt_off, 0,
                                   step_counter_floats(g.plan) * 4, stream));
    std::lock_guard<std::mutex> lk(g_rows_mu);
    g_rows[gradstate] = EpochRows{{0, 0, 0, 0, 0, 0, 0, 0}};
    return 0;
}

// forget the gradstate's slab-row table (the engine that owns the buffer is going away; the
// caching allocator may hand the same address to a new engine)
void flsim_pn1_release(void* gradstate) {
    pipe_release(gradstate);
    std::lock_guard<std::mutex> lk(g_rows_mu);
    g_rows.erase(gradstate);
}

static int run_chunk(void* gradstate, const WS& w, const float* theta, const WorkerRec* workers,
                     int n_chunk_workers, uint64_t seed, int dropout, int backward_pass,
                     float* worker_loss, hipStream_t stream,
                     float gscale = 1.f / SAMPLES_PER_WORKER) {
    const int S = n_chunk_workers * SAMPLES_PER_WORKER;
    GradState g = gs_layout((float*)gradstate);
    RC(forward(g, w, theta, S, workers, seed, dropout, stream));
    // linear3 + CrossEntropyLoss (models.py:46, main.py:107); dropout2 precedes linear3
    RC(head_and_loss<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, w.dlog, w.dh2,
                          S, backward_pass, dropout ? SCALE_P50 : 1.f, gscale, worker_loss,
                          stream, workers));
    if (backward_pass) {
        EpochRows* er = epoch_rows(gradstate);
        FLSIM_REQUIRE(er, "backward pass without flsim_pn1_begin_epoch on this gradstate");
        RC(backward(g, w, theta, S, dropout, stream, er));
    }
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
    RC(pipe_join(gradstate, stream));
    WS w = ws_layout((char*)workspace, max_samples);
    hipLaunchKernelGGL(k_fill_batch, dim3(S), dim3(256), 0, stream, pool, labels, list_a, len_a,
                       list_b, len_b, workers, n_workers_total, seed, lut, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    return run_chunk(gradstate, w, theta, workers, n_chunk_workers, seed, dropout, backward_pass,
                     worker_loss, stream);
}

// the same chunk, pipelined: fill + forward + head on `stream`, the backward on the gradstate's
// backward stream after this forward and after the previous chunk's backward; `workspace` must
// not be the one the previous call used (alternate two).  Losses are ordered on `stream`; the
// gradients are complete for any later entry point on the gradstate (pipe_join).
}  // extern "C"

// one pipelined pass: `front` (batch fill, forward, loss) on `stream`, then the backward on the
// gradstate's backward stream; a forward waits for the backward that last read its workspace
// (g_pipe_mu held) the gradstate's pipe, its stream and events created on first use
static int pipe_of(void* gradstate, Pipe** out) {
    Pipe& p = g_pipes[gradstate];
    if (!p.bs) {
        // the lowest priority: the caller's forwards (the facade's per-call forward, whose loss
        // the caller waits for) get the CUs first as the backward's blocks retire
        int least = 0, greatest = 0;
        FLSIM_CHECK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        FLSIM_CHECK_HIP(hipStreamCreateWithPriority(&p.bs, hipStreamNonBlocking, least));
        FLSIM_CHECK_HIP(hipEventCreateWithFlags(&p.fwd_done, hipEventDisableTiming));
        FLSIM_CHECK_HIP(hipEventCreateWithFlags(&p.bwd_tail, hipEventDisableTiming));
    }
    *out = &p;
    return 0;
}

// (g_pipe_mu held) the backward of workspace rows [0, S) on the gradstate's backward stream,
// after everything queued on `stream` so far; the workspace's event marks its end
static int queue_backward(void* gradstate, Pipe& p, hipEvent_t& ws_ev, void* workspace,
                          int max_samples, const float* theta, int S, int dropout,
                          hipStream_t stream, EpochRows* er) {
    WS w = ws_layout((char*)workspace, max_samples);
    GradState g = gs_layout((float*)gradstate);
    FLSIM_CHECK_HIP(hipEventRecord(p.fwd_done, stream));
    FLSIM_CHECK_HIP(hipStreamWaitEvent(p.bs, p.fwd_done, 0));
    RC(backward(g, w, theta, S, dropout, p.bs, er));
    FLSIM_CHECK_HIP(hipEventRecord(ws_ev, p.bs));
    p.pending = true;
    return 0;
}

template <class Front>
static int run_pipelined(void* gradstate, void* workspace, int max_samples, const float* theta,
                         int S, int dropout, hipStream_t stream, Front&& front) {
    EpochRows* er = epoch_rows(gradstate);
    FLSIM_REQUIRE(er, "backward pass without flsim_pn1_begin_epoch on this gradstate");
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    Pipe* p = nullptr;
    RC(pipe_of(gradstate, &p));
    hipEvent_t& ws_ev = p->ws_free[workspace];
    if (!ws_ev) FLSIM_CHECK_HIP(hipEventCreateWithFlags(&ws_ev, hipEventDisableTiming));
    else FLSIM_CHECK_HIP(hipStreamWaitEvent(stream, ws_ev, 0));   // its last backward is done
    WS w = ws_layout((char*)workspace, max_samples);
    GradState g = gs_layout((float*)gradstate);
    RC(front(g, w));
    return queue_backward(gradstate, *p, ws_ev, workspace, max_samples, theta, S, dropout, stream,
                          er);
}

// rows a queued backward still reads are not overwritten: `stream` waits for the last backward
// that read this workspace
static int wait_workspace(void* gradstate, void* workspace, hipStream_t stream) {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    auto it = g_pipes.find(gradstate);
    if (it != g_pipes.end()) {
        auto e = it->second.ws_free.find(workspace);
        if (e != it->second.ws_free.end() && e->second)
            FLSIM_CHECK_HIP(hipStreamWaitEvent(stream, e->second, 0));
    }
    return 0;
}

extern "C" {

int flsim_pn1_fwd_bwd_chunk_async(void* gradstate, void* workspace, int max_samples,
                                  const float* theta, const uint8_t* pool, const int32_t* labels,
                                  const int32_t* list_a, int len_a, const int32_t* list_b,
                                  int len_b, const float* lut, const WorkerRec* workers,
                                  int n_chunk_workers, int n_workers_total, uint64_t seed,
                                  int dropout, float* worker_loss, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && pool && labels && list_a && list_b && lut &&
                  workers && worker_loss, "null pointer");
    FLSIM_REQUIRE(n_chunk_workers > 0, "empty chunk");
    const int S = n_chunk_workers * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE(S <= max_samples, "chunk of %d samples exceeds workspace (%d)", S, max_samples);
    FLSIM_REQUIRE(S <= 16384, "chunk of %d samples exceeds the 32-bit index budget", S);
    FLSIM_REQUIRE(len_a > 0 && len_b > 0, "empty class list");
    return run_pipelined(gradstate, workspace, max_samples, theta, S, dropout, stream,
                         [&](const GradState& g, const WS& w) -> int {
        hipLaunchKernelGGL(k_fill_batch, dim3(S), dim3(256), 0, stream, pool, labels, list_a,
                           len_a, list_b, len_b, workers, n_workers_total, seed, lut, w.x0, w.y);
        FLSIM_LAUNCH_CHECK();
        RC(forward(g, w, theta, S, workers, seed, dropout, stream));
        return head_and_loss<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s,
                                  w.dlog, w.dh2, S, 1, dropout ? SCALE_P50 : 1.f,
                                  1.f / SAMPLES_PER_WORKER, worker_loss, stream, workers);
    });
}

// the explicit-batch form pipelined (the Worker.fwd_bkwd facade): the call's loss is ready on
// `stream` after its forward; its backward overlaps the next call's forward
int flsim_pn1_fwd_bwd_input_async(void* gradstate, void* workspace, int max_samples,
                                  const float* theta, const float* x, const int64_t* y,
                                  int n_samples, const WorkerRec* workers, uint64_t seed,
                                  int dropout, float* worker_loss, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && x && y && workers && worker_loss,
                  "null pointer");
    FLSIM_REQUIRE(n_samples > 0, "empty batch");
    const int S = ceil_div(n_samples, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE(S <= max_samples, "batch of %d samples exceeds workspace (%d)", n_samples,
                  max_samples);
    FLSIM_REQUIRE(S <= 16384, "batch of %d samples exceeds the 32-bit index budget", n_samples);
    return run_pipelined(gradstate, workspace, max_samples, theta, S, dropout, stream,
                         [&](const GradState& g, const WS& w) -> int {
        hipLaunchKernelGGL(k_load_input, dim3(S), dim3(256), 0, stream, x, y, n_samples, w.x0,
                           w.y);
        FLSIM_LAUNCH_CHECK();
        RC(forward(g, w, theta, S, workers, seed, dropout, stream));
        return head_and_loss<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s,
                                  w.dlog, w.dh2, S, 1, dropout ? SCALE_P50 : 1.f,
                                  1.f / (float)n_samples, worker_loss, stream, workers);
    });
}

// The facade's deferred backward (Worker.fwd_bkwd, agents.py:32-40, with the backward of up to a
// chunk of calls batched into one pass): every fwd_bkwd call of an epoch runs on the same theta_t
// (main.py:154,159,169), so each call's forward + loss runs alone -- the loss is all the call
// must return now (agents.py:40) -- into workspace rows [row0, row0 + S) (ws_layout's row view),
// and one backward over rows [0, n_rows) later adds the whole chunk's gradient to the slabs, at
// the batched engine's rates.  The forward kernels are the per-call facade's (bit-identical
// losses); the backward is FLSimulation's over the same rows.
int flsim_pn1_fwd_rows(void* gradstate, void* workspace, int max_samples, int row0,
                       const float* theta, const float* x, const int64_t* y, int n_samples,
                       const WorkerRec* workers, uint64_t seed, int dropout, float* worker_loss,
                       hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && x && y && workers && worker_loss,
                  "null pointer");
    FLSIM_REQUIRE(n_samples > 0, "empty batch");
    FLSIM_REQUIRE(row0 >= 0 && row0 % SAMPLES_PER_WORKER == 0,
                  "row0 %d is not a multiple of %d", row0, SAMPLES_PER_WORKER);
    const int S = ceil_div(n_samples, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE((long)row0 + S <= max_samples, "rows [%d, %d) exceed workspace (%d)", row0,
                  row0 + S, max_samples);
    FLSIM_REQUIRE(max_samples <= 16384, "workspace of %d samples exceeds the 32-bit index budget",
                  max_samples);
    FLSIM_REQUIRE(epoch_rows(gradstate), "forward rows without flsim_pn1_begin_epoch");
    RC(wait_workspace(gradstate, workspace, stream));
    WS w = ws_layout((char*)workspace, max_samples, row0);
    GradState g = gs_layout((float*)gradstate);
    hipLaunchKernelGGL(k_load_input, dim3(S), dim3(256), 0, stream, x, y, n_samples, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    RC(forward(g, w, theta, S, workers, seed, dropout, stream));
    return head_and_loss<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, w.dlog,
                              w.dh2, S, 1, dropout ? SCALE_P50 : 1.f, 1.f / (float)n_samples,
                              worker_loss, stream, workers);
}

// The facade's deferred forward (Worker.fwd_bkwd of 128-sample batches): a call only stages its
// batch into workspace rows [row0, row0 + 128) now (flsim_pn1_load_rows); the forward + loss of a
// run of staged rows then runs as ONE worker-batched pass (flsim_pn1_fwd_loaded_rows), when a
// loss is read or the chunk's backward is due.  The kernels are the batched engine's: the same
// sums per output as the one-call forward of flsim_pn1_fwd_rows (the tiles' K order does not
// depend on the row count, linear1's split-K is fixed), so the losses are bit-identical.
int flsim_pn1_load_rows(void* gradstate, void* workspace, int max_samples, int row0,
                        const float* x, const int64_t* y, int n_samples, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && x && y, "null pointer");
    FLSIM_REQUIRE(n_samples > 0, "empty batch");
    FLSIM_REQUIRE(row0 >= 0 && row0 % SAMPLES_PER_WORKER == 0,
                  "row0 %d is not a multiple of %d", row0, SAMPLES_PER_WORKER);
    const int S = ceil_div(n_samples, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE((long)row0 + S <= max_samples, "rows [%d, %d) exceed workspace (%d)", row0,
                  row0 + S, max_samples);
    FLSIM_REQUIRE(max_samples <= 16384, "workspace of %d samples exceeds the 32-bit index budget",
                  max_samples);
    RC(wait_workspace(gradstate, workspace, stream));
    WS w = ws_layout((char*)workspace, max_samples, row0);
    hipLaunchKernelGGL(k_load_input, dim3(S), dim3(256), 0, stream, x, y, n_samples, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    return 0;
}

// forward + CrossEntropyLoss of rows [row0, row0 + n_rows) staged by flsim_pn1_load_rows, every
// 128-row group one full batch: workers[n_rows / 128] the groups' dropout keys, worker_loss[g] =
// group g's mean loss (agents.py:40's lossval of that call)
int flsim_pn1_fwd_loaded_rows(void* gradstate, void* workspace, int max_samples, int row0,
                              int n_rows, const float* theta, const WorkerRec* workers,
                              uint64_t seed, int dropout, float* worker_loss, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && workers && worker_loss, "null pointer");
    FLSIM_REQUIRE(row0 >= 0 && row0 % SAMPLES_PER_WORKER == 0 && n_rows > 0 &&
                  n_rows % SAMPLES_PER_WORKER == 0, "bad rows [%d, +%d)", row0, n_rows);
    FLSIM_REQUIRE((long)row0 + n_rows <= max_samples, "rows [%d, %d) exceed workspace (%d)", row0,
                  row0 + n_rows, max_samples);
    FLSIM_REQUIRE(max_samples <= 16384, "workspace of %d samples exceeds the 32-bit index budget",
                  max_samples);
    FLSIM_REQUIRE(epoch_rows(gradstate), "forward rows without flsim_pn1_begin_epoch");
    RC(wait_workspace(gradstate, workspace, stream));
    WS w = ws_layout((char*)workspace, max_samples, row0);
    GradState g = gs_layout((float*)gradstate);
    RC(forward(g, w, theta, n_rows, workers, seed, dropout, stream));
    return head_and_loss<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, w.dlog,
                              w.dh2, n_rows, 1, dropout ? SCALE_P50 : 1.f,
                              1.f / SAMPLES_PER_WORKER, worker_loss, stream, workers);
}

// the backward of rows [0, n_rows) written by flsim_pn1_fwd_rows with this theta and dropout
// flag, on the gradstate's backward stream after everything queued on `stream` (so the next
// chunk's forwards -- into another workspace -- overlap it); every other entry point on the
// gradstate joins it first (pipe_join)
int flsim_pn1_bwd_rows(void* gradstate, void* workspace, int max_samples, int n_rows,
                       const float* theta, int dropout, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta, "null pointer");
    FLSIM_REQUIRE(n_rows > 0 && n_rows % SAMPLES_PER_WORKER == 0 && n_rows <= max_samples &&
                  n_rows <= 16384, "bad row count %d (workspace %d)", n_rows, max_samples);
    EpochRows* er = epoch_rows(gradstate);
    FLSIM_REQUIRE(er, "backward pass without flsim_pn1_begin_epoch on this gradstate");
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    Pipe* p = nullptr;
    RC(pipe_of(gradstate, &p));
    hipEvent_t& ws_ev = p->ws_free[workspace];
    if (!ws_ev) FLSIM_CHECK_HIP(hipEventCreateWithFlags(&ws_ev, hipEventDisableTiming));
    return queue_backward(gradstate, *p, ws_ev, workspace, max_samples, theta, n_rows, dropout,
                          stream, er);
}

// explicit batch (the Worker.fwd_bkwd(inp, outp) facade, agents.py:32-35): x NCHW fp32, y int64,
// any n_samples (main.py:43-44 --batch_size); the batch is padded to whole 128-sample groups
// (padding has zero loss and gradient) and the CE gradient is the mean over the n samples.
// workers[ceil(n/128)] give each group's dropout key; worker_loss[g] = group g's loss sum / 128.
int flsim_pn1_fwd_bwd_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                            const float* x, const int64_t* y, int n_samples,
                            const WorkerRec* workers, uint64_t seed, int dropout,
                            int backward_pass, float* worker_loss, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && x && y && workers && worker_loss,
                  "null pointer");
    FLSIM_REQUIRE(n_samples > 0, "empty batch");
    const int S = ceil_div(n_samples, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
    FLSIM_REQUIRE(S <= max_samples, "batch of %d samples exceeds workspace (%d)", n_samples,
                  max_samples);
    FLSIM_REQUIRE(S <= 16384, "batch of %d samples exceeds the 32-bit index budget", n_samples);
    RC(pipe_join(gradstate, stream));
    WS w = ws_layout((char*)workspace, max_samples);
    hipLaunchKernelGGL(k_load_input, dim3(S), dim3(256), 0, stream, x, y, n_samples, w.x0, w.y);
    FLSIM_LAUNCH_CHECK();
    return run_chunk(gradstate, w, theta, workers, S / SAMPLES_PER_WORKER, seed, dropout,
                     backward_pass, worker_loss, stream, 1.f / (float)n_samples);
}

// Evaluation of an explicit batch (util.py:31-45: model(images) after central.model.eval(),
// main.py:190): x NCHW fp32 [n][3][32][32] -> argmax predictions pred[n].  Re-packs theta.
int flsim_pn1_eval_input(void* gradstate, void* workspace, int max_samples, const float* theta,
                         const float* x, int n_images, int32_t* pred, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && workspace && theta && x && pred, "null pointer");
    FLSIM_REQUIRE(n_images > 0, "empty batch");
    FLSIM_REQUIRE(max_samples >= SAMPLES_PER_WORKER && max_samples % SAMPLES_PER_WORKER == 0,
                  "max_samples must be a positive multiple of %d", SAMPLES_PER_WORKER);
    GradState g = gs_layout((float*)gradstate);
    RC(pipe_join(gradstate, stream));
    WS w = ws_layout((char*)workspace, max_samples);
    RC(pack_weights(g, theta, stream));
    const int cap = max_samples < 16384 ? max_samples : 16384;
    for (int c0 = 0; c0 < n_images; c0 += cap) {
        const int n = n_images - c0 < cap ? n_images - c0 : cap;
        const int S = ceil_div(n, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
        hipLaunchKernelGGL(k_load_input, dim3(S), dim3(256), 0, stream, x + (long)c0 * 3072,
                           (const int64_t*)nullptr, n, w.x0, w.y);
        FLSIM_LAUNCH_CHECK();
        RC(forward(g, w, theta, S, nullptr, 0, 0, stream));
        RC(head_predict<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, S,
                             pred + c0, n, stream));
    }
    return 0;
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
    RC(pipe_join(gradstate, stream));
    WS w = ws_layout((char*)workspace, max_samples);
    RC(pack_weights(g, theta, stream));
    const int cap = max_samples < 16384 ? max_samples : 16384;   // 32-bit index budget
    for (int c0 = 0; c0 < n_images; c0 += cap) {
        const int n = n_images - c0 < cap ? n_images - c0 : cap;
        const int S = ceil_div(n, SAMPLES_PER_WORKER) * SAMPLES_PER_WORKER;
        hipLaunchKernelGGL(k_fill_seq, dim3(S), dim3(256), 0, stream, pool, first + c0, n, lut,
                           w.x0, w.y);
        FLSIM_LAUNCH_CHECK();
        RC(forward(g, w, theta, S, nullptr, 0, 0, stream));
        RC(head_predict<256>(w.e2, theta + P_OFF[16], theta + P_OFF[17], w.y, w.loss_s, S,
                             pred + c0, n, stream));
    }
    return 0;
}

// S_t (torch named_parameters layout, P floats) = sum of the epoch's slabs (fixed order)
int flsim_pn1_end_epoch(void* gradstate, float* grad_out, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && grad_out, "null pointer");
    RC(pipe_join(gradstate, stream));
    GradState g = gs_layout((float*)gradstate);
    return slab_step_launch((float*)gradstate, plan_in_use(g, gradstate), g.cnt_off, g.part_off,
                            grad_out, nullptr, nullptr, nullptr, nullptr, nullptr, P_TOTAL, stream);
}

// the same reduction fused with rule() + Adam (world = 1)
int flsim_pn1_server_step(void* gradstate, float* S_out, const flsim_rule* rule, float* p,
                          float* m, float* v, long step, double lr, double beta1, double beta2,
                          double eps, hipStream_t stream) {
    FLSIM_REQUIRE(gradstate && rule && p && m && v, "null pointer");
    RC(pipe_join(gradstate, stream));
    GradState g = gs_layout((float*)gradstate);
    RuleProg R;
    RC(make_rule(rule, &R));
    AdamConst ac;
    RC(make_adam_const(rule->k, step, lr, beta1, beta2, eps, &ac));
    return slab_step_launch((float*)gradstate, plan_in_use(g, gradstate), g.cnt_off, g.part_off,
                            S_out, &R, &ac, p, m, v, P_TOTAL, stream);
}

}  // extern "C"
