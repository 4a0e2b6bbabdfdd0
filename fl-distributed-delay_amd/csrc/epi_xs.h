// GEMM epilogues that write their output in the split-bf16 form (split.h) and / or read their
// ReLU / dropout mask operand from a split tensor, for the PerformantNet1 passes whose outputs feed
// split-bf16 GEMMs.  All of them are staged through LDS (gemm_core.h STAGED): the
// block's accumulator tile goes to LDS, and each thread then takes whole 4-channel units of a row,
// so every output unit is split once, by one thread, and leaves as one 16-B HM store and one 8-B L
// store.  PARTIAL epilogues accept a tile narrower than the output row (columns [n0, n0 + bn)).
#pragma once
#include "loaders.h"
#include "split.h"

namespace flsim {

// a unit of 4 values of a split tensor as an fp32 > 0 mask (h > 0, split.h xs_pos4)
__device__ __forceinline__ f32x4 mask4(f32x4 t, uint32_t pos) {
    return f32x4{(pos & 1) ? t.x : 0.f, (pos & 2) ? t.y : 0.f, (pos & 4) ? t.z : 0.f,
                 (pos & 8) ? t.w : 0.f};
}

// In-LDS ReLU mask of a staged tile (rows [m0, m0 + rows), units [n0 / 4, n0 / 4 + n4) of NC
// channels) from a channel-slice-major split act (split.h xs_unit): threads walk the tile slice by
// slice, rows fastest, so their act reads are contiguous in the slice-major layout.  Ends with a
// block barrier (every thread of the block calls it: staged epilogues run block-wide).
template <int NC, int AHW>
__device__ __forceinline__ void mask_tile_sm(float* tile, int ld, const float* act, int m0, int rows,
                                             int n0, int n4, int tid, int nt) {
    // (no runtime division and no batched loads: this runs in the GEMM kernels' epilogues, whose
    // register peak sets their occupancy; r04zb measured a batched form at 104 against 80 VGPRs)
    const f32x2* a2 = reinterpret_cast<const f32x2*>(act);
    for (int s = 0; 4 * s < n4; ++s) {
        for (int q = tid; q < rows * 4; q += nt) {
            const int r = q >> 2, c = 4 * s + (q & 3);
            const f32x2 a = a2[2 * xs_unit<NC, AHW, true>((unsigned)(m0 + r), n0 / 4 + c)];
            f32x4* t = reinterpret_cast<f32x4*>(tile + r * ld + 4 * c);
            *t = mask4(*t, xs_pos4(a));
        }
    }
    __syncthreads();
}

// conv forward: Y = relu(acc + bias) over NC channels, written split (conv3 -> a3, conv5 -> a5);
// SM: Y channel-slice-major over HW pixels per image (split.h xs_unit)
template <int NC, bool SM = false, int HW = 1>
struct EpiBiasReluXs {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr bool PARTIAL = true;
    static constexpr int NCOL = NC;
    float* Yhm;
    float* Yl;
    const float* bias;
    int M;
    float* Yf = nullptr;   // fp32 copy, same layout (split.h xs_store_f), or none
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int n0, int bn, int tid,
                               int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        const int n4 = bn / 4;
        for (int q = tid; q < rows * n4; q += nt) {
            const int r = q / n4, c = q - r * n4;
            const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
            const f32x4 b = *reinterpret_cast<const f32x4*>(bias + n0 + 4 * c);
            const f32x4 v = {fmaxf(t.x + b.x, 0.f), fmaxf(t.y + b.y, 0.f), fmaxf(t.z + b.z, 0.f),
                             fmaxf(t.w + b.w, 0.f)};
            xs_store_f(Yhm, Yl, Yf, xs_unit<NC, HW, SM>((unsigned)(m0 + r), n0 / 4 + c), v);
        }
    }
};

// data gradient through a ReLU: Y = acc * (act > 0), act split; Y split (OUT_XS: dz5, dz3) or
// fp32 (dz1, read by conv1's fp32 weight gradient); ASM: act channel-slice-major over AHW pixels
// per image (Y stays pixel-major)
template <int NC, bool OUT_XS, bool ASM = false, int AHW = 1>
struct EpiMaskXs {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr bool PARTIAL = true;
    static constexpr int NCOL = NC;
    float* Y;          // HM part (OUT_XS) or the fp32 output
    float* Yl;         // L part (OUT_XS)
    const float* act;  // HM part of the mask operand
    int M;
    static constexpr int BATCH = 8;
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int n0, int bn, int tid,
                               int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        const int n4 = bn / 4;
        const int total = rows * n4;
        if constexpr (ASM) {
            static_assert(NC % 16 == 0, "");
            // slice-major act: mask in LDS (act reads in its order), then store in row order
            mask_tile_sm<NC, AHW>(const_cast<float*>(tile), ld, act, m0, rows, n0, n4, tid, nt);
            for (int q = tid; q < total; q += nt) {
                const int r = q / n4, c = q - r * n4;
                const f32x4 o = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
                const long u = ((long)(m0 + r) * NC + n0) / 4 + c;
                if constexpr (OUT_XS)
                    xs_store(Y, Yl, u, o);
                else
                    st_nt4(Y + 4 * u, o);
            }
            return;
        }
        auto unit = [&](int q, f32x2 a) {
            const int r = q / n4, c = q - r * n4;
            const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
            const f32x4 o = mask4(t, xs_pos4(a));
            const long u = ((long)(m0 + r) * NC + n0) / 4 + c;
            if constexpr (OUT_XS)
                xs_store(Y, Yl, u, o);
            else
                st_nt4(Y + 4 * u, o);
        };
        // the mask units (their h parts) of a thread's first BATCH units are loaded before any is
        // used (one round trip; EpiMaskRows)
        auto mask_of = [&](int q) {
            const int r = q / n4, c = q - r * n4;
            return reinterpret_cast<const f32x2*>(act)[2 * (((long)(m0 + r) * NC + n0) / 4 + c)];
        };
        f32x2 av[BATCH];
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) av[it] = mask_of(q);
        }
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) unit(q, av[it]);
        }
        for (int q = tid + BATCH * nt; q < total; q += nt) unit(q, mask_of(q));
    }
};

// EpiDropScatterRows (loaders.h) over split tensors: the masked, scaled gradient of pooled element
// (m, n) goes to its argmax position of the 2x2 window in the full-resolution dZ, zeros elsewhere;
// act (the pooled, dropped activation) is split, dZ is written split (OUT_XS) or fp32.  Full rows
// (BN == NC).  ASM: act channel-slice-major (split.h xs_unit).
template <int PH, int PW, int NC, bool OUT_XS = true, bool ASM = false>
struct EpiDropScatterXs {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr int NCOL = NC;
    static_assert(NC % 4 == 0, "float4 rows");
    float* dZhm;          // HM part (OUT_XS) or the fp32 dZ
    float* dZl;           // L part (OUT_XS)
    const float* act;     // HM part
    const uint8_t* idx;
    float scale;
    int M;
    static constexpr int BATCH = 8;
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int N4 = NC / 4;
        if constexpr (ASM)      // slice-major act: masked in LDS first, then every unit passes
            mask_tile_sm<NC, PH * PW>(const_cast<float*>(tile), ld, act, m0, rows, 0, N4, tid, nt);
        const f32x2* a2 = reinterpret_cast<const f32x2*>(act) + 2 * (long)m0 * N4;   // h parts
        auto act_h = [&](int q) -> f32x2 {
            if constexpr (ASM)
                return __builtin_bit_cast(f32x2, u32x2{0x3f803f80u, 0x3f803f80u});   // h = 1: pass
            else
                return a2[2 * q];
        };
        const uint32_t* i4 = reinterpret_cast<const uint32_t*>(idx + (long)m0 * NC);
        const int total = rows * N4;
        f32x2 av[BATCH];
        uint32_t iv[BATCH];
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) {
                av[it] = act_h(q);
                iv[it] = i4[q];
            }
        }
#pragma unroll
        for (int it = 0; it < BATCH; ++it) {
            const int q = tid + it * nt;
            if (q < total) unit(tile, ld, m0, q, av[it], iv[it]);
        }
        for (int q = tid + BATCH * nt; q < total; q += nt) unit(tile, ld, m0, q, act_h(q), i4[q]);
    }
    __device__ void unit(const float* tile, int ld, int m0, int q, f32x2 a, uint32_t id) const {
        constexpr int N4 = NC / 4;
        const int r = q / N4, c = q - r * N4;
        const f32x4 t = *reinterpret_cast<const f32x4*>(tile + r * ld + 4 * c);
        const f32x4 g = mask4(f32x4{t.x * scale, t.y * scale, t.z * scale, t.w * scale},
                              xs_pos4(a));
        const unsigned mm = (unsigned)(m0 + r);
        const unsigned img = mm / (PH * PW);
        const unsigned rem = mm - img * (PH * PW);
        const unsigned ph = rem / PW, pw = rem - ph * PW;
        const long u0 = ((((long)img * (2 * PH) + 2 * ph) * (2 * PW) + 2 * pw) * NC) / 4 + c;
#pragma unroll
        for (int pos = 0; pos < 4; ++pos) {
            f32x4 o;
            o.x = (id & 0xffu) == (uint32_t)pos ? g.x : 0.f;
            o.y = ((id >> 8) & 0xffu) == (uint32_t)pos ? g.y : 0.f;
            o.z = ((id >> 16) & 0xffu) == (uint32_t)pos ? g.z : 0.f;
            o.w = (id >> 24) == (uint32_t)pos ? g.w : 0.f;
            const long u = u0 + ((pos >> 1) * (2 * PW) + (pos & 1)) * (long)N4;
            if constexpr (OUT_XS)
                xs_store(dZhm, dZl, u, o);
            else
                st_nt4(dZhm + 4 * u, o);
        }
    }
};

// conv forward + bias + ReLU + 2x2 max-pool + dropout (EpiPoolDrop, loaders.h) staged through LDS
// and written split (NHWC: conv2 -> d1, conv4 -> d2).  Tile rows are in pool-window order
// (Im2colKC / Im2colDirect WIN), so rows 4p .. 4p + 3 of the tile are pooled pixel p's window; a
// thread takes (pooled pixel, 4 channels): the same per-element max / first-argmax / dropout as
// EpiPoolDrop, one split unit of d and one 4-byte argmax word.  Full rows (BN == C).  SM: d
// channel-slice-major (split.h xs_unit; the argmax words stay pixel-major).
template <int PH, int PW, int C, bool SM = false>
struct EpiPoolDropXs {
    static constexpr bool ASUM = false;
    static constexpr bool STAGED = true;
    static constexpr int NCOL = C;
    float* dhm;
    float* dl;
    uint8_t* idx;
    const float* bias;
    const WorkerRec* workers;
    uint64_t seed;
    uint32_t site, thr;
    float scale;
    int dropout;
    int M;
    float* df = nullptr;   // fp32 copy of d, same layout (split.h xs_store_f), or none
    __device__ float value(int, float v) const { return v; }
    __device__ void store_rows(const float* tile, int ld, int m0, int bm, int tid, int nt) const {
        const int rows = M - m0 < bm ? M - m0 : bm;
        constexpr int C4 = C / 4;
        const int total = rows / 4 * C4;
        for (int u = tid; u < total; u += nt) {
            const int pl = u / C4, c = u - pl * C4;        // local pooled pixel, channel unit
            const f32x4 b = *reinterpret_cast<const f32x4*>(bias + 4 * c);
            f32x4 x[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f32x4 t = *reinterpret_cast<const f32x4*>(tile + (4 * pl + r) * ld + 4 * c);
                x[r] = f32x4{fmaxf(t.x + b.x, 0.f), fmaxf(t.y + b.y, 0.f), fmaxf(t.z + b.z, 0.f),
                             fmaxf(t.w + b.w, 0.f)};
            }
            const int q = (m0 >> 2) + pl;                 // pooled pixel (s, ph, pw)
            const int pw = q % PW;
            const int ph = (q / PW) % PH;
            const int s = q / (PW * PH);
            f32x4 out;
            uint32_t id = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float mv = x[0][e];
                int mi = 0;
#pragma unroll
                for (int r = 1; r < 4; ++r)
                    if (x[r][e] > mv) { mv = x[r][e]; mi = r; }
                float o = mv;
                if (dropout) {
                    const int w = s / SAMPLES_PER_WORKER;
                    const int nl = s - w * SAMPLES_PER_WORKER;
                    const WorkerRec wr = workers[w];
                    const uint32_t en = (uint32_t)(((nl * C + 4 * c + e) * PH + ph) * PW + pw);
                    o = philox_word(seed, wr.t, wr.i, site, en) >= thr ? mv * scale : 0.f;
                }
                out[e] = o;
                id |= (uint32_t)mi << (8 * e);
            }
            const long eo = (long)q * C + 4 * c;
            *reinterpret_cast<uint32_t*>(idx + eo) = id;
            xs_store_f(dhm, dl, df, xs_unit<C, PH * PW, SM>((unsigned)q, c), out);
        }
    }
};

}  // namespace flsim
