// conv1 forward lab (development tool): the product's direct k_conv1_fwd (pn1_net.hip) with its
// stores (MODE 1) or its MFMAs (MODE 2) taken out, and several grid sizes: where the time goes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I include
//         -I fl-distributed-delay_amd/csrc tools/lab/conv1_lab.hip -o tools/lab/conv1_lab
#include "lab_common.h"

constexpr int C1_ROWS = 32;     // output pixels per wave iteration (two 16-row tiles)
constexpr int C1_LD = 52;       // staging row stride (floats): 16-B aligned, rows on different banks
template <int MODE, int NT = 0>
__global__ void __launch_bounds__(256)
k_conv1_fwd(const float* __restrict__ x0, const float* __restrict__ W, const float* __restrict__ bias,
            float* __restrict__ a1, long units) {
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
    auto load = [&](long u, f32x4 (&xa)[2][2], float (&x8)[2]) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const long m = u * C1_ROWS + 16 * t + i;
            const long smp = m / 1156;
            const int rem = (int)(m - smp * 1156);
            const int oh = rem / 34, ow = rem - (rem / 34) * 34;
            const float* xs = x0 + smp * 4096;
#pragma unroll
            for (int sx = 0; sx < 2; ++sx) {
                const int tap = 4 * sx + g;
                const int ih = oh + tap / 3 - 2, iw = ow + tap % 3 - 2;
                xa[t][sx] = ((unsigned)ih < 32u && (unsigned)iw < 32u)
                                ? *reinterpret_cast<const f32x4*>(xs + (ih * 32 + iw) * 4) : zero4();
            }
            x8[t] = (oh < 32 && ow < 32) ? xs[(oh * 32 + ow) * 4 + g] : 0.f;   // tap 8: (ih, iw) = (oh, ow)
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
                    for (int kk = 0; kk < 4; ++kk) {
                        if (MODE == 2) c[kk] += xa[t][sx][kk] + wb[j][sx][kk];
                        else c = mfma16(xa[t][sx][kk], wb[j][sx][kk], c);
                    }
                acc[t][j] = MODE == 2 ? c + x8[t] * w8[j] : mfma16(x8[t], w8[j], c);
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
        f32x4* dst = reinterpret_cast<f32x4*>(a1 + u * C1_ROWS * 48);
#pragma unroll
        for (int q0 = 0; q0 < C1_ROWS * 12; q0 += 64) {
            const int q = q0 + lane, row = q / 12, c4 = q - (q / 12) * 12;
            const f32x4 v = *reinterpret_cast<const f32x4*>(st + row * C1_LD + 4 * c4);
            if (MODE == 1) { if (v.x == 123.f) dst[q] = v; }
            else if (NT) __builtin_nontemporal_store(v, dst + q);
            else dst[q] = v;
        }
        __builtin_amdgcn_wave_barrier();
    }
}


template <int MODE, int NT = 0>
static void run(const char* tag, const float* x0, const float* W, const float* b, float* a1, int S,
                int grid) {
    const long units = (long)S * 34 * 34 / C1_ROWS;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((k_conv1_fwd<MODE, NT>), dim3(grid), dim3(256), 0, 0, x0, W, b, a1, units);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k_conv1_fwd<MODE, NT>), dim3(grid), dim3(256), 0, 0, x0, W, b, a1, units);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    const double wbytes = (double)S * 34 * 34 * 48 * 4;
    printf("%-22s grid %6d  %7.3f ms  write %5.2f TB/s  %5.1f TF/s(27)\n", tag, grid, ms,
           wbytes / ms / 1e9, 2.0 * S * 34 * 34 * 48 * 27 / ms / 1e9);
    fflush(stdout);
}

int main() {
    const int S = 16384;
    float* x0 = dalloc((size_t)S * 4096, 1.f);
    float* W = dalloc(1296, 0.1f);
    float* b = dalloc(48, 0.01f);
    float* a1 = dalloc((size_t)S * 34 * 34 * 48, 0.f);
    for (int grid : {1024, 2048, 4096, 8192}) run<0>("full", x0, W, b, a1, S, grid);
    run<1>("no stores", x0, W, b, a1, S, 4096);
    run<2>("no mfma", x0, W, b, a1, S, 4096);
    run<0, 1>("full nt", x0, W, b, a1, S, 4096);
    run<2, 1>("no mfma nt", x0, W, b, a1, S, 4096);
    run<0, 1>("full nt g2048", x0, W, b, a1, S, 2048);
    return 0;
}
