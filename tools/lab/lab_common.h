// Shared pieces of the GEMM labs (development tools, not part of libflsim.so).
#pragma once
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
        if constexpr (ORD == 1) {      // the product's order (loaders.h)
            Base::load(ks, r);
            return;
        }
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
    static_assert(ORD == 0, "the product's column order only");
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

