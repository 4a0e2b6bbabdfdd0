// Lab: throughput of the rule() cascade interpreter (cascade.h casc_run) alone, on a configs[3]-like
// general-order program (k = 8100 entries, 72 stale events among 6 arrays), over P = 5,596,090
// elements -- no slab reduction, so the time is the interpreter's (plus the element streams).
// Variants: elements per lane (1, 4, 8, 16) x program form (op words / macro words, MAC).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include -I fl-distributed-delay_amd/csrc \
//         tools/lab/casc_lab.hip -o tools/lab/casc_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "cascade.h"
#include "common.h"

using namespace flsim;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int NARR = 6;
__constant__ int32_t c_prog[16384];     // op words
__constant__ int32_t c_mac[16384];      // macro pairs

struct Prog {
    __device__ __forceinline__ int32_t operator[](int i) const { return c_prog[i]; }
};
struct Mac {
    __device__ __forceinline__ uint32_t lo(int i) const { return (uint32_t)c_mac[2 * i]; }
    __device__ __forceinline__ uint32_t hi(int i) const { return (uint32_t)c_mac[2 * i + 1]; }
};

// EPL consecutive elements per lane as W float4 words
template <int W>
struct vecw {
    f32x4 v[W];
    __host__ __device__ vecw() {}
    __host__ __device__ explicit vecw(float s) {
#pragma unroll
        for (int i = 0; i < W; ++i) v[i] = f32x4{s, s, s, s};
    }
    __host__ __device__ vecw& operator+=(const vecw& o) {
#pragma unroll
        for (int i = 0; i < W; ++i) v[i] += o.v[i];
        return *this;
    }
};

template <class T> struct Lane;
template <> struct Lane<float> {
    static constexpr int EPL = 1;
    __device__ static float ld(const float* p) { return __builtin_nontemporal_load(p); }
    __device__ static void st(float* p, float v) { __builtin_nontemporal_store(v, p); }
};
template <> struct Lane<f32x4> {
    static constexpr int EPL = 4;
    __device__ static f32x4 ld(const float* p) {
        return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    }
    __device__ static void st(float* p, f32x4 v) {
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
    }
};
template <int W> struct Lane<vecw<W>> {
    static constexpr int EPL = 4 * W;
    __device__ static vecw<W> ld(const float* p) {
        vecw<W> r;
#pragma unroll
        for (int i = 0; i < W; ++i)
            r.v[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
        return r;
    }
    __device__ static void st(float* p, const vecw<W>& v) {
#pragma unroll
        for (int i = 0; i < W; ++i)
            __builtin_nontemporal_store(v.v[i], reinterpret_cast<f32x4*>(p) + i);
    }
};

struct Args {
    const float* x;
    const float* ys[NARR];
    float* out;
    long n;            // elements (multiple of 16)
    int need, lp;
};

template <class T, int MAC, bool RUN>
__global__ void __launch_bounds__(256) k_casc(Args A) {
    constexpr int EPL = Lane<T>::EPL;
    const long e = ((long)blockIdx.x * 256 + threadIdx.x) * EPL;
    if (e >= A.n) return;
    const T x = Lane<T>::ld(A.x + e);
    T ys[NARR];
#pragma unroll
    for (int q = 0; q < NARR; ++q) ys[q] = Lane<T>::ld(A.ys[q] + e);
    T r;
    if constexpr (RUN) {
        auto yf = [&](int q) -> T {
            switch (q) {
                case 0: return ys[0];
                case 1: return ys[1];
                case 2: return ys[2];
                case 3: return ys[3];
                case 4: return ys[4];
                default: return ys[5];
            }
        };
        if constexpr (MAC) r = casc_run_macro<true>(Mac{}, 0, casc_values(x, A.need, A.lp), yf);
        else r = casc_run<1, true>(Prog{}, 0, casc_values(x, A.need, A.lp), yf);
    } else {
        r = x;
#pragma unroll
        for (int q = 0; q < NARR; ++q) r += ys[q];
    }
    Lane<T>::st(A.out + e, r);
}

template <class T, int MAC, bool RUN>
static void run(const char* name, Args A, const std::vector<float>& want, float* hout) {
    constexpr int EPL = Lane<T>::EPL;
    const unsigned nb = (unsigned)((A.n / EPL + 255) / 256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_casc<T, MAC, RUN><<<nb, 256>>>(A);
    CK(hipDeviceSynchronize());
    const int reps = getenv("LAB_ITERS") ? atoi(getenv("LAB_ITERS")) : 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_casc<T, MAC, RUN><<<nb, 256>>>(A);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    bool ok = true;
    if (RUN) {
        CK(hipMemcpy(hout, A.out, 4 * A.n, hipMemcpyDeviceToHost));
        for (long i = 0; i < A.n && ok; i += 997)
            ok = __builtin_memcmp(&hout[i], &want[i], 4) == 0;
    }
    const double us = ms * 1e3 / reps;
    printf("%-28s %8.1f us  %7.1f GB/s  %s\n", name, us, 4.0 * A.n * (NARR + 2) / us / 1e3,
           RUN ? (ok ? "bit-exact" : "MISMATCH") : "");
}

int main() {
    const long n = 5596096;       // P rounded up to 16
    const int k = 8100, nev = 72;
    // configs[3]-like events: 72 distinct positions, arrays 0..5
    std::vector<int32_t> pos, arr;
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
    while ((int)pos.size() < nev) {
        const int p = (int)(rnd() % k);
        if (std::find(pos.begin(), pos.end(), p) == pos.end()) pos.push_back(p);
    }
    std::sort(pos.begin(), pos.end());
    for (int j = 0; j < nev; ++j) arr.push_back((int32_t)(rnd() % NARR));
    std::vector<int32_t> prog(16384);
    CascInfo info;
    const int len = build_cascade_program(k, pos.data(), arr.data(), nev, prog.data(), 16000, &info);
    if (len <= 0) { printf("program build failed %d\n", len); return 1; }
    printf("program: %d words (main %d), need %d, lp %d\n", len, info.tail_off, info.need, info.lp);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_prog), prog.data(), 16384 * 4));
    std::vector<uint32_t> mac(16384);
    CascInfo minfo;
    const int mlen = build_macro_program(prog.data(), info, mac.data(), 8000, &minfo);
    if (mlen <= 0) { printf("macro build failed %d\n", mlen); return 1; }
    printf("macro program: %d pairs (main %d)\n", mlen, minfo.tail_off);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_mac), mac.data(), 16384 * 4));

    std::vector<float> hx(n), hy[NARR], want(n), hout(n);
    for (long i = 0; i < n; ++i) hx[i] = (float)((i * 2654435761u) % 2001) * 1e-3f - 1.f;
    for (int q = 0; q < NARR; ++q) {
        hy[q].resize(n);
        for (long i = 0; i < n; ++i) hy[q][i] = (float)(((i + 7 * q) * 40503u) % 1999) * 1e-3f - 1.f;
    }
    for (long i = 0; i < n; i += 997) {
        auto yf = [&](int q) -> float { return hy[q][i]; };
        want[i] = casc_run<1, true>(prog.data(), 0, casc_values(hx[i], info.need, info.lp), yf);
    }
    Args A{};
    A.n = n;
    A.need = info.need;
    A.lp = info.lp;
    float* d;
    CK(hipMalloc(&d, 4 * n * (NARR + 2)));
    CK(hipMemcpy(d, hx.data(), 4 * n, hipMemcpyHostToDevice));
    A.x = d;
    for (int q = 0; q < NARR; ++q) {
        CK(hipMemcpy(d + (q + 1) * n, hy[q].data(), 4 * n, hipMemcpyHostToDevice));
        A.ys[q] = d + (q + 1) * n;
    }
    A.out = d + (NARR + 1) * n;

    run<vecw<1>, 1, false>("stream only (x4)", A, want, hout.data());
    run<float, 0, true>("ops   epl 1", A, want, hout.data());
    run<vecw<1>, 0, true>("ops   epl 4", A, want, hout.data());
    run<vecw<2>, 0, true>("ops   epl 8", A, want, hout.data());
    run<float, 1, true>("macro epl 1", A, want, hout.data());
    run<vecw<1>, 1, true>("macro epl 4 (vecw)", A, want, hout.data());
    run<f32x4, 1, true>("macro epl 4 (f32x4)", A, want, hout.data());
    run<vecw<2>, 1, true>("macro epl 8", A, want, hout.data());
    run<vecw<4>, 1, true>("macro epl 16", A, want, hout.data());
    return 0;
}
