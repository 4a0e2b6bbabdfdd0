// Split-bf16 MFMA lab (development tool, not part of libflsim.so): can the fp32 GEMMs run as
// sums of bf16 MFMA products at fp32 accuracy, and how fast?
//
// Each fp32 operand x is split x = h + m + l (h = bf16_rne(x), m = bf16_rne(x - h),
// l = bf16_rne(x - h - m)); a product a*b is the sum of the partial products of the parts, each
// exact in the MFMA's fp32 accumulator.  bf16x3 keeps hh, hm, mh; bf16x6 adds mm, hl, lh; bf16x9
// keeps all nine.
//   accuracy: one wave, a 16 x 16 tile over K, |C - C_fp64| / sum_k |a b| against the native
//             fp32 MFMA (v_mfma_f32_16x16x4_f32);
//   rate:     a full grid of 4-wave blocks running the gemm_kernel inner loop (LDS fragment reads,
//             one barrier per stage) on resident tiles, effective fp32 TF/s.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I fl-distributed-delay_amd/csrc
//         tools/lab/bf16x_lab.hip -o tools/lab/bf16x_lab
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "gemm_core.h"

using namespace flsim;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Parts {
    bf16x4 h, m, l;
};

__device__ __forceinline__ Parts split3(f32x4 x) {
    Parts p;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const __bf16 h = (__bf16)x[e];
        const float r1 = x[e] - (float)h;
        const __bf16 m = (__bf16)r1;
        const float r2 = r1 - (float)m;
        p.h[e] = h;
        p.m[e] = m;
        p.l[e] = (__bf16)r2;
    }
    return p;
}

__device__ __forceinline__ f32x4 mfma_bf16x16(bf16x4 a, bf16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a),
                                                     __builtin_bit_cast(s16x4, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf16x32(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
    return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// TERMS 3 / 6 / 9, smallest partial products first
template <int TERMS>
__device__ __forceinline__ f32x4 split_mac16(const Parts& a, const Parts& b, f32x4 c) {
    if constexpr (TERMS >= 9) c = mfma_bf16x16(a.l, b.l, c);
    if constexpr (TERMS >= 9) c = mfma_bf16x16(a.m, b.l, c);
    if constexpr (TERMS >= 9) c = mfma_bf16x16(a.l, b.m, c);
    if constexpr (TERMS >= 6) c = mfma_bf16x16(a.m, b.m, c);
    if constexpr (TERMS >= 6) c = mfma_bf16x16(a.h, b.l, c);
    if constexpr (TERMS >= 6) c = mfma_bf16x16(a.l, b.h, c);
    c = mfma_bf16x16(a.m, b.h, c);
    c = mfma_bf16x16(a.h, b.m, c);
    c = mfma_bf16x16(a.h, b.h, c);
    return c;
}
template <int TERMS>
__device__ __forceinline__ f32x4 split_mac32(const Parts& a0, const Parts& a1, const Parts& b0,
                                             const Parts& b1, f32x4 c) {
    if constexpr (TERMS >= 9) c = mfma_bf16x32(cat(a0.l, a1.l), cat(b0.l, b1.l), c);
    if constexpr (TERMS >= 9) c = mfma_bf16x32(cat(a0.m, a1.m), cat(b0.l, b1.l), c);
    if constexpr (TERMS >= 9) c = mfma_bf16x32(cat(a0.l, a1.l), cat(b0.m, b1.m), c);
    if constexpr (TERMS >= 6) c = mfma_bf16x32(cat(a0.m, a1.m), cat(b0.m, b1.m), c);
    if constexpr (TERMS >= 6) c = mfma_bf16x32(cat(a0.h, a1.h), cat(b0.l, b1.l), c);
    if constexpr (TERMS >= 6) c = mfma_bf16x32(cat(a0.l, a1.l), cat(b0.h, b1.h), c);
    c = mfma_bf16x32(cat(a0.m, a1.m), cat(b0.h, b1.h), c);
    c = mfma_bf16x32(cat(a0.h, a1.h), cat(b0.m, b1.m), c);
    c = mfma_bf16x32(cat(a0.h, a1.h), cat(b0.h, b1.h), c);
    return c;
}

// ---- accuracy: one wave, C[16][16] = A[16][K] B[K][16] ----
// MODE 0: fp32 MFMA; 1..3: bf16x{3,6,9} on 16x16x16; 4..6: bf16x{3,6,9} on 16x16x32
template <int MODE>
__global__ void acc_kernel(const float* A, const float* B, float* C, int K) {
    const int l = threadIdx.x;
    const int row = l & 15, g = l >> 4;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    auto fa = [&](int ks) {
        f32x4 v;
        for (int j = 0; j < 4; ++j) v[j] = A[(long)row * K + ks * 16 + 4 * g + j];
        return v;
    };
    auto fb = [&](int ks) {
        f32x4 v;
        for (int j = 0; j < 4; ++j) v[j] = B[(long)(ks * 16 + 4 * g + j) * 16 + row];
        return v;
    };
    const int KS = K / 16;
    if constexpr (MODE == 0) {
        for (int ks = 0; ks < KS; ++ks) {
            const f32x4 a = fa(ks), b = fb(ks);
            for (int j = 0; j < 4; ++j) c = mfma16(a[j], b[j], c);
        }
    } else if constexpr (MODE <= 3) {
        constexpr int T = MODE == 1 ? 3 : MODE == 2 ? 6 : 9;
        for (int ks = 0; ks < KS; ++ks) c = split_mac16<T>(split3(fa(ks)), split3(fb(ks)), c);
    } else if constexpr (MODE >= 7) {
        // the product's pairing (gemm_x6.h): per 16-deep k-step A [h|m], [h|l] x B [h|m], [m|h],
        // [l|h]; MODE 8: the three MFMAs into a zero accumulator, added to c by a VALU add
        for (int ks = 0; ks < KS; ++ks) {
            const Parts a = split3(fa(ks)), b = split3(fb(ks));
            const bf16x8 ahm = cat(a.h, a.m), ahl = cat(a.h, a.l);
            const bf16x8 bhm = cat(b.h, b.m), bmh = cat(b.m, b.h), blh = cat(b.l, b.h);
            f32x4 t = MODE == 8 ? f32x4{0.f, 0.f, 0.f, 0.f} : c;
            t = mfma_bf16x32(ahl, blh, t);
            t = mfma_bf16x32(ahm, bmh, t);
            t = mfma_bf16x32(ahm, bhm, t);
            c = MODE == 8 ? c + t : t;
        }
    } else {
        constexpr int T = MODE == 4 ? 3 : MODE == 5 ? 6 : 9;
        for (int ks = 0; ks + 1 < KS; ks += 2)
            c = split_mac32<T>(split3(fa(ks)), split3(fa(ks + 1)), split3(fb(ks)),
                               split3(fb(ks + 1)), c);
    }
    for (int r = 0; r < 4; ++r) C[(4 * g + r) * 16 + row] = c[r];
}

// ---- rate: FM x FN fragments per wave, 2 x 2 waves, resident KC tiles, ITER k-steps ----
// MODE 0: fp32; 2: bf16x6 split at read on 16x16x16; 5: bf16x6 split at read on 16x16x32
// (two k-steps per stage); 7: fp32 with two k-steps per stage; 8: bf16x6 on 16x16x32 with
// pre-split LDS planes (no conversion: the upper bound of splitting at the LDS store)
template <int MODE, int FM, int FN>
__global__ void __launch_bounds__(256) rate_kernel(float* out, int iters) {
    constexpr int BM = 32 * FM, BN = 32 * FN;
    constexpr int TA = KCTile<BM>::FLOATS, TB = KCTile<BN>::FLOATS;
    __shared__ __attribute__((aligned(16))) float lds[2 * 2 * (TA + TB)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    for (int i = tid; i < 2 * 2 * (TA + TB); i += 256)
        lds[i] = (float)((i * 2654435761u + blockIdx.x) % 1000) * 1e-3f - 0.5f;
    __syncthreads();
    f32x4 acc[FM][FN];
    for (int i = 0; i < FM; ++i)
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int PER = (MODE == 5 || MODE == 7 || MODE == 8) ? 2 : 1;
    for (int it = 0; it < iters; it += PER) {
        const float* base = lds + (it & 2 ? 2 * (TA + TB) : 0);
        if constexpr (MODE == 0) {
            const float* Ab = base;
            const float* Bb = base + TA;
            f32x4 af[FM], bf[FN];
            for (int i = 0; i < FM; ++i) af[i] = read_frag<true, BM>(Ab, wm * 16 * FM + 16 * i, lane);
            for (int j = 0; j < FN; ++j) bf[j] = read_frag<true, BN>(Bb, wn * 16 * FN + 16 * j, lane);
            for (int kk = 0; kk < 4; ++kk)
                for (int i = 0; i < FM; ++i)
                    for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
        } else if constexpr (MODE == 7) {
            for (int s = 0; s < 2; ++s) {
                const float* Ab = base + s * (TA + TB);
                const float* Bb = Ab + TA;
                f32x4 af[FM], bf[FN];
                for (int i = 0; i < FM; ++i) af[i] = read_frag<true, BM>(Ab, wm * 16 * FM + 16 * i, lane);
                for (int j = 0; j < FN; ++j) bf[j] = read_frag<true, BN>(Bb, wn * 16 * FN + 16 * j, lane);
                for (int kk = 0; kk < 4; ++kk)
                    for (int i = 0; i < FM; ++i)
                        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i][kk], bf[j][kk], acc[i][j]);
            }
        } else if constexpr (MODE == 2) {
            const float* Ab = base;
            const float* Bb = base + TA;
            Parts bp[FN];
            for (int j = 0; j < FN; ++j) bp[j] = split3(read_frag<true, BN>(Bb, wn * 16 * FN + 16 * j, lane));
            for (int i = 0; i < FM; ++i) {
                const Parts ap = split3(read_frag<true, BM>(Ab, wm * 16 * FM + 16 * i, lane));
                for (int j = 0; j < FN; ++j) acc[i][j] = split_mac16<6>(ap, bp[j], acc[i][j]);
            }
        } else if constexpr (MODE == 5) {
            const float* A0 = base;
            const float* B0 = base + TA;
            const float* A1 = base + TA + TB;
            const float* B1 = A1 + TA;
            Parts bp0[FN], bp1[FN];
            for (int j = 0; j < FN; ++j) {
                bp0[j] = split3(read_frag<true, BN>(B0, wn * 16 * FN + 16 * j, lane));
                bp1[j] = split3(read_frag<true, BN>(B1, wn * 16 * FN + 16 * j, lane));
            }
            for (int i = 0; i < FM; ++i) {
                const Parts a0 = split3(read_frag<true, BM>(A0, wm * 16 * FM + 16 * i, lane));
                const Parts a1 = split3(read_frag<true, BM>(A1, wm * 16 * FM + 16 * i, lane));
                for (int j = 0; j < FN; ++j) acc[i][j] = split_mac32<6>(a0, a1, bp0[j], bp1[j], acc[i][j]);
            }
        } else {   // MODE 8: planes of bf16x8 per (row, plane), read as 16 B each
            const bf16x8* P = reinterpret_cast<const bf16x8*>(base);
            bf16x8 bh[FN], bm[FN], bl[FN];
            for (int j = 0; j < FN; ++j) {
                const int r = (wn * 16 * FN + 16 * j + (lane & 15)) * 4 + (lane >> 4);
                bh[j] = P[(r + 0 * 4 * BN) % (TA + TB) / 2];
                bm[j] = P[(r + 1 * 4 * BN) % (TA + TB) / 2];
                bl[j] = P[(r + 2 * 4 * BN) % (TA + TB) / 2];
            }
            for (int i = 0; i < FM; ++i) {
                const int r = (wm * 16 * FM + 16 * i + (lane & 15)) * 4 + (lane >> 4) + 7;
                const bf16x8 ah = P[(r + 0 * 4 * BM) % (TA + TB) / 2];
                const bf16x8 am = P[(r + 1 * 4 * BM) % (TA + TB) / 2];
                const bf16x8 al = P[(r + 2 * 4 * BM) % (TA + TB) / 2];
                for (int j = 0; j < FN; ++j) {
                    f32x4 c = acc[i][j];
                    c = mfma_bf16x32(am, bm[j], c);
                    c = mfma_bf16x32(ah, bl[j], c);
                    c = mfma_bf16x32(al, bh[j], c);
                    c = mfma_bf16x32(am, bh[j], c);
                    c = mfma_bf16x32(ah, bm[j], c);
                    c = mfma_bf16x32(ah, bh[j], c);
                    acc[i][j] = c;
                }
            }
        }
        __syncthreads();
    }
    float s = 0.f;
    for (int i = 0; i < FM; ++i)
        for (int j = 0; j < FN; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * 256 + tid] = s;
}

static double lcg(unsigned long& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (double)((s >> 11) & ((1ull << 53) - 1)) / (double)(1ull << 53);
}

template <int MODE>
static void run_acc(const char* name, const float* dA, const float* dB, float* dC, int K,
                    const std::vector<float>& A, const std::vector<float>& B) {
    hipLaunchKernelGGL(acc_kernel<MODE>, dim3(1), dim3(64), 0, 0, dA, dB, dC, K);
    CK(hipDeviceSynchronize());
    std::vector<float> C(256);
    CK(hipMemcpy(C.data(), dC, 1024, hipMemcpyDeviceToHost));
    double emax = 0, esum = 0, bias = 0, cabs = 0, rel2 = 0, ref2 = 0;
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            double ref = 0, mag = 0;
            for (int k = 0; k < K; ++k) {
                const double p = (double)A[(long)r * K + k] * (double)B[(long)k * 16 + c];
                ref += p;
                mag += fabs(p);
            }
            const double d = (double)C[r * 16 + c] - ref;
            const double e = fabs(d) / (mag > 0 ? mag : 1);
            emax = e > emax ? e : emax;
            esum += e;
            bias += d * (ref > 0 ? 1.0 : -1.0);   // < 0: errors lean toward zero (truncation)
            cabs += fabs(ref);
            rel2 += d * d;
            ref2 += ref * ref;
        }
    printf("acc %-12s K=%6d  max %.3e  mean %.3e  (x 2^-24: max %.2f mean %.2f)  rel-L2 %.3e  "
           "signed bias / mean|C| %+.3e\n", name, K, emax, esum / 256, emax * 16777216.0,
           esum / 256 * 16777216.0, sqrt(rel2 / ref2), bias / cabs);
}

template <int MODE, int FM, int FN>
static void run_rate(const char* name) {
    const int blocks = 256 * 8, iters = 4096;
    float* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((rate_kernel<MODE, FM, FN>), dim3(blocks), dim3(256), 0, 0, out, 64);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((rate_kernel<MODE, FM, FN>), dim3(blocks), dim3(256), 0, 0, out, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double flops = 2.0 * (32 * FM) * (32 * FN) * 16.0 * iters * blocks;
    printf("rate %-24s FM=%d FN=%d  %8.3f ms  %7.1f TF/s (fp32-equivalent)\n", name, FM, FN, best,
           flops / best / 1e9);
    CK(hipFree(out));
}

int main() {
    for (int K : {1728, 16384}) {
        for (int dist = 0; dist < 2; ++dist) {
            std::vector<float> A((size_t)16 * K), B((size_t)K * 16);
            unsigned long s = 12345 + K + dist;
            for (auto& v : A) {   // dist 0: post-ReLU activations (half zeros); 1: uniform [-1, 1)
                const double u = lcg(s);
                v = dist == 0 ? (u < 0.5 ? 0.f : (float)(2.0 * lcg(s))) : (float)(2.0 * u - 1.0);
            }
            for (auto& v : B) {
                const double u1 = lcg(s) + 1e-12, u2 = lcg(s);
                v = (float)(0.05 * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
            }
            float *dA, *dB, *dC;
            CK(hipMalloc(&dA, A.size() * 4));
            CK(hipMalloc(&dB, B.size() * 4));
            CK(hipMalloc(&dC, 1024));
            CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
            CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
            printf("-- K = %d, A %s\n", K, dist == 0 ? "relu-like" : "uniform");
            run_acc<0>("fp32", dA, dB, dC, K, A, B);
            run_acc<1>("bf16x3/x16", dA, dB, dC, K, A, B);
            run_acc<2>("bf16x6/x16", dA, dB, dC, K, A, B);
            run_acc<3>("bf16x9/x16", dA, dB, dC, K, A, B);
            run_acc<4>("bf16x3/x32", dA, dB, dC, K, A, B);
            run_acc<5>("bf16x6/x32", dA, dB, dC, K, A, B);
            run_acc<6>("bf16x9/x32", dA, dB, dC, K, A, B);
            run_acc<7>("x6 product", dA, dB, dC, K, A, B);
            run_acc<8>("x6 prod+add", dA, dB, dC, K, A, B);
            CK(hipFree(dA));
            CK(hipFree(dB));
            CK(hipFree(dC));
        }
    }
    if (getenv("ACC_ONLY")) return 0;
    run_rate<0, 4, 4>("fp32");
    run_rate<7, 4, 4>("fp32 2 k-steps/stage");
    run_rate<2, 4, 4>("bf16x6 x16 split@read");
    run_rate<5, 4, 4>("bf16x6 x32 split@read");
    run_rate<8, 4, 4>("bf16x6 x32 pre-split");
    run_rate<0, 2, 3>("fp32");
    run_rate<5, 2, 3>("bf16x6 x32 split@read");
    run_rate<8, 2, 3>("bf16x6 x32 pre-split");
    return 0;
}
