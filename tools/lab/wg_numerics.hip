// Accumulation numerics of a weight-gradient-shaped GEMM on the bf16 matrix cores (development
// tool, not part of libflsim.so).  C[16][16] = sum over P "pixels" of A[p][i] * B[p][j] per tile
// (A: a signed dZ-like operand, B: a post-ReLU activation-like one), the reduction split into Z
// chains of KC k-steps of 16 (the product's slab splits, net_kernels.h wsplit), the chains' sums
// added on the host in fp64 so that only the chain arithmetic differs.  Strategies:
//   f32     v_mfma_f32_16x16x4_f32 chain (an exact fmaf chain: the CPU fp32 port's arithmetic class)
//   x6      the product's bf16x6 chain (gemm_x6.h x6_step<false>): hl+lh, hm+mh, hh+mm into one acc
//   x6f     the same, fresh per k-step (x6_step<true>)
//   x6two   hh+mm into one accumulator, hm+mh and hl+lh into a second
//   sep     hh alone (16x16x16) into one accumulator; hm+mh, hl+lh (16x16x32) and mm (16x16x16)
//           into a second
//   sepf    sep with the hh accumulation fresh per k-step (VALU add)
// against the fp64 sum: rel-L2 and alpha = <err, ref> / <ref, ref> (a systematic shrink of the
// result shows as alpha < 0 with |alpha| ~ rel).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/wg_numerics.hip -o tools/lab/wg_numerics
//   tools/lab/wg_numerics [KC ...]
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int T = 16;             // independent 16x16 tiles (one wave each)
constexpr long P = 1L << 20;      // reduction length per tile

__device__ inline void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = __float2bfloat16(x);
    const float r1 = x - __bfloat162float(h);
    m = __float2bfloat16(r1);
    l = __float2bfloat16(r1 - __bfloat162float(m));
}

__device__ inline f32x4 m32(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ inline f32x4 m16(bf16x4 a, bf16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// A, B: [T][P][16] fp32 (row p of tile t); out: [T][Z][16][16]
template <int S>
__global__ void k_chain(const float* A, const float* B, float* out, int KC, int Z) {
    const int t = blockIdx.x / Z, z = blockIdx.x % Z;
    const int lane = threadIdx.x, i = lane & 15, g = lane >> 4;
    const float* a = A + (long)t * P * 16;
    const float* b = B + (long)t * P * 16;
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    const long p0 = (long)z * KC * 16;
    for (int ks = 0; ks < KC; ++ks) {
        const long pb = p0 + ks * 16 + 4 * g;     // this lane's 4 k: pb .. pb + 3
        float av[4], bv[4];
        for (int j = 0; j < 4; ++j) {
            av[j] = a[(pb + j) * 16 + i];
            bv[j] = b[(pb + j) * 16 + i];
        }
        if constexpr (S == 0) {
            for (int j = 0; j < 4; ++j)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
            continue;
        } else {
            __bf16 ah[4], am[4], al[4], bh[4], bm[4], bl[4];
            for (int j = 0; j < 4; ++j) {
                split3(av[j], ah[j], am[j], al[j]);
                split3(bv[j], bh[j], bm[j], bl[j]);
            }
            bf16x8 Ahm, Ahl, Bhm, Bmh, Blh;
            bf16x4 Ah, Am, Bh, Bm;
            for (int j = 0; j < 4; ++j) {
                Ahm[j] = ah[j]; Ahm[4 + j] = am[j];
                Ahl[j] = ah[j]; Ahl[4 + j] = al[j];
                Bhm[j] = bh[j]; Bhm[4 + j] = bm[j];
                Bmh[j] = bm[j]; Bmh[4 + j] = bh[j];
                Blh[j] = bl[j]; Blh[4 + j] = bh[j];
                Ah[j] = ah[j]; Am[j] = am[j]; Bh[j] = bh[j]; Bm[j] = bm[j];
            }
            if constexpr (S == 1) {
                acc = m32(Ahl, Blh, acc);
                acc = m32(Ahm, Bmh, acc);
                acc = m32(Ahm, Bhm, acc);
            } else if constexpr (S == 2) {
                f32x4 u = m32(Ahl, Blh, f32x4{0, 0, 0, 0});
                u = m32(Ahm, Bmh, u);
                u = m32(Ahm, Bhm, u);
                acc += u;
            } else if constexpr (S == 3) {
                acc2 = m32(Ahl, Blh, acc2);
                acc2 = m32(Ahm, Bmh, acc2);
                acc = m32(Ahm, Bhm, acc);
            } else if constexpr (S == 4) {
                acc2 = m32(Ahl, Blh, acc2);
                acc2 = m16(Am, Bm, acc2);
                acc2 = m32(Ahm, Bmh, acc2);
                acc = m16(Ah, Bh, acc);
            } else {
                acc2 = m32(Ahl, Blh, acc2);
                acc2 = m16(Am, Bm, acc2);
                acc2 = m32(Ahm, Bmh, acc2);
                acc += m16(Ah, Bh, f32x4{0, 0, 0, 0});
            }
        }
    }
    float* o = out + ((long)t * Z + z) * 256;
    for (int r = 0; r < 4; ++r) o[(4 * g + r) * 16 + i] = acc[r] + acc2[r];
}

// fp64 reference: one thread per output
__global__ void k_ref(const float* A, const float* B, double* ref) {
    const int t = blockIdx.x, o = threadIdx.x, r = o / 16, c = o % 16;
    const float* a = A + (long)t * P * 16;
    const float* b = B + (long)t * P * 16;
    double s = 0;
    for (long p = 0; p < P; ++p) s += (double)a[p * 16 + r] * (double)b[p * 16 + c];
    ref[t * 256 + o] = s;
}

int main(int argc, char** argv) {
    std::vector<int> kcs;
    for (int a = 1; a < argc; ++a) kcs.push_back(atoi(argv[a]));
    if (kcs.empty()) kcs = {32, 256, 1024};     // KC must divide P / 16
    const size_t n = (size_t)T * P * 16;
    std::vector<float> hA(n), hB(n);
    std::mt19937_64 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::uniform_real_distribution<float> ud(0.f, 1.f);
    for (int t = 0; t < T; ++t) {
        float dirA[16], dirB[16];
        for (int j = 0; j < 16; ++j) { dirA[j] = nd(rng); dirB[j] = fabsf(nd(rng)); }
        for (long p = 0; p < P; ++p) {
            // a pixel's scale (heavy-tailed), a shared factor (the coherent part of the gradient)
            const float sa = expf(1.5f * nd(rng)) * 1e-3f, sb = expf(nd(rng));
            const float f = nd(rng);
            for (int j = 0; j < 16; ++j) {
                const size_t q = ((size_t)t * P + p) * 16 + j;
                const float x = fmaxf(0.f, nd(rng) + 0.3f * dirB[j] * f) * sb;
                hB[q] = ud(rng) < 0.3f ? 0.f : x;
                const float d = (nd(rng) + 0.2f * dirA[j] * f) * sa;
                hA[q] = ud(rng) < 0.4f ? 0.f : d;
            }
        }
    }
    float *A, *B, *out;
    double* ref;
    CK(hipMalloc(&A, n * 4));
    CK(hipMalloc(&B, n * 4));
    CK(hipMalloc(&ref, T * 256 * 8));
    CK(hipMemcpy(A, hA.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), n * 4, hipMemcpyHostToDevice));
    k_ref<<<T, 256>>>(A, B, ref);
    CK(hipDeviceSynchronize());
    std::vector<double> hr(T * 256);
    CK(hipMemcpy(hr.data(), ref, T * 256 * 8, hipMemcpyDeviceToHost));
    const char* names[] = {"f32", "x6", "x6f", "x6two", "sep", "sepf"};
    for (int KC : kcs) {
        const int Z = (int)(P / (16L * KC));
        CK(hipMalloc(&out, (size_t)T * Z * 256 * 4));
        std::vector<float> ho((size_t)T * Z * 256);
        printf("KC = %d k-steps per chain (%d pixels), Z = %d chains per tile, P = %ld\n", KC,
               16 * KC, Z, P);
        for (int s = 0; s < 6; ++s) {
            auto run = [&](auto kern) { kern<<<T * Z, 64>>>(A, B, out, KC, Z); };
            switch (s) {
                case 0: run(k_chain<0>); break;
                case 1: run(k_chain<1>); break;
                case 2: run(k_chain<2>); break;
                case 3: run(k_chain<3>); break;
                case 4: run(k_chain<4>); break;
                default: run(k_chain<5>); break;
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
            double e2 = 0, r2 = 0, er = 0;
            for (int t = 0; t < T; ++t)
                for (int o = 0; o < 256; ++o) {
                    double s2 = 0;
                    for (int z = 0; z < Z; ++z) s2 += ho[((size_t)t * Z + z) * 256 + o];
                    const double rv = hr[t * 256 + o], e = s2 - rv;
                    e2 += e * e; r2 += rv * rv; er += e * rv;
                }
            printf("  %-6s rel %.3e  alpha %+.3e\n", names[s], sqrt(e2 / r2), er / r2);
        }
        CK(hipFree(out));
    }
    return 0;
}
