// Lab (development tool, not part of libflsim.so): an exact-accumulation fp32 GEMM on the int8
// matrix cores (Ozaki-style slices), on the shape of PerformantNet1's conv6 data gradient
// (K = 9 taps x 192 channels = 1728, N = 192; M = rows of the lab, a slice of the 16k-sample
// chunk's S * 169).  VERDICT r05 item 3.
//
// Each fp32 row of A (a dZ im2col row) and column of B (a packed weight column) gets one
// power-of-two scale over the whole K, e = ilogb(max |x|) + 2, so |x 2^-e| < 1/2; the value is
// cut into S int8 slices by round-to-nearest-even steps of 2^-7 (each |slice| <= 64), so
// x = 2^e (sum_t q_t 2^-7t + r) with |r| <= 2^-7S / 2 (unbiased).  The slice products q_i q_j with
// i + j <= S + 1 are summed EXACTLY in int32 (v_mfma_i32_16x16x64_i8; the class sum is bounded by
// pairs * K * 64^2 < 2^31), one accumulator per class c = i + j, and only the end converts:
// C = 2^(eA + eB) sum_c 2^-7c float(acc_c) (round to nearest: no truncation bias at any K).
// The i8 MFMA issues at 2x the bf16 rate (~5 POPS dense), so with P = S(S+1)/2 products per
// fp32 product the issue-bound fp32-equivalent peak is 5000 / P TF/s.
//
// Reports, per S: time and fp32-equivalent TF/s of the GEMM kernel (slicing not timed: the
// product's producers would write the slices, as they write the split-bf16 form today), and the
// accuracy on the first 1024 rows against fp64, beside a sequential fp32 fmaf chain's (the CPU
// fp32 port's arithmetic class): rel-L2, alpha = <err, ref>/<ref, ref> (coherent bias), and the
// per-column sums' rel error (what the next layer's bias gradient sees).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/i8_lab.hip -o tools/lab/i8_lab
//   tools/lab/i8_lab [M]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int K = 1728, N = 192, KB = K / 64;
constexpr int BROWS = 64, BCOLS = 64;          // block tile per row fragment: 4 waves x 16 rows
constexpr int LDB = 64 + 16;                   // LDS row stride (bytes) of a B slice plane

// per-row exponents: e = ilogb(max |x|) + 2 (0 for an all-zero row)
__global__ void k_rowexp(const float* X, int rows, int* e) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float m = 0.f;
    for (int k = 0; k < K; ++k) m = fmaxf(m, fabsf(X[(long)r * K + k]));
    e[r] = m > 0.f ? ilogbf(m) + 2 : 0;
}

// slices q[t][r][k] (int8), t < S
__global__ void k_slice(const float* X, int rows, const int* e, int S, signed char* q) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)rows * K) return;
    const int r = (int)(i / K);
    float v = ldexpf(X[i], -e[r]);
    for (int t = 0; t < S; ++t) {
        const float s = rintf(v * 128.f);
        q[(long)t * rows * K + i] = (signed char)s;
        v = v * 128.f - s;
    }
}

// C[M][N] = A[M][K] B[N][K]^T from the slices; 4 waves, each RF x 16 rows x 64 columns (RF row
// fragments share each B fragment read from LDS); grid (M / (64 RF)) x (N / 64)
template <int S, int RF>
__global__ void __launch_bounds__(256) k_gemm(const signed char* qa, const signed char* qb,
                                              const int* ea, const int* eb, float* C, int M) {
    constexpr int NCLS = S;                    // classes c = i + j = 2 .. S + 1
    __shared__ __attribute__((aligned(16))) signed char sb[2][S][BCOLS * LDB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m0 = blockIdx.x * BROWS * RF, n0 = blockIdx.y * BCOLS;
    const int i = lane & 15, g = lane >> 4;
    i32x4 acc[NCLS][RF][4];
#pragma unroll
    for (int c = 0; c < NCLS; ++c)
#pragma unroll
        for (int f = 0; f < RF; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[c][f][j] = i32x4{0, 0, 0, 0};
    // B staging: 64 columns x 64 k bytes per slice = 256 x 16 B: thread -> (column, 16-B chunk)
    const int scol = tid >> 2, sch = tid & 3;
    auto stage = [&](int kb, int buf) {
#pragma unroll
        for (int t = 0; t < S; ++t) {
            const i32x4 v = *reinterpret_cast<const i32x4*>(
                qb + (long)t * N * K + (long)(n0 + scol) * K + kb * 64 + 16 * sch);
            *reinterpret_cast<i32x4*>(&sb[buf][t][scol * LDB + 16 * sch]) = v;
        }
    };
    // A's slices come straight from global memory (each lane 16 B per slice: one row, 16 k),
    // loaded one k-block ahead so their latency hides behind the current block's MFMAs
    auto load_a = [&](int kb, i32x4 (&a)[RF][S]) {
#pragma unroll
        for (int f = 0; f < RF; ++f) {
            const int row = m0 + (wave * RF + f) * 16 + i;
#pragma unroll
            for (int t = 0; t < S; ++t)
                a[f][t] = *reinterpret_cast<const i32x4*>(qa + (long)t * M * K + (long)row * K +
                                                           kb * 64 + 16 * g);
        }
    };
    i32x4 an[RF][S];
    load_a(0, an);
    stage(0, 0);
    __syncthreads();
    for (int kb = 0; kb < KB; ++kb) {
        const int cur = kb & 1;
        i32x4 a[RF][S];
#pragma unroll
        for (int f = 0; f < RF; ++f)
#pragma unroll
            for (int t = 0; t < S; ++t) a[f][t] = an[f][t];
        if (kb + 1 < KB) {
            load_a(kb + 1, an);
            stage(kb + 1, cur ^ 1);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            i32x4 b[S];
#pragma unroll
            for (int t = 0; t < S; ++t)
                b[t] = *reinterpret_cast<const i32x4*>(&sb[cur][t][(16 * j + i) * LDB + 16 * g]);
#pragma unroll
            for (int f = 0; f < RF; ++f)
#pragma unroll
                for (int ti = 0; ti < S; ++ti)
#pragma unroll
                    for (int tj = 0; tj < S; ++tj)
                        if (ti + tj <= S - 1)  // slices 1-based: (ti+1) + (tj+1) <= S + 1
                            acc[ti + tj][f][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                a[f][ti], b[tj], acc[ti + tj][f][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // C = 2^(eA + eB) sum_c 2^-7(c+2) acc_c; output layout: col = lane & 15, row = 4 g + r
#pragma unroll
    for (int f = 0; f < RF; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + 16 * j + i;
            const int ecol = eb[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int orow = m0 + (wave * RF + f) * 16 + 4 * g + r;
                float v = 0.f;
#pragma unroll
                for (int c = NCLS - 1; c >= 0; --c)      // smallest terms first
                    v += ldexpf((float)acc[c][f][j][r], -7 * (c + 2));
                C[(long)orow * N + col] = ldexpf(v, ea[orow] + ecol);
            }
        }
}

// references on the first R rows: fp64 dot, and a sequential fp32 fmaf chain
__global__ void k_ref(const float* A, const float* B, int R, double* r64, float* r32) {
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= R * N) return;
    const int m = o / N, n = o % N;
    double s = 0;
    float f = 0.f;
    for (int k = 0; k < K; ++k) {
        s += (double)A[(long)m * K + k] * (double)B[(long)n * K + k];
        f = fmaf(A[(long)m * K + k], B[(long)n * K + k], f);
    }
    r64[o] = s;
    r32[o] = f;
}

struct Err { double rel, alpha, colsum; };
static Err err_of(const float* c, const double* r, int R) {
    double e2 = 0, r2 = 0, er = 0;
    std::vector<double> cs(N, 0.0), rs(N, 0.0);
    for (int o = 0; o < R * N; ++o) {
        const double e = (double)c[o] - r[o];
        e2 += e * e; r2 += r[o] * r[o]; er += e * r[o];
        cs[o % N] += c[o]; rs[o % N] += r[o];
    }
    double ce = 0, cr = 0;
    for (int n = 0; n < N; ++n) { ce += (cs[n] - rs[n]) * (cs[n] - rs[n]); cr += rs[n] * rs[n]; }
    return Err{sqrt(e2 / r2), er / r2, sqrt(ce / cr)};
}

template <int S, int RF>
static void run(int M, const float* dA, const float* dB, const int* ea, const int* eb,
                const double* r64, const std::vector<float>& h32, int R) {
    signed char *qa, *qb;
    float* C;
    CK(hipMalloc(&qa, (size_t)S * M * K));
    CK(hipMalloc(&qb, (size_t)S * N * K));
    CK(hipMalloc(&C, (size_t)M * N * 4));
    k_slice<<<(unsigned)(((long)M * K + 255) / 256), 256>>>(dA, M, ea, S, qa);
    k_slice<<<(N * K + 255) / 256, 256>>>(dB, N, eb, S, qb);
    CK(hipDeviceSynchronize());
    const dim3 grid(M / (BROWS * RF), N / BCOLS);
    k_gemm<S, RF><<<grid, 256>>>(qa, qb, ea, eb, C, M);     // warm-up
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = 10;
    CK(hipEventRecord(e0));
    for (int r = 0; r < it; ++r) k_gemm<S, RF><<<grid, 256>>>(qa, qb, ea, eb, C, M);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    std::vector<float> hc((size_t)R * N);
    CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
    std::vector<double> hr((size_t)R * N);
    CK(hipMemcpy(hr.data(), r64, hr.size() * 8, hipMemcpyDeviceToHost));
    const Err e = err_of(hc.data(), hr.data(), R), f = err_of(h32.data(), hr.data(), R);
    const double tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12;
    printf("S=%d RF=%d  products %2d  issue-bound peak %6.0f TF/s | %8.3f ms  %6.1f TF/s  (x %.1f to a "
           "16,384-sample conv6 launch: %.2f ms) | rel %.2e alpha %+.1e colsum %.2e  [fp32 chain: "
           "rel %.2e alpha %+.1e colsum %.2e]\n",
           S, RF, S * (S + 1) / 2, 5000.0 / (S * (S + 1) / 2), ms, tf, 16384.0 * 169 / M,
           ms * 16384.0 * 169 / M, e.rel, e.alpha, e.colsum, f.rel, f.alpha, f.colsum);
    CK(hipFree(qa));
    CK(hipFree(qb));
    CK(hipFree(C));
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 1 << 18;      // multiple of 64
    const int R = 1024;
    std::mt19937_64 rng(11);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::uniform_real_distribution<float> ud(0.f, 1.f);
    // A: im2col rows of a pooled, dropped-out dZ: 9 tap blocks of 192 channels, each tap a
    // neighbouring pixel with its own (log-normal) scale, about half the entries zero
    std::vector<float> hA((size_t)M * K), hB((size_t)N * K);
    for (int m = 0; m < M; ++m)
        for (int tap = 0; tap < 9; ++tap) {
            const float s = expf(nd(rng)) * 1e-4f;
            for (int c = 0; c < 192; ++c)
                hA[(size_t)m * K + tap * 192 + c] = ud(rng) < 0.5f ? 0.f : nd(rng) * s;
        }
    for (auto& b : hB) b = nd(rng) * 0.02f;                // packed weights
    float *dA, *dB, *r32;
    double* r64;
    int *ea, *eb;
    CK(hipMalloc(&dA, hA.size() * 4));
    CK(hipMalloc(&dB, hB.size() * 4));
    CK(hipMalloc(&ea, M * 4));
    CK(hipMalloc(&eb, N * 4));
    CK(hipMalloc(&r64, (size_t)R * N * 8));
    CK(hipMalloc(&r32, (size_t)R * N * 4));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
    k_rowexp<<<(M + 255) / 256, 256>>>(dA, M, ea);
    k_rowexp<<<1, N>>>(dB, N, eb);
    k_ref<<<(R * N + 255) / 256, 256>>>(dA, dB, R, r64, r32);
    CK(hipDeviceSynchronize());
    std::vector<float> h32((size_t)R * N);
    CK(hipMemcpy(h32.data(), r32, h32.size() * 4, hipMemcpyDeviceToHost));
    printf("M = %d rows, N = %d, K = %d (conv6 data gradient; the product's fp32 direct kernel: "
           "12.7 ms per 16,384-sample launch, 140 TF/s)\n", M, N, K);
    run<3, 1>(M, dA, dB, ea, eb, r64, h32, R);
    run<3, 2>(M, dA, dB, ea, eb, r64, h32, R);
    run<4, 1>(M, dA, dB, ea, eb, r64, h32, R);
    run<4, 2>(M, dA, dB, ea, eb, r64, h32, R);
    run<5, 1>(M, dA, dB, ea, eb, r64, h32, R);
    run<5, 2>(M, dA, dB, ea, eb, r64, h32, R);
    run<6, 1>(M, dA, dB, ea, eb, r64, h32, R);
    return 0;
}
