// How v_mfma_f32_16x16x32_bf16 rounds (development tool, not part of libflsim.so): one wave, one
// instruction per case, every lane's A/B pair chosen so that output (0,0) receives a known set of
// exact products on top of a known accumulator; the result is compared with the exact sum rounded
// to nearest even (RNE), toward zero (RTZ) and with a sequential fmaf chain.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/lab/mfma_numerics.hip -o tools/lab/mfma_numerics
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// A[16][32], B[32][16] bf16 row-major; C in [16][16]; one MFMA
__global__ void k_one(const __bf16* A, const __bf16* B, const float* Cin, float* Cout) {
    const int lane = threadIdx.x;
    const int r = lane & 15, g = lane >> 4;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[r * 32 + 8 * g + j];
        b[j] = B[(8 * g + j) * 16 + r];
    }
    f32x4 c;
    for (int i = 0; i < 4; ++i) c[i] = Cin[(4 * g + i) * 16 + r];
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) Cout[(4 * g + i) * 16 + r] = c[i];
}

static __bf16 bf(float x) {   // exact for the values used here
    uint32_t u;
    memcpy(&u, &x, 4);
    const uint16_t h = (uint16_t)(u >> 16);
    __bf16 r;
    memcpy(&r, &h, 2);
    return r;
}

struct Case {
    const char* name;
    float c;
    std::vector<std::pair<float, float>> ab;   // products for output (0,0): a_k * b_k
};

int main() {
    const float u = ldexpf(1.f, -23);          // ulp of 1.0
    std::vector<Case> cases = {
        {"c=1, one product 0.75 ulp", 1.f, {{0.75f * u, 1.f}}},
        {"c=1, one product 0.5 ulp (tie, even -> 1)", 1.f, {{0.5f * u, 1.f}}},
        {"c=1+ulp, one product 0.5 ulp (tie, even -> 1+2ulp)", 1.f + u, {{0.5f * u, 1.f}}},
        {"c=1, one product -0.75 ulp", 1.f, {{-0.75f * u, 1.f}}},
        {"c=1, 24 products of 2^-28 (1.5 ulp/2)", 1.f, std::vector<std::pair<float, float>>(24, {ldexpf(1.f, -28), 1.f})},
        {"c=1, 32 products of 2^-30 (0.125 ulp)", 1.f, std::vector<std::pair<float, float>>(32, {ldexpf(1.f, -30), 1.f})},
        {"c=0, 1.0 + 31 x 2^-26", 0.f, {}},
        {"c=0, 2^20 + 1 + 30 x (-1/32)", 0.f, {}},
        {"c=1, 16 x 2^-26 and 16 x -2^-27", 1.f, {}},
        {"c=2^-30, one product 1.0", ldexpf(1.f, -30), {{1.f, 1.f}}},
        {"c=0, products 1, 2^-24, 2^-24", 0.f, {{1.f, 1.f}, {ldexpf(1.f, -24), 1.f}, {ldexpf(1.f, -24), 1.f}}},
        {"c=1, products 2^-25 x 8", 1.f, std::vector<std::pair<float, float>>(8, {ldexpf(1.f, -25), 1.f})},
        {"c=1, products 2^-26 x 16", 1.f, std::vector<std::pair<float, float>>(16, {ldexpf(1.f, -26), 1.f})},
        {"c=1, products 2^-27 x 32", 1.f, std::vector<std::pair<float, float>>(32, {ldexpf(1.f, -27), 1.f})},
        {"c=0, 2^8 + products 2^-16 x 2 (needs 25 bits)", 0.f, {{256.f, 1.f}, {ldexpf(1.f, -16), 1.f}, {ldexpf(1.f, -16), 1.f}}},
        {"c=0, 2^8 + products 2^-17 x 2", 0.f, {{256.f, 1.f}, {ldexpf(1.f, -17), 1.f}, {ldexpf(1.f, -17), 1.f}}},
        {"c=0, 2^8 + products 2^-18 x 4", 0.f, {{256.f, 1.f}, {ldexpf(1.f, -18), 1.f}, {ldexpf(1.f, -18), 1.f}, {ldexpf(1.f, -18), 1.f}, {ldexpf(1.f, -18), 1.f}}},
    };
    // fill the composite cases
    cases[6].ab.push_back({1.f, 1.f});
    for (int i = 0; i < 31; ++i) cases[6].ab.push_back({ldexpf(1.f, -26), 1.f});
    cases[7].ab.push_back({1048576.f, 1.f});
    cases[7].ab.push_back({1.f, 1.f});
    for (int i = 0; i < 30; ++i) cases[7].ab.push_back({-1.f / 32, 1.f});
    for (int i = 0; i < 16; ++i) cases[8].ab.push_back({ldexpf(1.f, -26), 1.f});
    for (int i = 0; i < 16; ++i) cases[8].ab.push_back({-ldexpf(1.f, -27), 1.f});

    __bf16 *dA, *dB;
    float *dC, *dO;
    CK(hipMalloc(&dA, 16 * 32 * 2));
    CK(hipMalloc(&dB, 32 * 16 * 2));
    CK(hipMalloc(&dC, 256 * 4));
    CK(hipMalloc(&dO, 256 * 4));
    for (const Case& cs : cases) {
        std::vector<__bf16> A(16 * 32, bf(0.f)), B(32 * 16, bf(0.f));
        std::vector<float> C(256, 0.f), O(256);
        C[0] = cs.c;
        double exact = cs.c;
        float chain = cs.c;
        for (size_t k = 0; k < cs.ab.size(); ++k) {
            A[k] = bf(cs.ab[k].first);
            B[k * 16] = bf(cs.ab[k].second);
            exact += (double)cs.ab[k].first * cs.ab[k].second;
            chain = fmaf(cs.ab[k].first, cs.ab[k].second, chain);
        }
        CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, dA, dB, dC, dO);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(O.data(), dO, 1024, hipMemcpyDeviceToHost));
        const float rne = (float)exact;
        // toward zero
        float rtz = rne;
        if (fabs((double)rne) > fabs(exact)) rtz = nextafterf(rne, 0.f);
        const double ulp = (double)nextafterf(fabsf(rne), INFINITY) - fabsf(rne);
        printf("%-52s mfma %.10e | exact %.10e | rne %.10e rtz %.10e fmaf-chain %.10e | (mfma-exact)/ulp %+.3f  %s\n",
               cs.name, O[0], exact, rne, rtz, chain, ((double)O[0] - exact) / ulp,
               O[0] == rne ? "=RNE" : (O[0] == rtz ? "=RTZ" : (O[0] == chain ? "=chain" : "other")));
    }
    return 0;
}
