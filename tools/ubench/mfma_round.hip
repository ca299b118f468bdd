// Rounding behaviour of the bf16 MFMA's accumulation (v_mfma_f32_32x32x16_bf16 /
// v_mfma_f32_16x16x32_bf16): each case puts chosen bf16 products in row 0 / column 0 of the tile
// and a chosen C, and prints D[0][0] next to the RN and RZ results of the exact sum.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/mfma_round.hip -o tools/ubench/mfma_round
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <cmath>
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k16(const uint16_t* a, const uint16_t* b, float c0, float* out) {
    // 16x16x32: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]
    const int l = threadIdx.x;
    v8s av, bv;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (l >> 4) + j;
        av[j] = (l & 15) == 0 ? (short)a[k] : 0;
        bv[j] = (l & 15) == 0 ? (short)b[k] : 0;
    }
    v4f c = {0.f, 0.f, 0.f, 0.f};
    if (l == 0) c[0] = c0;  // C/D: col = l&15, row = 4(l>>4)+r
    const v4f d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
    if (l == 0) out[0] = d[0];
}
__global__ void k32(const uint16_t* a, const uint16_t* b, float c0, float* out) {
    // 32x32x16: lane l (r = l&31, h = l>>5) holds A[row r][k 8h+j], B[k 8h+j][col r]
    const int l = threadIdx.x;
    v8s av, bv;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (l >> 5) + j;
        av[j] = (l & 31) == 0 ? (short)a[k] : 0;
        bv[j] = (l & 31) == 0 ? (short)b[k] : 0;
    }
    v16f c = {};
    if (l == 0) c[0] = c0;  // col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5)
    const v16f d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
    if (l == 0) out[0] = d[0];
}
static uint16_t bf(float x) { uint32_t u; memcpy(&u, &x, 4); return (uint16_t)(u >> 16); }  // exact inputs only
static float rz(double x) { float f = (float)x; if (fabs((double)f) > fabs(x)) f = nextafterf(f, 0.f); return f; }
int main() {
    uint16_t *da, *db; float* dout;
    hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dout, 4);
    struct Case { const char* name; int n; float a[32]; float c0; };
    const float u = ldexpf(1.f, -24);
    Case cs[] = {
        {"1 + 0.75 ulp (products)", 2, {1.f, 1.5f * u}, 0.f},
        {"-(1 + 0.75 ulp)", 2, {-1.f, -1.5f * u}, 0.f},
        {"C=1, products 0.75 ulp", 1, {1.5f * u}, 1.f},
        {"C=1, products 0.25 ulp", 1, {0.5f * u}, 1.f},
        {"1 + 16 x 2^-26", 17, {1.f, ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26),
                               ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26),
                               ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26)}, 0.f},
        {"C=1 + 8 x 2^-26", 8, {ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26), ldexpf(1,-26),
                                ldexpf(1,-26), ldexpf(1,-26)}, 1.f},
        {"2^20 - 2^20 + 2^-10 (cancel)", 3, {1048576.f, -1048576.f, ldexpf(1,-10)}, 0.f},
        {"1 + 2^-24 (tie, even down)", 2, {1.f, u}, 0.f},
        {"1 + 3*2^-24 (tie, even up)", 2, {1.f, 3 * u}, 0.f},
    };
    for (auto& c : cs) {
        uint16_t a[32] = {}, b[32] = {};
        double ex = c.c0;
        for (int i = 0; i < c.n; ++i) { a[i] = bf(c.a[i]); b[i] = bf(1.f); ex += c.a[i]; }
        hipMemcpy(da, a, 64, hipMemcpyHostToDevice); hipMemcpy(db, b, 64, hipMemcpyHostToDevice);
        float r16 = NAN, r32 = NAN;
        if (c.n <= 32) { hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, c.c0, dout); hipMemcpy(&r16, dout, 4, hipMemcpyDeviceToHost); }
        if (c.n <= 16) { hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, da, db, c.c0, dout); hipMemcpy(&r32, dout, 4, hipMemcpyDeviceToHost); }
        printf("%-32s exact %.10e  RN %.10e RZ %.10e | 16x16x32 %.10e  32x32x16 %.10e\n", c.name, ex, (double)(float)ex,
               (double)rz(ex), (double)r16, (double)r32);
    }
    return 0;
}
