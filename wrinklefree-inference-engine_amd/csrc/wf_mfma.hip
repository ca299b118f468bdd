// wf_mfma.hip -- ternary x int8 GEMM on the gfx950 matrix cores (batched decode M >= 16, prefill).
//
// Y[m, n] = float(sum_k enc(W[n, k]) * A[m, k]) * scale   (sgl-kernel bitnet_gemm semantics,
// tests/test_bitnet_core.py:149-167), W in the reference's blocked I2_S layout [N][K/4]
// (cache/bitnet_converter.py:26-77), A int8 [M][lda].
//
// v_mfma_i32_16x16x64_i8: lane l holds 16 int8 of A (row l & 15) and 16 of B (column l & 15) for
// its quarter q = l >> 4 of the 64-deep k step; A and B use the same (quarter, element) -> k map,
// so ANY consistent assignment of the 64 k of a step to (q, j) computes the same dot product. We
// pick the assignment the I2_S bytes give for free: the 16 bytes [32b + 16h, +16) of a weight row
// hold the 64 weights k = 128b + 16h + j + 32g (g = 0..3 at bit offsets 6, 4, 2, 0), so quarter q
// takes bit offset 6 - 2q -- one 16-byte load and four shift/masks per lane give the whole B
// fragment -- and its A fragment is the 16 contiguous activations at k = 128b + 16h + 32q.
// C/D layout (dtype-independent on gfx950): lane l holds D[row 4q + r][col l & 15], r < 4.
// The int32 sums are exact, so the result is bit-exact with the oracle for any tile order.
#include <hip/hip_runtime.h>

#include "wf_common.h"
#include "wf_device.h"
#include "wf_mfma.h"

namespace wf {


// Raw sgl-kernel epilogue: Y[m, n] = float(sum) * scale.
struct EpiRaw {
    float* Y;
    int64_t ldy;
    float scale;
    int M, N;
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) {
        const int n = c0 + l16;
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r0 + 4 * q + r;
            if (m < M) Y[(int64_t)m * ldy + n] = (float)acc[r] * scale;
        }
    }
};

template <int WR, int P>
__global__ __launch_bounds__(256) void k_tgemm_lds(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                   int64_t lda, float scale, int M, int N, int K, float* __restrict__ Y,
                                                   int64_t ldy) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[P * kTgStageBytes];
    EpiRaw e{Y, ldy, scale, M, N};
    tgemm_tile<WR, P>(W, A, lda, M, N, K, blockIdx.y * 128, blockIdx.x * 64 * (4 / WR), lds, e);
}

// M >= 16, I2_S, K % 128 == 0, 16-byte aligned rows (checked by the caller).
int launch_tgemm_mfma(const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K, float* y,
                      int64_t ldy, hipStream_t st) {
    if (M >= 512) {  // prefill-sized: 128 x 128 tiles (2 x 2 waves of 4 x 4 MFMA tiles)
        hipLaunchKernelGGL((k_tgemm_lds<2, kTgStagesWide>), dim3((N + 127) / 128, (M + 127) / 128), dim3(256), 0, st, w,
                           a, lda, scale, M, N, K, y, ldy);
    } else {  // batched decode: 128 x 64 tiles (4 x 1 waves of 2 x 4 MFMA tiles), twice the blocks
        hipLaunchKernelGGL((k_tgemm_lds<4, kTgStagesDeep>), dim3((N + 63) / 64, (M + 127) / 128), dim3(256), 0, st, w, a,
                           lda, scale, M, N, K, y, ldy);
    }
    return check_launch("tgemm_mfma");
}

}  // namespace wf
