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

namespace wf {

typedef int v4i __attribute__((ext_vector_type(4)));

// Block = 4 waves arranged WR x WC; each wave owns TMW x TNW 16x16 tiles:
// block tile = (WR * TMW * 16) rows x (WC * TNW * 16) columns.
template <int WR, int WC, int TMW, int TNW>
__global__ __launch_bounds__(256) void k_tgemm_mfma(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                    int64_t lda, float scale, int M, int N, int K,
                                                    float* __restrict__ Y, int64_t ldy) {
    static_assert(WR * WC == 4, "4 waves per block");
    constexpr int BM = WR * TMW * 16, BN = WC * TNW * 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int l16 = lane & 15, q = lane >> 4;
    const int wr = wave / WC, wc = wave % WC;
    const int m_base = blockIdx.y * BM + wr * TMW * 16;
    const int n_base = blockIdx.x * BN + wc * TNW * 16;
    const int64_t wrow = K / 4;

    const uint8_t* wp[TNW];
#pragma unroll
    for (int j = 0; j < TNW; ++j) wp[j] = W + (int64_t)min(n_base + 16 * j + l16, N - 1) * wrow;
    const int8_t* ap[TMW];
#pragma unroll
    for (int i = 0; i < TMW; ++i) ap[i] = A + (int64_t)min(m_base + 16 * i + l16, M - 1) * lda + 32 * q;
    const int sh = 6 - 2 * q;

    v4i acc[TMW][TNW];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = v4i{0, 0, 0, 0};

    const int steps = K / 64;  // K % 128 == 0
#pragma unroll 2
    for (int c = 0; c < steps; ++c) {
        const int boff = 32 * (c >> 1) + 16 * (c & 1);   // byte offset of the 64-weight group
        const int koff = 128 * (c >> 1) + 16 * (c & 1);  // its first activation
        v4i bf[TNW];
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            const uint4 w = ldg_nt(wp[j] + boff);
            bf[j] = v4i{(int)((w.x >> sh) & 0x03030303u), (int)((w.y >> sh) & 0x03030303u),
                        (int)((w.z >> sh) & 0x03030303u), (int)((w.w >> sh) & 0x03030303u)};
        }
        v4i af[TMW];
#pragma unroll
        for (int i = 0; i < TMW; ++i) af[i] = *reinterpret_cast<const v4i*>(ap[i] + koff);
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            const int n = n_base + 16 * j + l16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m_base + 16 * i + 4 * q + r;
                if (m < M && n < N) Y[(int64_t)m * ldy + n] = (float)acc[i][j][r] * scale;
            }
        }
}

// M >= 16, I2_S, K % 128 == 0, 16-byte aligned rows (checked by the caller).
int launch_tgemm_mfma(const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K, float* y,
                      int64_t ldy, hipStream_t st) {
    if (M >= 512) {  // prefill-sized: 128 x 128 block tiles, 2 x 2 waves of 4 x 4 MFMA tiles
        const dim3 grid((N + 127) / 128, (M + 127) / 128);
        hipLaunchKernelGGL((k_tgemm_mfma<2, 2, 4, 4>), grid, dim3(256), 0, st, w, a, lda, scale, M, N, K, y, ldy);
    } else {  // batched decode: 128 x 16 block tiles -> N / 16 blocks
        const dim3 grid((N + 15) / 16, (M + 127) / 128);
        hipLaunchKernelGGL((k_tgemm_mfma<4, 1, 2, 1>), grid, dim3(256), 0, st, w, a, lda, scale, M, N, K, y, ldy);
    }
    return check_launch("tgemm_mfma");
}

}  // namespace wf
