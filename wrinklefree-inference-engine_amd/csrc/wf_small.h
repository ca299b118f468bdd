// wf_small.h -- small-M ternary GEMM on the int8 matrix cores over row-major operands (gfx950),
// shared by the raw GEMM (wf_gemv.hip, sgl_kernel bitnet_gemm) and the fused BitNetLinear
// (wf_decode.hip wf_bitnet_linear_fused).
//
// The 128 x 64 LDS-DMA tiles of the batched GEMM stage 128 activation rows through a one-CU ring and
// give the 2560-row down projection 40 blocks (41 us at M = 16), while the VALU stream re-reads the
// activations from LDS once per row (7.8 / 12.4 us at M = 4 / 8; scripts/benchmark_kernels.py:140,
// 162-170 sweeps M 1-32 on that layer). Here a block owns TNT 16-row weight tiles and TMT 16-row
// activation tiles: v_mfma_i32_16x16x64_i8 with B = the weight rows, A = the activation rows, so every
// product is useful; 8 waves split the row's 64-byte chunks. Lane (n, q) loads bytes [64 j + 16 q, +16)
// of weight row n (16 rows x 64 contiguous bytes per instruction) and masks each I2_S group in place
// (32 / 16 / 4 / 1 x code, one accumulator per group, divided out exactly at the end); the group-g
// fields of its four dwords are the codes of k = 256 j + 128 (q >> 1) + 16 (q & 1) + 32 g + 0..15,
// sixteen consecutive activation bytes lane (m, q) loads from row m. The waves' int32 tiles meet in
// LDS and wave (t, c) hands output tile (t, c) to the epilogue in the MFMA C layout (lane (n, q): rows
// 4 q .. 4 q + 3 of column n). Integer sums: bit-exact with any k order.
#pragma once
#include "wf_device.h"

namespace wf {

typedef int v4i_t __attribute__((ext_vector_type(4)));
#ifndef WF_GS_MAXM  // study: largest M on the small-M kernel (above: the 128 x 64 / 128 x 128 LDS-DMA tiles)
#define WF_GS_MAXM 256
#endif
constexpr int kSmallMaxM = WF_GS_MAXM;

template <int TMT, int TNT, int PRE, class Epi>
__global__ __launch_bounds__(512) void k_gemm_small_mfma(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                         int64_t lda, int M, int N, int K, Epi e) {
    constexpr int NW = 8;
    static_assert(TMT * TNT <= NW, "one output tile per storing wave");
    __shared__ v4i_t red[NW][TMT * TNT][64];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16 * TNT, m0 = blockIdx.y * 16 * TMT;
    const int rb = K >> 2, J = (rb + 63) >> 6;  // 64-byte chunks per weight row (the last may be half)
    const uint8_t* wr[TNT];
#pragma unroll
    for (int c = 0; c < TNT; ++c) wr[c] = W + (int64_t)min(n0 + 16 * c + l16, N - 1) * rb;
    const int8_t* ar[TMT];
#pragma unroll
    for (int t = 0; t < TMT; ++t) ar[t] = A + (int64_t)min(m0 + 16 * t + l16, M - 1) * lda;
    v4i_t ac[TMT][TNT][4];
#pragma unroll
    for (int t = 0; t < TMT; ++t)
#pragma unroll
        for (int c = 0; c < TNT; ++c)
#pragma unroll
            for (int g = 0; g < 4; ++g) ac[t][c][g] = v4i_t{0, 0, 0, 0};
    for (int j0 = wave; j0 < J; j0 += NW * PRE) {
        uint4 w[PRE][TNT];
        v4i_t af[PRE][TMT][4];
#pragma unroll
        for (int u = 0; u < PRE; ++u) {  // clamped loads (vmcnt stays exact); invalid chunks zeroed below
            const int j = min(j0 + NW * u, J - 1);
#pragma unroll
            for (int c = 0; c < TNT; ++c) w[u][c] = ldg_nt(wr[c] + min(64 * j + 16 * q, rb - 16));
            const int k0 = 256 * j + 128 * (q >> 1) + 16 * (q & 1);
#pragma unroll
            for (int t = 0; t < TMT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) af[u][t][g] = *reinterpret_cast<const v4i_t*>(ar[t] + min(k0 + 32 * g, K - 16));
        }
#pragma unroll
        for (int u = 0; u < PRE; ++u) {
            const int j = j0 + NW * u;
            if (j >= J) break;  // wave-uniform
            const bool valid = 64 * j + 16 * q < rb;
#pragma unroll
            for (int c = 0; c < TNT; ++c) {
                const uint4 x = valid ? w[u][c] : make_uint4(0, 0, 0, 0);
                const v4i_t bf[4] = {
                    v4i_t{(int)((x.x >> 1) & 0x60606060u), (int)((x.y >> 1) & 0x60606060u), (int)((x.z >> 1) & 0x60606060u),
                          (int)((x.w >> 1) & 0x60606060u)},
                    v4i_t{(int)(x.x & 0x30303030u), (int)(x.y & 0x30303030u), (int)(x.z & 0x30303030u), (int)(x.w & 0x30303030u)},
                    v4i_t{(int)(x.x & 0x0c0c0c0cu), (int)(x.y & 0x0c0c0c0cu), (int)(x.z & 0x0c0c0c0cu), (int)(x.w & 0x0c0c0c0cu)},
                    v4i_t{(int)(x.x & 0x03030303u), (int)(x.y & 0x03030303u), (int)(x.z & 0x03030303u), (int)(x.w & 0x03030303u)}};
#pragma unroll
                for (int t = 0; t < TMT; ++t)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        ac[t][c][g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[u][t][g], bf[g], ac[t][c][g], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < TMT; ++t)
#pragma unroll
        for (int c = 0; c < TNT; ++c)
            red[wave][t * TNT + c][lane] = (ac[t][c][0] + 2 * ac[t][c][1] + 8 * ac[t][c][2] + 32 * ac[t][c][3]) >> 5;
    __syncthreads();
    if (wave >= TMT * TNT) return;  // wave = output tile (t, c): lane (n, q) holds rows 4 q .. 4 q + 3 of column n
    v4i_t sum = red[0][wave][lane];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) sum += red[w2][wave][lane];
    const int t = wave / TNT, c = wave % TNT;
    e.apply(m0 + 16 * t, n0 + 16 * c, sum, l16, q);
}

// Tile policy (same-box sweep on the down projection, tools/ab_gemm_sweep.sh, us per call at M = 2 /
// 4 / 8 / 16 / 32 / 64 / 128): 16 x 16 tiles 4.4 / 4.8 / 5.5 / 6.8 (16 x 32: 5.3 / 5.8 / 6.9 / 8.9);
// 32 x 16 at M = 32 10.8 (32 x 32: 13.0); 32 x 32 at M = 64 / 128 12.7 / 23.7 (32 x 16: 19.8 / --;
// the 128 x 64 LDS-DMA tiles: 42.4 / 44.0) -- about 160 blocks for the 2560-row projection. At
// K = 2560 (BitNetLinear, tools/ab_linear.sh) 32 x 32 is the faster tile at M = 32 as well.
// Whether (M, N) belongs on this kernel: up to 128 rows, up to kSmallMaxM on narrow layers (at M = 256
// the 6912-row gate|up projection is faster on the 128 x 128 tiles: 33 vs 48 us, tools/ab_linear.sh).
inline bool gemm_small_ok(int M, int N) { return M >= 2 && M <= kSmallMaxM && (M <= 128 || N < 4096); }
template <class Epi>
void launch_gemm_small_mfma(const uint8_t* w, const int8_t* a, int64_t lda, int M, int N, int K, const Epi& e,
                            hipStream_t st) {
#define WF_GS(TMTV, TNTV, PREV)                                                                                          \
    hipLaunchKernelGGL((k_gemm_small_mfma<TMTV, TNTV, PREV, Epi>), dim3((N + 16 * TNTV - 1) / (16 * TNTV), (M + 16 * TMTV - 1) / (16 * TMTV)), \
                       dim3(512), 0, st, w, a, lda, M, N, K, e)
    if (K > 4096) {  // long rows (the down projection): the sweep's tiles
        if (M <= 16) WF_GS(1, 1, 4);
        else if (M <= 32) WF_GS(2, 1, 4);
        else WF_GS(2, 2, 2);
    } else {  // K <= 4096: 32 weight rows per block from M = 2 on (half the blocks, twice the work each)
        if (M <= 16) WF_GS(1, 2, 2);
        else WF_GS(2, 2, 2);
    }
#undef WF_GS
}

}  // namespace wf
