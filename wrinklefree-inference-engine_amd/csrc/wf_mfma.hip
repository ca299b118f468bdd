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

#include <algorithm>

#include "wf_common.h"
#include "wf_device.h"
#include "wf_norm.h"
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

template <int TNW, int ALG = 0>
__global__ __launch_bounds__(512) void k_pgemm_t(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                 float scale, int M, int N, int K, float* __restrict__ Y, int64_t ldy,
                                                 int nbm, int nbn) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[PgCfg<TNW, ALG>::LDS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    int bm, bn;
    WF_STAMP(0);
    pg_tile_of(blockIdx.x, nbm, nbn, bm, bn);
    v4i_t acc[4][TNW];
    pg_main<TNW, ALG>(W, A, M, N, K, bm, bn, lds, acc);
    WF_STAMP(11);
    // Epilogue through LDS, 64 rows x 256 columns at a time: the fp32 tile (row stride 272 floats:
    // the four lane quarters, 4 rows apart, land 16 banks apart) is written by fragment, then stored
    // as whole rows, one KiB per wave-instruction (the fragment layout would store 64-byte pieces).
    constexpr int kRs = 272;
    static_assert(64 * kRs * 4 <= PgCfg<TNW, ALG>::LDS, "epilogue tile fits the ring");
    float* tile = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int hh = 0; hh < TNW / 4; ++hh) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
            __syncthreads();  // every wave is done reading the ring / the previous piece
#pragma unroll
            for (int j = 0; j < TNW; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    constexpr bool CW = PgCfg<TNW, ALG>::CW;
                    const int rt = pg_frag_rt<TNW, CW>(wave, i, j);
                    const int ct = pg_frag_ct<TNW, CW>(wave, i, j) - 16 * hh;  // inside this 256-column half
                    if ((rt >> 2) != pr || ct < 0 || ct >= 16) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        tile[((rt & 3) * 16 + 4 * q + r) * kRs + ct * 16 + l16] = (float)acc[i][j][r] * scale;
                }
            __syncthreads();
            const int col = bn * pg_block_cols<TNW>() + hh * 256 + lane * 4;
            for (int rr = wave; rr < 64; rr += 8) {
                const int row = bm * 128 + 64 * pr + rr;
                const float4 v = *reinterpret_cast<const float4*>(tile + rr * kRs + lane * 4);
                if (row < M && col < N) *reinterpret_cast<float4*>(Y + (int64_t)row * ldy + col) = v;
            }
        }
    }
}

// int8 codes [M][lda] -> tile order (one thread per 16-byte output piece; rows >= M are zero).
__global__ void k_codes_to_tiles(const int8_t* __restrict__ a, int64_t lda, int M, int K, int8_t* __restrict__ out,
                                 int64_t pieces) {
    const int nkb = K >> 7;
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < pieces; o += (int64_t)gridDim.x * blockDim.x) {
        const int l = (int)(o & 63), h = (int)((o >> 6) & 1);
        const int64_t tb = o >> 7;  // (row tile, block)
        const int kb = (int)(tb % nkb), rt = (int)(tb / nkb);
        const int row = 16 * rt + (l & 15), q = l >> 4;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
        if (row < M) {
            const int8_t* src = a + (int64_t)row * lda + 128 * kb + 16 * h + 4 * q;
#pragma unroll
            for (int g = 0; g < 4; ++g) v[g] = *reinterpret_cast<const uint32_t*>(src + 32 * g);
        }
        *reinterpret_cast<uint4*>(out + 16 * o) = make_uint4(v[0], v[1], v[2], v[3]);
    }
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

using namespace wf;

WF_STAMP_READER(wf_debug_stamps_mfma)

extern "C" int wf_codes_to_tiles(const int8_t* a, int64_t lda, int M, int K, int8_t* out, void* stream) {
    WF_REQUIRE(a && out && M > 0 && K > 0 && K % 128 == 0 && lda >= K && lda % 4 == 0 && ((uintptr_t)a & 3u) == 0,
               "codes_to_tiles: bad arguments (K %% 128 == 0, 4-byte aligned rows)");
    const int64_t pieces = (int64_t)(M + 15) / 16 * (K / 128) * 128;
    const int grid = (int)std::min<int64_t>((pieces + 255) / 256, 8192);
    hipLaunchKernelGGL(k_codes_to_tiles, dim3(grid), dim3(256), 0, as_stream(stream), a, lda, M,
                       K, out, pieces);
    return check_launch("codes_to_tiles");
}

extern "C" int wf_bitnet_gemm_tiled(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y,
                                    int64_t ldy, void* stream) {
    WF_REQUIRE(w && a && y && M > 0 && N > 0 && K > 0, "gemm_tiled: bad arguments");
    WF_REQUIRE(K % 128 == 0 && N % 16 == 0, "gemm_tiled: K %% 128 == 0 and N %% 16 == 0 required (K=%d N=%d)", K, N);
    WF_REQUIRE(ldy >= N && ldy % 4 == 0 && aligned16(a) && aligned16(w) && aligned16(y),
               "gemm_tiled: bad ldy or unaligned operands (ldy %% 4 == 0, 16-byte aligned pointers)");
    const int nbm = (M + 127) / 128;
#define WF_PGT(TNWV, ALGV, NBN) \
    hipLaunchKernelGGL((k_pgemm_t<TNWV, ALGV>), dim3(nbm * (NBN)), dim3(512), 0, as_stream(stream), w, a, scale, M, N, K, y, \
                       ldy, nbm, NBN)
    if (pg_wide(N))  // 512-column tiles: column-wave (CW) main loop (standalone gate|up 565 -> 523 us)
        WF_PGT(8, 3, (N + 511) / 512);
    else  // 256-column tiles: 2 x 4 wave grid (CW reads all 8 A row tiles per stage: over the LDS rate)
        WF_PGT(4, 0, (N + 255) / 256);
#undef WF_PGT
    return check_launch("gemm_tiled");
}
