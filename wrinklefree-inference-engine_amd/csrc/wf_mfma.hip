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

// ---------------------------------------------------------------------------------------------
// Prefill GEMM on the matrix-core tile layouts (BASELINE configs[2]: M = 2048 x 8 token rows).
// Operands as the batched decode step keeps them: W in WF_FMT_I2S_MFMA (512 contiguous bytes per
// (16-column tile, I2_S block)), A in tile-ordered codes (wf_norm.h tile_code_pos: 1 KiB per
// (16-row tile, block, half)). Every LDS-DMA wave-instruction therefore moves whole 128-byte lines
// (A: one contiguous KiB; W: two contiguous 512-byte runs), unlike the row-major A of k_tgemm_lds
// (16 rows x 64 bytes per instruction).
//
// Block = 8 waves, tile 128 rows x 256 columns (the weight columns are the wide side: the int8
// codes cost 1 byte per k and row, the weights 1/4 byte per k and column, so bytes per MAC =
// 1/BN + 1/(4 BM) = 0.0059 -> ~24 B/clk/CU from L2 at the full MFMA rate). Wave (wr, wc), wr < 2,
// wc < 4, owns row tiles [4 wr, +4) x column tiles [4 wc, +4): 16 accumulators, 32
// v_mfma_i32_16x16x64_i8 per I2_S block. One pipeline stage = one I2_S block (k = 128):
// A 8 row tiles x 2 KiB + W 16 column tiles x 512 B = 24 KiB; every wave issues exactly 3 LDS-DMA
// loads per stage (its row tile's two halves and column tiles 2w, 2w+1), so a counted
// `s_waitcnt vmcnt(3 (P-2))` + s_barrier publishes a stage with P-2 more in flight (the wf_mfma.h
// scheme). Blocks are mapped XCD-aware: the launch's round-robin dispatch gives XCD x a contiguous
// range of logical tiles, walked in groups of 4 row blocks x all column blocks, so the A slabs and
// weight columns a XCD's 32 resident blocks share stay in its L2.
// ---------------------------------------------------------------------------------------------
constexpr int kPgStage = 8 * 2048 + 16 * 512;  // 24 KiB
constexpr int kPgStages = 6;                    // 144 KiB: one block per CU, 4 stages in flight
constexpr int kPgGroupRows = 4;

// XCD-aware grouped tile order (measured: 4 % less time than plain row-major order)
__device__ __forceinline__ void pg_tile_of(int bid, int nbm, int nbn, int& bm, int& bn) {
    const int nblk = nbm * nbn, full = nblk / 8 * 8;
    const int L = bid < full ? (bid % 8) * (nblk / 8) + bid / 8 : bid;
    const int g = L / (kPgGroupRows * nbn), t = L % (kPgGroupRows * nbn);
    const int rows = min(kPgGroupRows, nbm - g * kPgGroupRows);
    bm = g * kPgGroupRows + t % rows;
    bn = t / rows;
}

// Fragments of one stage for one wave: A row tiles 4 wr + i (both halves), W column tiles 4 wc + j.
struct PgFrag {
    v4i_t a[2][4];
    uint2 w[4];
};

// The fragments of stage c are read from LDS one iteration ahead (while the MFMAs of stage c - 1
// run), so the matrix pipe never waits on an LDS round trip after the barrier. Iteration c: wait
// for stage c + 1 (vmcnt: stages c + 2 .. c + P - 2 may stay in flight), barrier, refill the slot
// of stage c - 1 (its fragments were consumed by the MFMAs of iteration c - 1, before the
// barrier), read stage c + 1's fragments, run stage c's MFMAs.
template <int P>
__global__ __launch_bounds__(512) void k_pgemm_t(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                 float scale, int M, int N, int K, float* __restrict__ Y, int64_t ldy,
                                                 int nbm, int nbn) {
    static_assert(P >= 4, "two stages in flight beyond the one being read");
    __shared__ __attribute__((aligned(16))) uint8_t lds[P * kPgStage];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int wr = wave >> 2, wc = wave & 3;
    int bm, bn;
    pg_tile_of(blockIdx.x, nbm, nbn, bm, bn);
    const int nkb = K >> 7, nrt = (M + 15) >> 4, nct = N >> 4;
    // DMA sources: A row tile 8 bm + wave (both halves), W column tiles 16 bn + 2 wave + (lane >= 32)
    const int rt = min(bm * 8 + wave, nrt - 1);
    const int8_t* asrc = A + ((int64_t)rt * nkb << 11) + lane * 16;
    const int ct = min(bn * 16 + 2 * wave + (lane >> 5), nct - 1);
    const uint8_t* wsrc = W + ((int64_t)ct * nkb << 9) + (lane & 31) * 16;
    auto issue = [&](int kb) {
        uint8_t* st = lds + (kb % P) * kPgStage;
        glds16_asm(asrc + ((int64_t)kb << 11), st + wave * 2048);
        glds16_asm(asrc + ((int64_t)kb << 11) + 1024, st + wave * 2048 + 1024);
        glds16_asm(wsrc + ((int64_t)kb << 9), st + 16384 + wave * 1024);
    };
    auto read = [&](PgFrag& f, int kb) {
        const uint8_t* st = lds + (kb % P) * kPgStage;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.w[j] = *reinterpret_cast<const uint2*>(st + 16384 + (4 * wc + j) * 512 + lane * 8);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                f.a[h][i] = *reinterpret_cast<const v4i_t*>(st + (4 * wr + i) * 2048 + h * 1024 + lane * 16);
    };
    v4i_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v4i_t{0, 0, 0, 0};
    auto mma = [&](const PgFrag& f) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            v4i_t bf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t w = h ? f.w[j].y : f.w[j].x;
                bf[j] = v4i_t{(int)((w >> 6) & 0x03030303u), (int)((w >> 4) & 0x03030303u),
                              (int)((w >> 2) & 0x03030303u), (int)(w & 0x03030303u)};
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[h][i], bf[j], acc[i][j], 0, 0, 0);
        }
    };
    // one iteration: stage c + 1 published and read into `nxt`, stage c computed from `cur`
    auto step = [&](int c, PgFrag& cur, PgFrag& nxt) {
        if (c + 1 < nkb) {
            if (c + P - 2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (P - 3)) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (c + P - 1 < nkb) issue(c + P - 1);
            read(nxt, c + 1);
        }
        mma(cur);
    };
#pragma unroll
    for (int c = 0; c < P - 1; ++c)
        if (c < nkb) issue(c);
    PgFrag f0, f1;
    if (P - 2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (P - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    read(f0, 0);
    int c = 0;
    for (; c + 1 < nkb; c += 2) {
        step(c, f0, f1);
        step(c + 1, f1, f0);
    }
    if (c < nkb) step(c, f0, f1);
    // Epilogue through LDS: the 128 x 256 fp32 tile (row stride 272 floats: the four lane quarters,
    // 4 rows apart, land 16 banks apart) is written by fragment, then stored as whole rows, one KiB
    // per wave-instruction (the fragment layout would store 64-byte pieces of 4 rows each).
    constexpr int kRs = 272;
    static_assert(128 * kRs * 4 <= P * kPgStage, "epilogue tile fits the ring");
    float* tile = reinterpret_cast<float*>(lds);
    __syncthreads();  // every wave is done reading the ring
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                tile[((4 * wr + i) * 16 + 4 * q + r) * kRs + (4 * wc + j) * 16 + l16] = (float)acc[i][j][r] * scale;
    __syncthreads();
    const int col = bn * 256 + lane * 4;
    for (int rr = wave; rr < 128; rr += 8) {
        const int row = bm * 128 + rr;
        const float4 v = *reinterpret_cast<const float4*>(tile + rr * kRs + lane * 4);
        if (row < M && col < N) *reinterpret_cast<float4*>(Y + (int64_t)row * ldy + col) = v;
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
    const int nbm = (M + 127) / 128, nbn = (N + 255) / 256;
    hipLaunchKernelGGL((k_pgemm_t<kPgStages>), dim3(nbm * nbn), dim3(512), 0, as_stream(stream), w, a, scale, M, N, K,
                       y, ldy, nbm, nbn);
    return check_launch("gemm_tiled");
}
