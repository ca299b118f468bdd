// wf_mfma.h -- LDS-DMA pipelined ternary x int8 GEMM on the gfx950 matrix cores (prefill and
// batched decode). Included by wf_mfma.hip (raw sgl-kernel epilogue) and wf_decode.hip (fused
// decode-step epilogues).
//
// Fragments (v_mfma_i32_16x16x64_i8; see wf_mfma.hip's header): in k-step c (64 weights) lane
// (l16 = lane & 15, q = lane >> 4) multiplies A[row l16][k = koff + 32q + 0..15] with
// enc(W[col l16][same k]); the I2_S bytes [boff, boff + 16) of a weight row hold all 64 weights of
// the step (quarter q at bit offset 6 - 2q), koff = 128(c>>1) + 16(c&1), boff = 32(c>>1) + 16(c&1).
//
// Block = 4 waves = WR x WC, tile 128 rows x (64 WC) columns; wave (wr, wc) owns row tiles
// [wr * 8/WR, +8/WR) and column tiles [4 wc, +4). Every k-step is one pipeline stage in LDS:
//   A: 8 KiB = 8 wave-loads (`global_load_lds_dwordx4`: a wave writes 1 KiB in lane order), wave w
//      loads row tiles 2w, 2w+1; slot (t, lane) <- A[16t + (lane & 15)][koff + 32 (lane >> 4)], so
//      the MFMA fragment of row tile t is the contiguous KiB t (conflict-free ds_read_b128).
//   B: 1 KiB per wave (its 64 columns' 16-byte weight groups; waves sharing wc load the same bytes
//      into their own slot), fragment of column tile j = slot 16j + l16 (4-lane broadcast).
// Every wave issues exactly 3 LDS-DMA loads per stage, so one counted `s_waitcnt vmcnt(3 (P-2))`
// retires its share of stage s with P-2 stages still in flight; a raw s_barrier then publishes the
// stage to all waves (no __syncthreads: it would drain the pipeline with vmcnt(0)). The stage the
// loop refills is the one every wave finished computing before that barrier.
#pragma once
#include "wf_device.h"

namespace wf {

typedef int v4i_t __attribute__((ext_vector_type(4)));

constexpr int kTgStageBytes = 8 * 1024 + 4 * 1024;  // A 8 KiB + 4 waves x 1 KiB of B
// LDS ring depth P: 4 (48 KiB, 3 blocks per CU) when the grid fills the chip (prefill); 12 (144 KiB,
// one block per CU, 11 stages = 132 KiB in flight) for the batched-decode grids of 20-200 blocks,
// whose time is the HBM/L2 latency of a shallow pipeline otherwise.
constexpr int kTgStagesWide = 4;
constexpr int kTgStagesDeep = 12;

__device__ __forceinline__ void glds16(const void* g, void* lds) {
    __builtin_amdgcn_global_load_lds(const_cast<void*>(g), reinterpret_cast<__attribute__((address_space(3))) void*>(
                                                               reinterpret_cast<uintptr_t>(lds)),
                                     16, 0, 0);
}

// The same LDS-DMA as inline asm: hipcc does not see it write LDS, so it does not put a
// `s_waitcnt vmcnt(0)` in front of every ds_read that might alias the DMA destination (with the
// builtin it does, which drains the whole ring before each stage's fragment reads). The caller
// counts completion with its own vmcnt + barrier (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void glds16_asm(const void* g, const void* lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(dst)
                 : "memory");
}

// The same with the non-temporal hint, for streams read once (the batched LM head's embedding tiles)
__device__ __forceinline__ void glds16_asm_nt(const void* g, const void* lds) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(dst)
                 : "memory");
}

// Epi::apply(i_tile_row0, j_tile_col0, acc, l16, q): called once per 16x16 output tile with its
// first row / column; lane holds D[row0 + 4q + r][col0 + l16], r < 4. k-steps [c_begin, c_end)
// (a split-K slice; the whole K is [0, K/64)).
template <int WR, int P, class Epi>
__device__ __forceinline__ void tgemm_tile(const uint8_t* __restrict__ W, const int8_t* __restrict__ A, int64_t lda,
                                           int M, int N, int K, int m0, int n0, uint8_t* lds, Epi& epi,
                                           int c_begin = 0, int c_end = -1) {
    constexpr int WC = 4 / WR;
    constexpr int TM = 8 / WR;  // row tiles per wave
    constexpr int TN = 4;       // column tiles per wave
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int wr = wave / WC, wc = wave % WC;
    if (c_end < 0) c_end = K / 64;
    const int steps = c_end - c_begin;
    // per-lane DMA sources: A rows of tiles 2w, 2w+1; B column of this wave's 64
    const int8_t* asrc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) asrc[u] = A + (int64_t)min(m0 + 16 * (2 * wave + u) + l16, M - 1) * lda + 32 * q;
    const uint8_t* bsrc = W + (int64_t)min(n0 + 64 * wc + lane, N - 1) * (K / 4);

    auto issue = [&](int cl) {  // cl: step within the slice
        uint8_t* st = lds + (cl % P) * kTgStageBytes;
        const int c = c_begin + cl;
        const int koff = 128 * (c >> 1) + 16 * (c & 1), boff = 32 * (c >> 1) + 16 * (c & 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) glds16_asm(asrc[u] + koff, st + (2 * wave + u) * 1024);
        glds16_asm(bsrc + boff, st + 8192 + wave * 1024);
    };

    v4i_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = v4i_t{0, 0, 0, 0};

#pragma unroll
    for (int c = 0; c < P - 1; ++c)
        if (c < steps) issue(c);
    const int sh = 6 - 2 * q;
    for (int c = 0; c < steps; ++c) {
        if (c + P - 2 < steps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (P - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (c + P - 1 < steps) issue(c + P - 1);
        const uint8_t* st = lds + (c % P) * kTgStageBytes;
        v4i_t af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const v4i_t*>(st + (wr * TM + i) * 1024 + lane * 16);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const uint4 w = *reinterpret_cast<const uint4*>(st + 8192 + wave * 1024 + (16 * j + l16) * 16);
            bf[j] = v4i_t{(int)((w.x >> sh) & 0x03030303u), (int)((w.y >> sh) & 0x03030303u),
                          (int)((w.z >> sh) & 0x03030303u), (int)((w.w >> sh) & 0x03030303u)};
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) epi.apply(m0 + 16 * (wr * TM + i), n0 + 64 * wc + 16 * j, acc[i][j], l16, q);
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
constexpr int kPgStage = 8 * 2048 + 16 * 512;  // 24 KiB (TNW = 4)
constexpr int kPgStages = 6;                    // 144 KiB: one block per CU, 4 stages in flight
constexpr int kPgGroupRows = 4;
// TNW column tiles per wave: 4 -> 128 x 256 block tiles (kPgStage, kPgStages), 8 -> 128 x 512 (a
// third fewer L2 -> LDS bytes per MAC: 1/512 + 1/512 instead of 1/256 + 1/512; 32 KiB stages)
template <int TNW>
constexpr int pg_stage_bytes() { return 8 * 2048 + TNW * 4 * 512; }
template <int TNW>
constexpr int pg_stages() { return TNW == 4 ? kPgStages : 4; }
template <int TNW>
constexpr int pg_block_cols() { return TNW * 64; }
// 512-column tiles where N fills them and there are enough of them for the chip
constexpr int kPgWideMinN = 8192;
inline bool pg_wide(int N) { return N % 512 == 0 && N >= kPgWideMinN; }

// XCD-aware grouped tile order (measured: 4 % less time than plain row-major order)
__device__ __forceinline__ void pg_tile_of(int bid, int nbm, int nbn, int& bm, int& bn) {
    const int nblk = nbm * nbn, full = nblk / 8 * 8;
    const int L = bid < full ? (bid % 8) * (nblk / 8) + bid / 8 : bid;
    const int g = L / (kPgGroupRows * nbn), t = L % (kPgGroupRows * nbn);
    const int rows = min(kPgGroupRows, nbm - g * kPgGroupRows);
    bm = g * kPgGroupRows + t % rows;
    bn = t / rows;
}

// The B fragments of one I2_S code pair (x: k-half 0, y: k-half 1): quarter q of each 32-bit word is
// (word >> (6 - 2q)) & 0x03030303. One 64-bit shift of (y:x) serves both words: the bits of y that
// enter x's top land in bits >= 26, above every kept 2-bit field (3 shifts + 8 ANDs for two
// fragments instead of 6 + 8). Inline asm: the compiler's demanded-bits pass splits a C++ 64-bit
// shift back into two 32-bit ones.
__device__ __forceinline__ void pg_decode_pair(uint2 wp, v4i_t& b0, v4i_t& b1) {
    const uint64_t w = ((uint64_t)wp.y << 32) | wp.x;
    uint64_t s6, s4, s2;
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(s6) : "v"(w));
    asm("v_lshrrev_b64 %0, 4, %1" : "=v"(s4) : "v"(w));
    asm("v_lshrrev_b64 %0, 2, %1" : "=v"(s2) : "v"(w));
    constexpr uint32_t M = 0x03030303u;
    b0 = v4i_t{(int)((uint32_t)s6 & M), (int)((uint32_t)s4 & M), (int)((uint32_t)s2 & M), (int)(wp.x & M)};
    b1 = v4i_t{(int)((uint32_t)(s6 >> 32) & M), (int)((uint32_t)(s4 >> 32) & M), (int)((uint32_t)(s2 >> 32) & M),
               (int)(wp.y & M)};
}

// Fragments of one stage for one wave: A row tiles 4 wr + i (both halves), W column tiles TNW wc + j.
// At TNW = 8 the 128 accumulators leave no room for a second fragment set: each stage reads its
// own fragments after its barrier (at TNW = 4 they are read one stage ahead).
#ifndef WF_PG_AHEAD8  // study switch: 1 = TNW 8 also reads its fragments one stage ahead (254 VGPRs
#define WF_PG_AHEAD8 0  // once the paired decode freed registers): gate|up 526 -> 525 us, not kept
#endif
// Fragments read one stage ahead (below): TNW = 4
template <int TNW>
constexpr bool pg_ahead() { return TNW == 4 || WF_PG_AHEAD8; }
template <int TNW>
struct PgFrag {
    v4i_t a[2][4];
    uint2 w[pg_ahead<TNW>() ? TNW : 1];
};

// The fragments of stage c are read from LDS one iteration ahead (while the MFMAs of stage c - 1
// run), so the matrix pipe never waits on an LDS round trip after the barrier. Iteration c: wait
// for stage c + 1 (vmcnt: stages c + 2 .. c + P - 2 may stay in flight), barrier, refill the slot
// of stage c - 1 (its fragments were consumed by the MFMAs of iteration c - 1, before the
// barrier), read stage c + 1's fragments, run stage c's MFMAs.
// Main loop of one 128 x (64 TNW) tile (bm, bn): int32 sums of wave (wr, wc) = (wave >> 2, wave & 3)
// in acc[i][j] = rows (4 wr + i) * 16 .., columns (TNW wc + j) * 16 .. of the tile (C/D layout).
// CW (column waves, ALG 3): the same stages and DMAs, but wave w owns every row tile (0..7) of the
// column tiles (TNW / 2) w + c, c < TNW / 2: each decoded weight fragment (7 VALU per 32-bit code
// word) feeds 8 MFMAs instead of 4. Two waves per SIMD issue into one matrix pipe and share its
// vector issue slots; an MFMA holds the issue for 8 of its 16 cycles, so at 4 MFMAs per decode the
// pair needs ~1900 issue cycles per 2048 MFMA cycles (measured ~55 % MFMA busy); at 8 per decode
// ~1500. acc[i][j] then holds row tile i + 4 (j / (TNW / 2)), column tile (TNW / 2) w + j % (TNW / 2)
// (pg_frag_rt / pg_frag_ct).
template <int TNW, bool CW>
__device__ __forceinline__ int pg_frag_rt(int wave, int i, int j) {
    return CW ? i + 4 * (j / (TNW / 2)) : 4 * (wave >> 2) + i;
}
template <int TNW, bool CW>
__device__ __forceinline__ int pg_frag_ct(int wave, int i, int j) {
    return CW ? (TNW / 2) * wave + j % (TNW / 2) : TNW * (wave & 3) + j;
}

// LDS-DMA sources of one 128 x (64 TNW) tile and its stage issue (3 or 4 DMAs per wave per stage)
template <int P, int TNW>
struct PgDma {
    static constexpr int SB = pg_stage_bytes<TNW>();
    const int8_t* asrc;
    const uint8_t* wsrc[TNW / 4];
    // A row tile 8 bm + wave (both halves); W column tiles 4 TNW bn + (TNW / 2) wave + 2 u + (lane >=
    // 32), u < TNW / 4 (two 512-byte column tiles per KiB piece)
    __device__ __forceinline__ PgDma(const uint8_t* __restrict__ W, const int8_t* __restrict__ A, int M, int N, int K,
                                     int bm, int bn) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int nkb = K >> 7, nrt = (M + 15) >> 4, nct = N >> 4;
        const int rt = min(bm * 8 + wave, nrt - 1);
        asrc = A + ((int64_t)rt * nkb << 11) + lane * 16;
#pragma unroll
        for (int u = 0; u < TNW / 4; ++u) {
            const int ct = min(bn * 4 * TNW + (TNW / 2) * wave + 2 * u + (lane >> 5), nct - 1);
            wsrc[u] = W + ((int64_t)ct * nkb << 9) + (lane & 31) * 16;
        }
    }
    __device__ __forceinline__ void issue(uint8_t* lds, int kb) const {
        const int wave = threadIdx.x >> 6;
        uint8_t* st = lds + (kb % P) * SB;
        glds16_asm(asrc + ((int64_t)kb << 11), st + wave * 2048);
        glds16_asm(asrc + ((int64_t)kb << 11) + 1024, st + wave * 2048 + 1024);
#pragma unroll
        for (int u = 0; u < TNW / 4; ++u) glds16_asm(wsrc[u] + ((int64_t)kb << 9), st + 16384 + ((TNW / 4) * wave + u) * 1024);
    }
    // the ring's first P - 1 stages (pgemm_tile<.., PRE = true> expects them issued)
    __device__ __forceinline__ void prologue(uint8_t* lds, int K) const {
#pragma unroll
        for (int c = 0; c < P - 1; ++c)
            if (c < (K >> 7)) issue(lds, c);
    }
};

// PRE: the caller issued the ring's first P - 1 stages (PgDma::prologue) before other vector-memory
// work of its own (a persistent block's previous epilogue: loads and stores count in the same
// vmcnt), so the first wait drains everything (vmcnt(0)) instead of counting.
template <int P, int TNW = 4, bool CW = false, bool PRE = false>
__device__ __forceinline__ void pgemm_tile(const uint8_t* __restrict__ W, const int8_t* __restrict__ A, int M, int N,
                                           int K, int bm, int bn, uint8_t* lds, v4i_t (&acc)[4][TNW]) {
    static_assert(P >= 4, "two stages in flight beyond the one being read");
    static_assert(TNW == 4 || TNW == 8, "256- or 512-column block tiles");
    constexpr int SB = pg_stage_bytes<TNW>(), NDMA = 2 + TNW / 4;  // DMAs per wave per stage
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int nkb = K >> 7;
    const PgDma<P, TNW> dma(W, A, M, N, K, bm, bn);
    auto issue = [&](int kb) { dma.issue(lds, kb); };
    auto read_w = [&](uint2 (&w)[TNW], int kb) {
        const uint8_t* st = lds + (kb % P) * SB;
#pragma unroll
        for (int j = 0; j < TNW; ++j) w[j] = *reinterpret_cast<const uint2*>(st + 16384 + (TNW * wc + j) * 512 + lane * 8);
    };
    auto read = [&](PgFrag<TNW>& f, int kb) {
        const uint8_t* st = lds + (kb % P) * SB;
        if constexpr (pg_ahead<TNW>()) read_w(f.w, kb);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                f.a[h][i] = *reinterpret_cast<const v4i_t*>(st + (4 * wr + i) * 2048 + h * 1024 + lane * 16);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = v4i_t{0, 0, 0, 0};
    auto mma_cw = [&](int kb) {  // CW: fragments read here, each decoded B feeds 8 MFMAs
        constexpr int CT = TNW / 2;
        const uint8_t* st = lds + (kb % P) * SB;
        uint2 wl[CT];
#pragma unroll
        for (int j = 0; j < CT; ++j) wl[j] = *reinterpret_cast<const uint2*>(st + 16384 + (CT * wave + j) * 512 + lane * 8);
        // CT <= 2: both halves decoded at once (pg_decode_pair); at CT = 4 they would spill
        constexpr int NH = CT <= 2 ? 2 : 1;
        v4i_t bf[NH][CT];
        if constexpr (NH == 2)
#pragma unroll
            for (int j = 0; j < CT; ++j) pg_decode_pair(wl[j], bf[0][j], bf[1][j]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            v4i_t fa[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) fa[r] = *reinterpret_cast<const v4i_t*>(st + r * 2048 + h * 1024 + lane * 16);
#pragma unroll
            for (int j = 0; j < CT; ++j) {
                if constexpr (NH == 1) {
                    const uint32_t w = h ? wl[j].y : wl[j].x;
                    bf[0][j] = v4i_t{(int)((w >> 6) & 0x03030303u), (int)((w >> 4) & 0x03030303u),
                                     (int)((w >> 2) & 0x03030303u), (int)(w & 0x03030303u)};
                }
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    acc[r & 3][(r >> 2) * CT + j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[r], bf[NH == 2 ? h : 0][j], acc[r & 3][(r >> 2) * CT + j], 0, 0, 0);
            }
        }
    };
    auto mma = [&](const PgFrag<TNW>& fc, int kb) {
        if constexpr (CW) {
            mma_cw(kb);
            return;
        }
        uint2 wl[TNW];
        PgFrag<TNW> fl;  // !pg_ahead: this stage's A fragments, read here (no second set in registers)
        if constexpr (pg_ahead<TNW>()) {
#pragma unroll
            for (int j = 0; j < TNW; ++j) wl[j] = fc.w[j];
        } else {
            read_w(wl, kb);
            read(fl, kb);
        }
        const PgFrag<TNW>& f = pg_ahead<TNW>() ? fc : fl;
#ifdef WF_PG_DEC32  // study: one 32-bit code word decoded per half (3 shifts + 4 ANDs per B fragment)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < TNW; ++j) {
                const uint32_t w = h ? wl[j].y : wl[j].x;
                const v4i_t bf = v4i_t{(int)((w >> 6) & 0x03030303u), (int)((w >> 4) & 0x03030303u),
                                       (int)((w >> 2) & 0x03030303u), (int)(w & 0x03030303u)};
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[h][i], bf, acc[i][j], 0, 0, 0);
            }
#else
        // a column tile's two halves decoded together (pg_decode_pair), then its 8 MFMAs
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            v4i_t b0, b1;
            pg_decode_pair(wl[j], b0, b1);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[0][i], b0, acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[1][i], b1, acc[i][j], 0, 0, 0);
        }
#endif
    };
    // one iteration: stage c + 1 published and read into `nxt`, stage c computed from `cur`
#ifdef WF_STAMPS
#define WF_PG_STAMP(i) \
    if (c == 8 || c == 9) WF_STAMP((i) + 5 * (c - 8))
#else
#define WF_PG_STAMP(i)
#endif
    auto step = [&](int c, PgFrag<TNW>& cur, PgFrag<TNW>& nxt) {
        WF_PG_STAMP(1);
        if (c + 1 < nkb) {
            if (c + P - 2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA * (P - 3)) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            WF_PG_STAMP(2);
            __builtin_amdgcn_s_barrier();
            WF_PG_STAMP(3);
#if !defined(WF_PG_STUDY) || WF_PG_STUDY != 1  // diagnostic build 1: no ring refills
            if (c + P - 1 < nkb) issue(c + P - 1);
#endif
            if constexpr (pg_ahead<TNW>() && !CW) read(nxt, c + 1);
        }
        WF_PG_STAMP(4);
        mma(cur, c);
        WF_PG_STAMP(5);
    };
#if defined(WF_PG_STUDY) && WF_PG_STUDY == 5  // diagnostic build 5: no main loop (epilogue cost)
    return;
#endif
    if constexpr (!PRE)
#pragma unroll
        for (int c = 0; c < P - 1; ++c)
            if (c < nkb) issue(c);
    PgFrag<TNW> f0, f1;
    if (!PRE && P - 2 < nkb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA * (P - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (pg_ahead<TNW>() && !CW) read(f0, 0);
    int c = 0;
    for (; c + 1 < nkb; c += 2) {
        step(c, f0, f1);
        step(c + 1, f1, f0);
    }
    if (c < nkb) step(c, f0, f1);
#undef WF_PG_STAMP
}

// Main-loop choice of the prefill GEMM kernels: ALG 0 = pgemm_tile with waves 2 (rows) x 4
// (columns), ALG 3 = the CW form (waves own column strips; each decoded weight fragment feeds 8
// MFMAs). Measured at 16384 x 13824 x 2560: the standalone fp32-output GEMM (k_pgemm_t) 565 -> 527 us
// with CW; the fused gate|up (k_pgemm_fused) 570 -> 580 us, and CW at 256-column tiles is slower
// (every wave reads all 8 A row tiles: LDS-read bound), so CW is the default only for k_pgemm_t's
// 512-column tiles. (Also measured and removed: two I2_S blocks per stage, a ping-pong form with
// the two waves of a SIMD alternating compute / load half-steps, and a software-pipelined CW form
// with the DMA pieces spread between the MFMAs -- none faster end to end; DESIGN.md.)
template <int TNW, int ALG>
struct PgCfg {
    static_assert(ALG == 0 || ALG == 3, "main-loop forms");
    static constexpr int P = pg_stages<TNW>();
    static constexpr int SB = pg_stage_bytes<TNW>();
    static constexpr int LDS = P * SB;
    static constexpr bool CW = ALG == 3;  // fragment -> tile mapping: pg_frag_rt / pg_frag_ct
};
template <int TNW, int ALG, bool PRE = false>
__device__ __forceinline__ void pg_main(const uint8_t* __restrict__ W, const int8_t* __restrict__ A, int M, int N,
                                        int K, int bm, int bn, uint8_t* lds, v4i_t (&acc)[4][TNW]) {
    pgemm_tile<PgCfg<TNW, ALG>::P, TNW, PgCfg<TNW, ALG>::CW, PRE>(W, A, M, N, K, bm, bn, lds, acc);
}
}  // namespace wf
