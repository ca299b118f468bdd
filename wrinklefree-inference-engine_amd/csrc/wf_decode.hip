// wf_decode.hip -- fused BitNet b1.58 decode step for gfx950.
//
// One decode token per sequence, per layer five launches:
//   QKV : rms_norm(input_layernorm) + quantize (block prologue) -> ternary GEMV over rows q|k|v ->
//         reference correction, RoPE (θ=5e5, half-split), q -> qbuf, k/v -> cache[pos]
//   ATTN: split-K GQA decode attention (wf_attn.hip), single launch, last-arriver merge
//   O   : rms_norm(attn_sub_norm) + quantize (prologue) -> GEMV + correction + residual
//         (h_b = h_a + o)
//   GU  : rms_norm(post_attention_layernorm) + quantize (prologue) -> GEMV over gate/up rows
//         interleaved in 8-row tiles; relu(gate)^2 * up
//   DN  : rms_norm(ffn_sub_norm) + quantize (prologue) -> GEMV (K = 6912) + correction + residual
//         (h_a = h_b + d)
// plus embed and the tied bf16 LM head (after the final norm) with a fused greedy argmax.
// At batch 1 every GEMV block normalises + quantises its input row itself (wf_norm.h) while its
// first weight chunks are in flight, so no launch carries a serial norm tail; at batch > 1 one
// k_rownorm launch per op produces the int8 codes instead. Every float op follows
// scripts/direct_inference_full.py:181-302 (bf16 tensors between ops); results match the oracle
// up to fp32 reduction order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <new>

#include "wf_common.h"
#include "wf_device.h"
#include "wf_norm.h"
#include "wf_mfma.h"
#include "wf_small.h"

namespace wf {
int prefill_attention_check(int Hq, int Hkv, int pps);
int prefill_attention(const uint16_t* q, int64_t q_rs, const uint16_t* k, const uint16_t* v, int64_t kv_sb,
                      int64_t kv_sh, int Hq, int Hkv, const int32_t* row_pos, const int32_t* row_slot, int M,
                      float sm_scale, const int32_t* pt, int pps, int npages, int64_t kv_pgs, uint16_t* out,
                      int64_t o_rs, hipStream_t st, int kv8, float k_scale, float v_scale);
int decode_attention_partials(const uint16_t* q, int64_t q_sb, const uint16_t* k, const uint16_t* v, int64_t kv_sb,
                              int64_t kv_sh, int B, int Hq, int Hkv, int S, const int32_t* seq_lens, float sm_scale,
                              float2* ml, float* o, hipStream_t st, bool kv_tiled, const int32_t* pt = nullptr,
                              int pps = 0, int npages = 0, int64_t kv_pgs = 0, int kv8 = 0, float k_scale = 1.f,
                              float v_scale = 1.f, uint16_t* merged_row = nullptr,
                              unsigned* merge_cnt = nullptr, uint64_t* xmax = nullptr,
                              const int32_t* order = nullptr, const SdpaBufs* sb = nullptr);
int seq_order(const int32_t* seq_lens, int B, int S, int32_t* order, hipStream_t st);

// study switches (same-box A/B builds, tools/build_var.sh; measured r04, profiles/ab_r04.txt):
// WF_NO_XTOK restores the batch-1 embed launch (-0.5 %); WF_OLD_EPI the LDS-round O/DN epilogue
// (+-0.1 %). Measured and removed with the round-4 attention kernels: the batched attention forming
// the O input row in its per-sequence tail (batch 128 -2.2 %: attention +7.5 us, k_rownorm_attn
// -4.5 us per layer).
#ifdef WF_NO_XTOK
constexpr bool kXTok = false;
#else
constexpr bool kXTok = true;
#endif
#ifdef WF_OLD_EPI
constexpr bool kPermEpi = false;
#else
constexpr bool kPermEpi = true;
#endif

#ifndef WF_XFIRST  // batch-1 GEMV: a workgroup barrier between the input-row loads and the weight stream
#define WF_XFIRST 1
#endif
constexpr bool kXFirst = WF_XFIRST;
enum { MODE_QKV = 0, MODE_O = 1, MODE_GU = 2, MODE_DN = 3, MODE_LINEAR = 4 };  // LINEAR: BitNetLinear drop-in
constexpr int kNT = 512;  // threads per GEMV / row-norm block (8 waves: 2 per SIMD hide the input-stage latency)

struct GemvArgs {
    // input row(s): bf16 x + norm weight (PPT > 0: normalised + quantised in the block prologue)
    const uint16_t* x;
    int64_t x_stride;
    const uint16_t* nw;
    float eps;
    // or int8 codes from k_rownorm (PPT == 0)
    const int8_t* q8;          // [B, q8_stride]
    int64_t q8_stride;
    const float* act_sf;       // [B] float(act scale)
    const int* act_sum;        // [B] sum of codes
    const uint8_t* w;          // packed rows
    int N, K, B;
    float ws0, ws1, ws2;       // weight scales (QKV: q,k,v; GU: gate,up; O/DN: ws0)
    // epilogue
    const uint16_t* resid;     // O/DN residual input [B, out_stride]
    uint16_t* out;             // O/DN hidden out; GU act; QKV q
    int64_t out_stride;
    // QKV extras (MODE_LINEAR: row segments of wf_bitnet_linear_fused -- rows [0, Hq) scale ws0 ->
    // out / out_stride, [Hq, Hq + Hkv) ws1 -> kc / kv_b_stride, [Hq + Hkv, N) ws2 -> vc / kv_pgs; see
    // lin_seg())
    int Hq, Hkv, S;
    const int32_t* positions;
    int* ws;                   // batched decode: split-K int32 partials
    size_t ws_ints;
    const uint16_t* rope_cos;
    const uint16_t* rope_sin;
    uint16_t* kc;
    uint16_t* vc;
    int64_t kv_b_stride;
    int kv_t;  // K/V caches in the matrix-core tile layouts (wf_attn.hip kv_tile_off; batched decode)
    // paged K/V (kv_t only): page of block t >> 5 of sequence m = pt[m * pps + (t >> 5)], page
    // stride kv_pgs elements, kv head stride 32 * 128 inside a page
    const int32_t* pt;
    int pps, npages;
    int64_t kv_pgs;
    // prefill: row m of the GEMM is a token of KV slot row_slot[m] (nullptr: row m = slot m)
    const int32_t* row_slot;
    // FP8 (e4m3fn) K/V cache: stored code = e4m3(clamp(y / scale, +-448)), RNE
    int kv8;
    float k_div, v_div;  // K / V scales: code = rne(y / scale) exactly as the header, the oracle and the reference
    // batched decode with the row norm fused into the GEMM launch (k_dec_gemm_t PRO != 0): arrival
    // and pass words per 32-sequence tile ([kSeamTiles] each), zero between launches
    unsigned* seam;
    // batch 1, layer 0 (k_gemv PPT > 0): the input row (QKV) / residual row (O) is the token's row
    // of the embedding table (x / resid = the table, row clamp(x_tok[b], 0, vocab - 1)) -- no embed
    // launch; QKV also sets seq_out[b] = positions[b] + 1 (what k_embed did)
    const int32_t* x_tok;
    int vocab;
    int32_t* seq_out;
};
constexpr int kSeamTiles = 8;  // 32-sequence tiles: batch <= 256 (kDecGemmMaxB)
// one 128-byte line per seam word: memory-side atomics and polls on one line serialise (the batch-1
// QKV + attention study measured ~5 us per hand-off with 20 counters sharing a line)
constexpr int kSeamLine = 32;

__device__ __forceinline__ uint8_t to_fp8(float y) {
    const float c = fminf(fmaxf(y, -448.f), 448.f);
    return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(c, c, 0, false) & 0xffu);
}
// A decode step's K/V cache element store, write-through (sc1). A new key's row lands in the tile
// layouts as 16 (K) and 128 (V) scattered 2-byte pieces, each dirtying its own cache line: plain
// stores left ~12 MB of partly dirty lines for the launch boundary to write back (batch 128; the
// attention launch then started 3.9 us after the QKV launch ended). Write-through: QKV op 13.3 ->
// 12.5 us, step 4.00 -> 3.96 ms (same-box A/B, round 3).
template <class T>
__device__ __forceinline__ void kv_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one-byte K/V code of y (already divided by the layer's scale): kvq 1 = OCP e4m3fn (RNE, saturating),
// 2 = int8 (the reference's INT8 KVCacheDtype: clamp(rne(y), -127, 127), kv_cache/kv_cache.py:159-185)
__device__ __forceinline__ uint8_t to_kv8(float y, int kvq) {
    if (kvq == 2) return (uint8_t)(int8_t)(int)fminf(fmaxf(__builtin_rintf(y), -127.f), 127.f);
    return to_fp8(y);
}

// MODE_LINEAR output n -> its row segment (wf_bitnet_linear_fused; one segment: Hq = N): the
// segment's weight scale, output base, row stride and column within the segment
struct LinSeg {
    float ws;
    uint16_t* out;
    int64_t ld;
    int col;
};
__device__ __forceinline__ LinSeg lin_seg(const GemvArgs& a, int n) {
    if (n < a.Hq) return {a.ws0, a.out, a.out_stride, n};
    if (n < a.Hq + a.Hkv) return {a.ws1, a.kc, a.kv_b_stride, n - a.Hq};
    return {a.ws2, a.vc, a.kv_pgs, n - a.Hq - a.Hkv};
}

// Reference correction (direct_inference_full.py:201-208) for one output:
// raw = fl32(S * f(ws)); c = f(ws * act_sum); out = fl32(fl32(raw - c) * f(s))
__device__ __forceinline__ float corrected(int S, float ws, int asum, float sf) {
    const float raw = (float)S * ws;
    const float c = ws * (float)asum;  // exact product rounded once == float(double(ws)*asum)
    return (raw - c) * sf;
}

// Block = kNT threads; LPR lanes per weight row -> kNT/LPR rows per block; MB activation rows.
// PPT > 0 (MB == 1): the block normalises + quantises its input row itself (wf_norm.h) while its
// first weight chunks stream in; PPT = 8-element pieces per thread (padded K <= 2048 * PPT).
// PPT == 0: the codes come from k_rownorm (batch > 1).
// TQ dot on the int8 matrix cores (batch 1, kTqMf): a TQ chunk's digit i is sixteen CONSECUTIVE
// codes (k = 80 c + 16 i + 0..15), i.e. one v_mfma_i32_16x16x64_i8 B fragment as decoded. The block's
// rows are 16-row tiles (8 / tiles waves per tile split the row's 4-chunk groups); lane (n, q) loads
// chunk 4 g + q of weight row n (16 rows x 64 contiguous bytes per instruction), decodes it and issues
// MFMA (g, i) with A = x[80 (4 g + q) + 16 i, +16) in every A row (plain LDS image; every output row
// is the weight row's dot). The five v_dot4 per decoded word leave the VALU.
// WF_TQ_MFMA: 0 off, 1 QKV / O / gate|up, 2 every batch-1 op. WF_TQ_CONTIG: a wave takes consecutive
// 4-chunk groups of its rows (1) instead of every kWpt-th (0).
#ifndef WF_TQ_MFMA
#define WF_TQ_MFMA 1
#endif
#ifndef WF_TQ_CONTIG
#define WF_TQ_CONTIG 0
#endif
template <int MODE>
constexpr int tq_mf_pre() { return MODE == MODE_GU ? 4 : (MODE == MODE_DN ? 3 : 1); }
typedef int v4i_tq __attribute__((ext_vector_type(4)));
template <class F, int MODE, int LPR, int MB, int PPT>
__global__ __launch_bounds__(kNT) void k_gemv(GemvArgs a) {
    static_assert(PPT == 0 || MB == 1, "the norm prologue handles one activation row");
    constexpr int RPB = kNT / LPR;
    constexpr bool kTqMf = (WF_TQ_MFMA == 2 || (WF_TQ_MFMA == 1 && MODE != MODE_DN)) && MB == 1 && PPT > 0 && MODE != MODE_LINEAR && __is_same(F, FmtTQ);
    constexpr int kTiles = RPB >= 16 ? RPB / 16 : 1, kWpt = (kNT / 64) / kTiles;
    constexpr int kTqPre = tq_mf_pre<MODE>();
    // 16-byte weight chunks in flight per lane (K = 2560 TQ: 1 per lane at LPR 32, 4 at LPR 8;
    // K = 6912 at LPR 32: 3)
    constexpr int kPrefetch = LPR >= 32 ? 4 : (LPR == 16 ? 4 : 8);
    extern __shared__ __attribute__((aligned(16))) int8_t smem[];
    __shared__ float red[2 * kNT / 64];
    __shared__ int red_i[kNT / 64];
    __shared__ float s_out[MB][RPB];

    const int K = a.K, N = a.N;
    const int img = lds_image_bytes<F>(K);
    const int b0 = blockIdx.y * MB;
    const int lrow = threadIdx.x / LPR, sub = threadIdx.x % LPR;
    const int row = blockIdx.x * RPB + lrow;
    const int C = F::chunks(K);
    WF_STAMP_BASE(512u * MODE);  // stamps build: one region per op
    WF_STAMP(0);

    // 1) the input row (issued first: vmcnt retires in order), 2) the weight stream, 3) residual
    constexpr int kNormPPT = PPT == 0 ? 1 : PPT;
    NormRow<kNormPPT, kNT> nr;
    constexpr int kMaxPiecesPerThread = 8192 / 16 / kNT;  // staged int8: K_pad <= 8192
    uint4 apre[MB][kMaxPiecesPerThread];
    const int pieces16 = F::k_pad(K) / 16;
    if constexpr (PPT > 0 && MODE == MODE_LINEAR) {
        nr.issue_x(a.x + (int64_t)b0 * a.x_stride, K);
    } else if constexpr (PPT > 0) {
        const int xrow = (MODE == MODE_QKV && a.x_tok) ? min(max(a.x_tok[b0], 0), a.vocab - 1) : b0;  // scalar load
        nr.issue(a.x + (int64_t)xrow * a.x_stride, a.nw, K);
    } else {
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int i = 0; i < kMaxPiecesPerThread; ++i) {
                const int p = threadIdx.x + kNT * i;
                apre[m][i] = (p < pieces16 && 16 * p < K)
                                 ? *reinterpret_cast<const uint4*>(a.q8 + (int64_t)(b0 + m) * a.q8_stride + 16 * p)
                                 : make_uint4(0, 0, 0, 0);
            }
    }
    // every wave's input-row loads reach the CU's load pipe before any wave's weight stream: a wave
    // whose row loads queued behind the other waves' weights held the norm's first barrier
    if constexpr (PPT > 0 && kXFirst) __builtin_amdgcn_s_barrier();
    const uint8_t* wr = a.w + (int64_t)min(row, N - 1) * F::row_bytes(K);
    uint4 wpre[kTqMf ? 1 : kPrefetch];
    uint4 wq[kTqMf ? kTqPre : 1];
    const int tq_wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), tq_l16 = threadIdx.x & 15,
              tq_q = (threadIdx.x >> 4) & 3;
    const int tq_part = tq_wave / kTiles, tq_G = (C + 3) >> 2;  // 4-chunk groups per row
    const int tq_gpw = (tq_G + kWpt - 1) / kWpt;                  // groups per wave
    // wave part's u-th group (may be >= tq_G or, contiguous, past the part's share: see tq_ok)
    const auto tq_g = [&](int u) { return WF_TQ_CONTIG ? tq_part * tq_gpw + u : tq_part + kWpt * u; };
    const auto tq_ok = [&](int u) { return tq_g(u) < tq_G && (!WF_TQ_CONTIG || u < tq_gpw); };
    const uint8_t* wqr = a.w + (int64_t)min((int)blockIdx.x * RPB + 16 * (tq_wave % kTiles) + tq_l16, N - 1) * F::row_bytes(K);
    if constexpr (kTqMf) {
#pragma unroll
        for (int u = 0; u < kTqPre; ++u)  // unconditional (clamped): vmcnt stays exact
            wq[u] = ldg_nt(wqr + 16 * (int64_t)min(4 * min(tq_g(u), tq_G - 1) + tq_q, C - 1));
    } else {
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u)  // clamped (no branch): lanes past the row re-read its last chunk
            wpre[u] = ldg_nt(wr + (int64_t)min(LPR * u + sub, C - 1) * 16);
    }
    // residual: unconditional (clamped) load -- a load under a lane condition makes hipcc wait
    // vmcnt(0) right there, i.e. for the whole weight prefetch before the prologue can start
    uint16_t resid_raw[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        resid_raw[m] = 0;
        if constexpr (MODE == MODE_O || MODE == MODE_DN) {
            const int rrow = (MODE == MODE_O && MB == 1 && a.x_tok) ? min(max(a.x_tok[b0], 0), a.vocab - 1) : b0 + m;
            resid_raw[m] = a.resid[(int64_t)rrow * a.out_stride + min(row, N - 1)];
        }
    }
    // batch 1 QKV: the RoPE entries of the epilogue (position: a scalar load, so the wait for it
    // does not drain the vector loads above)
    uint16_t rope_c = 0, rope_s = 0;
    if constexpr (MODE == MODE_QKV && MB == 1) {
        const int pos = min(max(a.positions[b0], 0), a.S - 1);
        const int d0 = 8 * (blockIdx.x & 7) + (threadIdx.x & 7);
        rope_c = a.rope_cos[(int64_t)pos * 64 + d0];
        rope_s = a.rope_sin[(int64_t)pos * 64 + d0];
    }
    // every load above is in flight before any input-stage arithmetic (hipcc would otherwise hoist
    // that math above the weight stream to save registers)
    if constexpr (PPT > 0) {
        nr.fence(true, MODE != MODE_LINEAR);
    }
    __builtin_amdgcn_sched_barrier(0);
    float sf[MB];
    int asum[MB];
    if constexpr (PPT > 0) {
        float y[PPT][8];
        if constexpr (MODE == MODE_LINEAR) {  // quantize x itself (no norm)
            unpack_row(nr, K, y);
            sf[0] = absmax_scale<PPT, kNT>(y, red);
        } else {
            sf[0] = norm_row<kNormPPT, kNT, 512u * MODE>(nr, K, a.eps, y, red);
        }
        const auto lds_at = [](int p) { return kTqMf ? 8 * p : F::lds_off(8 * p); };  // kTqMf: codes in k order
        int as = quant_row<PPT, kNT, decltype(lds_at), 512u * MODE>(y, sf[0], F::k_pad(K) / 8, smem, lds_at);
        as = wave_sum_i(as);
        if ((threadIdx.x & 63) == 0) red_i[threadIdx.x >> 6] = as;
    } else {
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int i = 0; i < kMaxPiecesPerThread; ++i) {
                const int p = threadIdx.x + kNT * i;
                if (p < pieces16) *reinterpret_cast<uint4*>(smem + m * img + F::lds_off(16 * p)) = apre[m][i];
            }
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            sf[m] = a.act_sf[b0 + m];
            asum[m] = a.act_sum[b0 + m];
        }
    }
    __syncthreads();
    if constexpr (PPT > 0) {
        asum[0] = 0;
#pragma unroll
        for (int i = 0; i < kNT / 64; ++i) asum[0] += red_i[i];
    }
    WF_STAMP(1);
    WF_STAMP_DRAIN(13);

    int acc[MB];
    if constexpr (kTqMf) {
        __shared__ int tq_red[kNT / 64][16];
        v4i_tq ac = v4i_tq{0, 0, 0, 0};
        const int limg = lds_image_bytes<F>(K) - 16;
        auto tq_group = [&](uint4 w, int g) __attribute__((always_inline)) {
            const int c = 4 * g + tq_q;
            Decoded<F> d;
            d.load(c < C ? w : make_uint4(0, 0, 0, 0));
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const v4i_tq bf = v4i_tq{(int)d.e[i][0], (int)d.e[i][1], (int)d.e[i][2], (int)d.e[i][3]};
                const v4i_tq af = *reinterpret_cast<const v4i_tq*>(smem + min(80 * c + 16 * i, limg));
                ac = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, ac, 0, 0, 0);
            }
        };
#pragma unroll
        for (int u = 0; u < kTqPre; ++u)
            if (tq_ok(u)) tq_group(wq[u], tq_g(u));  // wave-uniform
        for (int u = kTqPre; tq_ok(u); ++u)  // rows longer than the prefetch
            tq_group(ldg_nt(wqr + 16 * (int64_t)min(4 * tq_g(u) + tq_q, C - 1)), tq_g(u));
        if (tq_q == 0) tq_red[tq_wave][tq_l16] = ac[0];
        __syncthreads();
        int sum = 0;
#pragma unroll
        for (int p = 0; p < kWpt; ++p) sum += tq_red[(lrow >> 4) + kTiles * p][lrow & 15];
        acc[0] = sum;
        WF_STAMP(2);
    } else {
    DotAcc<F> dacc[MB];
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
        const int c = LPR * u + sub;
        if (c < C) {
            Decoded<F> d;
            d.load(wpre[u]);
            const int8_t* ab = smem + ((c >> 4) * F::kGroups) * 256 + (c & 15) * 16;
#pragma unroll
            for (int m = 0; m < MB; ++m) chunk_dot<F>(d, ab + m * img, dacc[m]);
        }
    }
    for (int c0 = LPR * kPrefetch; c0 < C; c0 += LPR * kPrefetch) {
        uint4 w[kPrefetch];
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u)
            w[u] = ldg_nt(wr + (int64_t)min(c0 + LPR * u + sub, C - 1) * 16);
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u) {
            const int c = c0 + LPR * u + sub;
            if (c < C) {
                Decoded<F> d;
                d.load(w[u]);
                const int8_t* ab = smem + ((c >> 4) * F::kGroups) * 256 + (c & 15) * 16;
#pragma unroll
                for (int m = 0; m < MB; ++m) chunk_dot<F>(d, ab + m * img, dacc[m]);
            }
        }
    }
    WF_STAMP(2);
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = group_reduce<LPR>(dacc[m].total(), OpAdd{});
    }

    if constexpr (MODE == MODE_QKV) {
        // rows per head permuted: block t of head h = dims {8t..8t+7, 64+8t..64+8t+7} (RPB == 16)
        static_assert(RPB == 16, "QKV epilogue pairs RoPE halves inside one 16-row block");
        const int head = blockIdx.x >> 3, tt = blockIdx.x & 7;
        const int proj = head < a.Hq ? 0 : (head < a.Hq + a.Hkv ? 1 : 2);
        const float wsp = proj == 0 ? a.ws0 : (proj == 1 ? a.ws1 : a.ws2);
        if (sub == 0) {
#pragma unroll
            for (int m = 0; m < MB; ++m) s_out[m][lrow] = rbf(corrected(acc[m], wsp, asum[m], sf[m]));
        }
        __syncthreads();
        if (MB == 1 && a.seq_out && blockIdx.x == 0 && threadIdx.x == 0) a.seq_out[b0] = a.positions[b0] + 1;
        if (threadIdx.x < 8 * MB) {
            const int m = threadIdx.x >> 3, i = threadIdx.x & 7;
            const int bi = b0 + m;
            const int d0 = 8 * tt + i;  // first-half dim; partner d0 + 64
            float x1 = s_out[m][i], x2 = s_out[m][8 + i];
            const int pos = min(max(a.positions[bi], 0), a.S - 1);  // never write outside the cache
            if (proj < 2) {  // RotaryEmbedding._rotate (direct_inference_full.py:58-70)
                const float c = bf2f(MB == 1 ? rope_c : a.rope_cos[(int64_t)pos * 64 + d0]);
                const float s = bf2f(MB == 1 ? rope_s : a.rope_sin[(int64_t)pos * 64 + d0]);
                const float r1 = rbf(rbf(x1 * c) - rbf(x2 * s));
                const float r2 = rbf(rbf(x1 * s) + rbf(x2 * c));
                x1 = r1;
                x2 = r2;
            }
            if (proj == 0) {
                uint16_t* qo = a.out + (int64_t)bi * a.out_stride + head * 128;
                qo[d0] = f2bf(x1);
                qo[d0 + 64] = f2bf(x2);
            } else {
                const int g = head - a.Hq - (proj == 2 ? a.Hkv : 0);
                uint16_t* cache = (proj == 1 ? a.kc : a.vc) + (int64_t)bi * a.kv_b_stride + ((int64_t)g * a.S + pos) * 128;
                cache[d0] = f2bf(x1);
                cache[d0 + 64] = f2bf(x2);
            }
        }
        WF_STAMP(7);
        return;
    } else if constexpr (MODE == MODE_LINEAR) {
        // BitNetLinear (direct_inference_full.py:186-208): y = bf16(fl32(fl32(raw - ws*sum(q)) * s))
        if (sub == 0) {
#pragma unroll
            for (int m = 0; m < MB; ++m) s_out[m][lrow] = corrected(acc[m], lin_seg(a, row).ws, asum[m], sf[m]);
        }
        __syncthreads();
        if (threadIdx.x < MB * RPB) {
            const int m = threadIdx.x / RPB, i = threadIdx.x % RPB;
            const int n = blockIdx.x * RPB + i;
            if (n < N) {
                const LinSeg g = lin_seg(a, n);
                g.out[(int64_t)(b0 + m) * g.ld + g.col] = f2bf(s_out[m][i]);
            }
        }
    } else if constexpr (kPermEpi && (MODE == MODE_O || MODE == MODE_DN) && MB == 1 && LPR == 32) {
        // O/DN at batch 1: a wave holds rows 2w (lanes 0-31) and 2w + 1 (lanes 32-63), every lane of a
        // row has its sum; lane 0 takes its partner's value by v_permlane32_swap and stores the pair
        // as one 4-byte word -- no LDS round and no block barrier before the store
        const float v = rbf(bf2f(resid_raw[0]) + rbf(corrected(acc[0], a.ws0, asum[0], sf[0])));
        const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        if ((threadIdx.x & 63) == 0) {
            uint16_t* o = a.out + (int64_t)b0 * a.out_stride + row;
            if (row + 1 < N)
                *reinterpret_cast<uint32_t*>(o) = pk_bf16(__uint_as_float(pr[0]), __uint_as_float(pr[1]));
            else if (row < N)
                *o = f2bf(__uint_as_float(pr[0]));
        }
        WF_STAMP(3);
    } else {
        // O/DN: out[row] = bf16(resid + bf16(o)); GU: act[8t+i] = bf16(bf16(relu(g)^2) * u)
        if (sub == 0) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                if constexpr (MODE == MODE_GU)
                    s_out[m][lrow] = rbf(corrected(acc[m], (lrow & 15) < 8 ? a.ws0 : a.ws1, asum[m], sf[m]));
                else
                    s_out[m][lrow] = rbf(bf2f(resid_raw[m]) + rbf(corrected(acc[m], a.ws0, asum[m], sf[m])));
            }
        }
        __syncthreads();
        constexpr int NOUT = (MODE == MODE_GU) ? RPB / 2 : RPB;  // outputs per block per row
        static_assert(NOUT % 8 == 0, "16-byte output granules");
        if (threadIdx.x < MB * (NOUT / 8)) {
            const int m = threadIdx.x / (NOUT / 8), j = threadIdx.x % (NOUT / 8);
            uint32_t pk[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                float lo, hi;
                if constexpr (MODE == MODE_GU) {
                    // 8-row tile j of the block: gate rows 16j..16j+7, up rows 16j+8..16j+15
                    const float* tg = &s_out[m][16 * j];
                    const float g0 = fmaxf(tg[2 * t], 0.f), g1 = fmaxf(tg[2 * t + 1], 0.f);
                    lo = rbf(rbf(g0 * g0) * tg[8 + 2 * t]);
                    hi = rbf(rbf(g1 * g1) * tg[8 + 2 * t + 1]);
                } else {
                    lo = s_out[m][8 * j + 2 * t];
                    hi = s_out[m][8 * j + 2 * t + 1];
                }
                pk[t] = pk_bf16(lo, hi);
            }
            const int64_t first = (int64_t)blockIdx.x * NOUT + 8 * j;
            if (first < a.out_stride)
                *reinterpret_cast<uint4*>(a.out + (int64_t)(b0 + m) * a.out_stride + first) =
                    make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
        WF_STAMP(3);
    }
}

// ---------------------------------------------------------------------------------------------
// Batched decode (B >= 16): int8-MFMA ternary GEMM (wf_mfma.hip's fragment scheme) over the codes
// of k_rownorm, with the same fused epilogues as k_gemv. Block = 4 waves x 2 16-row MFMA tiles =
// 128 sequences, one 16-weight-row column tile (so QKV's RoPE partner dims and GU's gate/up pairs
// sit in lanes l and l ^ 8 of the same tile).
// ---------------------------------------------------------------------------------------------
constexpr int kDecMfmaMinB = 16;
constexpr int kDecGemmMaxB = 256;  // whole-K register GEMM up to here, split-K LDS-DMA tiles above

// Fused decode-step epilogue of one 16 x 16 output tile (rows = sequences, columns = 16 weight rows
// = one QKV RoPE block / one gate-up tile): lane holds rows r0 + 4q + r of column c0 + l16.
// The per-row inputs of the epilogue (scale, code sum, position + RoPE entries, residual) can be
// loaded before the GEMM's result exists (load(), issued next to the fragment loads).
struct EpiIn {
    float sf[4];
    int as[4];
    int pos[4];
    float cs[4], sn[4];
    uint16_t res[4];
};
template <int MODE>
struct EpiDec {
    const GemvArgs* a;
    // independent per-row loads (issue before the fragment loads) ...
    // SC1: the scale / code sum were published in this launch (fused row norm): sc1 loads
    template <bool SC1 = false>
    __device__ __forceinline__ void load(int r0, int c0, int l16, int q, EpiIn& in) const {
        const GemvArgs& g = *a;
        const int n = min(c0 + l16, g.N - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int mc = min(r0 + 4 * q + r, g.B - 1);
            in.sf[r] = SC1 ? ld_sc1(g.act_sf + mc) : g.act_sf[mc];
            in.as[r] = SC1 ? ld_sc1(g.act_sum + mc) : g.act_sum[mc];
            if constexpr (MODE == MODE_QKV) in.pos[r] = g.positions[mc];
            if constexpr (MODE == MODE_O || MODE == MODE_DN) in.res[r] = g.resid[(int64_t)mc * g.out_stride + n];
        }
    }
    // ... and the RoPE entries, which depend on the position (issue after them)
    __device__ __forceinline__ void load_rope(int c0, int l16, EpiIn& in) const {
        if constexpr (MODE == MODE_QKV) {
            const GemvArgs& g = *a;
            const int d0 = 8 * ((c0 >> 4) & 7) + (l16 & 7);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int pos = min(max(in.pos[r], 0), g.S - 1);
                in.pos[r] = pos;
                in.cs[r] = bf2f(g.rope_cos[(int64_t)pos * 64 + d0]);
                in.sn[r] = bf2f(g.rope_sin[(int64_t)pos * 64 + d0]);
            }
        }
    }
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) {
        EpiIn in;
        load(r0, c0, l16, q, in);
        load_rope(c0, l16, in);
        apply(r0, c0, acc, l16, q, in);
    }
    // GU: act = bf16(bf16(relu(g)^2) * u) of the fragment's rows, quad-transposed: lane (quad k <
    // 2, qi) gets row 4q + qi, act columns 4k .. 4k + 3 of the fragment's 8, as 4 packed bf16
    // (rows in pairs through the packed-fp32 VALU: v_pk_mul_f32 / v_pk_add_f32 round each lane like
    // the scalar ops, so the float sequence of corrected() and the activation is unchanged)
    __device__ __forceinline__ uint2 gu_pack(const v4i_t& acc, const EpiIn& in, int l16) const {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const GemvArgs& g = *a;
        const float ws = l16 < 8 ? g.ws0 : g.ws1;
        const f2 W = {ws, ws};
        uint32_t yp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f2 S = {(float)acc[2 * h], (float)acc[2 * h + 1]};
            const f2 C = W * f2{(float)in.as[2 * h], (float)in.as[2 * h + 1]};
            const f2 SF = {in.sf[2 * h], in.sf[2 * h + 1]};
            const f2 u = (S * W - C) * SF;  // corrected(): fl32(fl32(S ws) - fl32(ws asum)) * sf
            const uint32_t vp = pk_bf16(u.x, u.y);
            const f2 v = {bf_lo(vp), bf_hi(vp)};
            const f2 pv = {dpp_f<DPP_ROW_ROR8>(v.x), dpp_f<DPP_ROW_ROR8>(v.y)};  // partner column l16 ^ 8
            const f2 gt = {fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
            const uint32_t gp = pk_bf16((gt * gt).x, (gt * gt).y);
            const f2 y = f2{bf_lo(gp), bf_hi(gp)} * pv;
            yp[h] = pk_bf16(y.x, y.y);
        }
        return quad_transpose_pk(yp[0], yp[1], l16 & 3);
    }
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q, const EpiIn& in) {
        const GemvArgs& g = *a;
        const int tile = c0 >> 4, n = c0 + l16, B = g.B, N = g.N;
        if constexpr (MODE == MODE_GU) {
            // 16-column fragment = gate columns 8 tile .. + 7 (lanes l16 < 8) and their up columns (l16
            // + 8): act rows 4q + r, 8 columns. The 4 x 4 blocks of act values in each lane quad are
            // transposed (4 DPP moves) so that lane (quad k, qi) holds row 4q + qi, columns 4k .. 4k + 3:
            // one 8-byte store per lane instead of four 2-byte ones (the stores were the epilogue's cost:
            // a quarter of them took the prefill gate|up GEMM from 570 to 472 us per layer).
            if (((g.out_stride & 3) | (reinterpret_cast<uintptr_t>(g.out) & 7)) == 0) {
                const int qi = l16 & 3, m = r0 + 4 * q + qi;
                const uint2 pk = gu_pack(acc, in, l16);
                if (l16 < 8 && m < B && tile * 16 < N)
                    *reinterpret_cast<uint2*>(g.out + (int64_t)m * g.out_stride + tile * 8 + 4 * (l16 >> 2)) = pk;
                return;
            }
        }
        float ws = g.ws0;
        int proj = 0, head = 0, tt = 0;
        if constexpr (MODE == MODE_QKV) {
            head = tile >> 3;
            tt = tile & 7;
            proj = head < g.Hq ? 0 : (head < g.Hq + g.Hkv ? 1 : 2);
            ws = proj == 0 ? g.ws0 : (proj == 1 ? g.ws1 : g.ws2);
        } else if constexpr (MODE == MODE_GU) {
            ws = l16 < 8 ? g.ws0 : g.ws1;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r0 + 4 * q + r;
            const float v = rbf(corrected(acc[r], ws, in.as[r], in.sf[r]));
            if constexpr (MODE == MODE_QKV || MODE == MODE_GU) {
                const float pv = __shfl_xor(v, 8, 64);  // partner column l16 ^ 8 (same rows)
                if (m >= B || tile * 16 >= N) continue;
                if constexpr (MODE == MODE_GU) {
#ifdef WF_GU_EPI_STUDY  // diagnostic build: a quarter of the act stores (store-issue cost)
                    if (r != 0) continue;
#endif
                    if (l16 < 8) {
                        const float gt = fmaxf(v, 0.f);
                        g.out[(int64_t)m * g.out_stride + tile * 8 + l16] = f2bf(rbf(rbf(gt * gt) * pv));
                    }
                } else {
                    const int d0 = 8 * tt + (l16 & 7);
                    const float x1 = l16 < 8 ? v : pv, x2 = l16 < 8 ? pv : v;
                    const int pos = in.pos[r];
                    float y = v;
                    if (proj < 2) {  // RotaryEmbedding._rotate (direct_inference_full.py:58-70)
                        const float cs = in.cs[r], sn = in.sn[r];
                        y = l16 < 8 ? rbf(rbf(x1 * cs) - rbf(x2 * sn)) : rbf(rbf(x1 * sn) + rbf(x2 * cs));
                    }
                    const int d = d0 + (l16 < 8 ? 0 : 64);
                    if (proj == 0) {
                        g.out[(int64_t)m * g.out_stride + head * 128 + d] = f2bf(y);
                    } else {
                        const int kvh = head - g.Hq - (proj == 2 ? g.Hkv : 0);
                        const int slot = g.row_slot ? g.row_slot[m] : m;
                        if (g.kv8) {  // FP8 / int8 tile-layout cache (element offsets are byte offsets)
                            uint8_t* c8 = reinterpret_cast<uint8_t*>(proj == 1 ? g.kc : g.vc);
                            int64_t off;
                            if (g.pt) {
                                const int pg = min(max(g.pt[(int64_t)slot * g.pps + (pos >> 5)], 0), g.npages - 1);
                                off = pg * g.kv_pgs + (int64_t)kvh * 4096 + (proj == 1 ? k_tile_off(pos & 31, d) : v_tile_off(pos & 31, d));
                            } else {
                                off = (int64_t)slot * g.kv_b_stride + (int64_t)kvh * g.S * 128 +
                                      (proj == 1 ? k_tile_off(pos, d) : v_tile_off(pos, d));
                            }
                            kv_store(c8 + off, to_kv8(y / (proj == 1 ? g.k_div : g.v_div), g.kv8));
                            continue;
                        }
                        if (g.pt) {  // paged: block pos >> 5 lives in page pt[slot][pos >> 5]
                            const int pg = min(max(g.pt[(int64_t)slot * g.pps + (pos >> 5)], 0), g.npages - 1);
                            uint16_t* cache = (proj == 1 ? g.kc : g.vc) + pg * g.kv_pgs + (int64_t)kvh * 4096;
                            kv_store(cache + (proj == 1 ? k_tile_off(pos & 31, d) : v_tile_off(pos & 31, d)), f2bf(y));
                            continue;
                        }
                        uint16_t* cache = (proj == 1 ? g.kc : g.vc) + (int64_t)slot * g.kv_b_stride + (int64_t)kvh * g.S * 128;
                        if (g.kv_t) kv_store(cache + (proj == 1 ? k_tile_off(pos, d) : v_tile_off(pos, d)), f2bf(y));
                        else cache[(int64_t)pos * 128 + d] = f2bf(y);
                    }
                }
            } else {  // O / DN: out = bf16(resid + bf16(o))
                if (m >= B || n >= N) continue;
                const int64_t o = (int64_t)m * g.out_stride + n;
                g.out[o] = f2bf(rbf(bf2f(in.res[r]) + v));
            }
        }
    }
};

// Batched decode GEMM, split-K: block (j, s, rb) = 128 sequences x 128 weight rows over k-step
// slice s (wf_mfma.h LDS-DMA pipeline), exact int32 partial sums to ws[s][B][N]; k_dec_epi adds
// the slices (fixed order, exact) and runs the fused epilogue. Splitting K spreads the 20-108
// column blocks of a layer over ~256+ CUs (one CU's LDS-DMA stream alone is ~25-30 GB/s).
struct EpiPartial {
    int* ws;
    int B, N;
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) {
        const int n = c0 + l16;
        if (n >= N) return;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r0 + 4 * q + r;
            if (m < B) ws[(int64_t)m * N + n] = acc[r];
        }
    }
};

__global__ __launch_bounds__(256) void k_dec_mfma_part(GemvArgs a, int* __restrict__ ws, int steps_per_split) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kTgStagesWide * kTgStageBytes];
    const int s = blockIdx.y;
    const int c0 = s * steps_per_split, c1 = min(c0 + steps_per_split, a.K / 64);
    EpiPartial e{ws + (int64_t)s * a.B * a.N, a.B, a.N};
    tgemm_tile<2, kTgStagesWide>(a.w, a.q8, a.q8_stride, a.B, a.N, a.K, blockIdx.z * 128, blockIdx.x * 128, lds, e, c0,
                                 c1);
}

// Batched decode GEMM without split-K (B up to a few hundred): block (column block, row block) =
// 16 TMT sequences x 16 TNT weight rows over the whole K. Its kDgWaves waves split K by I2_S blocks
// of 128 (wave w: blocks w, w + kDgWaves, ...); fragments go straight from global memory (L2: the
// codes are shared by every column block) into registers, two blocks in flight per wave (the
// whole K of a 2560-deep GEMM is in flight at once). The waves' exact int32 sums are added through
// LDS and each wave runs the fused EpiDec epilogue on one 16 x 16 tile: no partial slabs, no
// second launch. Fragment mapping as wf_mfma.h: lane (l16, q) takes A[row][128 kb + 16 h + 32 q,
// +16) and weight bytes [32 kb + 16 h, +16) of its column, bit offset 6 - 2q.
constexpr int kDgWaves = 8;
template <int TMT, int TNT, int NB, int MODE>
__global__ __launch_bounds__(kDgWaves * 64) void k_dec_gemm(GemvArgs a) {
    static_assert(TMT * TNT == kDgWaves, "one epilogue tile per wave");
    __shared__ v4i_t red[kDgWaves][TMT * TNT][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16 * TNT, m0 = blockIdx.y * 16 * TMT;
    const int K = a.K, nkb = K >> 7;
    const int8_t* ap[TMT];
    const uint8_t* wp[TNT];
#pragma unroll
    for (int i = 0; i < TMT; ++i) ap[i] = a.q8 + (int64_t)min(m0 + 16 * i + l16, a.B - 1) * a.q8_stride + 32 * q;
#pragma unroll
    for (int j = 0; j < TNT; ++j) wp[j] = a.w + (int64_t)min(n0 + 16 * j + l16, a.N - 1) * (K >> 2);
    v4i_t acc[TMT][TNT];
#pragma unroll
    for (int i = 0; i < TMT; ++i)
#pragma unroll
        for (int j = 0; j < TNT; ++j) acc[i][j] = v4i_t{0, 0, 0, 0};
    uint4 fa[NB][TMT][2], fw[NB][TNT][2];
    auto load = [&](uint4 (&la)[TMT][2], uint4 (&lw)[TNT][2], int kb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int i = 0; i < TMT; ++i) la[i][h] = *reinterpret_cast<const uint4*>(ap[i] + 128 * kb + 16 * h);
#pragma unroll
            for (int j = 0; j < TNT; ++j) lw[j][h] = *reinterpret_cast<const uint4*>(wp[j] + 32 * kb + 16 * h);
        }
    };
    const int sh = 6 - 2 * q;
    auto mma = [&](const uint4 (&la)[TMT][2], const uint4 (&lw)[TNT][2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            v4i_t bf[TNT];
#pragma unroll
            for (int j = 0; j < TNT; ++j) {
                const uint4 w = lw[j][h];
                bf[j] = v4i_t{(int)((w.x >> sh) & 0x03030303u), (int)((w.y >> sh) & 0x03030303u),
                              (int)((w.z >> sh) & 0x03030303u), (int)((w.w >> sh) & 0x03030303u)};
            }
#pragma unroll
            for (int i = 0; i < TMT; ++i) {
                const v4i_t af = __builtin_bit_cast(v4i_t, la[i][h]);
#pragma unroll
                for (int j = 0; j < TNT; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[j], acc[i][j], 0, 0, 0);
            }
        }
    };
    // wave w: I2_S blocks w + kDgWaves t, t < cnt; NB of them in flight
    const int cnt = (nkb - wave + kDgWaves - 1) / kDgWaves;
    WF_STAMP(0);
    // the epilogue's per-row inputs, around the fragment loads
    EpiDec<MODE> e{&a};
    const int er0 = m0 + 16 * (wave / TNT), ec0 = n0 + 16 * (wave % TNT);
    EpiIn ein;
    e.load(er0, ec0, l16, q, ein);
#pragma unroll
    for (int b = 0; b < NB; ++b)
        if (b < cnt) load(fa[b], fw[b], wave + kDgWaves * b);
    e.load_rope(ec0, l16, ein);
    WF_STAMP(1);
    for (int t0 = 0; t0 < cnt; t0 += NB) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int t = t0 + b;
            if (t < cnt) {
                mma(fa[b], fw[b]);
                if (t == 0) WF_STAMP(2);
                if (t + NB < cnt) load(fa[b], fw[b], wave + kDgWaves * (t + NB));
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TMT; ++i)
#pragma unroll
        for (int j = 0; j < TNT; ++j) red[wave][i * TNT + j][lane] = acc[i][j];
    WF_STAMP(3);
    __syncthreads();
    WF_STAMP(4);
    v4i_t sum = red[0][wave][lane];
#pragma unroll
    for (int w = 1; w < kDgWaves; ++w) sum += red[w][wave][lane];
    e.apply(er0, ec0, sum, l16, q, ein);
    WF_STAMP(5);
    WF_STAMP_DRAIN(6);
}

// The same GEMM on the matrix-core tile layouts (WF_FMT_I2S_MFMA weights, tile-ordered codes from
// k_rownorm<..., TL>): every fragment load is one contiguous wave-instruction (A: 1 KiB of codes per
// (row tile, I2_S block, half); B: 512 B of weight dwords per (column tile, I2_S block)), so the CU's
// load pipeline moves whole cache lines (tools/ubench/load_rates: ~4 cycles per distinct line per
// wave-instruction, whatever the bytes used). Lane (l16, q), block kb, half h: A = 16 codes of
// k = 128 kb + 16 h + 4 q + jj + 32 g at [4g + jj]; B dword h = I2_S bytes [32 kb + 16 h + 4 q, +4)
// of its column, decoded into the 4 groups g by shift 6 - 2g -- the same k for both operands.
// PRO != 0: the row norm of the GEMM's input is fused into the launch (no k_rownorm launch and no
// kernel boundary before the GEMM). Block (x, y) with x < rows of sequence tile y normalises and
// quantises row 32 y + x exactly like k_rownorm (the 512-thread tree; 4-wave blocks
// replay it with two chains per lane), stores its codes, scale and code sum write-through (sc1),
// drains, and bumps the tile's arrival word; every block of the tile waits for all of its rows
// (one polling lane, bounded), then reads the codes with sc1 loads. The weight fragments are issued
// before the norm, so the weight stream overlaps it. The last block of the tile to pass the wait
// re-arms both words (arrivals / passes), so the words are zero at every launch boundary. Needs the
// whole grid co-resident (host: wf_model_create checks the occupancy, else the two-launch form) and
// gridDim.x >= 32. PRO 1: rms_norm of x (a.x, a.nw; for O, x = the attention's bf16 rows).
constexpr unsigned kSeamSpin = 1u << 22;  // polls before a waiting block gives up (never in a valid launch)
// codes of the NT-thread pieces into the tile layout, write-through (the in-launch hand-off)
template <int PPT, int NT>
__device__ __forceinline__ int quant_row_tiled_wt(const float (&y)[PPT][8], float sf, int npad, int8_t* base, int row,
                                                  int nkb) {
    const float inv = rcp_1ulp(sf);
    int asum = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int p = (int)threadIdx.x + NT * i;
        const uint2 qv = quant8(y[i], sf, inv, asum);
        if (p < npad) {
            st_sc1(reinterpret_cast<uint32_t*>(base + tile_code_pos(row, 8 * p, nkb)), qv.x);
            st_sc1(reinterpret_cast<uint32_t*>(base + tile_code_pos(row, 8 * p + 4, nkb)), qv.y);
        }
    }
    return asum;
}

// The input row r of the fused GEMM (PRO 1 / 2): codes, scale and code sum published write-through.
template <int PRO, int PP, int NW>
__device__ __forceinline__ void dec_row_prologue(const GemvArgs& a, int r, float* red, int* red_i) {
    constexpr int NT = NW * 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, K = a.K, nkb = K >> 7;
    int8_t* q8 = const_cast<int8_t*>(a.q8);
    float sf;
    int as;
    if constexpr (NT == 512) {
        NormRow<PP, 512> nr;
        float y[PP][8];
        nr.issue(a.x + (int64_t)r * a.x_stride, a.nw, K);
        sf = norm_row(nr, K, a.eps, y, red);
        as = quant_row_tiled_wt<PP, 512>(y, sf, K / 8, q8, r, nkb);
    } else {
        static_assert(NT == 256 && PRO == 1, "4-wave blocks: rms_norm of x only");
        constexpr int PP2 = 2 * PP;
        NormRow<PP2, 256> nr;
        nr.issue(a.x + (int64_t)r * a.x_stride, a.nw, K);
        float y[PP2][8];
        unpack_row(nr, K, y);
        sf = norm_core_e512(nr, K, a.eps, y, red);
        as = quant_row_tiled_wt<PP2, 256>(y, sf, K / 8, q8, r, nkb);
    }
    as = wave_sum_i(as);
    if (lane == 0) red_i[wave] = as;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) t += red_i[i];
        st_sc1(const_cast<int*>(a.act_sum) + r, t);
        st_sc1(const_cast<float*>(a.act_sf) + r, sf);
    }
}

// (measured, not kept: a 1-D grid placing a column block's row blocks on one XCD so the weight
// fragments they all decode come from one L2 -- batch 128 36.2k -> 35.5k tok/s, every GEMM 0.1-0.9 us
// slower; the GEMMs are latency-bound, not HBM-bound)
#ifndef WF_DG_WNT  // study: batched decode GEMM weight loads non-temporal, 1 for o / down, 2 for all
#define WF_DG_WNT 0  // (all: gate|up 15.8 -> 17.1 us; o / down alone: no change; ab_kv_nt_r04.txt)
#endif
template <int TMT, int TNT, int NB, int MODE, int NW = kDgWaves, int PRO = 0, int PP = 1>
__global__ __launch_bounds__(NW * 64, 2) void k_dec_gemm_t(GemvArgs a) {  // 2 waves / SIMD: 4-wave blocks 2 per CU
    constexpr int EPT = TMT * TNT / NW;  // epilogue tiles per wave
    static_assert(EPT * NW == TMT * TNT, "whole epilogue tiles per wave");
    __shared__ v4i_t red[NW][TMT * TNT][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int ct0 = blockIdx.x * TNT, rt0 = blockIdx.y * TMT;
    const int nkb = a.K >> 7;
    const int nct = a.N >> 4, nrt = (a.B + 15) >> 4;
    const int8_t* ap[TMT];
    const uint8_t* wp[TNT];
#pragma unroll
    for (int i = 0; i < TMT; ++i) ap[i] = a.q8 + ((int64_t)min(rt0 + i, nrt - 1) * nkb << 11) + lane * 16;
#pragma unroll
    for (int j = 0; j < TNT; ++j) wp[j] = a.w + ((int64_t)min(ct0 + j, nct - 1) * nkb << 9) + lane * 8;
    v4i_t acc[TMT][TNT];
#pragma unroll
    for (int i = 0; i < TMT; ++i)
#pragma unroll
        for (int j = 0; j < TNT; ++j) acc[i][j] = v4i_t{0, 0, 0, 0};
    uint4 fa[NB][TMT][2];
    uint2 fw[NB][TNT];
    // PRO: the codes were written in this launch -> sc1 loads (buffer offsets: the code tensor < 2 GB)
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(a.q8);
    auto load_a = [&](uint4 (&la)[TMT][2], int kb) {
#pragma unroll
        for (int i = 0; i < TMT; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if constexpr (PRO != 0)
                    la[i][h] = ld16_sc1(rq, (int)(ap[i] - a.q8) + (kb << 11) + (h << 10));
                else
                    la[i][h] = *reinterpret_cast<const uint4*>(ap[i] + ((int64_t)kb << 11) + (h << 10));
            }
    };
    auto load_w = [&](uint2 (&lw)[TNT], int kb) {
#pragma unroll
        for (int j = 0; j < TNT; ++j) {
            if constexpr (WF_DG_WNT == 2 || (WF_DG_WNT == 1 && (MODE == MODE_O || MODE == MODE_DN))) {
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(wp[j] + ((int64_t)kb << 9)));
                lw[j] = make_uint2(v.x, v.y);
            } else {
                lw[j] = *reinterpret_cast<const uint2*>(wp[j] + ((int64_t)kb << 9));
            }
        }
    };
    auto mma = [&](const uint4 (&la)[TMT][2], const uint2 (&lw)[TNT]) {
        // TNT <= 4: both halves of each code pair decoded at once (wf_mfma.h pg_decode_pair); at
        // TNT = 8 the second half's fragments would not fit beside the accumulators (spills)
        constexpr int NH = TNT <= 4 ? 2 : 1;
        v4i_t bf[NH][TNT];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (NH == 2) {
                if (h == 0)
#pragma unroll
                    for (int j = 0; j < TNT; ++j) pg_decode_pair(lw[j], bf[0][j], bf[1][j]);
            } else {
#pragma unroll
                for (int j = 0; j < TNT; ++j) {
                    const uint32_t w = h ? lw[j].y : lw[j].x;
                    bf[0][j] = v4i_t{(int)((w >> 6) & 0x03030303u), (int)((w >> 4) & 0x03030303u),
                                     (int)((w >> 2) & 0x03030303u), (int)(w & 0x03030303u)};
                }
            }
#pragma unroll
            for (int i = 0; i < TMT; ++i) {
                const v4i_t af = __builtin_bit_cast(v4i_t, la[i][h]);
#pragma unroll
                for (int j = 0; j < TNT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[NH == 2 ? h : 0][j], acc[i][j], 0, 0, 0);
            }
        }
    };
    const int cnt = (nkb - wave + NW - 1) / NW;
    WF_STAMP_BASE(512u * MODE);  // stamps build: one region per op (batch > 1; k_gemv's at batch 1)
    WF_STAMP(0);
    EpiDec<MODE> e{&a};
    int er0[EPT], ec0[EPT];
    EpiIn ein[EPT];
#pragma unroll
    for (int x = 0; x < EPT; ++x) {
        const int tile = wave * EPT + x;
        er0[x] = (rt0 + tile / TNT) * 16;
        ec0[x] = (ct0 + tile % TNT) * 16;
    }
    if constexpr (PRO != 0) {
        __shared__ float s_red[16];
        __shared__ int s_red_i[NW];
        const int ty = blockIdx.y, rows = min(32, a.B - 32 * ty);
        unsigned* arrive = a.seam + ty * kSeamLine;
        const bool producer = (int)blockIdx.x < rows;
        // blocks that only wait start their weight stream now; a producing block first normalises its
        // row (its loads must not queue behind the weights: loads return in order) and publishes
        // (the drain before the arrival waits for every load in flight, weights included)
        // wave 0 polls: its loads return in order, so it issues its own weights only after the wait
        if (producer) {
            dec_row_prologue<PRO, PP, NW>(a, 32 * ty + blockIdx.x, s_red, s_red_i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's sc1 stores are done
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (wave != 0) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
                if (b < cnt) load_w(fw[b], wave + NW * b);
        }
        WF_STAMP(14);
        if (threadIdx.x == 0) {
            unsigned spins = 0;
            while (ld_sc1(arrive) < (unsigned)rows && ++spins < kSeamSpin) __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int b = 0; b < NB; ++b)
                if (b < cnt) load_w(fw[b], wave + NW * b);
        }
        WF_STAMP(15);
#pragma unroll
        for (int x = 0; x < EPT; ++x) e.template load<true>(er0[x], ec0[x], l16, q, ein[x]);
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (b < cnt) load_a(fa[b], wave + NW * b);
    } else {
#pragma unroll
        for (int x = 0; x < EPT; ++x) e.load(er0[x], ec0[x], l16, q, ein[x]);
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (b < cnt) {
                load_a(fa[b], wave + NW * b);
                load_w(fw[b], wave + NW * b);
            }
    }
#pragma unroll
    for (int x = 0; x < EPT; ++x) e.load_rope(ec0[x], l16, ein[x]);
    WF_STAMP(1);
    for (int t0 = 0; t0 < cnt; t0 += NB) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int t = t0 + b;
            if (t < cnt) {
                mma(fa[b], fw[b]);
                if (t == 0) WF_STAMP(2);
                if (t + NB < cnt) {
                    load_a(fa[b], wave + NW * (t + NB));
                    load_w(fw[b], wave + NW * (t + NB));
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TMT; ++i)
#pragma unroll
        for (int j = 0; j < TNT; ++j) red[wave][i * TNT + j][lane] = acc[i][j];
    WF_STAMP(3);
    __syncthreads();
    WF_STAMP(4);
#pragma unroll
    for (int x = 0; x < EPT; ++x) {
        const int tile = wave * EPT + x;
        v4i_t sum = red[0][tile][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) sum += red[w][tile][lane];
        e.apply(er0[x], ec0[x], sum, l16, q, ein[x]);
    }
    if constexpr (PRO != 0) {
        // re-arm: every block of the tile is past its wait once all have counted in here (the add is
        // at the end so its return does not hold this block's loads)
        if (threadIdx.x == 0) {
            unsigned* arrive = a.seam + blockIdx.y * kSeamLine;
            unsigned* passed = a.seam + (kSeamTiles + blockIdx.y) * kSeamLine;
            const unsigned old = __hip_atomic_fetch_add(passed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == gridDim.x - 1u) {
                st_sc1(arrive, 0u);
                st_sc1(passed, 0u);
            }
        }
    }
    WF_STAMP(5);
    WF_STAMP_DRAIN(6);
}

// Prefill q|k|v epilogue, staged through the (idle) LDS ring: the decode step's EpiDec<MODE_QKV>
// float sequence, but (1) the per-row inputs (scale, code sum, position, slot, page) are loaded
// once per row into LDS; (2) every wave writes its 16 fragments' corrected bf16 values into a
// 128 x 256 LDS tile in the GEMM's column order (a 16-column tile = dims 8 tt .. +7 and 64 + 8 tt ..
// +7 of one head: both RoPE halves of 8 dims are 32 contiguous LDS bytes); (3) the block then
// writes whole pieces: q rows and K tile rows as 16-byte pieces of 8 dims (RoPE from 16-byte cos /
// sin loads), V tile pieces of 8 consecutive keys of one dim (one 16-byte store when the 8 rows
// are positions 8a .. 8a + 7 of one slot, else per element). The per-fragment form (scattered
// 2-byte stores, two dependent loads per fragment) spilled its accumulators (272 B per lane).
constexpr int kPfEpiRS = 256 * 2 + 16;  // LDS row stride of the staged tile (bytes)
template <bool CW>
__device__ __forceinline__ void pf_qkv_epilogue(const GemvArgs& g, int bm, int bn, const v4i_t (&acc)[4][4],
                                                uint8_t* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    uint8_t* tile = lds;                                              // [128][kPfEpiRS]
    float* s_sf = reinterpret_cast<float*>(lds + 128 * kPfEpiRS);     // [128]
    int* s_as = reinterpret_cast<int*>(s_sf + 128);                    // [128]
    int* s_pos = s_as + 128;                                           // [128] clamped position
    int* s_slot = s_pos + 128;                                         // [128]
    int* s_pg = s_slot + 128;                                          // [128] page of the position (paged)
    __syncthreads();  // every wave is done with the ring
    if (threadIdx.x < 128) {
        const int mc = min(bm * 128 + (int)threadIdx.x, g.B - 1);
        s_sf[threadIdx.x] = g.act_sf[mc];
        s_as[threadIdx.x] = g.act_sum[mc];
        const int pos = min(max(g.positions[mc], 0), g.S - 1);
        const int slot = g.row_slot ? g.row_slot[mc] : mc;
        s_pos[threadIdx.x] = pos;
        s_slot[threadIdx.x] = slot;
        s_pg[threadIdx.x] = g.pt ? min(max(g.pt[(int64_t)slot * g.pps + (pos >> 5)], 0), g.npages - 1) : 0;
    }
    __syncthreads();
    const int head0 = bn * 2, nheads = g.Hq + 2 * g.Hkv;
    // the row tile of fragment (i, j) does not depend on j in the 2 x 4 wave grid: its rows' scale
    // and code sum are read from LDS once per (i, r), not once per fragment
    float sfv[4][4];
    int asv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rl = pg_frag_rt<4, CW>(wave, i, 0) * 16 + 4 * q + r;
            sfv[i][r] = s_sf[rl];
            asv[i][r] = s_as[rl];
        }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ct = pg_frag_ct<4, CW>(wave, i, j), head = head0 + (ct >> 3);
            const float ws = head < g.Hq ? g.ws0 : (head < g.Hq + g.Hkv ? g.ws1 : g.ws2);
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // rows in pairs (pf_tile_epilogue's packed form)
                const int rl = pg_frag_rt<4, CW>(wave, i, j) * 16 + 4 * q + 2 * h;
                const uint32_t vp =
                    CW ? corrected_pk(acc[i][j][2 * h], acc[i][j][2 * h + 1], ws, s_as[rl], s_as[rl + 1], s_sf[rl], s_sf[rl + 1])
                       : corrected_pk(acc[i][j][2 * h], acc[i][j][2 * h + 1], ws, asv[i][2 * h], asv[i][2 * h + 1],
                                      sfv[i][2 * h], sfv[i][2 * h + 1]);
                const uint32_t np = (uint32_t)dpp_i<DPP_QP_1032>((int)vp);  // column l16 ^ 1, same rows
                if (!(l16 & 1)) {
                    *reinterpret_cast<uint32_t*>(tile + rl * kPfEpiRS + (16 * ct + l16) * 2) = __builtin_amdgcn_perm(np, vp, 0x05040100u);
                    *reinterpret_cast<uint32_t*>(tile + (rl + 1) * kPfEpiRS + (16 * ct + l16) * 2) =
                        __builtin_amdgcn_perm(np, vp, 0x07060302u);
                }
            }
        }
    }
    __syncthreads();
    const int8_t kv8 = (int8_t)g.kv8;
    // q and k heads: item = (row, column tile) -> 8 dims of each RoPE half. Every item's cos / sin
    // pieces are in flight before the first item is processed (a load inside the item loop waited
    // one L2 round trip per item: its stores may alias the tables)
    constexpr int kQkItems = 128 * 16 / 512;
    uint4 csv[kQkItems], snv[kQkItems];
#pragma unroll
    for (int k = 0; k < kQkItems; ++k) {
        const int it = threadIdx.x + 512 * k, rl = it >> 4, tt = it & 7;
        const int pos = s_pos[rl];
        csv[k] = *reinterpret_cast<const uint4*>(g.rope_cos + (int64_t)pos * 64 + 8 * tt);
        snv[k] = *reinterpret_cast<const uint4*>(g.rope_sin + (int64_t)pos * 64 + 8 * tt);
    }
#pragma unroll
    for (int k = 0; k < kQkItems; ++k) {
        const int it = threadIdx.x + 512 * k;
        const int rl = it >> 4, ct = it & 15, tt = ct & 7, head = head0 + (ct >> 3);
        const int m = bm * 128 + rl;
        if (m >= g.B || head >= g.Hq + g.Hkv) continue;
        const uint4 lo = *reinterpret_cast<const uint4*>(tile + rl * kPfEpiRS + ct * 32);
        const uint4 hi = *reinterpret_cast<const uint4*>(tile + rl * kPfEpiRS + ct * 32 + 16);
        const int pos = s_pos[rl];
        const uint4 cs = csv[k];
        const uint4 sn = snv[k];
        const uint32_t x1[4] = {lo.x, lo.y, lo.z, lo.w}, x2[4] = {hi.x, hi.y, hi.z, hi.w};
        const uint32_t c4[4] = {cs.x, cs.y, cs.z, cs.w}, s4[4] = {sn.x, sn.y, sn.z, sn.w};
        // RotaryEmbedding._rotate (direct_inference_full.py:58-70) on packed bf16 pairs: y1 = x1 c -
        // x2 s, y2 = x1 s + x2 c, every product and sum rounded to bf16 (rope_pk)
        uint32_t p1[4], p2[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) rope_pk(x1[t], x2[t], c4[t], s4[t], p1[t], p2[t]);
        float y1[8], y2[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            y1[e] = (e & 1) ? bf_hi(p1[e >> 1]) : bf_lo(p1[e >> 1]);
            y2[e] = (e & 1) ? bf_hi(p2[e >> 1]) : bf_lo(p2[e >> 1]);
        }
        if (head < g.Hq) {
            uint16_t* qo = g.out + (int64_t)m * g.out_stride + head * 128 + 8 * tt;
            *reinterpret_cast<uint4*>(qo) = make_uint4(p1[0], p1[1], p1[2], p1[3]);
            *reinterpret_cast<uint4*>(qo + 64) = make_uint4(p2[0], p2[1], p2[2], p2[3]);
            continue;
        }
        const int kvh = head - g.Hq;
        const int64_t base = g.pt ? (int64_t)s_pg[rl] * g.kv_pgs + (int64_t)kvh * 4096
                                  : (int64_t)s_slot[rl] * g.kv_b_stride + (int64_t)kvh * g.S * 128;
        const int t = g.pt ? (pos & 31) : pos;
        const int64_t o1 = base + k_tile_off(t, 8 * tt), o2 = base + k_tile_off(t, 64 + 8 * tt);
        if (kv8) {
            uint8_t* c8 = reinterpret_cast<uint8_t*>(g.kc);
            uint32_t b1[2] = {0u, 0u}, b2[2] = {0u, 0u};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                b1[e >> 2] |= (uint32_t)to_kv8(y1[e] / g.k_div, kv8) << (8 * (e & 3));
                b2[e >> 2] |= (uint32_t)to_kv8(y2[e] / g.k_div, kv8) << (8 * (e & 3));
            }
            *reinterpret_cast<uint2*>(c8 + o1) = make_uint2(b1[0], b1[1]);
            *reinterpret_cast<uint2*>(c8 + o2) = make_uint2(b2[0], b2[1]);
        } else {
            *reinterpret_cast<uint4*>(g.kc + o1) = make_uint4(p1[0], p1[1], p1[2], p1[3]);
            *reinterpret_cast<uint4*>(g.kc + o2) = make_uint4(p2[0], p2[1], p2[2], p2[3]);
        }
    }
    // v heads: item = (8-row group, dim) -> one V tile piece of 8 keys
    for (int it = threadIdx.x; it < 16 * 256; it += 512) {
        const int g8 = it >> 8, col = it & 255, d = col & 127, head = head0 + (col >> 7);
        if (head < g.Hq + g.Hkv || head >= nheads) continue;
        const int kvh = head - g.Hq - g.Hkv;
        const int lc = 16 * ((col >> 7) * 8 + ((d & 63) >> 3)) + (d & 7) + (d >= 64 ? 8 : 0);  // staged column
        uint16_t vv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vv[e] = *reinterpret_cast<const uint16_t*>(tile + (8 * g8 + e) * kPfEpiRS + lc * 2);
        const int r0 = 8 * g8, m0 = bm * 128 + r0;
        const int p0 = s_pos[r0], sl0 = s_slot[r0];
        bool whole = m0 + 7 < g.B && (p0 & 7) == 0;
#pragma unroll
        for (int e = 1; e < 8; ++e) whole = whole && s_pos[r0 + e] == p0 + e && s_slot[r0 + e] == sl0;
        if (whole) {
            const int64_t base = g.pt ? (int64_t)s_pg[r0] * g.kv_pgs + (int64_t)kvh * 4096
                                      : (int64_t)sl0 * g.kv_b_stride + (int64_t)kvh * g.S * 128;
            const int64_t off = base + v_tile_off(g.pt ? (p0 & 31) : p0, d);
            if (kv8) {
                uint32_t b[2] = {0u, 0u};
#pragma unroll
                for (int e = 0; e < 8; ++e) b[e >> 2] |= (uint32_t)to_kv8(bf2f(vv[e]) / g.v_div, kv8) << (8 * (e & 3));
                *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(g.vc) + off) = make_uint2(b[0], b[1]);
            } else {
                *reinterpret_cast<uint4*>(g.vc + off) = make_uint4(vv[0] | (uint32_t)vv[1] << 16, vv[2] | (uint32_t)vv[3] << 16,
                                                                   vv[4] | (uint32_t)vv[5] << 16, vv[6] | (uint32_t)vv[7] << 16);
            }
            continue;
        }
        for (int e = 0; e < 8; ++e) {  // ragged group: per element
            const int rl = r0 + e;
            if (bm * 128 + rl >= g.B) break;
            const int pos = s_pos[rl];
            const int64_t base = g.pt ? (int64_t)s_pg[rl] * g.kv_pgs + (int64_t)kvh * 4096
                                      : (int64_t)s_slot[rl] * g.kv_b_stride + (int64_t)kvh * g.S * 128;
            const int64_t off = base + v_tile_off(g.pt ? (pos & 31) : pos, d);
            if (kv8) reinterpret_cast<uint8_t*>(g.vc)[off] = to_kv8(bf2f(vv[e]) / g.v_div, kv8);
            else g.vc[off] = vv[e];
        }
    }
}

// Prefill GU / O / DN epilogue, staged through the (idle) LDS ring: EpiDec's float sequence, but the
// per-row inputs are loaded once per row into LDS, every wave writes its fragments' bf16 results
// (GU: the act = bf16(bf16(relu(g)^2) * u) values) into a 128-row LDS tile, and the block then
// stores whole 16-byte pieces of rows (O / DN: + the residual, read as 16-byte pieces). The
// per-fragment form stored 2-byte elements, 32 or 64 per wave-instruction: measured with the main
// loop removed, the GU epilogue alone took 103 us per layer at 16384 rows (store-issue bound;
// ~28 us of HBM writes), O / DN 64 us, and with one block per CU it is not overlapped by MFMAs.
// Needs out_stride % 8 == 0 and a 16-byte aligned out / resid (checked by the host).
template <int MODE, int TNW>
constexpr int pf_tile_epilogue_bytes() {  // staged tile + per-row scale / code sum
    return 128 * ((MODE == MODE_GU ? pg_block_cols<TNW>() / 2 : pg_block_cols<TNW>()) * 2 + 32) + 128 * 8;
}
template <int MODE, int TNW, bool CW>
__device__ __forceinline__ void pf_tile_epilogue(const GemvArgs& g, int bm, int bn, const v4i_t (&acc)[4][TNW],
                                                 uint8_t* lds) {
    static_assert(MODE == MODE_GU || MODE == MODE_O || MODE == MODE_DN, "row-tile epilogues");
    constexpr int BC = pg_block_cols<TNW>();
    constexpr int OC = MODE == MODE_GU ? BC / 2 : BC;  // output columns of the block
    constexpr int RS = OC * 2 + 32;                     // LDS row stride: 4 rows of a fragment 8 banks apart
    constexpr int PPR = OC / 8;                         // 16-byte pieces per row
    static_assert(pf_tile_epilogue_bytes<MODE, TNW>() <= PgCfg<TNW, CW ? 3 : 0>::LDS, "staged tile fits the ring");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    constexpr int IT = 128 * PPR / 512;                 // store items per thread
    static_assert(IT * 512 == 128 * PPR, "whole items per thread");
    uint8_t* tile = lds;
    float* s_sf = reinterpret_cast<float*>(lds + 128 * RS);
    int* s_as = reinterpret_cast<int*>(s_sf + 128);
    const int limit = MODE == MODE_GU ? g.N / 2 : g.N;
    // O / DN: every residual piece of this thread in flight before the LDS phase (a load inside the
    // store loop would wait one HBM round trip per item: stores may alias it)
    uint4 rsv[MODE == MODE_GU ? 1 : IT];
    if constexpr (MODE != MODE_GU) {
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int it = threadIdx.x + 512 * k, rl = it / PPR, pc = it % PPR;
            const int m = min(bm * 128 + rl, g.B - 1), n = min(bn * OC + pc * 8, limit - 8);
            rsv[k] = *reinterpret_cast<const uint4*>(g.resid + (int64_t)m * g.out_stride + n);
        }
    }
    __syncthreads();  // every wave is done with the ring
    if (threadIdx.x < 128) {
        const int mc = min(bm * 128 + (int)threadIdx.x, g.B - 1);
        s_sf[threadIdx.x] = g.act_sf[mc];
        s_as[threadIdx.x] = g.act_sum[mc];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TNW; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rt = pg_frag_rt<TNW, CW>(wave, i, j), ct = pg_frag_ct<TNW, CW>(wave, i, j);
            const float ws = (MODE == MODE_GU && l16 >= 8) ? g.ws1 : g.ws0;
#pragma unroll
            for (int r = 0; r < 4 && MODE == MODE_GU; ++r) {
                const int rl = rt * 16 + 4 * q + r;
                const float v = rbf(corrected(acc[i][j][r], ws, s_as[rl], s_sf[rl]));
                if constexpr (MODE == MODE_GU) {
                    const float pv = __shfl_xor(v, 8, 64);  // up column l16 + 8 of the same row
                    const float gt = fmaxf(v, 0.f);
                    const float y = rbf(rbf(gt * gt) * pv);
                    const float ny = dpp_f<DPP_QP_1032>(y);  // column l16 ^ 1
                    if (l16 < 8 && !(l16 & 1)) *reinterpret_cast<uint32_t*>(tile + rl * RS + (ct * 8 + l16) * 2) = pk_bf16(y, ny);
                }
            }
            if constexpr (MODE != MODE_GU) {
                // rows in pairs: one packed correction, one DPP for both rows' column l16 ^ 1, and
                // the (column l16, l16 ^ 1) words of each row assembled by v_perm
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int rl = rt * 16 + 4 * q + 2 * h;
                    const uint32_t vp = corrected_pk(acc[i][j][2 * h], acc[i][j][2 * h + 1], ws, s_as[rl], s_as[rl + 1],
                                                     s_sf[rl], s_sf[rl + 1]);
                    const uint32_t np = (uint32_t)dpp_i<DPP_QP_1032>((int)vp);  // column l16 ^ 1, same rows
                    if (!(l16 & 1)) {
                        *reinterpret_cast<uint32_t*>(tile + rl * RS + (ct * 16 + l16) * 2) = __builtin_amdgcn_perm(np, vp, 0x05040100u);
                        *reinterpret_cast<uint32_t*>(tile + (rl + 1) * RS + (ct * 16 + l16) * 2) =
                            __builtin_amdgcn_perm(np, vp, 0x07060302u);
                    }
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int it = threadIdx.x + 512 * k, rl = it / PPR, pc = it % PPR;
        const int m = bm * 128 + rl, n = bn * OC + pc * 8;
        if (m >= g.B || n >= limit) continue;
        uint4 v = *reinterpret_cast<const uint4*>(tile + rl * RS + pc * 16);
        if constexpr (MODE != MODE_GU) {  // out = bf16(resid + bf16(o))
            const uint4 rs = rsv[k];
            uint32_t ov[4] = {v.x, v.y, v.z, v.w};
            const uint32_t rv[4] = {rs.x, rs.y, rs.z, rs.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                ov[e] = bf16_add_pk(rv[e], ov[e]);
            v = make_uint4(ov[0], ov[1], ov[2], ov[3]);
        }
        *reinterpret_cast<uint4*>(g.out + (int64_t)m * g.out_stride + n) = v;
    }
}

// Prefill GEMM (rows = prompt tokens) on the tile layouts with the decode step's fused epilogues:
// the wf_mfma.h 128 x 256 tile main loop (pgemm_tile), then EpiDec<MODE> per 16 x 16 fragment
// (correction, RoPE + K/V cache write through row_slot, residual, ReLU^2 * up).
// Per-fragment epilogue of a prefill GEMM tile (gate|up, or any mode without the staged tile)
template <int MODE, int TNW, bool CW>
__device__ __forceinline__ void pf_frag_epilogue(const GemvArgs& a, int bm, int bn, v4i_t (&acc)[4][TNW]) {
    constexpr int BC = pg_block_cols<TNW>();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    (void)lane;
    if constexpr (MODE == MODE_GU && !CW && TNW % 2 == 0) {
        // gate|up, 16-byte stores: fragments j, j + 1 hold act columns 8 T .. 8 T + 15 of the same
        // rows (T = their first 16-column tile, even). After gu_pack lane quad 0 has columns 0-3 and
        // quad 1 columns 4-7 of each; quad 0 takes quad 1's part of fragment j (DPP row_shl:4), quad 1
        // quad 0's part of fragment j + 1 (row_shr:4), and each stores 8 columns = one dwordx4: half
        // the store instructions of one dwordx2 per fragment (the epilogue is store-issue-bound)
        if (((a.out_stride & 7) | (reinterpret_cast<uintptr_t>(a.out) & 15)) == 0) {
            EpiDec<MODE> e{&a};
            const int k = (l16 >> 2) & 1, qi = l16 & 3;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r0 = bm * 128 + pg_frag_rt<TNW, CW>(wave, i, 0) * 16, m = r0 + 4 * q + qi;
                EpiIn in;
                e.load(r0, bn * BC + pg_frag_ct<TNW, CW>(wave, i, 0) * 16, l16, q, in);
#pragma unroll
                for (int p = 0; p < TNW / 2; ++p) {
                    const uint2 y0 = e.gu_pack(acc[i][2 * p], in, l16), y1 = e.gu_pack(acc[i][2 * p + 1], in, l16);
                    // both exchanges in every lane (a DPP inside a divergent branch reads disabled lanes as 0)
                    const int sx = (int)(k ? y0.x : y1.x), sy = (int)(k ? y0.y : y1.y);
                    const uint32_t ux = (uint32_t)dpp_i<0x104>(sx), uy = (uint32_t)dpp_i<0x104>(sy);  // lane + 4
                    const uint32_t dx = (uint32_t)dpp_i<0x114>(sx), dy = (uint32_t)dpp_i<0x114>(sy);  // lane - 4
                    const uint32_t rx = k ? dx : ux, ry = k ? dy : uy;
                    const uint4 o = k ? make_uint4(rx, ry, y1.x, y1.y) : make_uint4(y0.x, y0.y, rx, ry);
                    const int T = (bn * BC + pg_frag_ct<TNW, CW>(wave, i, 2 * p) * 16) / 16 + k;
                    if (l16 < 8 && m < a.B && T * 16 < a.N)
                        *reinterpret_cast<uint4*>(a.out + (int64_t)m * a.out_stride + T * 8) = o;
                }
            }
            return;
        }
    }
    // epilogue per row tile: the column tiles' per-row inputs (scale, code sum, residual) are all
    // issued before the first store -- one round trip per row tile instead of per fragment (stores
    // in between would pin the loads behind them): o 159 -> 141, down 291 -> 274 us
    EpiDec<MODE> e{&a};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        EpiIn in[TNW];
#pragma unroll
        for (int j = 0; j < TNW; ++j)
            e.load(bm * 128 + pg_frag_rt<TNW, CW>(wave, i, j) * 16, bn * BC + pg_frag_ct<TNW, CW>(wave, i, j) * 16, l16, q, in[j]);
#pragma unroll
        for (int j = 0; j < TNW; ++j)
            e.apply(bm * 128 + pg_frag_rt<TNW, CW>(wave, i, j) * 16, bn * BC + pg_frag_ct<TNW, CW>(wave, i, j) * 16, acc[i][j], l16,
                    q, in[j]);
    }
}

// Prefill GEMM (rows = prompt tokens) on the tile layouts with the decode step's fused epilogues:
// the wf_mfma.h 128 x 256 tile main loop (pgemm_tile), then EpiDec<MODE> per 16 x 16 fragment
// (correction, RoPE + K/V cache write through row_slot, residual, ReLU^2 * up).
template <int MODE, int TNW = 4, int ALG = 0, bool STAGED = false>
__global__ __launch_bounds__(512) void k_pgemm_fused(GemvArgs a, int nbm, int nbn) {
    static_assert(MODE != MODE_QKV || TNW == 4, "the q|k|v epilogue stages 256 columns (two heads)");
    __shared__ __attribute__((aligned(16))) uint8_t lds[PgCfg<TNW, ALG>::LDS];
    constexpr bool CW = PgCfg<TNW, ALG>::CW;
    int bm, bn;
    pg_tile_of(blockIdx.x, nbm, nbn, bm, bn);
    v4i_t acc[4][TNW];
    pg_main<TNW, ALG>(a.w, a.q8, a.B, a.N, a.K, bm, bn, lds, acc);
    if constexpr (MODE == MODE_QKV) {
        pf_qkv_epilogue<CW>(a, bm, bn, acc, lds);
    } else if constexpr (STAGED) {
        pf_tile_epilogue<MODE, TNW, CW>(a, bm, bn, acc, lds);
    } else {
        pf_frag_epilogue<MODE, TNW, CW>(a, bm, bn, acc);
    }
}

// The same GEMM as a persistent tile loop (per-fragment epilogues only: the staged epilogues use the
// ring's LDS): one block per CU takes tiles blockIdx.x + i gridDim.x (gridDim.x % 8 == 0 keeps every
// tile on the XCD pg_tile_of gives it), and the next tile's first P - 1 ring stages are issued before
// this tile's epilogue, so their HBM / L2 latency overlaps the epilogue's VALU and stores instead of
// following them (one-shot blocks pay it after the previous block on the CU has exited).
template <int MODE, int TNW>
__global__ __launch_bounds__(512) void k_pgemm_fused_pt(GemvArgs a, int nbm, int nbn) {
    constexpr int P = PgCfg<TNW, 0>::P;
    __shared__ __attribute__((aligned(16))) uint8_t lds[PgCfg<TNW, 0>::LDS];
    const int nt = nbm * nbn;
    int t = blockIdx.x, bm, bn;
    if (t >= nt) return;  // whole block
    pg_tile_of(t, nbm, nbn, bm, bn);
    PgDma<P, TNW>(a.w, a.q8, a.B, a.N, a.K, bm, bn).prologue(lds, a.K);
    for (;;) {
        v4i_t acc[4][TNW];
        pg_main<TNW, 0, true>(a.w, a.q8, a.B, a.N, a.K, bm, bn, lds, acc);
        const int tn = t + (int)gridDim.x;
        int bm2 = 0, bn2 = 0;
        __builtin_amdgcn_s_barrier();  // every wave's last fragment reads are done: the ring is free
        if (tn < nt) {
            pg_tile_of(tn, nbm, nbn, bm2, bn2);
            PgDma<P, TNW>(a.w, a.q8, a.B, a.N, a.K, bm2, bn2).prologue(lds, a.K);
        }
        pf_frag_epilogue<MODE, TNW, false>(a, bm, bn, acc);
        if (tn >= nt) break;
        t = tn;
        bm = bm2;
        bn = bn2;
    }
}

// One wave per 16 x 16 output tile: lane (l16, q) sums the nsplit int32 partials of rows
// r0 + 4q + r, column c0 + l16 and runs EpiDec on them (same fragment layout as the GEMM).
template <int MODE>
__global__ __launch_bounds__(256) void k_dec_epi(GemvArgs a, const int* __restrict__ ws, int nsplit) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int c0 = (blockIdx.x * 4 + wave) * 16, r0 = blockIdx.y * 16;
    if (c0 >= a.N) return;  // whole wave
    const int n = min(c0 + l16, a.N - 1);
    v4i_t acc = {0, 0, 0, 0};
    const int64_t plane = (int64_t)a.B * a.N;
    for (int s = 0; s < nsplit; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += ws[s * plane + (int64_t)min(r0 + 4 * q + r, a.B - 1) * a.N + n];
    EpiDec<MODE> e{&a};
    e.apply(r0, c0, acc, l16, q);
}

// BitNetLinear for many rows: per-row int8 codes (k_quant_rows_lin) -> MFMA GEMM -> this epilogue.
struct EpiLinear {
    const GemvArgs* a;
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) {
        const GemvArgs& g = *a;
        const int n = c0 + l16;
        if (n >= g.N) return;
        const LinSeg sg = lin_seg(g, n);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r0 + 4 * q + r;
            if (m < g.B) sg.out[(int64_t)m * sg.ld + sg.col] = f2bf(corrected(acc[r], sg.ws, g.act_sum[m], g.act_sf[m]));
        }
    }
};
// the same epilogue by value for the small-M kernel (wf_small.h)
struct EpiLinearSmall {
    GemvArgs a;
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) const {
        EpiLinear{&a}.apply(r0, c0, acc, l16, q);
    }
};
__global__ __launch_bounds__(256) void k_linear_mfma(GemvArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kTgStagesWide * kTgStageBytes];
    EpiLinear e{&a};
    tgemm_tile<2, kTgStagesWide>(a.w, a.q8, a.q8_stride, a.B, a.N, a.K, blockIdx.y * 128, blockIdx.x * 128, lds, e);
}
// per-row activation quantizer of BitNetLinear: codes, float scale, code sum
// BitNet MLP activation (direct_inference_full.py:258): g <- bf16(bf16(relu(g)^2) * u), 8 elements per
// thread (n % 8 == 0, 16-byte aligned rows)
__global__ __launch_bounds__(256) void k_relu2_mul(uint16_t* __restrict__ g, const uint16_t* __restrict__ u, int64_t n8) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const uint4 gv = reinterpret_cast<const uint4*>(g)[i], uv = reinterpret_cast<const uint4*>(u)[i];
    const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, uw[4] = {uv.x, uv.y, uv.z, uv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float g0 = fmaxf(bf_lo(gw[j]), 0.f), g1 = fmaxf(bf_hi(gw[j]), 0.f);
        o[j] = pk_bf16(rbf(rbf(g0 * g0) * bf_lo(uw[j])), rbf(rbf(g1 * g1) * bf_hi(uw[j])));
    }
    reinterpret_cast<uint4*>(g)[i] = make_uint4(o[0], o[1], o[2], o[3]);
}

template <int PPT>
__global__ __launch_bounds__(kNT) void k_quant_rows_lin(const uint16_t* __restrict__ x, int64_t xs, int K,
                                                        int8_t* __restrict__ q8, int64_t q8s, float* __restrict__ sf,
                                                        int* __restrict__ asum) {
    __shared__ float red[2 * kNT / 64];
    __shared__ int red_i[kNT / 64];
    const int b = blockIdx.x;
    NormRow<PPT, kNT> nr;
    const int npk = K >> 3;
#pragma unroll
    for (int i = 0; i < PPT; ++i) nr.x[i] = *reinterpret_cast<const uint4*>(x + b * xs + 8 * min((int)threadIdx.x + kNT * i, npk - 1));
    float y[PPT][8];
    unpack_row(nr, K, y);
    const float s = absmax_scale<PPT, kNT>(y, red);
    int as = quant_row<PPT, kNT>(y, s, K / 8, q8 + (int64_t)b * q8s, [](int p) { return 8 * p; });
    as = wave_sum_i(as);
    if ((threadIdx.x & 63) == 0) red_i[threadIdx.x >> 6] = as;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < kNT / 64; ++i) t += red_i[i];
        asum[b] = t;
        sf[b] = s;
    }
}

// [R][H] bf16 -> the fragment layout (bf_tile_off), one thread per 8-element piece (R % 16 == 0).
__global__ void k_bf_tile(const uint16_t* __restrict__ src, int R, int H, uint16_t* __restrict__ dst) {
    const int64_t np = (int64_t)R * (H >> 3);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < np; t += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / (H >> 3)), p = (int)(t % (H >> 3));
        *reinterpret_cast<uint4*>(dst + bf_tile_off(r, p, H)) = *reinterpret_cast<const uint4*>(src + t * 8);
    }
}

// Batched LM head: logits[b, v] = bf16(sum_k hn[b, k] E[v, k]) on v_mfma_f32_16x16x32_bf16 (fp32
// accumulation; lane quarter q takes k = 32s + 8q + 0..7 of step s for both operands). Block = 128
// sequences x 256 vocabulary rows, 4 waves x 64 rows; each k-step is an LDS-DMA pipeline stage
// (wf_mfma.h scheme): A = hn 8 KiB (wave w loads row tiles 2w, 2w+1), B = the wave's 64 embedding
// rows x 64 B = 4 KiB; 6 DMA loads per wave per stage. E is read from HBM exactly once.
// Per (row, block) the (max, first index) of the block's 256 logits goes to `part`.
typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef float v4f_t __attribute__((ext_vector_type(4)));
// NW waves of 64 vocabulary rows per block (round 4: 8 waves = 512 rows): every block re-reads the
// whole 640 KB A (hn) from L2 through LDS, so at 256 rows A was a third of the LDS-DMA traffic the
// launch is bound by (984 MB for 657 MB of E); at 512 rows a fifth (816 MB). P stages in the ring
// (3 at 8 waves: 40 KiB stages).
#ifndef WF_LM_WAVES  // study builds only (tools/build_var.sh)
#define WF_LM_WAVES 8
#endif
constexpr int kLmWaves = WF_LM_WAVES;
constexpr int kLmStages = kLmWaves == 4 ? 4 : 3;
template <int NW>
constexpr int lm_stage_bytes() { return 8 * 1024 + NW * 4096; }
#ifndef WF_LM_NT  // study: 0 = the batched LM head's embedding DMAs without the non-temporal hint
#define WF_LM_NT 1
#endif
template <int NW, int P>
__global__ __launch_bounds__(NW * 64) void k_lm_head_mfma(const uint16_t* __restrict__ E, const uint16_t* __restrict__ hn,
                                                          int H, int V, int B, uint16_t* __restrict__ logits,
                                                          uint2* __restrict__ part, int nblk) {
    static_assert(NW == 4 || NW == 8, "A row tiles: 2 per wave at 4 waves, 1 at 8");
    constexpr int SB = lm_stage_bytes<NW>(), AU = 8 / NW, NDMA = AU + 4;
    __shared__ __attribute__((aligned(16))) uint8_t lds[P * SB];
    __shared__ float s_val[NW][128];
    __shared__ int s_idx[NW][128];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const int m0 = blockIdx.y * 128, n0 = blockIdx.x * (64 * NW) + wave * 64;
    const int steps = H / 32;
    // both operands in the fragment layout (bf_tile_off): fragment (tile, k-step c) of this lane at
    // tile_base + 512 c elements -- one contiguous KiB per wave-instruction
    const int nrt = (B + 15) >> 4, nvt = V >> 4;
    const uint16_t* asrc[AU];
#pragma unroll
    for (int u = 0; u < AU; ++u) asrc[u] = hn + (((int64_t)min((m0 >> 4) + AU * wave + u, nrt - 1) * steps) << 9) + lane * 8;
    const uint16_t* bsrc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bsrc[j] = E + (((int64_t)min((n0 >> 4) + j, nvt - 1) * steps) << 9) + lane * 8;
    auto issue = [&](int c) {
        uint8_t* st = lds + (c % P) * SB;
#pragma unroll
        for (int u = 0; u < AU; ++u) glds16_asm(asrc[u] + 512 * c, st + (AU * wave + u) * 1024);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // embedding tiles: read once per step (non-temporal); hn is re-read
            if constexpr (WF_LM_NT) glds16_asm_nt(bsrc[j] + 512 * c, st + 8192 + wave * 4096 + j * 1024);
            else glds16_asm(bsrc[j] + 512 * c, st + 8192 + wave * 4096 + j * 1024);
        }
    };
    v4f_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v4f_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < P - 1; ++c)
        if (c < steps) issue(c);
    for (int c = 0; c < steps; ++c) {
        if (c + P - 2 < steps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA * (P - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (c + P - 1 < steps) issue(c + P - 1);
        const uint8_t* st = lds + (c % P) * SB;
        v8s_t bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const v8s_t*>(st + 8192 + wave * 4096 + j * 1024 + lane * 16);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const v8s_t af = *reinterpret_cast<const v8s_t*>(st + i * 1024 + lane * 16);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
        }
    }
    // epilogue: bf16 logits; per row the (max, first index) over this wave's 64 columns
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * i + 4 * q + r, m = m0 + row;
            float bv = -INFINITY;
            int bi = 0x7fffffff;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + 16 * j + l16;
                const uint16_t lb = f2bf(acc[i][j][r]);
                if (m < B && n < V) logits[(int64_t)m * V + n] = lb;
                const float v = n < V ? bf2f(lb) : -INFINITY;
                if (v > bv) { bv = v; bi = n; }  // columns ascend with j: first index kept on ties
            }
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {
                const float ov = __shfl_xor(bv, o, 64);
                const int oi = __shfl_xor(bi, o, 64);
                if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
            }
            if (l16 == 0) {
                s_val[wave][row] = bv;
                s_idx[wave][row] = bi;
            }
        }
    __syncthreads();
    if (threadIdx.x < 128 && m0 + (int)threadIdx.x < B) {
        const int row = threadIdx.x;
        float bv = s_val[0][row];
        int bi = s_idx[0][row];
        for (int w = 1; w < NW; ++w)
            if (s_val[w][row] > bv || (s_val[w][row] == bv && s_idx[w][row] < bi)) { bv = s_val[w][row]; bi = s_idx[w][row]; }
        part[(int64_t)(m0 + row) * nblk + blockIdx.x] = make_uint2(__float_as_uint(bv), (uint32_t)bi);
    }
}

// Greedy token per row from the LM-head partials; advances the position.
__global__ __launch_bounds__(256) void k_argmax_rows(const uint2* __restrict__ part, int nblk, int32_t* tokens,
                                                     int32_t* positions, int max_seq) {
    __shared__ float r_val[256];
    __shared__ int r_idx[256];
    const int b = blockIdx.x;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        const uint2 v = part[(int64_t)b * nblk + i];
        const float fv = __uint_as_float(v.x);
        const int id = (int)v.y;
        if (fv > best || (fv == best && id < bi)) { best = fv; bi = id; }
    }
    r_val[threadIdx.x] = best;
    r_idx[threadIdx.x] = bi;
    __syncthreads();
    for (int s2 = 128; s2 > 0; s2 >>= 1) {
        if (threadIdx.x < s2) {
            const float v2 = r_val[threadIdx.x + s2];
            const int i2 = r_idx[threadIdx.x + s2];
            if (v2 > r_val[threadIdx.x] || (v2 == r_val[threadIdx.x] && i2 < r_idx[threadIdx.x])) {
                r_val[threadIdx.x] = v2;
                r_idx[threadIdx.x] = i2;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tokens[b] = r_idx[0];
        positions[b] = min(positions[b] + 1, max_seq - 1);
    }
}

// ---------------------------------------------------------------------------------------------
// embed, standalone row norm (batch > 1 codes; final norm), LM head with fused greedy argmax
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_embed(const uint16_t* __restrict__ embed, const int32_t* __restrict__ tokens,
                                               int H, int V, uint16_t* __restrict__ h,
                                               const int32_t* __restrict__ positions, int32_t* __restrict__ seq_lens) {
    const int b = blockIdx.x;
    const int tok = min(max(tokens[b], 0), V - 1);  // never read outside the table
    const uint16_t* src = embed + (int64_t)tok * H;
    for (int i = threadIdx.x; i < H / 8; i += blockDim.x)
        reinterpret_cast<uint4*>(h + (int64_t)b * H)[i] = reinterpret_cast<const uint4*>(src)[i];
    if (threadIdx.x == 0) seq_lens[b] = positions[b] + 1;
}

// One block per row: rms_norm + quantize -> q8/sf/asum (Y16 = false), or the final norm -> bf16.
template <int PPT, bool Y16, bool TL = false>
__global__ __launch_bounds__(kNT) void k_rownorm(const uint16_t* __restrict__ x, int64_t xs,
                                                 const uint16_t* __restrict__ nw, int K, float eps,
                                                 int8_t* __restrict__ q8, int64_t q8s, float* __restrict__ sf,
                                                 int* __restrict__ asum, uint16_t* __restrict__ y16, int64_t ys) {
    __shared__ float red[2 * kNT / 64];
    __shared__ int red_i[kNT / 64];
    const int b = blockIdx.x;
    // stamps build: ln_in / ln_post share a region (the later one stays), ffn_sub and final apart
    WF_STAMP_BASE(Y16 ? 3072u : (PPT == 1 ? 2048u : 2304u));
    WF_STAMP(0);
    NormRow<PPT, kNT> nr;
    nr.issue(x + (int64_t)b * xs, nw, K);
    float y[PPT][8];
    if constexpr (Y16) {
        (void)norm_row(nr, K, eps, y, red, false);
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int p = threadIdx.x + kNT * i;
            if (p < K / 8)
                *reinterpret_cast<uint4*>(y16 + (TL ? bf_tile_off(b, p, K) : (int64_t)b * ys + 8 * p)) =
                    make_uint4(pk_bf16(y[i][0], y[i][1]), pk_bf16(y[i][2], y[i][3]), pk_bf16(y[i][4], y[i][5]),
                               pk_bf16(y[i][6], y[i][7]));
        }
    } else {
        const float s = norm_row(nr, K, eps, y, red);
        WF_STAMP(1);
        int as;
        if constexpr (TL) as = quant_row_tiled<PPT, kNT>(y, s, K / 8, q8, b, K >> 7);
        else as = quant_row<PPT, kNT>(y, s, K / 8, q8 + (int64_t)b * q8s, [](int p) { return 8 * p; });
        as = wave_sum_i(as);
        if ((threadIdx.x & 63) == 0) red_i[threadIdx.x >> 6] = as;
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int i = 0; i < kNT / 64; ++i) t += red_i[i];
            asum[b] = t;
            sf[b] = s;
        }
        WF_STAMP(2);
    }
}

// Prefill row norm (thousands of rows): block = 8 consecutive rows = one half of a 16-row code
// tile, one wave per row, no block-wide reductions. A wave replays k_rownorm's 512-thread tree for
// its row (bit-identical codes, scale and code sum): lane l holds pieces 8 (64 j + l), j < NP, i.e.
// piece j of "thread" 64 (j % 8) + l; the eight per-thread fma chains are kept apart, each goes
// through the same wave_sum, and tree_sum<8> adds them in wave order (max and the integer code sum
// are order-free). Codes land row-major in LDS (row stride K + 16 bytes); after one barrier the
// block writes its half-tiles in the tile_code_pos layout as whole 128-byte lines (lane = one
// 16-byte slot, its 4 dwords gathered by conflict-free ds_read_b32), so every line of the code
// tensor is written by one block of one XCD (the former 4-rows-per-block kernel split each line
// over four blocks' 4-byte stores: 76 us at K 2560, 98 us at K 6912 for 16384 rows).
#ifndef WF_RN8_NT  // FFN-width row loads with the non-temporal hint (that buffer is read only here): 71.0
#define WF_RN8_NT 1  // -> 70.1 us; the hidden-width rows are re-read as the residual (27.0 vs 26.2 us with it)
#endif
// FULL: the launcher saw K / 8 > 64 (NP - 1), so pieces j < NP - 1 exist for every lane (no per-piece
// bound checks; only the last piece is checked).
// Two blocks per CU (4 waves per SIMD, <= 128 VGPRs) up to K 7168, as the LDS allows; unbounded,
// hipcc gave a FULL K-6912 form 146 VGPRs, so one block per CU (72 -> 102 us).
template <int NP, bool FULL = false>
__global__ __launch_bounds__(512, NP <= 14 ? 4 : 1) void k_rownorm_tile8(const uint16_t* __restrict__ x, int64_t xs,
                                                       const uint16_t* __restrict__ nw, int K, float eps,
                                                       int8_t* __restrict__ q8, float* __restrict__ sf,
                                                       int* __restrict__ asum_out) {
    // LDS: the norm weight row (K bf16; kept out of the registers: two blocks per CU at K 6912),
    // then the codes [8][K + 16]
    extern __shared__ __attribute__((aligned(16))) int8_t s_dyn[];
    uint16_t* s_nw = reinterpret_cast<uint16_t*>(s_dyn);
    int8_t* s_codes = s_dyn + 2 * K;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, npk = K >> 3, KS = K + 16;
    const int row = blockIdx.x * 8 + wave;
    uint4 xv[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int pc = min(64 * j + lane, npk - 1);
        if constexpr (WF_RN8_NT && NP > 5) xv[j] = ldg_nt(reinterpret_cast<const uint8_t*>(x + (int64_t)row * xs + 8 * pc));
        else xv[j] = *reinterpret_cast<const uint4*>(x + (int64_t)row * xs + 8 * pc);
    }
    for (int p = threadIdx.x; p < npk; p += 512)
        reinterpret_cast<uint4*>(s_nw)[p] = reinterpret_cast<const uint4*>(nw)[p];
    float ss[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const bool valid = (FULL && j < NP - 1) || 64 * j + lane < npk;
        const uint32_t w4[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float lo = valid ? bf_lo(w4[e]) : 0.f, hi = valid ? bf_hi(w4[e]) : 0.f;
            ss[j & 7] = fmaf(lo, lo, ss[j & 7]);
            ss[j & 7] = fmaf(hi, hi, ss[j & 7]);
        }
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) reg_fence(xv[j]);  // pass 2 unpacks again (no 8 NP floats kept live)
    float W[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) W[v] = v < NP ? wave_sum(ss[v]) : 0.f;  // chains >= NP are +0
    __syncthreads();  // s_nw complete
    const float rr = rms_factor(div_rn(tree_sum<8>(W), (float)K, 1.0f / (float)K) + eps);
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) {  // xv[j] <- the normalised row, packed bf16 (0 past the row)
        const bool valid = (FULL && j < NP - 1) || 64 * j + lane < npk;
        const uint4 wv = reinterpret_cast<const uint4*>(s_nw)[min(64 * j + lane, npk - 1)];
        const uint32_t w4[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w}, n4[4] = {wv.x, wv.y, wv.z, wv.w};
        uint32_t o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t a = pk_bf16(bf_lo(w4[e]) * rr, bf_hi(w4[e]) * rr);
            const uint32_t b = valid ? pk_bf16(bf_lo(a) * bf_lo(n4[e]), bf_hi(a) * bf_hi(n4[e])) : 0u;
            m = fmaxf(m, fmaxf(fabsf(bf_lo(b)), fabsf(bf_hi(b))));
            o4[e] = b;
        }
        xv[j] = make_uint4(o4[0], o4[1], o4[2], o4[3]);
        if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // at most 4 norm-weight pieces in registers
    }
    // the codes pass re-reads the packed row (without the fence hipcc keeps all 8 NP floats live)
#pragma unroll
    for (int j = 0; j < NP; ++j) reg_fence(xv[j]);
    const float s = act_scale_f(wave_max(m));
    const float inv = rcp_1ulp(s);
    int as = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const uint2 c = quant8_bf16x8(xv[j], s, inv, as);
        const int p = 64 * j + lane;
        if (p < npk) *reinterpret_cast<uint2*>(s_codes + wave * KS + 8 * p) = c;
    }
    as = wave_sum_i(as);
    if (lane == 0) {
        sf[row] = s;
        asum_out[row] = as;
    }
    __syncthreads();
    // half-tiles (kb, h): 32 slots (r8, q) = 4 whole lines; lanes 0-31 one pair, 32-63 the next
    const int nkb = K >> 7, half8 = blockIdx.x & 1, rt = blockIdx.x >> 1;
    const int slot = threadIdx.x & 31, r8 = slot & 7, qq = slot >> 3;
    for (int pr = threadIdx.x >> 5; pr < 2 * nkb; pr += 16) {
        const int kb = pr >> 1, h = pr & 1;
        const int8_t* src = s_codes + r8 * KS + 128 * kb + 16 * h + 4 * qq;
        // u32x4 (not uint4, a struct the compiler stored as four dword stores): one dwordx4 per lane
        const u32x4 v = {*reinterpret_cast<const uint32_t*>(src), *reinterpret_cast<const uint32_t*>(src + 32),
                         *reinterpret_cast<const uint32_t*>(src + 64), *reinterpret_cast<const uint32_t*>(src + 96)};
        *reinterpret_cast<u32x4*>(q8 + ((((int64_t)rt * nkb + kb) * 2 + h) << 10) + (((r8 + 8 * half8) + 16 * qq) << 4)) = v;
    }
}

#ifndef WF_LM_U  // study builds only (tools/build_variant.sh): 16-byte chunks in flight per lane
#define WF_LM_U 4
#endif
constexpr int kLmU = WF_LM_U;
// logits[b, v] = bf16(sum_k hn[b,k] * E[v,k]) (F.linear, fp32 accumulation); 16 lanes per vocab
// row, 16 rows per block. Each block publishes its (max, first index) per row (sc1); the last
// block reduces them: greedy token (direct_inference_full.py:306-307; first index on ties), and
// advances the position.
template <int MB>
__global__ __launch_bounds__(256) void k_lm_head(const uint16_t* __restrict__ E, const uint16_t* __restrict__ hn, int H,
                                                 int V, int B, uint16_t* __restrict__ logits, uint2* __restrict__ part,
                                                 int nblk, unsigned* ticket, int32_t* tokens, int32_t* positions,
                                                 int max_seq) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sh[];
    __shared__ float s_val[MB][16];
    __shared__ int sh_flag;
    __shared__ float r_val[256];
    __shared__ int r_idx[256];
    const int b0 = blockIdx.y * MB;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int lrow = wave * 4 + (lane >> 4);
    const int row = blockIdx.x * 16 + lrow;
    const int C = H / 8;
    const uint16_t* er = E + (int64_t)min(row, V - 1) * H;
    WF_STAMP_BASE(4096u);
    WF_STAMP(0);
    constexpr int U = kLmU;
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // first weight chunks in flight before the activation staging
        const int c = 16 * u + sub;
        w[u] = (c < C) ? ldg_nt(reinterpret_cast<const uint8_t*>(er + 8 * c)) : make_uint4(0, 0, 0, 0);
    }
    for (int i = threadIdx.x; i < MB * H / 8; i += blockDim.x) {
        const int m = i / (H / 8), j = i - m * (H / 8);
        reinterpret_cast<uint4*>(sh + m * H)[j] = reinterpret_cast<const uint4*>(hn + (int64_t)(b0 + m) * H)[j];
    }
    __syncthreads();
    WF_STAMP(1);
    float acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = 0.f;
    for (int c0 = 0; c0 < C; c0 += 16 * U) {
        if (c0 > 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int c = c0 + 16 * u + sub;
                w[u] = (c < C) ? ldg_nt(reinterpret_cast<const uint8_t*>(er + 8 * c)) : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = c0 + 16 * u + sub;
            if (c < C) {
                const uint32_t wd[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                for (int m = 0; m < MB; ++m) {
                    const uint4 hv = *reinterpret_cast<const uint4*>(sh + m * H + 8 * c);
                    const uint32_t hd[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        acc[m] = fmaf(__uint_as_float(wd[t] << 16), __uint_as_float(hd[t] << 16), acc[m]);
                        acc[m] = fmaf(__uint_as_float(wd[t] & 0xffff0000u), __uint_as_float(hd[t] & 0xffff0000u), acc[m]);
                    }
                }
            }
        }
    }
    WF_STAMP(2);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        float v = acc[m];
        v = group_reduce<16>(v, OpAdd{});
        if (sub == 0) {
            const uint16_t lb = f2bf(v);
            if (row < V) logits[(int64_t)(b0 + m) * V + row] = lb;
            s_val[m][lrow] = row < V ? bf2f(lb) : -INFINITY;
        }
    }
    __syncthreads();
    if (threadIdx.x < MB) {
        const int m = threadIdx.x;
        float best = s_val[m][0];
        int bi = 0;
        for (int i = 1; i < 16; ++i)
            if (s_val[m][i] > best) { best = s_val[m][i]; bi = i; }
        const uint64_t pk = ((uint64_t)(uint32_t)(blockIdx.x * 16 + bi) << 32) | __float_as_uint(best);
        st_sc1(reinterpret_cast<uint64_t*>(part) + (int64_t)(b0 + m) * nblk + blockIdx.x, pk);
    }
    const bool last = ticket_arrive(ticket, gridDim.x * gridDim.y, linear_block_id(), &sh_flag);
    WF_STAMP(3);
    if (!last) return;
    constexpr int kAM = 32;  // partial records in flight per thread
    for (int b = 0; b < B; ++b) {
        float best = -INFINITY;
        int bi = 0x7fffffff;
        const uint64_t* pb = reinterpret_cast<const uint64_t*>(part) + (int64_t)b * nblk;
        for (int i0 = threadIdx.x; i0 < nblk; i0 += 256 * kAM) {
            uint64_t v[kAM];
#pragma unroll
            for (int u = 0; u < kAM; ++u) v[u] = ld_sc1(pb + min(i0 + 256 * u, nblk - 1));  // clamped: repeats are harmless
#pragma unroll
            for (int u = 0; u < kAM; ++u) {
                const float fv = __uint_as_float((uint32_t)v[u]);
                const int id = (int)(v[u] >> 32);
                if (fv > best || (fv == best && id < bi)) { best = fv; bi = id; }
            }
        }
        r_val[threadIdx.x] = best;
        r_idx[threadIdx.x] = bi;
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if (threadIdx.x < s) {
                const float v2 = r_val[threadIdx.x + s];
                const int i2 = r_idx[threadIdx.x + s];
                if (v2 > r_val[threadIdx.x] || (v2 == r_val[threadIdx.x] && i2 < r_idx[threadIdx.x])) {
                    r_val[threadIdx.x] = v2;
                    r_idx[threadIdx.x] = i2;
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            tokens[b] = r_idx[0];
            positions[b] = min(positions[b] + 1, max_seq - 1);
        }
        __syncthreads();
    }
    ticket_rearm(ticket);
    WF_STAMP(4);
}

// Batch < 16 LM head as one persistent stream with the final norm in its prologue (replaces a
// k_rownorm launch + 8016 one-shot k_lm_head blocks): grid = a few blocks per CU, block g takes the
// 32-row vocabulary tiles g, g + G, ...; every block first puts its first weight chunks in flight,
// then normalises the MB final hidden rows itself (norm_row at 512 threads: k_rownorm's tree, so hn
// and the logits are bit-identical to the two-launch form) into LDS, then streams its tiles with
// the next round's chunks in flight while the current ones are summed (each lane the same chunk
// order as k_lm_head: same fp32 sums). Logits bf16 per row; each lane-row keeps its running
// (max, first index); one (max, index) record per block and row, one ticket arrival per block, the
// last block reduces the G records (first index on ties) into the greedy token and advances the
// position.
template <int MB, int PPT>
__global__ __launch_bounds__(kNT) void k_lm_head_p(const uint16_t* __restrict__ E, const uint16_t* __restrict__ h,
                                                   const uint16_t* __restrict__ fnw, float eps, int H, int V, int B,
                                                   uint16_t* __restrict__ logits, uint2* __restrict__ part,
                                                   unsigned* ticket, int32_t* tokens, int32_t* positions, int max_seq,
                                                   uint16_t* __restrict__ hn_out) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sh[];  // [MB][H] normalised rows
    __shared__ float red[2 * kNT / 64];
    __shared__ float s_val[MB][32];
    __shared__ int s_idx[MB][32];
    __shared__ int sh_flag;
    __shared__ float r_val[kNT];
    __shared__ int r_idx[kNT];
    const int b0 = blockIdx.y * MB, G = gridDim.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int lrow = wave * 4 + (lane >> 4);  // 0..31
    const int C = H / 8;                      // 16-byte chunks per row
    constexpr int U = kLmU;
    const int R = (C + 16 * U - 1) / (16 * U);  // rounds per tile
    const int ntiles = (V + 31) / 32;
    WF_STAMP_BASE(4096u);
    WF_STAMP(0);
    auto load = [&](uint4 (&w)[U], int t, int r) {
        const uint16_t* er = E + (int64_t)min(32 * t + lrow, V - 1) * H;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = 16 * (U * r + u) + sub;
            w[u] = ldg_nt(reinterpret_cast<const uint8_t*>(er + 8 * min(c, C - 1)));
        }
    };
    uint4 wa[U], wb[U];
    int t = blockIdx.x, r = 0;
    if (t < ntiles) load(wa, t, 0);
    // the final norm of this block's MB rows (scripts/direct_inference_full.py:296-297)
#pragma unroll 1
    for (int m = 0; m < MB; ++m) {
        NormRow<PPT, kNT> nr;
        nr.issue(h + (int64_t)(b0 + m) * H, fnw, H);
        nr.fence(true, true);
        float y[PPT][8];
        (void)norm_row(nr, H, eps, y, red, false);
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int p = threadIdx.x + kNT * i;
            if (p < C) {
                const uint4 v = make_uint4(pk_bf16(y[i][0], y[i][1]), pk_bf16(y[i][2], y[i][3]), pk_bf16(y[i][4], y[i][5]),
                                           pk_bf16(y[i][6], y[i][7]));
                reinterpret_cast<uint4*>(sh + m * H)[p] = v;
                if (blockIdx.x == 0) reinterpret_cast<uint4*>(hn_out + (int64_t)(b0 + m) * H)[p] = v;
            }
        }
        __syncthreads();  // red reused by the next row
    }
    WF_STAMP(1);
    float acc[MB], best[MB];
    int bidx[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        acc[m] = 0.f;
        best[m] = -INFINITY;
        bidx[m] = 0x7fffffff;
    }
    while (t < ntiles) {
        int tn = t, rn = r + 1;
        if (rn == R) {
            rn = 0;
            tn = t + G;
        }
        if (tn < ntiles) load(wb, tn, rn);  // the next round's chunks in flight while these are summed
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = 16 * (U * r + u) + sub;
            if (c < C) {
                const uint32_t wd[4] = {wa[u].x, wa[u].y, wa[u].z, wa[u].w};
#pragma unroll
                for (int m = 0; m < MB; ++m) {
                    const uint4 hv = *reinterpret_cast<const uint4*>(sh + m * H + 8 * c);
                    const uint32_t hd[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        acc[m] = fmaf(__uint_as_float(wd[q] << 16), __uint_as_float(hd[q] << 16), acc[m]);
                        acc[m] = fmaf(__uint_as_float(wd[q] & 0xffff0000u), __uint_as_float(hd[q] & 0xffff0000u), acc[m]);
                    }
                }
            }
        }
        if (r == R - 1) {  // tile done: logits of this lane-row, running max (rows increase: first index kept)
            const int row = 32 * t + lrow;
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const float v = group_reduce<16>(acc[m], OpAdd{});
                acc[m] = 0.f;
                if (sub == 0 && row < V) {
                    const uint16_t lb = f2bf(v);
                    logits[(int64_t)(b0 + m) * V + row] = lb;
                    if (bf2f(lb) > best[m]) {
                        best[m] = bf2f(lb);
                        bidx[m] = row;
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = wb[u];
        t = tn;
        r = rn;
    }
    WF_STAMP(2);
    if (sub == 0) {
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            s_val[m][lrow] = best[m];
            s_idx[m][lrow] = bidx[m];
        }
    }
    __syncthreads();
    if (threadIdx.x < MB) {
        const int m = threadIdx.x;
        float bv = s_val[m][0];
        int bi = s_idx[m][0];
        for (int i = 1; i < 32; ++i)
            if (s_val[m][i] > bv || (s_val[m][i] == bv && s_idx[m][i] < bi)) { bv = s_val[m][i]; bi = s_idx[m][i]; }
        const uint64_t pk = ((uint64_t)(uint32_t)bi << 32) | __float_as_uint(bv);
        st_sc1(reinterpret_cast<uint64_t*>(part) + (int64_t)(b0 + m) * G + blockIdx.x, pk);
    }
    const bool last = ticket_arrive(ticket, gridDim.x * gridDim.y, linear_block_id(), &sh_flag);
    WF_STAMP(3);
    if (!last) return;
    for (int b = 0; b < B; ++b) {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        const uint64_t* pb = reinterpret_cast<const uint64_t*>(part) + (int64_t)b * G;
        for (int i = threadIdx.x; i < G; i += kNT) {
            const uint64_t v = ld_sc1(pb + i);
            const float fv = __uint_as_float((uint32_t)v);
            const int id = (int)(v >> 32);
            if (fv > bv || (fv == bv && id < bi)) { bv = fv; bi = id; }
        }
        r_val[threadIdx.x] = bv;
        r_idx[threadIdx.x] = bi;
        __syncthreads();
        for (int s2 = kNT / 2; s2 > 0; s2 >>= 1) {
            if (threadIdx.x < s2) {
                const float v2 = r_val[threadIdx.x + s2];
                const int i2 = r_idx[threadIdx.x + s2];
                if (v2 > r_val[threadIdx.x] || (v2 == r_val[threadIdx.x] && i2 < r_idx[threadIdx.x])) {
                    r_val[threadIdx.x] = v2;
                    r_idx[threadIdx.x] = i2;
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            tokens[b] = r_idx[0];
            positions[b] = min(positions[b] + 1, max_seq - 1);
        }
        __syncthreads();
    }
    ticket_rearm(ticket);
    WF_STAMP(4);
}

}  // namespace wf

WF_STAMP_READER(wf_debug_stamps_decode)

// =============================================================================================
// Model runtime
// =============================================================================================
// ticket slots, kTicketWords words each
enum { TK_LM = 0, TK_COUNT = 1 };

struct wf_model {
    wf_model_desc d;
    int qkv_rows;
    int32_t* tokens = nullptr;     // caller-owned (desc)
    int32_t* positions = nullptr;  // caller-owned (desc)
    uint16_t* logits = nullptr;    // caller-owned (desc)
    uint16_t *k_cache = nullptr, *v_cache = nullptr;  // caller-owned (desc)
    int32_t* seq_lens = nullptr;
    uint16_t *h_a = nullptr, *h_b = nullptr, *qbuf = nullptr, *act = nullptr, *hn = nullptr;
    int* dec_ws = nullptr;      // batched decode split-K partials
    size_t dec_ws_ints = 0;
    float2* part_ml = nullptr;  // attention partials [B, Hq, splits] (m, l); splits 16 below B 16, else 8
    float* part_o = nullptr;    // [B, Hq, splits, head_dim] unnormalised o
    int8_t* q8 = nullptr;   // batch > 1: activation codes of the next GEMV [B, q8_stride]
    float* act_sf = nullptr;
    int* act_sum = nullptr;
    unsigned* tickets = nullptr;
    unsigned* seam = nullptr;  // fused row-norm hand-off words (k_dec_gemm_t PRO), zero between launches
    unsigned* attn_cnt = nullptr;  // batched attention tail: one arrival counter per sequence (kTailLine apart)
    uint16_t* attn_row = nullptr;  // batch < 16 / untiled caches: the merged bf16 attention rows [B][H] (kMerge1)
    uint64_t* attn_xmax = nullptr;  // exchange granules: k_attn_sdpa {max, epoch} [B][Hq][splits][3]; k_attn_sdpa_mfma [B][Hkv][8]
    wf::SdpaBufs sdpa;              // the attention's error word and test hook
    unsigned* err_host = nullptr;   // host-mapped error word the attention raises on a poll timeout (wf_model_check)
    int32_t* attn_order = nullptr;  // batched attention: sequences by decreasing context (k_seq_order)
    int fuse[4] = {0, 0, 0, 0};  // per GEMM op (QKV, O, GU, DN): row norm fused into the GEMM launch
    uint2* am_part = nullptr;
    int lm_blocks = 0;
    int64_t q8_stride = 0;
    int kv_tiled = 0;  // batched MFMA decode: K/V caches in the tile layouts (include/wf_bitnet.h)
    uint16_t* embed_t = nullptr;  // batched LM head: the tied embedding in the fragment layout (copy)
    float* kv_scale = nullptr;    // host copy of the FP8 K/V scales [layers][2] (1.0 when bf16)
    // prefill workspace (wf_model_prefill_reserve): rows of prompt tokens
    int pf_rows = 0;
    uint16_t *pf_h_a = nullptr, *pf_h_b = nullptr, *pf_q = nullptr, *pf_attn = nullptr, *pf_act = nullptr;
    int8_t* pf_q8 = nullptr;
    float* pf_sf = nullptr;
    int* pf_asum = nullptr;
    int32_t* pf_seq = nullptr;
    hipStream_t cap = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

using namespace wf;
// (defined with the prefill launches below; the batched decode's row norm uses it too)
static void rownorm_tile8_launch(const uint16_t* x, int64_t xs, const uint16_t* nw, int K, int rows, float eps,
                                 int8_t* q8, float* sf, int* asum, hipStream_t st);

namespace {

// lanes per weight row of the kNT-thread GEMV blocks (QKV needs 16 rows per block for its RoPE
// pairing)
constexpr int kLprQKV = kNT / 16;  // 240 blocks at 2B
constexpr int kLprO = kNT / 16;    // 160 blocks
constexpr int kLprGU = 8;          // 64 rows = four gate/up tiles per block: 216 blocks at I = 6912
constexpr int kLprDN = kNT / 16;   // 160 blocks
// batch < 16 LM head stream: blocks of kNT threads (two per CU at 256 CUs)
#ifndef WF_LM_BLOCKS  // study builds: blocks of the batch < 16 LM head stream
#define WF_LM_BLOCKS 512
#endif
constexpr int kLmStreamBlocks = WF_LM_BLOCKS;

int64_t wrow_bytes(int fmt, int K) { return fmt == WF_FMT_TQ ? FmtTQ::row_bytes(K) : FmtI2S::row_bytes(K); }
int k_pad(int fmt, int K) { return fmt == WF_FMT_TQ ? FmtTQ::k_pad(K) : FmtI2S::k_pad(K); }
// 8-element pieces per thread of the norm prologue / k_rownorm
int norm_ppt(int kpad) { return kpad <= 8 * kNT ? 1 : 2; }

template <class F, int MODE, int LPR>
int launch_gemv(const GemvArgs& ga, hipStream_t st) {
    constexpr int RPB = kNT / LPR;
    const int img = lds_image_bytes<F>(ga.K);
    const int gx = (ga.N + RPB - 1) / RPB;
    const int B = ga.B;
#define WF_G(MBV, PPTV)                                                                                         \
    hipLaunchKernelGGL((k_gemv<F, MODE, LPR, MBV, PPTV>), dim3(gx, B / MBV), dim3(kNT),     \
                       (size_t)img * MBV, st, ga)
    if (B == 1) {
        if (norm_ppt(F::k_pad(ga.K)) == 1) WF_G(1, 1);
        else WF_G(1, 2);
    } else if (B % 8 == 0) WF_G(8, 0);
    else if (B % 4 == 0) WF_G(4, 0);
    else if (B % 2 == 0) WF_G(2, 0);
    else WF_G(1, 0);
#undef WF_G
    return check_launch("gemv");
}

// split-K factor of the batched decode GEMM: ~384 blocks of 128 x 128 over the layer's columns
int dec_split(int N, int K, int* steps_per_split) {
    const int cb = (N + 127) / 128, steps = K / 64;
    const int want = std::max(1, std::min(steps, (384 + cb - 1) / cb));
    const int sps = (steps + want - 1) / want;
    if (steps_per_split) *steps_per_split = sps;
    return (steps + sps - 1) / sps;
}

// The batched tile-layout GEMM's kernel for a shape, with or without the fused row norm (PRO: 0 none,
// else the op's input kind; PP = 8-element pieces per thread of the norm). One function so the
// launch and the host occupancy check name the same instantiation.
template <int MODE, int PRO, int PP>
const void* dec_gemm_kernel(int N, int K, int* threads) {
    if (N >= 8192) {  // wide layers (gate|up): 128-column tiles halve the code re-reads
        // 4 waves per block (64 KiB of LDS, two blocks per CU): the 108 x 4 blocks of the 2B
        // gate|up at batch 128 are resident in one round (8 waves + 128 KiB took two rounds).
        // Measured and not kept (round 3): 32 x 224 tiles, one 4-wave block per CU (248 blocks,
        // 220 KB of fragments each instead of 2 x 160 KB on 176 CUs): gate|up 16.3 -> 20.2 us per
        // op -- one wave per SIMD cannot hide its own 28-tile MFMA + decode stream.
        *threads = 4 * 64;
        if constexpr (PRO == 2) return nullptr;  // the attention input is never this wide
        else return reinterpret_cast<const void*>(&k_dec_gemm_t<2, 8, 3, MODE, 4, PRO, PP>);
    }
    *threads = kDgWaves * 64;
    if (K <= 3 * 128 * kDgWaves)  // the whole K in flight at once
        return reinterpret_cast<const void*>(&k_dec_gemm_t<2, 4, 3, MODE, kDgWaves, PRO, PP>);
    return reinterpret_cast<const void*>(&k_dec_gemm_t<2, 4, 2, MODE, kDgWaves, PRO, PP>);
}
dim3 dec_gemm_grid(int N, int B) {
    return N >= 8192 ? dim3((N + 127) / 128, (B + 31) / 32) : dim3(N / 64 + ((N & 63) ? 1 : 0), (B + 31) / 32);
}
template <int MODE>
const void* dec_gemm_kernel_pro(int pro, int K, int N, int* threads) {
    if (pro == 0) return dec_gemm_kernel<MODE, 0, 1>(N, K, threads);
#ifndef WF_FUSED_NORM
    return nullptr;  // the fused row norm is a study build (-DWF_FUSED_NORM)
#else
    const bool big = norm_ppt(K) != 1;
    if constexpr (MODE == MODE_O) {
        return big ? dec_gemm_kernel<MODE, 2, 2>(N, K, threads) : dec_gemm_kernel<MODE, 2, 1>(N, K, threads);
    } else {
        return big ? dec_gemm_kernel<MODE, 1, 2>(N, K, threads) : dec_gemm_kernel<MODE, 1, 1>(N, K, threads);
    }
#endif
}

template <int MODE, int LPR>
int launch_gemv_fmt(int fmt, const GemvArgs& ga, hipStream_t st, int pro = 0) {
    if (fmt == WF_FMT_I2S_MFMA) {  // batched decode on the matrix-core tile layouts
        int threads = 0;
        const void* fn = dec_gemm_kernel_pro<MODE>(pro, ga.K, ga.N, &threads);
        if (!fn) {
            set_error("dec_gemm_t: no fused kernel for this shape");
            return WF_EINVAL;
        }
        void* args[] = {const_cast<GemvArgs*>(&ga)};
        const hipError_t e = hipLaunchKernel(fn, dec_gemm_grid(ga.N, ga.B), dim3(threads), args, 0, st);
        if (e != hipSuccess) {
            set_error("dec_gemm_t launch: %s", hipGetErrorString(e));
            return WF_EHIP;
        }
        return check_launch("dec_gemm_t");
    }
    if (fmt == WF_FMT_I2S && ga.B >= kDecMfmaMinB) {  // batched decode on the matrix cores, split-K
        if (ga.B <= kDecGemmMaxB) {
            const dim3 grid((ga.N + 63) / 64, (ga.B + 31) / 32);
            if (ga.K <= 3 * 128 * kDgWaves)  // the whole K in flight at once
                hipLaunchKernelGGL((k_dec_gemm<2, 4, 3, MODE>), grid, dim3(kDgWaves * 64), 0, st, ga);
            else
                hipLaunchKernelGGL((k_dec_gemm<2, 4, 2, MODE>), grid, dim3(kDgWaves * 64), 0, st, ga);
            return check_launch("dec_gemm");
        }
        const int cb = (ga.N + 127) / 128;
        int sps = 0;
        const int nsplit = dec_split(ga.N, ga.K, &sps);
        if ((size_t)nsplit * ga.B * ga.N > ga.ws_ints) {
            set_error("dec_mfma: split-K workspace too small");
            return WF_EINVAL;
        }
        hipLaunchKernelGGL(k_dec_mfma_part, dim3(cb, nsplit, (ga.B + 127) / 128), dim3(256), 0, st, ga, ga.ws, sps);
        hipLaunchKernelGGL((k_dec_epi<MODE>), dim3((ga.N + 63) / 64, (ga.B + 15) / 16), dim3(256), 0, st, ga,
                           (const int*)ga.ws, nsplit);
        return check_launch("dec_mfma");
    }
    if (fmt == WF_FMT_TQ) return launch_gemv<FmtTQ, MODE, LPR>(ga, st);
    return launch_gemv<FmtI2S, MODE, LPR>(ga, st);
}

#ifndef WF_DEC_TILE8  // study: 1 = batch >= 16 GEMM inputs through the prefill row norm k_rownorm_tile8
#define WF_DEC_TILE8 0  // (bit-identical; 16 blocks at batch 128: 35.0k -> 32.3k tok/s, ab_dec_tile8_r04.txt)
#endif
// rows of x [B, xs] -> int8 codes in m->q8 (batch > 1), or bf16 into y16 (final norm)
void launch_rownorm(const wf_model* m, const uint16_t* x, int64_t xs, const uint16_t* nw, int K, uint16_t* y16,
                    hipStream_t st) {
    const wf_model_desc& d = m->d;
    const bool big = norm_ppt(K) != 1;
#define WF_RN(PPTV, Y, TL)                                                                                          \
    hipLaunchKernelGGL((k_rownorm<PPTV, Y, TL>), dim3(d.batch), dim3(kNT), 0, st, x, xs, nw, K, d.eps, m->q8, m->q8_stride, \
                       m->act_sf, m->act_sum, y16, (int64_t)K)
    const bool tl = d.wfmt == WF_FMT_I2S_MFMA;
    if (y16) {  // final norm: the matrix-core LM head reads it in the fragment layout
        if (m->embed_t) {
            if (big) WF_RN(2, true, true);
            else WF_RN(1, true, true);
        } else {
            if (big) WF_RN(2, true, false);
            else WF_RN(1, true, false);
        }
    } else if (tl) {
        // (study: the prefill row norm, one wave per row, whole 128-byte code lines)
        if (WF_DEC_TILE8 && d.batch % 16 == 0) rownorm_tile8_launch(x, xs, nw, K, d.batch, d.eps, m->q8, m->act_sf, m->act_sum, st);
        else if (big) WF_RN(2, false, true);
        else WF_RN(1, false, true);
    } else {
        if (big) WF_RN(2, false, false);
        else WF_RN(1, false, false);
    }
#undef WF_RN
}

// Which batched GEMMs take their row norm inside the launch (k_dec_gemm_t PRO). The hand-off needs
// every block of the grid resident at once (blocks of a 32-sequence tile wait for the tile's rows,
// which blocks 0..31 of that tile produce) and >= 32 column blocks: checked per op against the
// occupancy of the exact instantiation (the API's count, cross-checked with the block's registers,
// LDS and threads: the API can read one block per CU high, MI355X_MICROARCH.md). Otherwise the op
// keeps the k_rownorm launch.
//
// Measured and NOT the product (round 3, same-box bench at batch 128, ctx 1024): 31.5-32.5k ->
// 27.4k tok/s. In-graph stamps: producers publish their rows ~3.5-4.5 us after entry, but the tile's
// rows are seen ready only at 8-11 us -- the one polling lane's loads queue behind its CU's weight
// stream (MI355X_MICROARCH.md price table, handoff-flag under load) and the norm overlaps nothing,
// while the boundary it removes costs ~2 us. So only the study build -DWF_FUSED_NORM plans it.
void fused_norm_plan(wf_model* m) {
    for (int& f : m->fuse) f = 0;
#ifdef WF_FUSED_NORM
    const wf_model_desc& d = m->d;
    if (d.wfmt != WF_FMT_I2S_MFMA || d.batch < kDecMfmaMinB || d.batch > 32 * kSeamTiles) return;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return;
    const int shapes[4][2] = {{m->qkv_rows, d.hidden}, {d.hidden, d.hidden}, {2 * d.inter, d.hidden}, {d.hidden, d.inter}};
    for (int op = 0; op < 4; ++op) {
        const int N = shapes[op][0], K = shapes[op][1];
        int threads = 0;
        const void* fn = nullptr;
        switch (op) {
            case 0: fn = dec_gemm_kernel_pro<MODE_QKV>(1, K, N, &threads); break;
            case 1: fn = dec_gemm_kernel_pro<MODE_O>(1, K, N, &threads); break;
            case 2: fn = dec_gemm_kernel_pro<MODE_GU>(1, K, N, &threads); break;
            default: fn = dec_gemm_kernel_pro<MODE_DN>(1, K, N, &threads); break;
        }
        if (!fn) continue;
        const dim3 g = dec_gemm_grid(N, d.batch);
        int per_cu = 0;
        hipFuncAttributes fa{};
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) != hipSuccess ||
            hipFuncGetAttributes(&fa, fn) != hipSuccess)
            continue;
        // cross-check the API with the block's own limits (512 registers per SIMD lane, 4 SIMDs,
        // 160 KiB of LDS, 2048 threads per CU): the smaller count is the one relied on
        const int regs = std::max(8, (fa.numRegs + 7) / 8 * 8), waves_per_simd = threads / 64 / 4;
        const int by_regs = (512 / regs) / std::max(1, waves_per_simd);
        const int by_lds = fa.sharedSizeBytes ? (int)((160 * 1024) / fa.sharedSizeBytes) : 64;
        const int sure = std::min({per_cu, by_regs, by_lds, 2048 / threads});
        m->fuse[op] = (g.x >= 32 && (int64_t)sure * cus >= (int64_t)g.x * g.y) ? 1 : 0;
    }
    (void)hipGetLastError();
#endif
}

GemvArgs base_args(const wf_model* m, int l) {
    const wf_model_desc& d = m->d;
    GemvArgs a{};
    a.eps = d.eps;
    a.B = d.batch;
    a.q8 = m->q8;
    a.q8_stride = m->q8_stride;
    a.act_sf = m->act_sf;
    a.act_sum = m->act_sum;
    a.Hq = d.n_heads;
    a.Hkv = d.n_kv_heads;
    a.S = d.max_seq;
    a.positions = m->positions;
    a.ws = m->dec_ws;
    a.ws_ints = m->dec_ws_ints;
    a.rope_cos = d.rope_cos;
    a.rope_sin = d.rope_sin;
    const int64_t kvl = d.page_table ? (int64_t)d.num_pages * d.n_kv_heads * 32 * d.head_dim
                                     : (int64_t)d.batch * d.n_kv_heads * d.max_seq * d.head_dim;
    a.pt = d.page_table;
    a.pps = d.max_seq / 32;
    a.npages = d.num_pages;
    a.kv_pgs = (int64_t)d.n_kv_heads * 32 * d.head_dim;
    // FP8 caches hold one byte per element: the layer offset is in bytes, the kernels index bytes
    const int64_t esz = d.kv_quant ? 1 : 2;
    a.kc = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(m->k_cache) + l * kvl * esz);
    a.vc = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(m->v_cache) + l * kvl * esz);
    a.kv8 = d.kv_quant;
    a.k_div = d.kv_quant ? m->kv_scale[2 * l] : 1.0f;
    a.v_div = d.kv_quant ? m->kv_scale[2 * l + 1] : 1.0f;
    a.kv_b_stride = (int64_t)d.n_kv_heads * d.max_seq * d.head_dim;
    a.kv_t = m->kv_tiled;
    a.seam = m->seam;
    return a;
}

// input rows + norm weight of a GEMM whose launch normalises them itself (k_dec_gemm_t PRO 1)
void fused_input(GemvArgs& a, const uint16_t* x, int64_t xs, const uint16_t* nw) {
    a.x = x;
    a.x_stride = xs;
    a.nw = nw;
}

// input row + norm weight of a GEMV; batch > 1 normalises them in a k_rownorm launch first
int gemv_input(wf_model* m, GemvArgs& a, const uint16_t* x, int64_t xs, const uint16_t* nw, hipStream_t st) {
    a.x = x;
    a.x_stride = xs;
    a.nw = nw;
    if (m->d.batch > 1) {
        launch_rownorm(m, x, xs, nw, a.K, nullptr, st);
        return check_launch("rownorm");
    }
    return WF_OK;
}

// every decode attention path writes the bf16 row m->attn_row (k_attn_sdpa's merge ticket: batch
// < 16 or untiled caches; k_attn_sdpa_mfma: batch >= 16 on tile-layout caches); k_attn_sdpa also
// leaves its per-split (m, l, o) records (include/wf_bitnet.h attention view)
bool attn_sdpa_path(const wf_model* m) { return m->d.batch < 16 || !m->kv_tiled; }

// the host-visible error word the decode attention raises when a poll of its in-launch exchange
// times out (a sibling block never became resident): reported, and cleared, by the next call
int take_device_error(wf_model* m) {
    if (!m->err_host) return WF_OK;
    const unsigned e = __atomic_exchange_n(m->err_host, 0u, __ATOMIC_ACQ_REL);
    if (!e) return WF_OK;
    set_error("decode attention: an in-launch exchange timed out (code %u: %s); that step's attention rows are NaN", e,
              e == WF_ATTN_ERR_SDPA ? "k_attn_sdpa split maxima / records" : "k_attn_sdpa_mfma split-2 block max");
    return WF_EHIP;
}

// One op of the decode step (WF_OP_* in include/wf_bitnet.h).
int run_op(wf_model* m, int l, int op, hipStream_t st) {
    const wf_model_desc& d = m->d;
    const int B = d.batch, H = d.hidden, I = d.inter, D = d.head_dim, S = d.max_seq;
    const float* wsh = d.wscale + 7 * l;  // host copy made at create time
    GemvArgs a = base_args(m, l);
    int rc = WF_OK;
    switch (op) {
        case WF_OP_EMBED:
            hipLaunchKernelGGL(k_embed, dim3(B), dim3(256), 0, st, d.embed, m->tokens, H, d.vocab, m->h_a, m->positions,
                               m->seq_lens);
            break;
        case WF_OP_QKV:  // rms_norm(input_layernorm)(h_a) -> q|k|v, RoPE, cache
            a.w = d.w_qkv + (int64_t)l * m->qkv_rows * wrow_bytes(d.wfmt, H);
            a.N = m->qkv_rows; a.K = H; a.ws0 = wsh[0]; a.ws1 = wsh[1]; a.ws2 = wsh[2];
            a.out = m->qbuf; a.out_stride = (int64_t)d.n_heads * D;
            if (m->fuse[0]) return fused_input(a, m->h_a, H, d.ln_in + (int64_t)l * H), launch_gemv_fmt<MODE_QKV, kLprQKV>(d.wfmt, a, st, 1);
            if ((rc = gemv_input(m, a, m->h_a, H, d.ln_in + (int64_t)l * H, st))) return rc;
            if (kXTok && B == 1 && l == 0) {  // the token's embedding row itself (no embed launch at batch 1)
                a.x = d.embed; a.x_stride = H; a.x_tok = m->tokens; a.vocab = d.vocab; a.seq_out = m->seq_lens;
            }
            return launch_gemv_fmt<MODE_QKV, kLprQKV>(d.wfmt, a, st);
        case WF_OP_ATTN: {  // split partials; merged by the O projection's input stage or the tail
            if (m->kv_tiled && B >= 16 && l == 0 && (rc = seq_order(m->seq_lens, B, S, m->attn_order, st))) return rc;
            uint16_t* mrow = m->attn_row;
            unsigned* mcnt = m->attn_cnt;  // k_attn_sdpa's arrival counts
            if (a.pt)  // paged pool: kv head stride 32 * D inside a page
                return decode_attention_partials(m->qbuf, (int64_t)d.n_heads * D, a.kc, a.vc, 0, 32 * D, B, d.n_heads,
                                                 d.n_kv_heads, S, m->seq_lens, 1.0f / sqrtf((float)D), m->part_ml,
                                                 m->part_o, st, true, a.pt, a.pps, a.npages, a.kv_pgs, d.kv_quant,
                                                 m->kv_scale[2 * l], m->kv_scale[2 * l + 1], mrow, mcnt, m->attn_xmax,
                                                 m->attn_order, &m->sdpa);
            return decode_attention_partials(m->qbuf, (int64_t)d.n_heads * D, a.kc, a.vc, a.kv_b_stride, (int64_t)S * D,
                                             B, d.n_heads, d.n_kv_heads, S, m->seq_lens, 1.0f / sqrtf((float)D),
                                             m->part_ml, m->part_o, st, m->kv_tiled != 0, nullptr, 0, 0, 0, d.kv_quant,
                                             d.kv_quant ? m->kv_scale[2 * l] : 1.f, d.kv_quant ? m->kv_scale[2 * l + 1] : 1.f,
                                             mrow, mcnt, m->attn_xmax, m->attn_order, &m->sdpa);
        }
        case WF_OP_O:  // h_b = h_a + o_proj(rms_norm(attn_sub_norm)(attn))
            a.w = d.w_o + (int64_t)l * H * wrow_bytes(d.wfmt, H); a.N = H; a.K = H; a.ws0 = wsh[3];
            a.resid = m->h_a; a.out = m->h_b; a.out_stride = H;
            if (kXTok && B == 1 && l == 0) { a.resid = d.embed; a.x_tok = m->tokens; a.vocab = d.vocab; }
            a.x = m->attn_row;  // every attention path writes its bf16 output rows
            a.x_stride = H;
            a.nw = d.attn_sub + (int64_t)l * H;
            if (m->fuse[1]) return launch_gemv_fmt<MODE_O, kLprO>(d.wfmt, a, st, 1);  // x = the attention rows
            if (B > 1) {  // the attention's bf16 rows: the plain row norm
                launch_rownorm(m, m->attn_row, H, a.nw, H, nullptr, st);
                if ((rc = check_launch("rownorm_attn_row"))) return rc;
            }
            return launch_gemv_fmt<MODE_O, kLprO>(d.wfmt, a, st);
        case WF_OP_GATE_UP:  // act = relu(gate)^2 * up of rms_norm(post_attention_layernorm)(h_b)
            a.w = d.w_gu + (int64_t)l * 2 * I * wrow_bytes(d.wfmt, H); a.N = 2 * I; a.K = H;
            a.ws0 = wsh[4]; a.ws1 = wsh[5]; a.out = m->act; a.out_stride = I;
            if (m->fuse[2]) return fused_input(a, m->h_b, H, d.ln_post + (int64_t)l * H), launch_gemv_fmt<MODE_GU, kLprGU>(d.wfmt, a, st, 1);
            if ((rc = gemv_input(m, a, m->h_b, H, d.ln_post + (int64_t)l * H, st))) return rc;
            return launch_gemv_fmt<MODE_GU, kLprGU>(d.wfmt, a, st);
        case WF_OP_DOWN:  // h_a = h_b + down(rms_norm(ffn_sub_norm)(act))
            a.w = d.w_d + (int64_t)l * H * wrow_bytes(d.wfmt, I); a.N = H; a.K = I; a.ws0 = wsh[6];
            a.resid = m->h_b; a.out = m->h_a; a.out_stride = H;
            if (m->fuse[3]) return fused_input(a, m->act, I, d.ffn_sub + (int64_t)l * I), launch_gemv_fmt<MODE_DN, kLprDN>(d.wfmt, a, st, 1);
            if ((rc = gemv_input(m, a, m->act, I, d.ffn_sub + (int64_t)l * I, st))) return rc;
            return launch_gemv_fmt<MODE_DN, kLprDN>(d.wfmt, a, st);
        case WF_OP_LM_HEAD: {  // final norm -> hn, logits = hn @ embed^T, greedy token
            if (m->embed_t) {
                launch_rownorm(m, m->h_a, H, d.final_norm, H, m->hn, st);
                if ((rc = check_launch("final_norm"))) return rc;
                const int nb = (d.vocab + 64 * kLmWaves - 1) / (64 * kLmWaves);
                hipLaunchKernelGGL((k_lm_head_mfma<kLmWaves, kLmStages>), dim3(nb, (B + 127) / 128), dim3(64 * kLmWaves), 0,
                                   st, m->embed_t, m->hn, H, d.vocab, B, m->logits, m->am_part, nb);
                hipLaunchKernelGGL(k_argmax_rows, dim3(B), dim3(256), 0, st, m->am_part, nb, m->tokens, m->positions, S);
                break;
            }
            const size_t sh = (size_t)H * 2;
            // every block the same number of 32-row tiles (4008 tiles: 501 blocks x 8, not 512 blocks
            // of 7 or 8 -- the 8-tile blocks set the launch's end)
            const int ntl = (d.vocab + 31) / 32, per = (ntl + kLmStreamBlocks - 1) / kLmStreamBlocks;
            const int G = (ntl + per - 1) / per;
#define WF_LM(MBV, PPTV)                                                                                            \
    hipLaunchKernelGGL((k_lm_head_p<MBV, PPTV>), dim3(G, B / MBV), dim3(kNT), sh * MBV, st, d.embed, m->h_a,          \
                       d.final_norm, d.eps, H, d.vocab, B, m->logits, m->am_part, m->tickets + TK_LM * kTicketWords,  \
                       m->tokens, m->positions, S, m->hn)
            if (norm_ppt(H) == 1) {
                if (B % 4 == 0) WF_LM(4, 1);
                else if (B % 2 == 0) WF_LM(2, 1);
                else WF_LM(1, 1);
            } else {
                if (B % 4 == 0) WF_LM(4, 2);
                else if (B % 2 == 0) WF_LM(2, 2);
                else WF_LM(1, 2);
            }
#undef WF_LM
            break;
        }
        default:
            set_error("model op %d unknown", op);
            return WF_EINVAL;
    }
    return check_launch("model_op");
}

int model_step(wf_model* m, hipStream_t st) {
    // batch 1: layer 0's QKV / O read the token's embedding row themselves (GemvArgs::x_tok)
    int rc = (kXTok && m->d.batch == 1) ? WF_OK : run_op(m, 0, WF_OP_EMBED, st);
    for (int l = 0; l < m->d.layers && !rc; ++l)
        for (int op = WF_OP_QKV; op <= WF_OP_DOWN && !rc; ++op) rc = run_op(m, l, op, st);
    if (!rc) rc = run_op(m, 0, WF_OP_LM_HEAD, st);
    return rc;
}

}  // namespace

extern "C" {

int wf_model_create(const wf_model_desc* dp, wf_model** out) {
    WF_REQUIRE(dp && out, "model_create: null argument");
    const wf_model_desc& d = *dp;
    WF_REQUIRE(d.head_dim == 128, "model_create: head_dim must be 128 (got %d)", d.head_dim);
    WF_REQUIRE(d.hidden == d.n_heads * d.head_dim, "model_create: hidden != n_heads * head_dim");
    WF_REQUIRE(d.n_kv_heads > 0 && d.n_heads % d.n_kv_heads == 0, "model_create: bad GQA");
    WF_REQUIRE(d.n_heads / d.n_kv_heads <= 8, "model_create: GQA group %d > 8", d.n_heads / d.n_kv_heads);
    WF_REQUIRE(d.hidden % 128 == 0 && d.inter % 128 == 0, "model_create: hidden/inter must be multiples of 128");
    WF_REQUIRE(k_pad(d.wfmt, d.hidden) <= 8192 && k_pad(d.wfmt, d.inter) <= 8192,
               "model_create: hidden/inter (padded to the weight format) > 8192 not supported");
    WF_REQUIRE(d.batch >= 1 && d.batch <= 1024 && d.max_seq >= 1 && d.vocab >= 1 && d.layers >= 1,
               "model_create: bad sizes (batch 1..1024)");
    WF_REQUIRE(d.wfmt == WF_FMT_I2S || d.wfmt == WF_FMT_TQ || d.wfmt == WF_FMT_I2S_MFMA, "model_create: bad weight format");
    WF_REQUIRE(d.wfmt != WF_FMT_I2S_MFMA || (d.batch >= kDecMfmaMinB && d.hidden % 16 == 0 && d.inter % 16 == 0),
               "model_create: WF_FMT_I2S_MFMA weights need batch >= %d", kDecMfmaMinB);
    WF_REQUIRE(d.embed && d.final_norm && d.rope_cos && d.rope_sin && d.ln_in && d.ln_post && d.attn_sub && d.ffn_sub &&
                   d.w_qkv && d.w_o && d.w_gu && d.w_d && d.wscale,
               "model_create: null weight pointer");
    WF_REQUIRE(d.tokens && d.positions && d.logits && d.k_cache && d.v_cache, "model_create: null state pointer");
    wf_model* m = new (std::nothrow) wf_model();
    WF_REQUIRE(m, "model_create: out of host memory");
    m->d = d;
    float* ws = new float[7 * d.layers];  // host copy of the scales (read while recording launches)
    for (int i = 0; i < 7 * d.layers; ++i) ws[i] = d.wscale[i];
    m->d.wscale = ws;
    m->qkv_rows = (d.n_heads + 2 * d.n_kv_heads) * d.head_dim;
    m->tokens = d.tokens;
    m->positions = d.positions;
    m->logits = d.logits;
    m->k_cache = d.k_cache;
    m->v_cache = d.v_cache;
    const int B = d.batch;
    m->lm_blocks = (d.vocab + 15) / 16;
    m->q8_stride = ((d.hidden > d.inter ? d.hidden : d.inter) + 15) / 16 * 16;
    auto fail = [&](hipError_t e) {
        set_error("model_create: %s", hipGetErrorString(e));
        wf_model_destroy(m);
        return WF_EHIP;
    };
    hipError_t e;
#define WF_ALLOC(ptr, bytes) \
    if ((e = hipMalloc((void**)&(ptr), (bytes))) != hipSuccess) return fail(e)
    WF_ALLOC(m->seq_lens, sizeof(int32_t) * B);
    WF_ALLOC(m->h_a, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->h_b, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->qbuf, 2 * (size_t)B * d.hidden);
    m->kv_tiled = (B >= kDecMfmaMinB && (d.wfmt == WF_FMT_I2S || d.wfmt == WF_FMT_I2S_MFMA) && d.max_seq % 32 == 0) ? 1 : 0;
    m->kv_scale = new float[2 * d.layers];
    for (int i = 0; i < 2 * d.layers; ++i) m->kv_scale[i] = (d.kv_quant && d.kv_scale) ? d.kv_scale[i] : 1.0f;
    if (d.kv_quant < WF_KV_BF16 || d.kv_quant > WF_KV_INT8) {
        set_error("model_create: kv_quant must be WF_KV_BF16, WF_KV_FP8 or WF_KV_INT8 (got %d)", d.kv_quant);
        wf_model_destroy(m);
        return WF_EINVAL;
    }
    if (d.kv_quant && !(m->kv_tiled && d.head_dim == 128)) {
        set_error("model_create: FP8 / int8 K/V need the batched matrix-core decoder (batch >= %d, I2_S, head_dim 128, "
                  "max_seq %% 32 == 0)", kDecMfmaMinB);
        wf_model_destroy(m);
        return WF_EINVAL;
    }
    for (int i = 0; i < 2 * d.layers; ++i)
        if (!(m->kv_scale[i] > 0.f) || !std::isfinite(m->kv_scale[i])) {
            set_error("model_create: K/V scales must be positive and finite");
            wf_model_destroy(m);
            return WF_EINVAL;
        }
    if (d.page_table && !(m->kv_tiled && d.head_dim == 128 && d.num_pages >= 1)) {
        set_error("model_create: paged KV needs batch >= %d, I2_S weights, head_dim 128, max_seq %% 32 == 0 and "
                  "num_pages >= 1", kDecMfmaMinB);
        wf_model_destroy(m);
        return WF_EINVAL;
    }
    if (B >= kDecMfmaMinB && d.wfmt == WF_FMT_I2S) {
        const int shapes[4][2] = {{m->qkv_rows, d.hidden}, {d.hidden, d.hidden}, {2 * d.inter, d.hidden}, {d.hidden, d.inter}};
        for (auto& sh : shapes)
            m->dec_ws_ints = std::max(m->dec_ws_ints, (size_t)dec_split(sh[0], sh[1], nullptr) * B * sh[0]);
        WF_ALLOC(m->dec_ws, sizeof(int) * m->dec_ws_ints);
    }
    WF_ALLOC(m->part_ml, sizeof(float2) * (size_t)B * d.n_heads * kAttnPartSplitsMax);
    WF_ALLOC(m->part_o, sizeof(float) * (size_t)B * d.n_heads * kAttnPartSplitsMax * d.head_dim);
    WF_ALLOC(m->hn, 2 * (size_t)((B + 15) / 16 * 16) * d.hidden);  // fragment layout: whole row tiles
    if ((d.wfmt == WF_FMT_I2S || d.wfmt == WF_FMT_I2S_MFMA) && B >= kDecMfmaMinB && d.vocab % 16 == 0 &&
        d.hidden % 32 == 0) {
        WF_ALLOC(m->embed_t, 2 * (size_t)d.vocab * d.hidden);
        hipLaunchKernelGGL(k_bf_tile, dim3(4096), dim3(256), 0, nullptr, d.embed, d.vocab, d.hidden, m->embed_t);
        if ((e = hipStreamSynchronize(nullptr)) != hipSuccess) return fail(e);
    }
    WF_ALLOC(m->act, 2 * (size_t)B * d.inter);
    WF_ALLOC(m->q8, (size_t)((B + 15) / 16 * 16) * m->q8_stride);  // tile layout: whole 16-row tiles
    WF_ALLOC(m->act_sf, sizeof(float) * B);
    WF_ALLOC(m->act_sum, sizeof(int) * B);
    WF_ALLOC(m->tickets, sizeof(unsigned) * kTicketWords * TK_COUNT);
    WF_ALLOC(m->seam, sizeof(unsigned) * 2 * kSeamTiles * kSeamLine);
    // arrival lines: one per sequence (batched tail) or per (sequence, head) (kMerge1)
    // (the second half: k_attn_sdpa's exchange counters)
    WF_ALLOC(m->attn_cnt, 2 * sizeof(unsigned) * (size_t)B * d.n_heads * kTailLine);
    WF_ALLOC(m->attn_row, 2 * (size_t)B * d.hidden);
    // k_attn_sdpa: split maxima + merge granules; k_attn_sdpa_mfma: [B][Hkv][8] (fits the maxima part)
    const size_t xbytes = sizeof(uint64_t) * (size_t)(attn_sdpa_path(m) ? sdpa_xbuf_granules(B, d.n_heads)
                                                                         : sdpa_xmax_granules(B, d.n_heads));
    WF_ALLOC(m->attn_xmax, xbytes);
    if (attn_sdpa_path(m) && d.max_seq > kAttnPartSplits1 * 1024) {  // k_attn_sdpa: 8 splits of <= 1024 keys
        set_error("model_create: max_seq %d > %d: the batch-%d decode attention takes %d splits of <= 1024 keys", d.max_seq,
                  kAttnPartSplits1 * 1024, B, kAttnPartSplits1);
        wf_model_destroy(m);
        return WF_EINVAL;
    }
    if ((e = hipHostMalloc((void**)&m->err_host, 64, hipHostMallocMapped)) != hipSuccess) return fail(e);
    *m->err_host = 0u;
    if ((e = hipHostGetDevicePointer((void**)&m->sdpa.err, m->err_host, 0)) != hipSuccess) return fail(e);
    WF_ALLOC(m->attn_order, sizeof(int32_t) * (size_t)B);
    {  // identity order until the first step sorts the batch
        std::vector<int32_t> id(B);
        for (int b = 0; b < B; ++b) id[b] = b;
        if ((e = hipMemcpy(m->attn_order, id.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice)) != hipSuccess) return fail(e);
    }
    WF_ALLOC(m->am_part, sizeof(uint2) * B * m->lm_blocks);
#undef WF_ALLOC
    // tickets start at zero; every launch re-arms the ones it uses
    if ((e = hipMemset(m->tickets, 0, sizeof(unsigned) * kTicketWords * TK_COUNT)) != hipSuccess) return fail(e);
    if ((e = hipMemset(m->seam, 0, sizeof(unsigned) * 2 * kSeamTiles * kSeamLine)) != hipSuccess) return fail(e);
    if ((e = hipMemset(m->attn_cnt, 0, 2 * sizeof(unsigned) * (size_t)B * d.n_heads * kTailLine)) != hipSuccess) return fail(e);
    // granule tags start at 0; the first launch's epoch is 1
    if ((e = hipMemset(m->attn_xmax, 0, xbytes)) != hipSuccess) return fail(e);
    fused_norm_plan(m);
    if ((e = hipStreamCreateWithFlags(&m->cap, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    *out = m;
    return WF_OK;
}

int wf_model_destroy(wf_model* m) {
    if (!m) return WF_OK;
    if (m->exec) (void)hipGraphExecDestroy(m->exec);
    if (m->graph) (void)hipGraphDestroy(m->graph);
    if (m->cap) (void)hipStreamDestroy(m->cap);
    if (m->err_host) (void)hipHostFree(m->err_host);
    void* ptrs[] = {m->attn_cnt, m->attn_row, m->attn_xmax, m->attn_order, m->seq_lens, m->h_a, m->h_b, m->qbuf, m->part_ml, m->part_o, m->hn, m->act, m->q8, m->dec_ws,
                    m->act_sf, m->act_sum, m->tickets, m->seam, m->am_part, m->embed_t, m->pf_h_a, m->pf_h_b, m->pf_q,
                    m->pf_attn, m->pf_act, m->pf_q8, m->pf_sf, m->pf_asum, m->pf_seq};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete[] m->d.wscale;
    delete[] m->kv_scale;
    delete m;
    return WF_OK;
}

int wf_model_step(wf_model* m, void* stream) {
    WF_REQUIRE(m, "model_step: null model");
    if (int rc = take_device_error(m)) return rc;
    return model_step(m, as_stream(stream));
}

int wf_model_launch_op(wf_model* m, int layer, int op, void* stream) {
    WF_REQUIRE(m, "model_launch_op: null model");
    WF_REQUIRE(layer >= 0 && layer < m->d.layers, "model_launch_op: layer %d out of range", layer);
    if (int rc = take_device_error(m)) return rc;
    return run_op(m, layer, op, as_stream(stream));
}

int wf_model_check(wf_model* m) {
    WF_REQUIRE(m, "model_check: null model");
    return take_device_error(m);
}

int wf_model_debug_stall_attention(wf_model* m, int on) {
    WF_REQUIRE(m, "model_debug_stall_attention: null model");
    WF_REQUIRE(attn_sdpa_path(m), "model_debug_stall_attention: the model's decode attention has no in-launch exchange");
    m->sdpa.stall = on ? 1 : 0;
    return WF_OK;
}

int wf_model_fused_norm(const wf_model* m, int* flags4) {
    WF_REQUIRE(m && flags4, "model_fused_norm: null argument");
    for (int i = 0; i < 4; ++i) flags4[i] = m->fuse[i];
    return WF_OK;
}

int wf_model_attn_view(const wf_model* m, wf_attn_records* out) {
    WF_REQUIRE(m && out, "model_attn_view: null argument");
    out->q = m->qbuf;
    out->part_ml = reinterpret_cast<const float*>(m->part_ml);
    out->part_o = m->part_o;
    out->records = attn_sdpa_path(m) ? kAttnPartSplits1 : 0;
    out->attn_row = m->attn_row;
    return WF_OK;
}

// ---------------------------------------------------------------------------------------------
// Prefill: the prompt tokens of any KV slots as GEMM rows (BASELINE configs[2]). Per layer:
// row norm + quantize (tile order) -> fused prefill GEMM (k_pgemm_fused) for QKV (+ RoPE, K/V
// rows written into each token's slot / position), causal attention (k_attn_prefill_sdpa), row norm ->
// O (+ residual), row norm -> gate|up (ReLU^2 * up), row norm -> down (+ residual). The float
// sequence per token is the decode step's (same epilogues, same row norm); attention sums over the
// whole prefix in one pass instead of the decode step's 8 merged splits.
// ---------------------------------------------------------------------------------------------
int wf_model_prefill_reserve(wf_model* m, int rows) {
    WF_REQUIRE(m && rows > 0, "model_prefill_reserve: bad arguments");
    const wf_model_desc& d = m->d;
    WF_REQUIRE(m->kv_tiled && d.wfmt == WF_FMT_I2S_MFMA && d.head_dim == 128 && d.n_heads == 4 * d.n_kv_heads,
               "model_prefill: needs the batched matrix-core decoder (batch >= %d, I2_S weights), head_dim 128 "
               "and 4 query heads per kv head",
               kDecMfmaMinB);
    rows = (rows + 15) / 16 * 16;
    if (rows <= m->pf_rows) return WF_OK;
    void* old[] = {m->pf_h_a, m->pf_h_b, m->pf_q, m->pf_attn, m->pf_act, m->pf_q8, m->pf_sf, m->pf_asum, m->pf_seq};
    for (void* p : old)
        if (p) (void)hipFree(p);
    m->pf_rows = 0;
    const size_t H = d.hidden, I = d.inter, R = rows;
    hipError_t e = hipSuccess;
#define WF_PA(ptr, bytes) \
    if (e == hipSuccess) e = hipMalloc((void**)&(ptr), (bytes))
    WF_PA(m->pf_h_a, 2 * R * H);
    WF_PA(m->pf_h_b, 2 * R * H);
    WF_PA(m->pf_q, 2 * R * H);
    WF_PA(m->pf_attn, 2 * R * H);
    WF_PA(m->pf_act, 2 * R * I);
    WF_PA(m->pf_q8, R * (H > I ? H : I));
    WF_PA(m->pf_sf, sizeof(float) * R);
    WF_PA(m->pf_asum, sizeof(int) * R);
    WF_PA(m->pf_seq, sizeof(int32_t) * R);
#undef WF_PA
    if (e != hipSuccess) {
        set_error("model_prefill_reserve: %s", hipGetErrorString(e));
        return WF_EHIP;
    }
    m->pf_rows = rows;
    return WF_OK;
}

extern "C++" {
// k_rownorm_tile8 over `rows` rows (rows % 16 == 0) into the tile-layout codes q8 + sf / asum
static void rownorm_tile8_launch(const uint16_t* x, int64_t xs, const uint16_t* nw, int K, int rows, float eps,
                                 int8_t* q8, float* sf, int* asum, hipStream_t st) {
    const dim3 grid(rows / 8);
    const size_t lds = 2 * (size_t)K + 8 * (size_t)(K + 16);
    const int np = (K / 8 + 63) / 64;
#define WF_RN8(NPV, FV) \
    hipLaunchKernelGGL((k_rownorm_tile8<NPV, FV>), grid, dim3(512), lds, st, x, xs, nw, K, eps, q8, sf, asum)
    if (np == 5) {  // the 2B-4T hidden width (2560)
        WF_RN8(5, true);
    } else if (np < 5) {
        WF_RN8(5, false);
    } else if (np <= 14) {  // incl. the FFN width 6912 (FULL there: 128 VGPRs + a spill, measured slower)
        WF_RN8(14, false);
    } else {  // K up to 8192: 2 K + 8 (K + 16) bytes of LDS pass 64 KiB
        static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rownorm_tile8<16>),
                                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                                           2 * 8192 + 8 * (8192 + 16));
        (void)attr;
        WF_RN8(16, false);
    }
#undef WF_RN8
}
static void prefill_rownorm(const wf_model* m, const uint16_t* x, int64_t xs, const uint16_t* nw, int K, int rows,
                            hipStream_t st) {
    // rows % 16 == 0 (wf_model_prefill); 8 rows per block
    rownorm_tile8_launch(x, xs, nw, K, rows, m->d.eps, m->pf_q8, m->pf_sf, m->pf_asum, st);
}

// LDS-staged row-tile epilogue (pf_tile_epilogue) where the output rows are 16-byte pieces: o / down
// (256-column tiles; measured o 141 -> 131, down 275 -> 262 us per layer at 16384 rows); the
// 512-column gate|up tile stays per fragment (staged: 570 -> 614 us)
static bool pf_staged_ok(const GemvArgs& a, bool wide) {
    const bool al = a.out_stride % 8 == 0 && reinterpret_cast<uintptr_t>(a.out) % 16 == 0 &&
                    (!a.resid || reinterpret_cast<uintptr_t>(a.resid) % 16 == 0);
    return !wide && al;
}
#ifndef WF_PG_PERSIST  // 0 = one-shot gate|up blocks (one tile each): same time, bit-identical
#define WF_PG_PERSIST 1  // (ab_prefill_persist_r04.txt)
#endif
constexpr bool kPgPersist = WF_PG_PERSIST;
[[maybe_unused]] static int pg_cu_count() {  // queried once per device (every gate|up launch asks)
    static int cached[64] = {};
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev >= 0 && dev < 64 && cached[dev]) return cached[dev];
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (dev >= 0 && dev < 64) cached[dev] = n;
    return n;
}
template <int MODE, int TNW, int ALG>
static void pg_launch(const GemvArgs& a, int nbm, int nbn, hipStream_t st) {
    // (the 512-column o / down tile of a wide model does not fit the staged tile into the ring)
    constexpr bool kStaged = MODE != MODE_QKV && pf_tile_epilogue_bytes<MODE, TNW>() <= PgCfg<TNW, ALG>::LDS;
    if constexpr (kPgPersist && MODE == MODE_GU && TNW == 8 && ALG == 0) {  // gate|up: persistent tile loop
        const int nt = nbm * nbn, ncu = pg_cu_count() / 8 * 8;
        hipLaunchKernelGGL((k_pgemm_fused_pt<MODE, TNW>), dim3(ncu >= 8 ? min(nt, ncu) : nt), dim3(512), 0, st, a, nbm, nbn);
        return;
    }
    if (kStaged && pf_staged_ok(a, TNW == 8))
        hipLaunchKernelGGL((k_pgemm_fused<MODE, TNW, ALG, kStaged>), dim3(nbm * nbn), dim3(512), 0, st, a, nbm, nbn);
    else
        hipLaunchKernelGGL((k_pgemm_fused<MODE, TNW, ALG, false>), dim3(nbm * nbn), dim3(512), 0, st, a, nbm, nbn);
}
template <int MODE>
static void prefill_gemm(const GemvArgs& a, hipStream_t st) {
    const int nbm = (a.B + 127) / 128;
    if constexpr (MODE != MODE_QKV) {
        if (pg_wide(a.N)) {  // gate|up: 128 x 512 tiles
            pg_launch<MODE, 8, 0>(a, nbm, (a.N + 511) / 512, st);
            return;
        }
    }
    pg_launch<MODE, 4, 0>(a, nbm, (a.N + 255) / 256, st);
}
}  // extern "C++"

int wf_model_prefill_view(const wf_model* m, const uint16_t** q, const uint16_t** attn) {
    WF_REQUIRE(m && q && attn, "model_prefill_view: null argument");
    WF_REQUIRE(m->pf_rows > 0 && m->pf_q && m->pf_attn, "model_prefill_view: no prefill reservation");
    *q = m->pf_q;
    *attn = m->pf_attn;
    return WF_OK;
}

int wf_model_prefill(wf_model* m, const int32_t* tokens, const int32_t* row_slot, const int32_t* row_pos, int rows,
                     void* stream) {
    WF_REQUIRE(m && tokens && row_slot && row_pos, "model_prefill: null argument");
    WF_REQUIRE(rows > 0 && rows <= m->pf_rows, "model_prefill: %d rows exceed the reserved %d (wf_model_prefill_reserve)",
               rows, m->pf_rows);
    WF_REQUIRE(rows % kPrefillRowGroup == 0, "model_prefill: rows must come in aligned groups of %d of one slot (got %d rows)",
               kPrefillRowGroup, rows);
    const wf_model_desc& d = m->d;
    hipStream_t st = as_stream(stream);
    const int H = d.hidden, I = d.inter, D = d.head_dim;
    int rc;
    {  // every contract check before the first launch: a refused call leaves the K/V cache untouched
        const GemvArgs a0 = base_args(m, 0);
        if ((rc = prefill_attention_check(d.n_heads, d.n_kv_heads, d.page_table ? a0.pps : d.max_seq / 32))) return rc;
    }
    hipLaunchKernelGGL(k_embed, dim3(rows), dim3(256), 0, st, d.embed, tokens, H, d.vocab, m->pf_h_a, row_pos, m->pf_seq);
    for (int l = 0; l < d.layers; ++l) {
        const float* wsh = d.wscale + 7 * l;
        GemvArgs a = base_args(m, l);
        a.B = rows;
        a.q8 = m->pf_q8;
        a.act_sf = m->pf_sf;
        a.act_sum = m->pf_asum;
        a.positions = row_pos;
        a.row_slot = row_slot;
        // QKV (+ RoPE, K/V rows into the cache)
        prefill_rownorm(m, m->pf_h_a, H, d.ln_in + (int64_t)l * H, H, rows, st);
        a.w = d.w_qkv + (int64_t)l * m->qkv_rows * (H / 4); a.N = m->qkv_rows; a.K = H;
        a.ws0 = wsh[0]; a.ws1 = wsh[1]; a.ws2 = wsh[2]; a.out = m->pf_q; a.out_stride = H;
        prefill_gemm<MODE_QKV>(a, st);
        // causal attention over each token's slot prefix
        const bool paged = d.page_table != nullptr;
        if ((rc = prefill_attention(m->pf_q, H, a.kc, a.vc, paged ? 0 : a.kv_b_stride, paged ? 32 * D : (int64_t)d.max_seq * D,
                                    d.n_heads, d.n_kv_heads, row_pos, row_slot, rows, 1.0f / sqrtf((float)D), a.pt,
                                    a.pps, a.npages, a.kv_pgs, m->pf_attn, H, st, d.kv_quant,
                                    d.kv_quant ? m->kv_scale[2 * l] : 1.f, d.kv_quant ? m->kv_scale[2 * l + 1] : 1.f)))
            return rc;
        // O (+ residual)
        prefill_rownorm(m, m->pf_attn, H, d.attn_sub + (int64_t)l * H, H, rows, st);
        a.w = d.w_o + (int64_t)l * H * (H / 4); a.N = H; a.K = H; a.ws0 = wsh[3];
        a.resid = m->pf_h_a; a.out = m->pf_h_b; a.out_stride = H;
        prefill_gemm<MODE_O>(a, st);
        // gate|up
        prefill_rownorm(m, m->pf_h_b, H, d.ln_post + (int64_t)l * H, H, rows, st);
        a.w = d.w_gu + (int64_t)l * 2 * I * (H / 4); a.N = 2 * I; a.K = H; a.ws0 = wsh[4]; a.ws1 = wsh[5];
        a.out = m->pf_act; a.out_stride = I;
        prefill_gemm<MODE_GU>(a, st);
        // down (+ residual)
        prefill_rownorm(m, m->pf_act, I, d.ffn_sub + (int64_t)l * I, I, rows, st);
        a.w = d.w_d + (int64_t)l * H * (I / 4); a.N = H; a.K = I; a.ws0 = wsh[6];
        a.resid = m->pf_h_b; a.out = m->pf_h_a; a.out_stride = H;
        prefill_gemm<MODE_DN>(a, st);
        if ((rc = check_launch("prefill layer"))) return rc;
    }
    return WF_OK;
}

int64_t wf_bitnet_linear_ws_bytes(int M, int K) {
    if (M <= 0 || K <= 0) return 0;
    return (int64_t)M * ((K + 15) / 16 * 16) + 8 * (int64_t)M + 256;
}

// BitNetLinear.forward (scripts/direct_inference_full.py:186-208): per-row int8 quantization of x,
// ternary GEMM, the reference's correction, bf16 out. One launch for M < 16 (quantize in the GEMV
// prologue), else a quantize launch + the int8-MFMA GEMM (I2_S).
int wf_bitnet_linear_fused(int fmt, const uint8_t* w, int nseg, const int* n, const float* ws, const uint16_t* x,
                           int64_t ldx, int M, int K, uint16_t* const* y, const int64_t* ldy, void* workspace,
                           void* stream) {
    WF_REQUIRE(w && x && n && ws && y && ldy, "bitnet_linear: null pointer");
    WF_REQUIRE(nseg >= 1 && nseg <= 3, "bitnet_linear_fused: 1..3 segments (got %d)", nseg);
    int N = 0;
    for (int s = 0; s < nseg; ++s) {
        WF_REQUIRE(n[s] > 0 && y[s] && ldy[s] >= n[s], "bitnet_linear_fused: segment %d: bad rows / output / stride", s);
        N += n[s];
    }
    WF_REQUIRE(M > 0 && K > 0 && K % 128 == 0, "bitnet_linear: bad shape M=%d N=%d K=%d (K %% 128 == 0)", M, N, K);
    WF_REQUIRE(fmt == WF_FMT_I2S || fmt == WF_FMT_TQ, "bitnet_linear: unknown weight format %d", fmt);
    const int kp = fmt == WF_FMT_TQ ? FmtTQ::k_pad(K) : FmtI2S::k_pad(K);
    WF_REQUIRE(kp <= 8192, "bitnet_linear: K > 8192 not supported");
    WF_REQUIRE(ldx >= K && ldx % 8 == 0 && aligned16(x) && aligned16(w), "bitnet_linear: bad strides / alignment");
    hipStream_t st = as_stream(stream);
    GemvArgs a{};
    a.w = w; a.N = N; a.K = K; a.B = M;
    a.x = x; a.x_stride = ldx;
    // row segments (lin_seg): [0, Hq) -> out, [Hq, Hq + Hkv) -> kc, the rest -> vc
    a.Hq = n[0]; a.ws0 = ws[0]; a.out = y[0]; a.out_stride = ldy[0];
    a.Hkv = nseg > 1 ? n[1] : 0;
    if (nseg > 1) { a.ws1 = ws[1]; a.kc = y[1]; a.kv_b_stride = ldy[1]; }
    if (nseg > 2) { a.ws2 = ws[2]; a.vc = y[2]; a.kv_pgs = ldy[2]; }
    if (M < kDecMfmaMinB || fmt != WF_FMT_I2S) {
        constexpr int LPR = 32, RPB = kNT / LPR;
        const dim3 grid((N + RPB - 1) / RPB, M);
#define WF_LIN(F, PPTV) hipLaunchKernelGGL((k_gemv<F, MODE_LINEAR, LPR, 1, PPTV>), grid, dim3(kNT), (size_t)lds_image_bytes<F>(K), st, a)
        if (fmt == WF_FMT_TQ) { if (norm_ppt(kp) == 1) WF_LIN(FmtTQ, 1); else WF_LIN(FmtTQ, 2); }
        else { if (norm_ppt(kp) == 1) WF_LIN(FmtI2S, 1); else WF_LIN(FmtI2S, 2); }
#undef WF_LIN
        return check_launch("bitnet_linear");
    }
    WF_REQUIRE(workspace && ((uintptr_t)workspace & 15) == 0, "bitnet_linear: workspace of wf_bitnet_linear_ws_bytes() bytes required for M >= 16");
    const int64_t q8s = (K + 15) / 16 * 16;
    int8_t* q8 = reinterpret_cast<int8_t*>(workspace);
    float* sf = reinterpret_cast<float*>(q8 + (int64_t)M * q8s);
    int* asum = reinterpret_cast<int*>(sf + M);
    if (norm_ppt(K) == 1) hipLaunchKernelGGL(k_quant_rows_lin<1>, dim3(M), dim3(kNT), 0, st, x, ldx, K, q8, q8s, sf, asum);
    else hipLaunchKernelGGL(k_quant_rows_lin<2>, dim3(M), dim3(kNT), 0, st, x, ldx, K, q8, q8s, sf, asum);
    a.q8 = q8; a.q8_stride = q8s; a.act_sf = sf; a.act_sum = asum;
    if (gemm_small_ok(M, N))  // 16-32-row tiles (wf_small.h; the 128 x 128 tiles give N / 128 blocks)
        launch_gemm_small_mfma(w, q8, q8s, M, N, K, EpiLinearSmall{a}, st);
    else
        hipLaunchKernelGGL(k_linear_mfma, dim3((N + 127) / 128, (M + 127) / 128), dim3(256), 0, st, a);
    return check_launch("bitnet_linear");
}

int wf_bitnet_linear(int fmt, const uint8_t* w, const uint16_t* x, int64_t ldx, float ws, int M, int N, int K,
                     uint16_t* y, int64_t ldy, void* workspace, void* stream) {
    WF_REQUIRE(N > 0, "bitnet_linear: bad shape M=%d N=%d K=%d (K %% 128 == 0)", M, N, K);
    uint16_t* const ys[1] = {y};
    const int64_t lds[1] = {ldy};
    return wf_bitnet_linear_fused(fmt, w, 1, &N, &ws, x, ldx, M, K, ys, lds, workspace, stream);
}

int64_t wf_bitnet_mlp_ws_bytes(int M, int H, int I) {
    if (M <= 0 || H <= 0 || I <= 0) return 0;
    const int64_t act = ((int64_t)M * I * 2 + 255) / 256 * 256;
    return 2 * act + std::max(wf_bitnet_linear_ws_bytes(M, H), wf_bitnet_linear_ws_bytes(M, I));
}

// BitNet MLP (direct_inference_full.py:252-265): gate|up with one shared quantization, relu(g)^2 * u,
// rms_norm(ffn_sub_norm), down -- the reference's attempted bitnet_mlp_forward_cpu as one call.
int wf_bitnet_mlp(int fmt, const uint8_t* w_gate_up, const uint8_t* w_down, float ws_gate, float ws_up,
                  float ws_down, const uint16_t* ffn_sub_norm, float eps, const uint16_t* x, int64_t ldx, int M, int H,
                  int I, uint16_t* y, int64_t ldy, void* workspace, void* stream) {
    WF_REQUIRE(w_gate_up && w_down && ffn_sub_norm && x && y && workspace, "bitnet_mlp: null pointer");
    WF_REQUIRE(((uintptr_t)workspace & 255) == 0, "bitnet_mlp: workspace of wf_bitnet_mlp_ws_bytes() bytes, 256-byte aligned");
    WF_REQUIRE(M > 0 && H > 0 && I > 0 && H % 128 == 0 && I % 128 == 0 && I <= 8192,
               "bitnet_mlp: bad shape M=%d H=%d I=%d (multiples of 128, I <= 8192)", M, H, I);
    WF_REQUIRE(aligned16(ffn_sub_norm), "bitnet_mlp: ffn_sub_norm must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    const int64_t act = ((int64_t)M * I * 2 + 255) / 256 * 256;
    uint16_t* g = reinterpret_cast<uint16_t*>(workspace);
    uint16_t* u = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(workspace) + act);
    void* lin_ws = reinterpret_cast<uint8_t*>(workspace) + 2 * act;
    const int n[2] = {I, I};
    const float ws[2] = {ws_gate, ws_up};
    uint16_t* const ys[2] = {g, u};
    const int64_t lds[2] = {I, I};
    int rc = wf_bitnet_linear_fused(fmt, w_gate_up, 2, n, ws, x, ldx, M, H, ys, lds, lin_ws, stream);
    if (rc) return rc;
    const int64_t n8 = (int64_t)M * I / 8;
    hipLaunchKernelGGL(k_relu2_mul, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, g, u, n8);
    // rms_norm(ffn_sub_norm) of the activation rows (the decode step's row norm) -> u
    if (norm_ppt(I) == 1)
        hipLaunchKernelGGL((k_rownorm<1, true, false>), dim3(M), dim3(kNT), 0, st, g, (int64_t)I, ffn_sub_norm, I, eps,
                           nullptr, (int64_t)0, nullptr, nullptr, u, (int64_t)I);
    else
        hipLaunchKernelGGL((k_rownorm<2, true, false>), dim3(M), dim3(kNT), 0, st, g, (int64_t)I, ffn_sub_norm, I, eps,
                           nullptr, (int64_t)0, nullptr, nullptr, u, (int64_t)I);
    if ((rc = check_launch("bitnet_mlp"))) return rc;
    return wf_bitnet_linear(fmt, w_down, u, I, ws_down, M, H, I, y, ldy, lin_ws, stream);
}

int wf_model_graph_launch(wf_model* m, void* stream) {
    WF_REQUIRE(m, "model_graph_launch: null model");
    if (int rc = take_device_error(m)) return rc;
    if (!m->exec) {
        WF_HIP(hipStreamBeginCapture(m->cap, hipStreamCaptureModeThreadLocal));
        int rc = model_step(m, m->cap);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(m->cap, &g);
        if (rc) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        WF_HIP(e);
        m->graph = g;
        WF_HIP(hipGraphInstantiate(&m->exec, m->graph, nullptr, nullptr, 0));
    }
    WF_HIP(hipGraphLaunch(m->exec, as_stream(stream)));
    return WF_OK;
}

}  // extern "C"
