/*
 * wf_bitnet.h -- C-ABI of the MI355X (gfx950) BitNet 1.58-bit hot path.
 *
 * This is the drop-in boundary that replaces the sgl-kernel CPU ops of the reference
 * (extern/sglang-bitnet/sgl-kernel, un-vendored; API recovered in SURVEY.md §8b) and the kernels
 * behind src/wrinklefree_inference/{kernels,kv_cache}. Plain pointers and sizes only: device
 * pointers for tensor data, `stream` = a hipStream_t (NULL = the default stream). Every call is
 * stream-ordered with no hidden synchronisation and no allocation (graph-capturable), except
 * wf_model_* which own device memory.
 *
 * Return codes: WF_OK (0), WF_EINVAL (1, bad argument: the Python layer raises ValueError /
 * RuntimeError like the reference's TORCH_CHECKs), WF_EHIP (2, HIP error), WF_ENOTSUP (3).
 * wf_last_error() holds the message of the last failure on the calling thread.
 *
 * Packed-weight formats (enc = w + 1 in {0,1,2}):
 *   WF_FMT_I2S : blocked I2_S [N, K/4] (cache/bitnet_converter.py:26-77) -- the reference layout.
 *   WF_FMT_TQ  : ~1.6-bit [N, ceil(K/80)*16], 5 trits per byte (load-time bijection of I2_S).
 *   WF_FMT_I2S_MFMA: the I2_S bytes re-tiled for the int8 matrix cores (same size, N % 16 == 0):
 *                dword ((n/16 * K/128 + kb) * 64 + (n%16) + 16q) * 2 + h = I2_S bytes
 *                [32 kb + 16 h + 4 q, +4) of row n -- one contiguous KiB-class load per MFMA
 *                fragment set. Used by the batched (batch >= 16) decode step.
 */
#ifndef WF_BITNET_H
#define WF_BITNET_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WF_OK 0
#define WF_EINVAL 1
#define WF_EHIP 2
#define WF_ENOTSUP 3

enum { WF_F32 = 0, WF_BF16 = 1, WF_F16 = 2, WF_I8 = 3, WF_U8 = 4 };
enum { WF_FMT_I2S = 0, WF_FMT_TQ = 1, WF_FMT_I2S_MFMA = 2 };
/* K/V cache element types (wf_model_desc.kv_quant) */
enum { WF_KV_BF16 = 0, WF_KV_FP8 = 1, WF_KV_INT8 = 2 };

/* ---- library ------------------------------------------------------------------------------ */
const char* wf_last_error(void);
int wf_abi_version(void);
/* sgl_kernel.quantization.bitnet_check_kernel_available (kernels/bitnet_patch.py:22;
 * scripts/launch_sglang_bitnet.sh:44-50): 1 when a gfx950 device is visible and the kernels load. */
int wf_check_kernel_available(void);

/* ---- ternary GEMV / GEMM ------------------------------------------------ */
/* torch.ops.sgl_kernel.bitnet_gemv_cpu(packed_weights, activations, scale)
 * (docs/research/sglang_optimization_plan.md:61-64; call sites kernels/bitnet_patch.py:69,
 * scripts/benchmark_kernels.py:46): y[n] = float(sum_k enc(W[n,k]) * a[k]) * scale. K % 128 == 0. */
int wf_bitnet_gemv(const uint8_t* w, const int8_t* a, float scale, int N, int K, float* y, void* stream);
/* torch.ops.sgl_kernel.bitnet_gemm_cpu (sglang_optimization_plan.md:66-70; bitnet_patch.py:73):
 * Y[m,n] = float(sum_k enc(W[n,k]) * A[m,k]) * scale, one scale for the batch. */
int wf_bitnet_gemm(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y, void* stream);
/* Same contract, any weight format and strides (lda/ldy in elements, lda % 16 == 0). */
int wf_bitnet_gemm_ex(int fmt, const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K,
                      float* y, int64_t ldy, void* stream);
/* BitNetLinear.forward, fused (scripts/direct_inference_full.py:186-208, the layer the reference's
 * decode runs 7x per block; kernels/bitnet_patch.py:55-78 is the same contract without the
 * correction): per row m, s = double(max|x[m]|)/127, q = rne(x/float(s)), then
 * y[m,n] = bf16(fl32(fl32(sum_k enc(W[n,k]) q[k] - ws * sum_k q[k]) * s)).  x, y bf16 (row strides
 * ldx, ldy in elements; ldx % 8 == 0), W I2_S or TQ [N][row bytes], K % 128 == 0, K <= 8192.
 * M < 16 is one launch (quantize in the GEMV prologue); M >= 16 with I2_S needs a 16-byte aligned
 * workspace of wf_bitnet_linear_ws_bytes(M, K) bytes (per-row codes for the int8-MFMA GEMM). */
int64_t wf_bitnet_linear_ws_bytes(int M, int K);
int wf_bitnet_linear(int fmt, const uint8_t* w, const uint16_t* x, int64_t ldx, float ws, int M, int N, int K,
                     uint16_t* y, int64_t ldy, void* workspace, void* stream);
/* Fused projections with ONE shared activation quantization ("shared quantize
 * across fused QKV / gate-up"; the reference's attempted bitnet_qkv_forward_cpu / bitnet_mlp_forward_cpu,
 * docs/research/sglang_optimization_plan.md:326-331, and the q|k|v / gate|up projections of
 * scripts/direct_inference_full.py:212-214,254-256 that quantize the same input 3x / 2x). The nseg
 * (1..3) layers' packed weights are row-concatenated in w (segment s = the next n[s] rows, same format
 * and K), each with its own weight scale ws[s] and bf16 output y[s] (device pointer, row stride
 * ldy[s]); n, ws, y, ldy are host arrays of nseg entries. y[s] equals wf_bitnet_linear on segment s
 * bit for bit. M < 16: one launch for all segments; M >= 16 (I2_S): one row quantization and one
 * int8-MFMA GEMM over all segments (workspace of wf_bitnet_linear_ws_bytes(M, K) bytes). */
int wf_bitnet_linear_fused(int fmt, const uint8_t* w, int nseg, const int* n, const float* ws, const uint16_t* x,
                           int64_t ldx, int M, int K, uint16_t* const* y, const int64_t* ldy, void* workspace,
                           void* stream);
/* BitNet MLP (scripts/direct_inference_full.py:252-265; the reference's attempted
 * bitnet_mlp_forward_cpu, docs/research/sglang_optimization_plan.md:326-331): for each row of x
 * (bf16 [M, H], the post-attention-normed hidden state), y = down(rms_norm(relu(gate(x))^2 * up(x),
 * ffn_sub_norm)) with BitNetLinear gate / up / down (gate|up: one shared quantization, weights
 * row-concatenated [gate; up] as wf_bitnet_linear_fused), bf16 between ops as the reference. y bf16
 * [M, H] (row stride ldy); H, I multiples of 128, I <= 8192; workspace of wf_bitnet_mlp_ws_bytes(M, H, I)
 * bytes, 256-byte aligned. Four launches below 16 rows, six above. */
int64_t wf_bitnet_mlp_ws_bytes(int M, int H, int I);
int wf_bitnet_mlp(int fmt, const uint8_t* w_gate_up, const uint8_t* w_down, float ws_gate, float ws_up,
                  float ws_down, const uint16_t* ffn_sub_norm, float eps, const uint16_t* x, int64_t ldx, int M, int H,
                  int I, uint16_t* y, int64_t ldy, void* workspace, void* stream);
/* kernels/native.py:27-65 (wrinklefree_inference.kernels.native gemv/gemm): signed (bits-1) dot
 * on the LSB-interleaved layout byte[j] = w[4j] | w[4j+1]<<2 | ..., float(sum) * scale. */
int wf_bitnet_gemm_lsb(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y, void* stream);

/* ---- activation int8 quantizer --------------------------------------------- */
/* torch.ops.sgl_kernel.bitnet_quantize_activations_cpu (sglang_optimization_plan.md:72-74;
 * semantics tests/test_bitnet_core.py:139-146): per-tensor m = max|x|, s = m/127 (double; m -> 1
 * when m < 1e-6), q = clamp(rne(x / float(s)), -128, 127). Writes q and m (device float; the host
 * forms s = double(m)/127 exactly as the reference). `dtype` of x: WF_F32 / WF_BF16 / WF_F16. */
int wf_quantize_i8(const void* x, int dtype, int64_t n, int8_t* q, float* absmax, void* stream);
/* Per-row variant (one scale per token; used by batched decode): row_absmax [M]. */
int wf_quantize_i8_rows(const void* x, int dtype, int M, int K, int8_t* q, float* row_absmax, void* stream);
/* kernels/native.py:244-256 variant: float32 scale, truncating cast. */
int wf_quantize_i8_trunc(const void* x, int dtype, int64_t n, int8_t* q, float* absmax, void* stream);

/* ---- load-time weight formats -------------------------------- */
/* cache/bitnet_converter.py:26-77: float ternary weights [N,K] -> blocked I2_S [N,K/4]. */
int wf_pack_i2s(const void* w, int dtype, int N, int K, uint8_t* out, void* stream);
/* tests/test_bitnet_core.py:21-53 then :56-106: HF [N/4,K] uint8 -> I2_S [N,K/4]. */
int wf_hf_to_i2s(const uint8_t* hf, int Np, int K, uint8_t* out, void* stream);
/* I2_S [N,K/4] <-> TQ [N, ceil(K/80)*16] (bijection, K % 128 == 0). */
int wf_i2s_to_tq(const uint8_t* i2s, int N, int K, uint8_t* tq, void* stream);
int wf_tq_to_i2s(const uint8_t* tq, int N, int K, uint8_t* i2s, void* stream);
int64_t wf_tq_row_bytes(int K);
/* I2_S <-> WF_FMT_I2S_MFMA (bijection; N % 16 == 0, K % 128 == 0). */
int wf_i2s_to_mfma(const uint8_t* i2s, int N, int K, uint8_t* out, void* stream);
int wf_mfma_to_i2s(const uint8_t* mf, int N, int K, uint8_t* i2s, void* stream);
/* int8 activation codes [M][lda] -> the matrix-core tile order the batched decode step's row
 * quantizer writes: per (16-row tile rt, I2_S block kb, half h) one KiB, lane l16 + 16q holding
 * the codes of row 16rt + l16 at k = 128kb + 16h + 4q + jj + 32g in byte 4g + jj (csrc/wf_norm.h
 * tile_code_pos). out holds ceil(M/16)*16*K bytes; rows >= M are zero. K % 128 == 0. */
int wf_codes_to_tiles(const int8_t* a, int64_t lda, int M, int K, int8_t* out, void* stream);
/* bitnet_gemm (the sgl_kernel contract above: Y = float(sum enc(W) * A) * scale, fp32 out) for
 * prefill-sized M on the matrix-core tile layouts: w in WF_FMT_I2S_MFMA, a from wf_codes_to_tiles.
 * Bit-identical to wf_bitnet_gemm on the same logical operands. K % 128 == 0, N % 16 == 0. */
int wf_bitnet_gemm_tiled(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y, int64_t ldy,
                         void* stream);

/* ---- KV cache ----------------------------------------------------- */
/* sgl_kernel.kvcache.KVCacheManager.scatter_kv / gather_kv (tests/test_kv_cache_cpp.py:283-373;
 * Python twin :20-127): pool [max_pages, L, 2, H, D] of elem_bytes-sized elements; k/v [T, H*D].
 * gather writes into caller buffers. Page ids must be in [0, max_pages) (checked on device:
 * out-of-range tokens are skipped and counted in *bad if bad != NULL). */
int wf_kv_scatter(void* pool, int elem_bytes, int max_pages, int L, int H, int D, const void* k, const void* v,
                  const int32_t* pages, int T, int layer, int32_t* bad, void* stream);
int wf_kv_gather(const void* pool, int elem_bytes, int max_pages, int L, int H, int D, void* k_out, void* v_out,
                 const int32_t* pages, int T, int layer, int32_t* bad, void* stream);
/* The same two calls on the decode engine's own paged pool (wf_model_desc.page_table's pages, bf16):
 * k_pool / v_pool = one layer's [num_pages][H][32 * 128] of wf_model_desc.k_cache / v_cache; token
 * row t of k / v ([T, H*128]) at page pages[t], slot slots[t] in [0, 32) -- the reference's
 * slot_indices (tests/test_kv_cache_cpp.py:80-126), here the position within a 32-token page, stored
 * in the K / V tile layouts the batched attention reads. So sgl_kernel.kvcache.KVCacheManager can
 * hand out, fill and read the very pages the decode step attends over (invalid page / slot ids:
 * skipped, counted in *bad). head_dim 128. */
int wf_kv_scatter_tiles(void* k_pool, void* v_pool, int num_pages, int H, int D, const uint16_t* k, const uint16_t* v,
                        const int32_t* pages, const int32_t* slots, int T, int32_t* bad, void* stream);
int wf_kv_gather_tiles(const void* k_pool, const void* v_pool, int num_pages, int H, int D, uint16_t* k_out,
                       uint16_t* v_out, const int32_t* pages, const int32_t* slots, int T, int32_t* bad, void* stream);
/* KVCache._quantize_to_int8 / _quantize_to_fp8 (kv_cache/kv_cache.py:159-218): given m = max|x|
 * (device), q = clamp(rne(x * float(127/m')), -127, 127), m' = m or 1 if m < 1e-6. */
int wf_kv_quant_i8(const void* x, int dtype, int64_t n, const float* absmax, int8_t* q, void* stream);
/* _dequantize_* (kv_cache.py:187-228): out = (float(q) * scale[0]) rounded to out_dtype. */
int wf_kv_dequant_i8(const int8_t* q, int64_t n, const float* scale, void* out, int out_dtype, void* stream);

/* Split-K decode attention for one query token per sequence (kv_cache.py:316-369 without GQA;
 * scripts/direct_inference_full.py:229-244 with GQA). Strides are in elements.
 *   q   : [B, Hq, D] (q_dtype)            out : [B, Hq, D] (out_dtype)
 *   k,v : element (b, g, t, d) at b*kv_sb + g*kv_sh + t*kv_st + d (kv_dtype: BF16/F16/F32/I8;
 *         I8 caches are dequantized as rbf16(float(q) * k_scale) like kv_cache.py:220-228)
 *   seq_lens : [B] int32 device (NULL -> every sequence has S keys)
 *   ws : workspace of wf_decode_attention_ws_bytes(B, Hq, D, S) bytes.                           */
int64_t wf_decode_attention_ws_bytes(int B, int Hq, int D, int S);
int wf_decode_attention(const void* q, int q_dtype, int64_t q_sb, int64_t q_sh, const void* k, const void* v,
                        int kv_dtype, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale,
                        int B, int Hq, int Hkv, int D, int S, const int32_t* seq_lens, float sm_scale, void* out,
                        int out_dtype, int64_t o_sb, int64_t o_sh, void* ws, void* stream);

/* ---- SGLang BitNet linear method, MSB-interleaved layout ------------------- */
/* Layout (sglang_backend/bitnet_quantization.py:99-105, :128-133): byte j of row n =
 * code(w[4j])<<6 | code(w[4j+1])<<4 | code(w[4j+2])<<2 | code(w[4j+3]), code = w + 1.        */
/* weights.abs().max().item() (bitnet_quantization.py:84): *out = max|x| (device float).       */
int wf_absmax(const void* x, int dtype, int64_t n, float* out, void* stream);
/* quantize_to_bitnet (bitnet_quantization.py:69-109) given its scale (the caller maps a scale
 * < 1e-6 to 1.0 and raises for K % 128 != 0 like the reference's assert): normalized =
 * rnd_dtype(w / float(scale)); code 2 if > 0.5, 0 if < -0.5, else 1. out [N, K/4].            */
int wf_msb_ternarize(const void* w, int dtype, int N, int K, float scale, uint8_t* out, void* stream);
/* dequantize_bitnet (bitnet_quantization.py:211-252): out[n,k] = (code-1) * float(scale) in
 * out_dtype (F32/BF16/F16); K % 16 == 0, 16-byte aligned.                                    */
int wf_msb_dequant(const uint8_t* packed, int N, int K, float scale, void* out, int out_dtype, void* stream);
/* BitNetLinearMethod.apply (bitnet_quantization.py:366-409) computed from the packed bytes:
 * y[m,n] = rnd(rnd(ws * sum_k (code-1) x[m,k]) + bias[n]), ws = scale rounded to the compute
 * dtype (x_dtype: BF16 or F16; y and bias in the same dtype; bias may be NULL). fp32 accumulate.
 * WF_ENOTSUP when K % 64 != 0 or K > 16384 (the caller then multiplies the dequantised matrix). */
int wf_msb_linear(const uint8_t* w, float scale, const void* x, int x_dtype, int64_t ldx, int M, int N, int K,
                  const void* bias, void* y, int64_t ldy, void* stream);

/* ---- whole decode step (scripts/direct_inference_full.py:181-302) ------ */
typedef struct {
    int hidden, layers, n_heads, n_kv_heads, head_dim, inter, vocab, max_seq, batch;
    float eps;
    int wfmt;                     /* WF_FMT_I2S or WF_FMT_TQ for the ternary weights below         */
    const uint16_t* embed;        /* [vocab, hidden] bf16 (tied LM head)                          */
    const uint16_t* final_norm;   /* [hidden]                                                     */
    const uint16_t* rope_cos;     /* [max_seq, head_dim/2] bf16                                   */
    const uint16_t* rope_sin;
    const uint16_t* ln_in;        /* [layers, hidden]                                             */
    const uint16_t* ln_post;
    const uint16_t* attn_sub;
    const uint16_t* ffn_sub;      /* [layers, inter]                                              */
    const uint8_t* w_qkv;         /* [layers, (Hq+2Hkv)*D rows] packed, rows q|k|v                */
    const uint8_t* w_o;           /* [layers, hidden rows]                                        */
    const uint8_t* w_gu;          /* [layers, 2*inter rows], gate/up interleaved in 8-row tiles   */
    const uint8_t* w_d;           /* [layers, hidden rows] (K = inter)                            */
    const float* wscale;          /* HOST [layers, 7] q,k,v,o,gate,up,down (copied at create)      */
    /* caller-owned device state (read and written by every step)                                */
    int32_t* tokens;              /* [batch]: input token; the step stores the greedy next token   */
    int32_t* positions;           /* [batch]: position of the input token; the step increments it  */
    uint16_t* logits;             /* [batch, vocab] bf16                                           */
    uint16_t* k_cache;            /* [layers, batch, n_kv_heads, max_seq, head_dim] bf16           */
    uint16_t* v_cache;            /* same shape; for batch >= 16 with I2_S weights and max_seq % 32 == 0 it is
                                     stored transposed per (layer, sequence, kv head): [head_dim, max_seq] */
    int debug_flags;              /* reserved, must be 0 (latency studies use the stamp build,
                                     tools/stamps.py)                                             */
    /* Paged KV (optional; batched matrix-core decode only: batch >= 16, I2_S weights, head_dim 128,
     * max_seq % 32 == 0). Replaces the dense per-sequence planes of k_cache / v_cache above with a
     * shared pool of 32-token pages, the MI355X-native counterpart of sgl_kernel.kvcache's paged
     * pool (tests/test_kv_cache_cpp.py:283-373) for the attention of SURVEY §8f rank 2:
     *   k_cache, v_cache : [layers, num_pages, n_kv_heads, 32 * head_dim] bf16, each 32-token page
     *                      of one kv head in the K / V tile layout of one 32-key block;
     *   page_table       : [batch, max_seq / 32] int32, page of block t >> 5 of sequence b. It is
     *                      read by every step (caller-owned, device memory, may change between
     *                      steps); entries of blocks a step touches must be in [0, num_pages)
     *                      (out-of-range ids are clamped on the device: wrong keys, never a fault).
     * page_table == NULL keeps the dense layout. */
    const int32_t* page_table;
    int num_pages;
    /* One-byte K/V (optional; same decoders as paged KV), kv_quant:
     *   WF_KV_BF16 (0) bf16 K/V;
     *   WF_KV_FP8  (1) OCP e4m3fn bytes, code = e4m3(clamp(v / scale, +-448)) (RNE);
     *   WF_KV_INT8 (2) int8, code = clamp(rne(v / scale), -127, 127) -- the reference's default
     *                  KVCacheDtype.INT8 (kv_cache/kv_cache.py:30-37, 159-218) with a static
     *                  per-layer scale instead of its per-update absmax (one scale per layer there too).
     * Same tile layouts / pages with one byte per element -- half the attention bytes. kv_scale: HOST
     * [layers][2] (K, V) scales (NULL = 1.0), copied at create; the attention widens codes to bf16
     * exactly and folds the scales into the score scale and the partial sums. Quality bar (reference
     * docs/research/notebook.md:690-700): attention-output cosine >= 0.998 vs bf16 K/V. */
    int kv_quant;
    const float* kv_scale;
} wf_model_desc;

typedef struct wf_model wf_model;
/* Validates the descriptor and allocates the private workspaces (activations, attention partials). */
int wf_model_create(const wf_model_desc* d, wf_model** out);
int wf_model_destroy(wf_model* m);
/* One decode step for every sequence of the batch, stream-ordered; capturable into a HIP graph. */
int wf_model_step(wf_model* m, void* stream);
/* Capture wf_model_step into a graph once, then replay it (no host work per token). */
int wf_model_graph_launch(wf_model* m, void* stream);
/* Launch one op of the step (profiling / per-kernel timing). Ops, in step order: */
enum {
    WF_OP_EMBED = 0,      /* h = embed[token] (layer ignored; skipped at batch 1, see below)      */
    WF_OP_QKV = 1,        /* input_layernorm + quantize -> q|k|v ternary GEMV + correction + RoPE
                             + K/V cache write                                                    */
    WF_OP_ATTN = 2,       /* GQA decode attention with the reference's CPU bf16 SDPA arithmetic;
                             writes the bf16 attention row (wf_attn_records.attn_row)             */
    WF_OP_O = 3,          /* attn_sub_norm + quantize of that row -> o_proj + residual             */
    WF_OP_GATE_UP = 4,    /* post_attention_layernorm + quantize -> gate|up + relu^2 * up          */
    WF_OP_DOWN = 5,       /* ffn_sub_norm + quantize -> down_proj + residual                       */
    WF_OP_LM_HEAD = 6     /* final norm + tied bf16 LM head + greedy argmax + position advance
                             (layer ignored)                                                      */
    /* (batch > 1: each GEMM op's norm + quantize runs as a row-norm launch in front of it) */
};
/* Batch 1: wf_model_step skips WF_OP_EMBED and layer 0's WF_OP_QKV / WF_OP_O read the token's
 * embedding row (embed[token], the residual) themselves, so wf_model_launch_op(m, 0, WF_OP_QKV or
 * WF_OP_O) at batch 1 takes its input from tokens[0] (wf_model_desc.tokens), not from h. */
int wf_model_launch_op(wf_model* m, int layer, int op, void* stream);
/* Read-only view of the step's attention hand-off, for kernel-level checks (tests/, profiling):
 * after WF_OP_QKV and WF_OP_ATTN of a layer, q holds that layer's query rows after RoPE
 * ([batch, n_heads * head_dim] bf16) and the partial records of the split attention: per
 * (sequence b, query head h, record s < records), part_ml[2 ((b n_heads + h) records + s) + {0, 1}] =
 * (running max m, sum l) and the unnormalised output o[d] at part_o[((b n_heads + h) records + s) *
 * 128 + ((d >> 2) & 1) * 64 + (d >> 3) * 4 + (d & 3)] (head_dim 128). Batch < 16 and untiled caches:
 * records in one frame (m = 0; the reference's SDPA semantics), which each head's last attention
 * block sums into attn_row. Batch >= 16 on tile-layout caches: no records (records = 0). attn_row is
 * the bf16 attention output [batch, n_heads * head_dim] the O projection reads, on every path. Device
 * pointers owned by the model; valid until wf_model_destroy. */
typedef struct {
    const uint16_t* q;
    const float* part_ml;
    const float* part_o;
    int records;
    const uint16_t* attn_row;
} wf_attn_records;
int wf_model_attn_view(const wf_model* m, wf_attn_records* out);
/* The decode attention exchanges split maxima / records between the workgroups of one launch
 * (batch < 16 or untiled caches; batched split-2 sequences) and bounds every poll: if a sibling
 * workgroup never becomes resident (the device shared with other work that holds every CU), the
 * poll gives up after ~0.2-0.5 s, that launch's attention rows are NaN and the kernel raises a
 * host-visible error word. wf_model_step / wf_model_graph_launch / wf_model_launch_op report (and
 * clear) it at their next call with WF_EHIP; wf_model_check reports it without launching (call it
 * after synchronising the stream to check the steps launched so far). */
int wf_model_check(wf_model* m);
/* Test hook: with on != 0, the model's batch < 16 / untiled decode attention polls for a tag no
 * workgroup publishes, so its next EAGER launches (wf_model_step, wf_model_launch_op; a captured
 * graph keeps the flag of its capture) take the timeout path above. */
int wf_model_debug_stall_attention(wf_model* m, int on);
/* Read-only view of the last wf_model_prefill call's last layer, for kernel-level checks (tests/):
 * q = its query rows after RoPE and attn = its causal attention output rows, both [rows][n_heads *
 * head_dim] bf16 in the call's row order. Device pointers owned by the model; valid until the next
 * prefill or wf_model_destroy. WF_EINVAL before any prefill reservation. */
int wf_model_prefill_view(const wf_model* m, const uint16_t** q, const uint16_t** attn);
/* Which batched GEMM ops (flags[0..3] = QKV, O, gate|up, down) run their input row norm inside the
 * GEMM launch instead of a separate row-norm launch (batch >= 16 on WF_FMT_I2S_MFMA weights, when
 * the whole grid fits the device at once; decided at wf_model_create). Diagnostic / bench query:
 * the step's results do not depend on it. */
int wf_model_fused_norm(const wf_model* m, int* flags4);
/* Prefill (BASELINE configs[2]; the prompt pass that precedes scripts/direct_inference_full.py's
 * decode loop): run prompt tokens of any KV slots through all layers as GEMM rows and write their
 * K/V into the cache (dense planes or pages). Batched matrix-core decoders only (batch >= 16, I2_S
 * weights), head_dim 128, 4 query heads per kv head. Row r: token tokens[r] of slot row_slot[r] at
 * position row_pos[r] (device int32 arrays); every aligned group of WF_PREFILL_ROW_GROUP rows
 * belongs to one slot (pad a sequence by repeating its last row); a slot's earlier positions must already be in the
 * cache (earlier rows of the same call count). Does not touch tokens / positions / logits: the
 * decode step then runs the prompt's last token. reserve() allocates the row workspace once. */
#define WF_PREFILL_ROW_GROUP 32
int wf_model_prefill_reserve(wf_model* m, int rows);
int wf_model_prefill(wf_model* m, const int32_t* tokens, const int32_t* row_slot, const int32_t* row_pos, int rows,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif
