// wf_decode.hip -- fused BitNet b1.58 decode step for gfx950.
//
// One decode token per sequence = per layer four fused ternary-GEMV launches + split-K attention:
//   QKV : prologue rms_norm(input_layernorm) -> per-token int8 quantize (LDS image);
//         rows q|k|v; epilogue = reference correction, RoPE (θ=5e5, half-split), K/V -> cache.
//   ATT : split-K GQA decode attention over the cache (wf_attn.hip) -> attn [B, Hq*D] bf16.
//   O   : prologue rms_norm(attn_sub_norm) + quantize; epilogue correction + residual add.
//   GU  : prologue rms_norm(post_attention_layernorm) + quantize; rows gate/up interleaved in
//         8-row tiles; epilogue relu(gate)^2 * up (bf16 ops as the reference).
//   DN  : prologue rms_norm(ffn_sub_norm) over 6912 + quantize; epilogue correction + residual.
// then final rms_norm + tied bf16 LM head GEMV with a fused greedy argmax. Every float op follows
// scripts/direct_inference_full.py:181-302 (bf16 tensors between ops), so results match the oracle
// up to fp32 reduction order.
//
// The weights are streamed once per token (HBM-bound); activations never leave LDS/L2.
#include <hip/hip_runtime.h>

#include <new>

#include "wf_common.h"
#include "wf_device.h"

namespace wf {
int decode_attention_impl(const void* q, int q_dtype, int64_t q_sb, int64_t q_sh, const void* k, const void* v,
                          int kv_dtype, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int B,
                          int Hq, int Hkv, int D, int S, const int32_t* seq_lens, float sm_scale, void* out,
                          int out_dtype, int64_t o_sb, int64_t o_sh, void* ws, hipStream_t st);

enum { MODE_QKV = 0, MODE_O = 1, MODE_GU = 2, MODE_DN = 3 };
constexpr int kMaxVec = 8;              // prologue: up to 8 x 4 elements per thread -> K <= 8192
constexpr int kRowsPerBlockFused = 16;  // 4 waves x 4 rows, 16 lanes per row
constexpr int kPrefetch = 4;            // 16-byte weight chunks in flight per lane

struct LayerArgs {
    const uint16_t* x;        // [B, K] bf16 prologue input
    int64_t x_stride;
    const uint16_t* norm_w;   // [K] bf16
    const uint8_t* w;         // packed rows
    int N, K;
    float ws0, ws1, ws2;      // weight scales (QKV: q,k,v; GU: gate, up; O/DN: ws0)
    float eps;
    // epilogue
    const uint16_t* resid;    // O/DN: residual input [B, N]
    uint16_t* out;            // O/DN: hidden out [B, N]; GU: act [B, I]; QKV: q [B, Hq*D]
    int64_t out_stride;
    // QKV extras
    int Hq, Hkv, D, S;
    const int32_t* positions;
    const uint16_t* rope_cos;
    const uint16_t* rope_sin;
    uint16_t* kc;             // this layer's cache: [B][Hkv][S][D]
    uint16_t* vc;
    int64_t kv_b_stride;      // Hkv*S*D
};

// rms_norm + int8 quantize of one activation row into the block's LDS image, in three phases with
// one barrier each (per-wave partials in LDS, no reuse hazards):
//   load:   raw bf16 x and norm weight -> registers (issued before the weight stream)
//   finish: sum(x^2) -> r = bf16(rsqrt(mean + eps)); y = bf16(bf16(x*r)*w); max|y|; q = rne(y/s)
// Exact reference float sequence (direct_inference_full.py:181-184, 196; test_bitnet_core.py:139-146).
struct RowRaw {
    uint2 x[kMaxVec], w[kMaxVec];
};

__device__ __forceinline__ void prologue_load(const uint16_t* __restrict__ x, const uint16_t* __restrict__ nw, int K,
                                              RowRaw& r) {
    const int nvec = K / 4;
#pragma unroll
    for (int v = 0; v < kMaxVec; ++v) {
        const int e = threadIdx.x + v * blockDim.x;
        r.x[v] = make_uint2(0, 0);
        r.w[v] = make_uint2(0, 0);
        if (e < nvec) {
            r.x[v] = *reinterpret_cast<const uint2*>(x + 4 * e);
            r.w[v] = *reinterpret_cast<const uint2*>(nw + 4 * e);
        }
    }
}

template <class F>
__device__ __forceinline__ void prologue_finish(const RowRaw& r, int K, float eps, int8_t* img, float* red,
                                                int* redi_row, float* out_sf) {
    const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nvec = K / 4;
    float xv[kMaxVec][4];
    float ss = 0.f;
#pragma unroll
    for (int v = 0; v < kMaxVec; ++v) {
        xv[v][0] = __uint_as_float(r.x[v].x << 16); xv[v][1] = __uint_as_float(r.x[v].x & 0xffff0000u);
        xv[v][2] = __uint_as_float(r.x[v].y << 16); xv[v][3] = __uint_as_float(r.x[v].y & 0xffff0000u);
#pragma unroll
        for (int j = 0; j < 4; ++j) ss = fmaf(xv[v][j], xv[v][j], ss);
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    ss = red[0];
    for (int i = 1; i < nw; ++i) ss += red[i];
    const float rr = rbf(1.0f / sqrtf(ss / (float)K + eps));
    float mx = 0.f;
#pragma unroll
    for (int v = 0; v < kMaxVec; ++v) {
        const float w4[4] = {__uint_as_float(r.w[v].x << 16), __uint_as_float(r.w[v].x & 0xffff0000u),
                             __uint_as_float(r.w[v].y << 16), __uint_as_float(r.w[v].y & 0xffff0000u)};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xv[v][j] = rbf(rbf(xv[v][j] * rr) * w4[j]);
            mx = fmaxf(mx, fabsf(xv[v][j]));
        }
    }
    mx = wave_max(mx);
    if (lane == 0) red[16 + wave] = mx;
    __syncthreads();
    mx = red[16];
    for (int i = 1; i < nw; ++i) mx = fmaxf(mx, red[16 + i]);
    const float sf = (float)act_scale_from_max(mx);
    int asum = 0;
#pragma unroll
    for (int v = 0; v < kMaxVec; ++v) {
        const int e = threadIdx.x + v * blockDim.x;
        if (e < nvec) {
            uint32_t packed = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int8_t qv = quant_one(xv[v][j], sf);
                asum += qv;
                packed |= (uint32_t)(uint8_t)qv << (8 * j);
            }
            *reinterpret_cast<uint32_t*>(img + F::lds_off(4 * e)) = packed;
        }
    }
    for (int k = K + 4 * threadIdx.x; k < F::k_pad(K); k += 4 * blockDim.x)  // TQ pad weights see zeros
        *reinterpret_cast<uint32_t*>(img + F::lds_off(k)) = 0u;
    asum = wave_sum_i(asum);
    if (lane == 0) redi_row[wave] = asum;
    *out_sf = sf;
    // the caller's __syncthreads() publishes the image and the per-wave sums
}

// Reference correction (direct_inference_full.py:201-208) for one output:
// raw = fl32(S * f(ws)); c = f(ws * act_sum); out = fl32(fl32(raw - c) * f(s)) -> bf16
__device__ __forceinline__ float corrected(int S, float ws, int asum, float sf) {
    const float raw = (float)S * ws;
    const float c = ws * (float)asum;  // exact product rounded once == float(double(ws)*asum)
    return (raw - c) * sf;
}

template <class F, int MODE, int MB>
__global__ __launch_bounds__(256) void k_fused_gemv(LayerArgs a) {
    extern __shared__ __attribute__((aligned(16))) int8_t smem[];
    __shared__ float red[32];
    __shared__ int redi[MB][4];
    __shared__ float s_sf[MB];
    __shared__ float s_out[MB][16];

    const int K = a.K, N = a.N;
    const int img = lds_image_bytes<F>(K);
    const int b0 = blockIdx.y * MB;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int lrow = wave * 4 + (lane >> 4);                  // 0..15 within the block
    const int row = blockIdx.x * kRowsPerBlockFused + lrow;
    const int C = F::chunks(K);

    // activation row loads first, then the weight stream: vmcnt retires loads in order, so the
    // prologue only waits for its own (L2-near) data while the weights are in flight.
    RowRaw raw;
    prologue_load(a.x + (int64_t)b0 * a.x_stride, a.norm_w, K, raw);
    const uint8_t* wr = a.w + (int64_t)min(row, N - 1) * F::row_bytes(K) + sub * 16;
    uint4 wpre[kPrefetch];
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
        const int c = 16 * u + sub;
        wpre[u] = (c < C) ? ldg_nt(wr + (int64_t)(16 * u) * 16) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll 1
    for (int m = 0; m < MB; ++m) {
        if (m > 0) prologue_load(a.x + (int64_t)(b0 + m) * a.x_stride, a.norm_w, K, raw);
        float sf;
        prologue_finish<F>(raw, K, a.eps, smem + m * img, red, redi[m], &sf);
        if (threadIdx.x == 0) s_sf[m] = sf;
    }
    __syncthreads();
    int s_asum[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) s_asum[m] = redi[m][0] + redi[m][1] + redi[m][2] + redi[m][3];

    int acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = 0;
#pragma unroll
    for (int u = 0; u < kPrefetch; ++u) {
        const int c = 16 * u + sub;
        if (c < C) {
            Decoded<F> d;
            d.load(wpre[u]);
            const int8_t* ab = smem + ((c >> 4) * F::kGroups) * 256 + sub * 16;
#pragma unroll
            for (int m = 0; m < MB; ++m) acc[m] = chunk_dot<F>(d, ab + m * img, acc[m]);
        }
    }
    for (int c0 = 16 * kPrefetch; c0 < C; c0 += 16 * kPrefetch) {
        uint4 w[kPrefetch];
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u) {
            const int c = c0 + 16 * u + sub;
            w[u] = (c < C) ? ldg_nt(wr + (int64_t)(c0 + 16 * u) * 16) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u) {
            const int c = c0 + 16 * u + sub;
            if (c < C) {
                Decoded<F> d;
                d.load(w[u]);
                const int8_t* ab = smem + ((c >> 4) * F::kGroups) * 256 + sub * 16;
#pragma unroll
                for (int m = 0; m < MB; ++m) acc[m] = chunk_dot<F>(d, ab + m * img, acc[m]);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = group16_sum_i(acc[m]);

    // ---- epilogues ----
    if constexpr (MODE == MODE_O || MODE == MODE_DN) {
        if (sub == 0 && row < N) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const float o = rbf(corrected(acc[m], a.ws0, s_asum[m], s_sf[m]));
                const int64_t bi = b0 + m;
                const float h = bf2f(a.resid[bi * a.out_stride + row]);
                a.out[bi * a.out_stride + row] = f2bf(h + o);  // hidden + out (bf16 add)
            }
        }
    } else if constexpr (MODE == MODE_GU) {
        // block rows: [gate 8t..8t+7 | up 8t..8t+7], t = blockIdx.x
        if (sub == 0) {
#pragma unroll
            for (int m = 0; m < MB; ++m)
                s_out[m][lrow] = rbf(corrected(acc[m], lrow < 8 ? a.ws0 : a.ws1, s_asum[m], s_sf[m]));
        }
        __syncthreads();
        if (threadIdx.x < 8 * MB) {
            const int m = threadIdx.x >> 3, i = threadIdx.x & 7;
            const float g = s_out[m][i], u = s_out[m][8 + i];
            const float rl = g > 0.f ? g : 0.f;
            const int n = blockIdx.x * 8 + i;
            a.out[(int64_t)(b0 + m) * a.out_stride + n] = f2bf(rbf(rl * rl) * u);
        }
    } else {  // MODE_QKV: rows per head permuted: block t of head h = dims {8t'..8t'+7, 64+8t'..64+8t'+7}
        const int head = blockIdx.x >> 3, tt = blockIdx.x & 7;   // head in [0, Hq+2Hkv), D == 128
        const int proj = head < a.Hq ? 0 : (head < a.Hq + a.Hkv ? 1 : 2);
        const float wsp = proj == 0 ? a.ws0 : (proj == 1 ? a.ws1 : a.ws2);
        if (sub == 0) {
#pragma unroll
            for (int m = 0; m < MB; ++m) s_out[m][lrow] = rbf(corrected(acc[m], wsp, s_asum[m], s_sf[m]));
        }
        __syncthreads();
        if (threadIdx.x < 8 * MB) {
            const int m = threadIdx.x >> 3, i = threadIdx.x & 7;
            const int bi = b0 + m;
            const int d0 = 8 * tt + i;              // first-half dim; partner d0 + 64
            float x1 = s_out[m][i], x2 = s_out[m][8 + i];
            const int pos = min(max(a.positions[bi], 0), a.S - 1);  // never write outside the cache
            if (proj < 2) {  // RotaryEmbedding._rotate (direct_inference_full.py:58-70)
                const float c = bf2f(a.rope_cos[(int64_t)pos * 64 + d0]);
                const float s = bf2f(a.rope_sin[(int64_t)pos * 64 + d0]);
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
                uint16_t* cache = (proj == 1 ? a.kc : a.vc) + (int64_t)bi * a.kv_b_stride +
                                  ((int64_t)g * a.S + pos) * 128;
                cache[d0] = f2bf(x1);
                cache[d0 + 64] = f2bf(x2);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Small kernels: embedding gather, step bookkeeping, final norm, LM head + argmax.
// ---------------------------------------------------------------------------------------------
__global__ void k_embed(const uint16_t* __restrict__ embed, const int32_t* __restrict__ tokens, int H, int V,
                        uint16_t* __restrict__ h, const int32_t* __restrict__ positions, int32_t* __restrict__ seq_lens) {
    const int b = blockIdx.x;
    const int tok = min(max(tokens[b], 0), V - 1);  // never read outside the table
    const uint4* src = reinterpret_cast<const uint4*>(embed + (int64_t)tok * H);
    uint4* dst = reinterpret_cast<uint4*>(h + (int64_t)b * H);
    for (int i = threadIdx.x; i < H / 8; i += blockDim.x) dst[i] = src[i];
    if (threadIdx.x == 0) seq_lens[b] = positions[b] + 1;
}

__global__ __launch_bounds__(256) void k_final_norm(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                    int H, float eps, uint16_t* __restrict__ y) {
    __shared__ float red[16];
    const int b = blockIdx.x;
    const uint16_t* xr = x + (int64_t)b * H;
    float ss = 0.f;
    for (int k = threadIdx.x; k < H; k += blockDim.x) {
        const float v = bf2f(xr[k]);
        ss = fmaf(v, v, ss);
    }
    ss = block_sum(ss, red);
    const float r = rbf(1.0f / sqrtf(ss / (float)H + eps));
    for (int k = threadIdx.x; k < H; k += blockDim.x) y[(int64_t)b * H + k] = f2bf(rbf(bf2f(xr[k]) * r) * bf2f(w[k]));
}

// logits[b, v] = bf16(sum_k hn[b,k] * E[v,k]) (F.linear in bf16 with fp32 accumulation);
// 16 lanes per vocab row, 16 rows per block; per-block (max, first index) for the greedy argmax.
template <int MB>
__global__ __launch_bounds__(256) void k_lm_head(const uint16_t* __restrict__ E, const uint16_t* __restrict__ hn, int H,
                                                 int V, uint16_t* __restrict__ logits, float* __restrict__ pmax,
                                                 int32_t* __restrict__ pidx, int nblk) {
    extern __shared__ __attribute__((aligned(16))) uint16_t sh[];
    const int b0 = blockIdx.y * MB;
    for (int i = threadIdx.x; i < MB * H / 8; i += blockDim.x) {
        const int m = i / (H / 8), j = i - m * (H / 8);
        reinterpret_cast<uint4*>(sh + m * H)[j] = reinterpret_cast<const uint4*>(hn + (int64_t)(b0 + m) * H)[j];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int lrow = wave * 4 + (lane >> 4);
    const int row = blockIdx.x * 16 + lrow;
    float acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = 0.f;
    if (row < V) {
        const uint16_t* er = E + (int64_t)row * H;
        const int C = H / 8;
        for (int c0 = 0; c0 < C; c0 += 64) {
            uint4 w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + 16 * u + sub;
                w[u] = (c < C) ? ldg_nt(reinterpret_cast<const uint8_t*>(er + 8 * c)) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
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
    }
    __shared__ float s_val[MB][16];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        float v = acc[m];
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 1, 64);
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
        pmax[(int64_t)(b0 + m) * nblk + blockIdx.x] = best;
        pidx[(int64_t)(b0 + m) * nblk + blockIdx.x] = blockIdx.x * 16 + bi;
    }
}

// Greedy sampling (direct_inference_full.py:306-307 argmax; first index on ties) and step advance.
__global__ __launch_bounds__(256) void k_argmax_advance(const float* __restrict__ pmax, const int32_t* __restrict__ pidx,
                                                        int nblk, int32_t* __restrict__ tokens,
                                                        int32_t* __restrict__ positions, int max_seq) {
    __shared__ float sv[256];
    __shared__ int si[256];
    const int b = blockIdx.x;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
        const float v = pmax[(int64_t)b * nblk + i];
        const int id = pidx[(int64_t)b * nblk + i];
        if (v > best || (v == best && id < bi)) { best = v; bi = id; }
    }
    sv[threadIdx.x] = best;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const float v = sv[threadIdx.x + s];
            const int id = si[threadIdx.x + s];
            if (v > sv[threadIdx.x] || (v == sv[threadIdx.x] && id < si[threadIdx.x])) {
                sv[threadIdx.x] = v;
                si[threadIdx.x] = id;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tokens[b] = si[0];
        positions[b] = min(positions[b] + 1, max_seq - 1);
    }
}

}  // namespace wf

// =============================================================================================
// Model runtime
// =============================================================================================
struct wf_model {
    wf_model_desc d;
    int qkv_rows;
    int32_t* tokens = nullptr;     // caller-owned (desc)
    int32_t* positions = nullptr;  // caller-owned (desc)
    uint16_t* logits = nullptr;    // caller-owned (desc)
    uint16_t *k_cache = nullptr, *v_cache = nullptr;  // caller-owned (desc)
    int32_t* seq_lens = nullptr;
    uint16_t *h_a = nullptr, *h_b = nullptr, *qbuf = nullptr, *attn = nullptr, *act = nullptr, *hn = nullptr;
    float* attn_ws = nullptr;
    float* am_val = nullptr;
    int32_t* am_idx = nullptr;
    int lm_blocks = 0;
    hipStream_t cap = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

using namespace wf;

namespace {

int64_t wrow_bytes(int fmt, int K) { return fmt == WF_FMT_TQ ? FmtTQ::row_bytes(K) : FmtI2S::row_bytes(K); }

template <class F, int MODE>
int launch_fused(const LayerArgs& la, int rows_per_tile_out, int B, hipStream_t st) {
    const int img = lds_image_bytes<F>(la.K);
    const int gx = (la.N + kRowsPerBlockFused - 1) / kRowsPerBlockFused;
    (void)rows_per_tile_out;
#define WF_FUSED(MBV)                                                                                              \
    hipLaunchKernelGGL((k_fused_gemv<F, MODE, MBV>), dim3(gx, B / MBV), dim3(256), (size_t)img * MBV, st, la)
    if (B % 8 == 0) WF_FUSED(8);
    else if (B % 4 == 0) WF_FUSED(4);
    else if (B % 2 == 0) WF_FUSED(2);
    else WF_FUSED(1);
#undef WF_FUSED
    return check_launch("fused_gemv");
}

template <int MODE>
int launch_fused_fmt(int fmt, const LayerArgs& la, int B, hipStream_t st) {
    if (fmt == WF_FMT_TQ) return launch_fused<FmtTQ, MODE>(la, 0, B, st);
    return launch_fused<FmtI2S, MODE>(la, 0, B, st);
}

LayerArgs layer_args(const wf_model* m, int l) {
    const wf_model_desc& d = m->d;
    const int B = d.batch, D = d.head_dim, S = d.max_seq;
    const int64_t kvl = (int64_t)B * d.n_kv_heads * S * D;  // cache elements per layer
    LayerArgs la{};
    la.eps = d.eps;
    la.Hq = d.n_heads; la.Hkv = d.n_kv_heads; la.D = D; la.S = S;
    la.positions = m->positions; la.rope_cos = d.rope_cos; la.rope_sin = d.rope_sin;
    la.kc = m->k_cache + l * kvl; la.vc = m->v_cache + l * kvl;
    la.kv_b_stride = (int64_t)d.n_kv_heads * S * D;
    return la;
}

// One op of the decode step (WF_OP_* in include/wf_bitnet.h).
int run_op(wf_model* m, int l, int op, hipStream_t st) {
    const wf_model_desc& d = m->d;
    const int B = d.batch, H = d.hidden, I = d.inter, D = d.head_dim, S = d.max_seq;
    const float* wsh = d.wscale + 7 * l;  // host copy made at create time
    LayerArgs la = layer_args(m, l);
    switch (op) {
        case WF_OP_EMBED:
            hipLaunchKernelGGL(k_embed, dim3(B), dim3(256), 0, st, d.embed, m->tokens, H, d.vocab, m->h_a, m->positions,
                               m->seq_lens);
            break;
        case WF_OP_QKV:  // rms_norm(h_a) -> q (RoPE) -> qbuf ; k (RoPE), v -> cache[pos]
            la.x = m->h_a; la.x_stride = H; la.norm_w = d.ln_in + (int64_t)l * H;
            la.w = d.w_qkv + (int64_t)l * m->qkv_rows * wrow_bytes(d.wfmt, H);
            la.N = m->qkv_rows; la.K = H; la.ws0 = wsh[0]; la.ws1 = wsh[1]; la.ws2 = wsh[2];
            la.out = m->qbuf; la.out_stride = (int64_t)d.n_heads * D;
            return launch_fused_fmt<MODE_QKV>(d.wfmt, la, B, st);
        case WF_OP_ATTN:
            return decode_attention_impl(m->qbuf, WF_BF16, (int64_t)d.n_heads * D, D, la.kc, la.vc, WF_BF16,
                                         la.kv_b_stride, (int64_t)S * D, D, 1.f, 1.f, B, d.n_heads, d.n_kv_heads, D,
                                         S, m->seq_lens, 1.0f / sqrtf((float)D), m->attn, WF_BF16,
                                         (int64_t)d.n_heads * D, D, m->attn_ws, st);
        case WF_OP_O:  // h_b = h_a + o_proj(rms_norm(attn))
            la.x = m->attn; la.x_stride = (int64_t)d.n_heads * D; la.norm_w = d.attn_sub + (int64_t)l * H;
            la.w = d.w_o + (int64_t)l * H * wrow_bytes(d.wfmt, H); la.N = H; la.K = H; la.ws0 = wsh[3];
            la.resid = m->h_a; la.out = m->h_b; la.out_stride = H;
            return launch_fused_fmt<MODE_O>(d.wfmt, la, B, st);
        case WF_OP_GATE_UP:  // act = relu(gate)^2 * up of rms_norm(h_b)
            la.x = m->h_b; la.x_stride = H; la.norm_w = d.ln_post + (int64_t)l * H;
            la.w = d.w_gu + (int64_t)l * 2 * I * wrow_bytes(d.wfmt, H); la.N = 2 * I; la.K = H;
            la.ws0 = wsh[4]; la.ws1 = wsh[5]; la.out = m->act; la.out_stride = I;
            return launch_fused_fmt<MODE_GU>(d.wfmt, la, B, st);
        case WF_OP_DOWN:  // h_a = h_b + down(rms_norm(act))
            la.x = m->act; la.x_stride = I; la.norm_w = d.ffn_sub + (int64_t)l * I;
            la.w = d.w_d + (int64_t)l * H * wrow_bytes(d.wfmt, I); la.N = H; la.K = I; la.ws0 = wsh[6];
            la.resid = m->h_b; la.out = m->h_a; la.out_stride = H;
            return launch_fused_fmt<MODE_DN>(d.wfmt, la, B, st);
        case WF_OP_FINAL_NORM:
            hipLaunchKernelGGL(k_final_norm, dim3(B), dim3(256), 0, st, m->h_a, d.final_norm, H, d.eps, m->hn);
            break;
        case WF_OP_LM_HEAD: {
            const size_t sh = (size_t)H * 2;
#define WF_LM(MBV)                                                                                              \
    hipLaunchKernelGGL((k_lm_head<MBV>), dim3(m->lm_blocks, B / MBV), dim3(256), sh * MBV, st, d.embed, m->hn, \
                       H, d.vocab, m->logits, m->am_val, m->am_idx, m->lm_blocks)
            if (B % 4 == 0) WF_LM(4);
            else if (B % 2 == 0) WF_LM(2);
            else WF_LM(1);
#undef WF_LM
            break;
        }
        case WF_OP_ARGMAX:
            hipLaunchKernelGGL(k_argmax_advance, dim3(B), dim3(256), 0, st, m->am_val, m->am_idx, m->lm_blocks,
                               m->tokens, m->positions, S);
            break;
        default:
            set_error("model op %d unknown", op);
            return WF_EINVAL;
    }
    return check_launch("model_op");
}

int model_step(wf_model* m, hipStream_t st) {
    int rc = run_op(m, 0, WF_OP_EMBED, st);
    for (int l = 0; l < m->d.layers && !rc; ++l)
        for (int op = WF_OP_QKV; op <= WF_OP_DOWN && !rc; ++op) rc = run_op(m, l, op, st);
    for (int op = WF_OP_FINAL_NORM; op <= WF_OP_ARGMAX && !rc; ++op) rc = run_op(m, 0, op, st);
    return rc;
}

}  // namespace

extern "C" {

int wf_model_create(const wf_model_desc* dp, wf_model** out) {
    WF_REQUIRE(dp && out, "model_create: null argument");
    const wf_model_desc& d = *dp;
    WF_REQUIRE(d.head_dim == 128, "model_create: head_dim must be 128 (got %d)", d.head_dim);
    WF_REQUIRE(d.hidden == d.n_heads * d.head_dim, "model_create: hidden != n_heads * head_dim");
    WF_REQUIRE(d.n_kv_heads > 0 && d.n_heads % d.n_kv_heads == 0 && d.n_heads / d.n_kv_heads <= 8, "model_create: bad GQA");
    WF_REQUIRE(d.hidden % 128 == 0 && d.inter % 128 == 0 && d.inter % 8 == 0, "model_create: hidden/inter must be multiples of 128");
    WF_REQUIRE(d.hidden <= 8192 && d.inter <= 8192, "model_create: hidden/inter > 8192 not supported");
    WF_REQUIRE(d.batch >= 1 && d.max_seq >= 1 && d.vocab >= 1 && d.layers >= 1, "model_create: bad sizes");
    WF_REQUIRE(d.wfmt == WF_FMT_I2S || d.wfmt == WF_FMT_TQ, "model_create: bad weight format");
    WF_REQUIRE(d.embed && d.final_norm && d.rope_cos && d.rope_sin && d.ln_in && d.ln_post && d.attn_sub && d.ffn_sub &&
                   d.w_qkv && d.w_o && d.w_gu && d.w_d && d.wscale,
               "model_create: null weight pointer");
    WF_REQUIRE(d.tokens && d.positions && d.logits && d.k_cache && d.v_cache, "model_create: null state pointer");
    wf_model* m = new (std::nothrow) wf_model();
    WF_REQUIRE(m, "model_create: out of host memory");
    m->d = d;
    // keep a host copy of the scales (read while recording launches)
    float* ws = new float[7 * d.layers];
    for (int i = 0; i < 7 * d.layers; ++i) ws[i] = d.wscale[i];
    m->d.wscale = ws;
    m->qkv_rows = (d.n_heads + 2 * d.n_kv_heads) * d.head_dim;
    const int B = d.batch;
    m->lm_blocks = (d.vocab + 15) / 16;
    auto fail = [&](hipError_t e) {
        set_error("model_create: %s", hipGetErrorString(e));
        wf_model_destroy(m);
        return WF_EHIP;
    };
    hipError_t e;
#define WF_ALLOC(ptr, bytes) \
    if ((e = hipMalloc((void**)&(ptr), (bytes))) != hipSuccess) return fail(e)
    m->tokens = d.tokens;
    m->positions = d.positions;
    m->logits = d.logits;
    m->k_cache = d.k_cache;
    m->v_cache = d.v_cache;
    WF_ALLOC(m->seq_lens, sizeof(int32_t) * B);
    WF_ALLOC(m->h_a, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->h_b, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->qbuf, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->attn, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->hn, 2 * (size_t)B * d.hidden);
    WF_ALLOC(m->act, 2 * (size_t)B * d.inter);
    WF_ALLOC(m->attn_ws, (size_t)wf_decode_attention_ws_bytes(B, d.n_heads, d.head_dim, d.max_seq));
    WF_ALLOC(m->am_val, sizeof(float) * B * m->lm_blocks);
    WF_ALLOC(m->am_idx, sizeof(int32_t) * B * m->lm_blocks);
#undef WF_ALLOC
    // attention tickets must start at zero (every launch re-arms them)
    if ((e = hipMemset(m->attn_ws, 0, (size_t)wf_decode_attention_ws_bytes(B, d.n_heads, d.head_dim, d.max_seq))) !=
        hipSuccess)
        return fail(e);
    if ((e = hipStreamCreateWithFlags(&m->cap, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    *out = m;
    return WF_OK;
}

int wf_model_destroy(wf_model* m) {
    if (!m) return WF_OK;
    if (m->exec) (void)hipGraphExecDestroy(m->exec);
    if (m->graph) (void)hipGraphDestroy(m->graph);
    if (m->cap) (void)hipStreamDestroy(m->cap);
    void* ptrs[] = {m->seq_lens, m->h_a, m->h_b, m->qbuf, m->attn, m->hn, m->act, m->attn_ws, m->am_val, m->am_idx};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete[] m->d.wscale;
    delete m;
    return WF_OK;
}

int wf_model_step(wf_model* m, void* stream) {
    WF_REQUIRE(m, "model_step: null model");
    return model_step(m, as_stream(stream));
}

int wf_model_launch_op(wf_model* m, int layer, int op, void* stream) {
    WF_REQUIRE(m, "model_launch_op: null model");
    WF_REQUIRE(layer >= 0 && layer < m->d.layers, "model_launch_op: layer %d out of range", layer);
    return run_op(m, layer, op, as_stream(stream));
}

int wf_model_graph_launch(wf_model* m, void* stream) {
    WF_REQUIRE(m, "model_graph_launch: null model");
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
