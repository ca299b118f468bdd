// wf_attn.hip -- KV cache data movement and split-K decode attention for gfx950.
//
// Decode attention reads every cached K and V row of a sequence once: HBM-bound, algorithmic
// bytes per call = sum_b 2 * Hkv * S_b * D * sizeof(kv) (+ q and out). Each 16-lane group
// (D = 128) owns one key position at a time and every lane holds 8 consecutive elements of the
// head dimension, so one wave-instruction reads 4 contiguous 256-byte K rows (coalesced 1 KiB for
// the [.., S, D] layout). The G query heads of a GQA group share every K/V load.
#include <hip/hip_runtime.h>

#include "wf_common.h"
#include "wf_device.h"

namespace wf {

constexpr int kAttnThreads = 256;
constexpr int kAttnMinSplit = 64;   // keys per split (lower bound)
constexpr int kAttnTargetBlocks = 512;

static inline int attn_splits(int B, int Hkv, int S) {
    int target = (kAttnTargetBlocks + B * Hkv - 1) / (B * Hkv);
    if (target < 1) target = 1;
    int T = (S + target - 1) / target;
    if (T < kAttnMinSplit) T = kAttnMinSplit;
    return (S + T - 1) / T;
}
static inline int attn_split_len(int B, int Hkv, int S) {
    const int ns = attn_splits(B, Hkv, S);
    return (S + ns - 1) / ns;
}

// Load 8 consecutive KV elements as f32.
template <int KVDT>
__device__ __forceinline__ void load8(const void* base, int64_t off, float scale, float (&x)[8]) {
    if constexpr (KVDT == DT_BF16 || KVDT == DT_F16) {
        const uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + off);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if constexpr (KVDT == DT_BF16) {
                x[2 * i] = __uint_as_float(w[i] << 16);
                x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
            } else {
                x[2 * i] = h2f((uint16_t)(w[i] & 0xffffu));
                x[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
            }
        }
    } else if constexpr (KVDT == DT_F32) {
        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off);
        const float4 a = p[0], b = p[1];
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    } else {  // int8 cache: kv_cache.py:220-228 -> rbf16(float(q) * scale)
        const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const int8_t*>(base) + off);
        const uint32_t w[2] = {r.x, r.y};
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = rbf((float)(int8_t)(w[i >> 2] >> (8 * (i & 3))) * scale);
    }
}

// One block = one (sequence b, kv head g, split s). Partial results (m, l, o[D]) per query head
// go to the workspace; k_attn_combine merges the splits.
template <int D, int G, int KVDT>
__global__ __launch_bounds__(kAttnThreads) void k_attn_split(
    const void* __restrict__ q, int qdt, int64_t q_sb, int64_t q_sh, const void* __restrict__ K,
    const void* __restrict__ V, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int Hq,
    int Hkv, int S, const int32_t* __restrict__ seq_lens, float sm_scale, int NS, int T, float* __restrict__ ws) {
    constexpr int LP = D / 8;        // lanes per key position
    constexpr int PW = 64 / LP;      // positions per wave-instruction
    constexpr int NW = kAttnThreads / 64;
    const int s = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
    const int grp = Hq / Hkv;        // runtime group size (<= G)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int pg = lane / LP, li = lane % LP;
    const int Sb = seq_lens ? min(seq_lens[b], S) : S;
    const int t0 = s * T, t1 = min(Sb, t0 + T);

    float qv[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
#pragma unroll
        for (int j = 0; j < 8; ++j) qv[h][j] = 0.f;
        if (h < grp) {
            const int64_t qo = b * q_sb + (int64_t)(g * grp + h) * q_sh + li * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) qv[h][j] = load_as_f32(q, qo + j, qdt);
        }
    }
    float m[G], l[G], o[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        m[h] = -INFINITY;
        l[h] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[h][j] = 0.f;
    }
    const int64_t kvb = b * kv_sb + g * kv_sh + li * 8;
    for (int t = t0 + wave * PW + pg; t < t1; t += NW * PW) {
        float kx[8], vx[8];
        load8<KVDT>(K, kvb + t * kv_st, k_scale, kx);
        load8<KVDT>(V, kvb + t * kv_st, v_scale, vx);
        float sc[G];
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float d = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) d = fmaf(qv[h][j], kx[j], d);
#pragma unroll
            for (int off = LP / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            sc[h] = d * sm_scale;
        }
#pragma unroll
        for (int h = 0; h < G; ++h) {
            if (h < grp) {
                const float mn = fmaxf(m[h], sc[h]);
                const float al = __expf(m[h] - mn);
                const float p = __expf(sc[h] - mn);
                l[h] = l[h] * al + p;
#pragma unroll
                for (int j = 0; j < 8; ++j) o[h][j] = fmaf(p, vx[j], o[h][j] * al);
                m[h] = mn;
            }
        }
    }
    // merge the PW position groups of the wave (same li, different pg)
#pragma unroll
    for (int off = LP; off < 64; off <<= 1) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const float mo = __shfl_xor(m[h], off, 64), lo = __shfl_xor(l[h], off, 64);
            const float mn = fmaxf(m[h], mo);
            const float a = (m[h] == -INFINITY) ? 0.f : __expf(m[h] - mn);
            const float c = (mo == -INFINITY) ? 0.f : __expf(mo - mn);
            l[h] = l[h] * a + lo * c;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float oo = __shfl_xor(o[h][j], off, 64);
                o[h][j] = o[h][j] * a + oo * c;
            }
            m[h] = mn;
        }
    }
    // merge the NW waves through LDS (lanes with pg == 0 hold the wave's result)
    __shared__ float sm_m[NW][G], sm_l[NW][G];
    __shared__ float sm_o[NW][G][D];
    if (pg == 0) {
#pragma unroll
        for (int h = 0; h < G; ++h) {
            if (li == 0) { sm_m[wave][h] = m[h]; sm_l[wave][h] = l[h]; }
#pragma unroll
            for (int j = 0; j < 8; ++j) sm_o[wave][h][li * 8 + j] = o[h][j];
        }
    }
    __syncthreads();
    // thread -> (h, d): G*D outputs over 256 threads
    for (int idx = threadIdx.x; idx < grp * D; idx += kAttnThreads) {
        const int h = idx / D, d = idx - h * D;
        float mx = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; ++w) mx = fmaxf(mx, sm_m[w][h]);
        float ls = 0.f, os = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float a = (sm_m[w][h] == -INFINITY) ? 0.f : __expf(sm_m[w][h] - mx);
            ls += sm_l[w][h] * a;
            os += sm_o[w][h][d] * a;
        }
        const int hq = g * grp + h;
        float* po = ws + (((int64_t)b * Hq + hq) * NS + s) * (D + 2);
        po[2 + d] = os;
        if (d == 0) { po[0] = mx; po[1] = ls; }
    }
}

// Merge NS split partials per (b, query head) and write the output row.
__global__ void k_attn_combine(const float* __restrict__ ws, int Hq, int D, int NS, void* __restrict__ out, int odt,
                               int64_t o_sb, int64_t o_sh) {
    const int h = blockIdx.x, b = blockIdx.y;
    const float* p = ws + ((int64_t)b * Hq + h) * NS * (D + 2);
    float mx = -INFINITY;
    for (int s = 0; s < NS; ++s) mx = fmaxf(mx, p[s * (D + 2)]);
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        float ls = 0.f, os = 0.f;
        for (int s = 0; s < NS; ++s) {
            const float ms = p[s * (D + 2)];
            const float a = (ms == -INFINITY) ? 0.f : __expf(ms - mx);
            ls += p[s * (D + 2) + 1] * a;
            os += p[s * (D + 2) + 2 + d] * a;
        }
        store_from_f32(out, b * o_sb + (int64_t)h * o_sh + d, odt, os / ls);
    }
}

// ---------------------------------------------------------------------------------------------
// Paged KV scatter / gather (sgl_kernel.kvcache.KVCacheManager; tests/test_kv_cache_cpp.py:20-127)
// pool [P][L][2][H*D] elements; one block per (token, K|V), 4-byte copies.
// ---------------------------------------------------------------------------------------------
__global__ void k_kv_page_copy(uint8_t* __restrict__ pool, const uint8_t* __restrict__ src_k,
                               const uint8_t* __restrict__ src_v, uint8_t* __restrict__ dst_k,
                               uint8_t* __restrict__ dst_v, const int32_t* __restrict__ pages, int P, int L,
                               int64_t row_bytes, int layer, int scatter, int32_t* __restrict__ bad) {
    const int t = blockIdx.x, kv = blockIdx.y;
    const int page = pages[t];
    if (page < 0 || page >= P) {
        if (threadIdx.x == 0 && kv == 0 && bad) atomicAdd(bad, 1);
        return;
    }
    uint8_t* slot = pool + (((int64_t)page * L + layer) * 2 + kv) * row_bytes;
    const int64_t n4 = row_bytes / 4;
    if (scatter) {
        const uint32_t* s = reinterpret_cast<const uint32_t*>((kv ? src_v : src_k) + (int64_t)t * row_bytes);
        for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) reinterpret_cast<uint32_t*>(slot)[i] = s[i];
    } else {
        uint32_t* d = reinterpret_cast<uint32_t*>((kv ? dst_v : dst_k) + (int64_t)t * row_bytes);
        for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) d[i] = reinterpret_cast<const uint32_t*>(slot)[i];
    }
}

template <int D, int G, int KVDT>
static void launch_attn(dim3 grid, hipStream_t st, const void* q, int qdt, int64_t q_sb, int64_t q_sh, const void* k,
                        const void* v, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float ks, float vs, int Hq, int Hkv,
                        int S, const int32_t* sl, float sm, int NS, int T, float* ws) {
    hipLaunchKernelGGL((k_attn_split<D, G, KVDT>), grid, dim3(kAttnThreads), 0, st, q, qdt, q_sb, q_sh, k, v, kv_sb,
                       kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws);
}

template <int D, int G>
static int dispatch_kvdt(int kvdt, dim3 grid, hipStream_t st, const void* q, int qdt, int64_t q_sb, int64_t q_sh,
                         const void* k, const void* v, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float ks, float vs,
                         int Hq, int Hkv, int S, const int32_t* sl, float sm, int NS, int T, float* ws) {
    switch (kvdt) {
        case DT_BF16: launch_attn<D, G, DT_BF16>(grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws); return 0;
        case DT_F16: launch_attn<D, G, DT_F16>(grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws); return 0;
        case DT_F32: launch_attn<D, G, DT_F32>(grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws); return 0;
        case DT_I8: launch_attn<D, G, DT_I8>(grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws); return 0;
    }
    return 1;
}

template <int D>
static int dispatch_g(int grp, int kvdt, dim3 grid, hipStream_t st, const void* q, int qdt, int64_t q_sb, int64_t q_sh,
                      const void* k, const void* v, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float ks, float vs,
                      int Hq, int Hkv, int S, const int32_t* sl, float sm, int NS, int T, float* ws) {
    if (grp == 1) return dispatch_kvdt<D, 1>(kvdt, grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws);
    if (grp == 2) return dispatch_kvdt<D, 2>(kvdt, grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws);
    if (grp <= 4) return dispatch_kvdt<D, 4>(kvdt, grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws);
    if (grp <= 8) return dispatch_kvdt<D, 8>(kvdt, grid, st, q, qdt, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, ks, vs, Hq, Hkv, S, sl, sm, NS, T, ws);
    return 1;
}

int decode_attention_impl(const void* q, int q_dtype, int64_t q_sb, int64_t q_sh, const void* k, const void* v,
                          int kv_dtype, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int B,
                          int Hq, int Hkv, int D, int S, const int32_t* seq_lens, float sm_scale, void* out,
                          int out_dtype, int64_t o_sb, int64_t o_sh, void* ws, hipStream_t st) {
    const int NS = attn_splits(B, Hkv, S), T = attn_split_len(B, Hkv, S);
    const dim3 grid(NS, Hkv, B);
    const int grp = Hq / Hkv;
    float* wsf = reinterpret_cast<float*>(ws);
    int bad = 1;
    switch (D) {
        case 16: bad = dispatch_g<16>(grp, kv_dtype, grid, st, q, q_dtype, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, k_scale, v_scale, Hq, Hkv, S, seq_lens, sm_scale, NS, T, wsf); break;
        case 32: bad = dispatch_g<32>(grp, kv_dtype, grid, st, q, q_dtype, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, k_scale, v_scale, Hq, Hkv, S, seq_lens, sm_scale, NS, T, wsf); break;
        case 64: bad = dispatch_g<64>(grp, kv_dtype, grid, st, q, q_dtype, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, k_scale, v_scale, Hq, Hkv, S, seq_lens, sm_scale, NS, T, wsf); break;
        case 128: bad = dispatch_g<128>(grp, kv_dtype, grid, st, q, q_dtype, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, k_scale, v_scale, Hq, Hkv, S, seq_lens, sm_scale, NS, T, wsf); break;
    }
    WF_REQUIRE(!bad, "decode_attention: unsupported D=%d / group=%d / kv dtype=%d", D, grp, kv_dtype);
    hipLaunchKernelGGL(k_attn_combine, dim3(Hq, B), dim3(D < 64 ? 64 : D), 0, st, wsf, Hq, D, NS, out, out_dtype, o_sb,
                       o_sh);
    return check_launch("decode_attention");
}

}  // namespace wf

using namespace wf;

extern "C" {

int64_t wf_decode_attention_ws_bytes(int B, int Hq, int D, int S) {
    // worst case over Hkv >= 1: the split count grows as Hkv shrinks
    return (int64_t)B * Hq * attn_splits(B, 1, S) * (D + 2) * (int64_t)sizeof(float);
}

int wf_decode_attention(const void* q, int q_dtype, int64_t q_sb, int64_t q_sh, const void* k, const void* v,
                        int kv_dtype, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int B,
                        int Hq, int Hkv, int D, int S, const int32_t* seq_lens, float sm_scale, void* out,
                        int out_dtype, int64_t o_sb, int64_t o_sh, void* ws, void* stream) {
    WF_REQUIRE(q && k && v && out && ws, "decode_attention: null pointer");
    WF_REQUIRE(B > 0 && Hq > 0 && Hkv > 0 && Hq % Hkv == 0 && Hq / Hkv <= 8, "decode_attention: bad heads Hq=%d Hkv=%d", Hq, Hkv);
    WF_REQUIRE(S > 0, "decode_attention: S must be > 0");
    WF_REQUIRE(q_dtype == WF_F32 || q_dtype == WF_BF16 || q_dtype == WF_F16, "decode_attention: bad q dtype");
    WF_REQUIRE(out_dtype == WF_F32 || out_dtype == WF_BF16 || out_dtype == WF_F16, "decode_attention: bad out dtype");
    WF_REQUIRE(kv_st % 8 == 0 && kv_sh % 8 == 0 && kv_sb % 8 == 0, "decode_attention: KV strides must be multiples of 8");
    WF_REQUIRE(aligned16(k) && aligned16(v), "decode_attention: K/V must be 16-byte aligned");
    return decode_attention_impl(q, q_dtype, q_sb, q_sh, k, v, kv_dtype, kv_sb, kv_sh, kv_st, k_scale, v_scale, B, Hq,
                                 Hkv, D, S, seq_lens, sm_scale, out, out_dtype, o_sb, o_sh, ws, as_stream(stream));
}

static int kv_page_common(uint8_t* pool, int elem_bytes, int max_pages, int L, int H, int D, const void* k,
                          const void* v, void* ko, void* vo, const int32_t* pages, int T, int layer, int32_t* bad,
                          int scatter, void* stream) {
    WF_REQUIRE(pool && pages && T >= 0 && max_pages > 0 && L > 0 && H > 0 && D > 0, "kv_page: bad arguments");
    WF_REQUIRE(layer >= 0 && layer < L, "kv_page: layer %d out of range [0, %d)", layer, L);
    WF_REQUIRE(elem_bytes == 1 || elem_bytes == 2 || elem_bytes == 4, "kv_page: elem_bytes must be 1, 2 or 4");
    const int64_t row_bytes = (int64_t)H * D * elem_bytes;
    WF_REQUIRE(row_bytes % 4 == 0, "kv_page: H*D*elem_bytes must be a multiple of 4");
    if (T == 0) return WF_OK;
    hipLaunchKernelGGL(k_kv_page_copy, dim3(T, 2), dim3(256), 0, as_stream(stream), pool, (const uint8_t*)k,
                       (const uint8_t*)v, (uint8_t*)ko, (uint8_t*)vo, pages, max_pages, L, row_bytes, layer, scatter,
                       bad);
    return check_launch("kv_page_copy");
}

int wf_kv_scatter(void* pool, int elem_bytes, int max_pages, int L, int H, int D, const void* k, const void* v,
                  const int32_t* pages, int T, int layer, int32_t* bad, void* stream) {
    WF_REQUIRE(k && v, "kv_scatter: null k/v");
    return kv_page_common((uint8_t*)pool, elem_bytes, max_pages, L, H, D, k, v, nullptr, nullptr, pages, T, layer, bad,
                          1, stream);
}

int wf_kv_gather(const void* pool, int elem_bytes, int max_pages, int L, int H, int D, void* k_out, void* v_out,
                 const int32_t* pages, int T, int layer, int32_t* bad, void* stream) {
    WF_REQUIRE(k_out && v_out, "kv_gather: null outputs");
    return kv_page_common((uint8_t*)pool, elem_bytes, max_pages, L, H, D, nullptr, nullptr, k_out, v_out, pages, T,
                          layer, bad, 0, stream);
}

}  // extern "C"
