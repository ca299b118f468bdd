// wf_attn.hip -- KV cache data movement and split-K decode attention for gfx950.
//
// Decode attention reads every cached K and V row of a sequence once: HBM-bound, algorithmic
// bytes per call = sum_b 2 * Hkv * S_b * D * sizeof(kv) (+ q and out). Each 16-lane group
// (D = 128) owns one key position at a time and every lane holds 8 consecutive elements of the
// head dimension, so one wave-instruction reads 4 contiguous 256-byte K rows (coalesced 1 KiB for
// the [.., S, D] layout). The G query heads of a GQA group share every K/V load.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>

#include "wf_common.h"
#include "wf_device.h"
#include "wf_norm.h"
#include "wf_mfma.h"

namespace wf {

constexpr int kAttnThreads = 256;
constexpr int kAttnU = 4;  // key positions per lane group per split (all loads issued up front)
constexpr int kAttnMaxSplits = 256;  // splits per sequence (S <= 256 * split length)

// keys per split: kAttnU positions x (256 / (D/8)) lane groups  (D = 128 -> 64)
static inline int attn_split_len(int D) { return kAttnU * (kAttnThreads / (D / 8)); }
static inline int attn_splits(int D, int S) { return (S + attn_split_len(D) - 1) / attn_split_len(D); }
static inline int64_t attn_cnt_bytes(int B, int Hkv) { return (((int64_t)B * Hkv * 4) + 255) / 256 * 256; }
static inline int64_t attn_rec_floats(int D) { return D + 4; }

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

// Raw 16-byte KV load (decoded later, so every load of the split is in flight at once).
template <int KVDT>
struct KVRaw {
    uint4 a, b;  // b used by f32 only
    __device__ __forceinline__ void load(const void* base, int64_t off) {
        if constexpr (KVDT == DT_F32) {
            const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(base) + off);
            a = p[0];
            b = p[1];
        } else if constexpr (KVDT == DT_I8) {
            const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const int8_t*>(base) + off);
            a = make_uint4(r.x, r.y, 0, 0);
        } else {
            a = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + off);
        }
    }
    __device__ __forceinline__ void decode(float scale, float (&x)[8]) const {
        const uint32_t w[4] = {a.x, a.y, a.z, a.w};
        if constexpr (KVDT == DT_BF16) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { x[2 * i] = __uint_as_float(w[i] << 16); x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
        } else if constexpr (KVDT == DT_F16) {
#pragma unroll
            for (int i = 0; i < 4; ++i) { x[2 * i] = h2f((uint16_t)(w[i] & 0xffffu)); x[2 * i + 1] = h2f((uint16_t)(w[i] >> 16)); }
        } else if constexpr (KVDT == DT_F32) {
            x[0] = __uint_as_float(a.x); x[1] = __uint_as_float(a.y); x[2] = __uint_as_float(a.z); x[3] = __uint_as_float(a.w);
            x[4] = __uint_as_float(b.x); x[5] = __uint_as_float(b.y); x[6] = __uint_as_float(b.z); x[7] = __uint_as_float(b.w);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = rbf((float)(int8_t)(w[i >> 2] >> (8 * (i & 3))) * scale);
        }
    }
};

// store 4 consecutive outputs
__device__ __forceinline__ void store_out4(void* out, int64_t off, int odt, const float (&v)[4]) {
    if (odt == DT_BF16) {
        const uint2 pk = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(out) + off) = pk;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) store_from_f32(out, off + j, odt, v[j]);
    }
}

// One block = one (sequence b, kv head g, split s of T keys). Lane group `gid` (D/8 lanes, 8 head
// dims per lane) owns keys t0 + gid + NG*u, u < kAttnU, loads all of them first, then does a local
// softmax; groups merge by shuffles and through LDS. With NS > 1 the block publishes (m, l, o)
// partials write-through (sc1) and bumps a per-(b, g) ticket; the last arriver merges the splits
// and writes the output (MI355X_MICROARCH.md "Valid forms" row 1: sc1 stores, vmcnt(0) in every
// storing wave, a barrier, one agent-scope atomic add; sc1 loads in the last arriver). Its merge
// issues every (m, l) and o load of its share of the splits at once (one round trip), folds them
// with an online max, and combines the thread subsets through LDS. The last arriver also re-arms
// the ticket for the next launch.
template <int D, int G, int KVDT, int U = kAttnU>
__global__ __launch_bounds__(kAttnThreads) void k_attn_split(
    const void* __restrict__ q, int qdt, int64_t q_sb, int64_t q_sh, const void* __restrict__ K,
    const void* __restrict__ V, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int Hq,
    int Hkv, int S, const int32_t* __restrict__ seq_lens, float sm_scale, int NS, unsigned* __restrict__ cnt,
    float* __restrict__ part, void* __restrict__ out, int odt, int64_t o_sb, int64_t o_sh) {
    constexpr int LP = D / 8;                // lanes per key position
    constexpr int NG = kAttnThreads / LP;    // lane groups per block
    constexpr int T = U * NG;
    const int s = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
    const int grp = Hq / Hkv;
    const int gid = threadIdx.x / LP, li = threadIdx.x % LP;
    const int Sb = seq_lens ? min(seq_lens[b], S) : S;
    const int t0 = s * T;
    const int nact = (Sb + T - 1) / T;       // splits that hold keys for this sequence
    WF_STAMP(0);

    __shared__ float sm_m[NG][G], sm_l[NG][G];
    __shared__ __attribute__((aligned(16))) float sm_o[NG][G][D];
    __shared__ int sh_last;

    float m[G], l[G], o[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
        m[h] = -INFINITY;
        l[h] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[h][j] = 0.f;
    }
    if (t0 < Sb) {
        const int64_t kvb = b * kv_sb + g * kv_sh + li * 8;
        float qv[G][8];
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const int64_t qo = b * q_sb + (int64_t)(g * grp + min(h, grp - 1)) * q_sh + li * 8;
            if (qdt == DT_BF16) {
                const uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(q) + qo);
                const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) { qv[h][2 * i] = __uint_as_float(w[i] << 16); qv[h][2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) qv[h][j] = load_as_f32(q, qo + j, qdt);
            }
        }
        KVRaw<KVDT> kr[U], vr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = min(t0 + gid + NG * u, Sb - 1);
            kr[u].load(K, kvb + t * kv_st);
            vr[u].load(V, kvb + t * kv_st);
        }
        float sc[U][G];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float kx[8];
            kr[u].decode(k_scale, kx);
            const bool valid = t0 + gid + NG * u < Sb;
#pragma unroll
            for (int h = 0; h < G; ++h) {
                float d = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) d = fmaf(qv[h][j], kx[j], d);
                d = group_reduce<LP>(d, OpAdd{});
                sc[u][h] = valid ? d * sm_scale : -INFINITY;
            }
        }
        WF_STAMP(1);
#pragma unroll
        for (int h = 0; h < G; ++h) {
            float mx = sc[0][h];
#pragma unroll
            for (int u = 1; u < U; ++u) mx = fmaxf(mx, sc[u][h]);
            m[h] = mx;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float vx[8];
            vr[u].decode(v_scale, vx);
#pragma unroll
            for (int h = 0; h < G; ++h) {
                const float p = (sc[u][h] == -INFINITY) ? 0.f : __expf(sc[u][h] - m[h]);
                l[h] += p;
#pragma unroll
                for (int j = 0; j < 8; ++j) o[h][j] = fmaf(p, vx[j], o[h][j]);
            }
        }
    }
    // every lane group parks (m, l, o) in LDS; the block merges them per (h, d) below
    if (li == 0) {
#pragma unroll
        for (int h = 0; h < G; ++h) { sm_m[gid][h] = m[h]; sm_l[gid][h] = l[h]; }
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
        *reinterpret_cast<float4*>(&sm_o[gid][h][li * 8]) = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
        *reinterpret_cast<float4*>(&sm_o[gid][h][li * 8 + 4]) = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
    }
    __syncthreads();
    WF_STAMP(2);
    // block result per (h, 4 consecutive d)
    constexpr int D4 = D / 4;
    const int rec = D + 4;  // partial record: m, l, 0, 0, o[D]
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(part, (short)0, 0x7fffffff, 0x00020000);
    for (int idx = threadIdx.x; idx < grp * D4; idx += kAttnThreads) {
        const int h = idx / D4, d = (idx - h * D4) * 4;
        float mx = -INFINITY;
#pragma unroll
        for (int w = 0; w < NG; ++w) mx = fmaxf(mx, sm_m[w][h]);
        float ls = 0.f;
        float os[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < NG; ++w) {
            const float a = (sm_m[w][h] == -INFINITY) ? 0.f : __expf(sm_m[w][h] - mx);
            ls += sm_l[w][h] * a;
            const float4 ov = *reinterpret_cast<const float4*>(&sm_o[w][h][d]);
            os[0] += ov.x * a; os[1] += ov.y * a; os[2] += ov.z * a; os[3] += ov.w * a;
        }
        const int hq = g * grp + h;
        if (NS == 1) {
            const float ov[4] = {os[0] / ls, os[1] / ls, os[2] / ls, os[3] / ls};
            store_out4(out, b * o_sb + (int64_t)hq * o_sh + d, odt, ov);
        } else if (t0 < Sb) {
            const int off = (int)((((int64_t)b * Hq + hq) * NS + s) * rec) * 4;  // bytes
            const float4 ov = make_float4(os[0], os[1], os[2], os[3]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ov), rs, off + 16 + 4 * d, 0, 16 /*sc1*/);
            if (d == 0)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_float4(mx, ls, 0.f, 0.f)), rs,
                                                       off, 0, 16);
        }
    }
    if (NS == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(cnt + b * Hkv + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_last = (old == (unsigned)NS - 1u);
    }
    __syncthreads();
    WF_STAMP(3);
    if (!sh_last) return;
    // ---- last arriver: merge the active splits of every query head of this kv group ----
    const int na = min(nact, NS);  // <= kAttnMaxSplits (host check)
    const int nout = grp * D4;     // float4 outputs of this (b, g)
    const int nsub = max(1, kAttnThreads / nout);  // thread subsets over the splits
    constexpr int kMU = 8;         // splits in flight per thread per round
    float M = -INFINITY, Lsum = 0.f, O4[4] = {0.f, 0.f, 0.f, 0.f};
    const int oi = threadIdx.x % nout, sb = threadIdx.x / nout;
    if (sb < nsub) {
        const int h = oi / D4, d = (oi - h * D4) * 4;
        const int64_t rbase = (((int64_t)b * Hq + g * grp + h) * NS) * rec;
        for (int sp0 = sb; sp0 < na; sp0 += kMU * nsub) {
            float4 ml[kMU], ov[kMU];
#pragma unroll
            for (int u = 0; u < kMU; ++u) {  // every load of the round in flight at once
                const int sp = min(sp0 + u * nsub, na - 1);
                const int off = (int)((rbase + (int64_t)sp * rec) * 4);
                ml[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
                ov[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 + 4 * d, 0, 16));
            }
#pragma unroll
            for (int u = 0; u < kMU; ++u) {
                if (sp0 + u * nsub < na) {
                    const float nm = fmaxf(M, ml[u].x);
                    const float a = __expf(M - nm), c = __expf(ml[u].x - nm);  // M = -inf -> a = 0
                    Lsum = Lsum * a + ml[u].y * c;
                    O4[0] = O4[0] * a + ov[u].x * c;
                    O4[1] = O4[1] * a + ov[u].y * c;
                    O4[2] = O4[2] * a + ov[u].z * c;
                    O4[3] = O4[3] * a + ov[u].w * c;
                    M = nm;
                }
            }
        }
    }
    // combine the nsub subsets: [nsub][nout] x (M, L, O[4]) in the (now free) sm_o area
    float* cm = sm_o[0][0];
    float* cl = cm + nsub * nout;
    float4* co = reinterpret_cast<float4*>(cl + nsub * nout);
    if (sb < nsub) {
        cm[sb * nout + oi] = M;
        cl[sb * nout + oi] = Lsum;
        co[sb * nout + oi] = make_float4(O4[0], O4[1], O4[2], O4[3]);
    }
    __syncthreads();
    WF_STAMP(4);
    for (int o2 = threadIdx.x; o2 < nout; o2 += kAttnThreads) {
        const int h2 = o2 / D4, d2 = (o2 - h2 * D4) * 4;
        float MM = -INFINITY;
        for (int t = 0; t < nsub; ++t) MM = fmaxf(MM, cm[t * nout + o2]);
        float LL = 0.f, OO[4] = {0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < nsub; ++t) {
            const float wgt = (cm[t * nout + o2] == -INFINITY) ? 0.f : __expf(cm[t * nout + o2] - MM);
            LL += cl[t * nout + o2] * wgt;
            const float4 v4 = co[t * nout + o2];
            OO[0] += v4.x * wgt; OO[1] += v4.y * wgt; OO[2] += v4.z * wgt; OO[3] += v4.w * wgt;
        }
        const float inv = 1.0f / LL;
        const float ov4[4] = {OO[0] * inv, OO[1] * inv, OO[2] * inv, OO[3] * inv};
        store_out4(out, b * o_sb + (int64_t)(g * grp + h2) * o_sh + d2, odt, ov4);
    }
    if (threadIdx.x == 0) st_sc1(cnt + b * Hkv + g, 0u);  // re-arm the ticket for the next launch
    WF_STAMP(5);
}

// ---------------------------------------------------------------------------------------------
// Decode-step attention shared constants: k_attn_sdpa's block size and keys per lane group per chunk,
// and the K/V load form.
// ---------------------------------------------------------------------------------------------
#ifndef WF_AP_THREADS  // study builds only (tools/build_variant.sh): threads per block
#define WF_AP_THREADS 512
#endif
constexpr int kAttnPartThreads = WF_AP_THREADS;
// keys per lane group per chunk (chunk = (threads / 16) U keys): a split that one 160-key chunk
// covers (contexts <= 1280 at 8 splits) takes one load round; longer splits the double-buffered
// 128-key chunks. Round 6, k_attn_sdpa at ctx 1024 (same box, tools/ab_quick.sh): 256 threads x U 10
// 10.7 us, 1,014 tok/s; 512 x 5 9.3 us, 1,060 tok/s (half the keys per lane: the QK, P.V and
// permlane-merge chains of a wave halve, 2 waves per SIMD); 768 x 3 11.1 us; 512 x 5 at 4 splits
// 12.0 us. (Round 2, exact softmax without the exchange: 512 threads lost, 5.72 -> 6.10 us.)
// -DWF_AP_U=n: one U everywhere.
#ifdef WF_AP_U
constexpr int kApUShort = WF_AP_U, kApULong = WF_AP_U;
#else
constexpr int kApUShort = 160 / (kAttnPartThreads / 16), kApULong = 128 / (kAttnPartThreads / 16);
#endif
#ifndef WF_KV_NT  // decode-attention K/V loads with the non-temporal hint (each byte is read once per step)
#define WF_KV_NT 1
#endif
__device__ __forceinline__ uint4 kv_ld16(const uint16_t* p) {
    if constexpr (WF_KV_NT) return ldg_nt(reinterpret_cast<const uint8_t*>(p));
    else return *reinterpret_cast<const uint4*>(p);
}
#ifndef WF_KV_NT_B1  // study: 1 = the hint in the batch < 16 attention too (5.8 -> 6.4 us there: not kept)
#define WF_KV_NT_B1 0
#endif

// ---------------------------------------------------------------------------------------------
// The reference's attention AS IT RUNS (scripts/direct_inference_full.py:241: torch 2.10's CPU
// flash SDPA on bf16; restated in oracle/wf_oracle.c orc_attention_sdpa_cpu_bf16 and pinned by
// tests/golden/sdpa_cpu_bf16.npz): keys in 512-key blocks with a RUNNING max M_c (max over blocks
// <= c), probabilities e = fexp_u20(s - M_c) on the 16-key vector part of a block and expf on its
// tail, P = bf16(e) into P.V, the UNROUNDED e into the row sum, blocks combined by
// r_c = expf(M_{c-1} - M_c), out = bf16(dst * (1 / sum)).
//
// Decode step, batch < 16 and untiled caches: block (split s, query head, sequence), kAttnPartSplits1
// splits of T = round_up(ceil(S / NS), 16) keys read by 16-lane groups (8 dims per lane, a wave
// reads 4 contiguous 256-byte key rows), in two phases around an in-launch exchange of the 512-key
// block maxima:
//   1. q.k of the split's keys (products exact in fp32, summed in f64 and rounded once -- torch's
//      oneDNN GEMM is that close to exact, tests/golden/sdpa_probe.py), the split's per-block maxima
//      published as epoch-tagged granules; wave 0 polls the head's granules (all NS splits);
//   2. wave 0 folds the NS x 3 published maxima into M_c, r_c and the suffix products R, every
//      lane forms P and e of its keys, scales by the product of the r's after the key's block
//      (1.0 exactly inside the split's last block), and accumulates l = sum e and o = sum P v.
// Every record (m = 0, l, o) is then in the frame of the head's last block; the head's last block
// (merge ticket) sums the NS records and writes out = bf16(O * (1 / L)) into the bf16 attention row,
// resets the ticket and stores this launch's tag as the head's epoch word (the next launch's tag is
// that + 1). Merging in the O projection's input stage instead (round 5, same box): attention 10.4
// -> 9.0 us, O 4.4 -> 6.0 us per layer (every O block reads all 83 KB of records), 1019 -> 1011
// tok/s. Pipelined polls (four in flight, 256 clocks apart) did not shorten the exchange (2.2 ->
// 2.6 us).
// Residency: every split of a head must be resident while its siblings poll: the host launches
// at most kSdpaMaxBlocks blocks per launch (B = 1: 160), below the chip's resident count.
// ---------------------------------------------------------------------------------------------
#ifndef WF_SDPA_SLEEP
#define WF_SDPA_SLEEP 1
#endif
#ifndef WF_SDPA_WPE
#define WF_SDPA_WPE
#endif
// (measured, not kept: all splits of a head on one XCD with L2 polls -- the dispatcher does deal
// block b to XCD b % 8 (tools/ubench/xcd_map.hip), but no load without sc1 ever saw a granule another
// CU stored, whatever the store's policy bits, and an sc1 hand-off takes 0.6 us on one XCD and across
// two alike (tools/ubench/handoff.hip): the exchange's ~2.2 us is the siblings' QK skew (~0.9 us)
// plus that hand-off, not the distance)
constexpr int kSdpaMaxT = 1024;      // split length bound (max_seq <= 8192): a split spans <= 3 blocks
constexpr int kSdpaMaxSeq = kAttnPartSplits1 * kSdpaMaxT;
#ifndef WF_SDPA_SPIN  // poll bound (iterations of an sc1 load round trip + s_sleep): ~0.3-1 s, never in a valid launch
#define WF_SDPA_SPIN (1 << 20)
#endif
// a poll bound was hit (a sibling workgroup never became resident): raise the model's host-visible
// error word (WF_ATTN_ERR_*; wf_model_check and the next wf_model_step report it)
__device__ __forceinline__ void attn_fail(unsigned* err, unsigned code) {
    if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// torch Vectorized<float>::fexp_u20 (AVX512), bit for bit (x <= 0 here: no overflow branch)
__device__ __forceinline__ float fexp_u20(float x) {
    const float src = x * __uint_as_float(0x3fb8aa3bu);  // x * log2(e)
    const float fr = src - floorf(src);
    float r = fmaf(fr, -0.079204240219773236f, -0.22433836478672356f);
    r = fmaf(fr, r, 0.30354260500649682f);
    r = fmaf(fr, r, 0.00010703434948458272f);
    const float t = fmaf(8388608.0f, src - r, 1065353216.0f);
    const int ci = (int)t;  // v_cvt_i32_f32 truncates, as _mm512_cvttps_epi32
    return __int_as_float(x < __uint_as_float(0xc2aeac50u) ? 0 : ci);
}
// fexp_u20 on a packed pair: the same operations, two lanes per instruction where the VALU has
// packed fp32 forms (each lane rounds as the scalar op)
__device__ __forceinline__ f32x2_t fexp_u20_pk(f32x2_t x) {
    const f32x2_t src = x * __uint_as_float(0x3fb8aa3bu);
    const f32x2_t fr = src - f32x2_t{floorf(src.x), floorf(src.y)};
    f32x2_t r = __builtin_elementwise_fma(fr, f32x2_t{-0.079204240219773236f, -0.079204240219773236f},
                                          f32x2_t{-0.22433836478672356f, -0.22433836478672356f});
    r = __builtin_elementwise_fma(fr, r, f32x2_t{0.30354260500649682f, 0.30354260500649682f});
    r = __builtin_elementwise_fma(fr, r, f32x2_t{0.00010703434948458272f, 0.00010703434948458272f});
    const f32x2_t t = __builtin_elementwise_fma(f32x2_t{8388608.0f, 8388608.0f}, src - r,
                                                f32x2_t{1065353216.0f, 1065353216.0f});
    const float lo = __uint_as_float(0xc2aeac50u);
    return f32x2_t{__int_as_float(x.x < lo ? 0 : (int)t.x), __int_as_float(x.y < lo ? 0 : (int)t.y)};
}
// glibc expf (the scalar tail and the block rescale), within ~1 ulp: x = k ln2 + r (two-constant
// reduction, exact for |k| < 2^11), 2^(r log2 e) on v_exp_f32, scaled by 2^k (x <= 0 here). A 1-ulp
// difference moves a bf16 P once in ~2^15 keys; the f64 exp it replaced cost ~0.5 us per launch.
__device__ __forceinline__ float expf_rn(float x) {
    if (!(x > -104.0f)) return 0.0f;  // below the smallest subnormal (and -inf)
    const float k = rintf(x * 1.44269504f);
    float r = fmaf(-k, 0.693145752f, x);  // ln 2 high part (16 bits): k * hi exact
    r = fmaf(-k, 1.42860677e-06f, r);     // ln 2 low part
    return ldexpf(__builtin_amdgcn_exp2f(r * 1.44269504f), (int)k);
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)dpp_i<CTRL>((int)(uint32_t)u), hi = (uint32_t)dpp_i<CTRL>((int)(uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double group16_sum_d(double v) {
    v += dpp_d<DPP_QP_1032>(v);
    v += dpp_d<DPP_QP_2301>(v);
    v += dpp_d<DPP_HALF_MIRROR>(v);
    v += dpp_d<DPP_MIRROR>(v);
    return v;
}

// k_attn_sdpa's per-chunk steps as plain functions: lambdas capturing the kernel's locals by reference
// left their closure objects (pointers to the locals) in scratch
template <int U>
__device__ __forceinline__ void sdpa_load(uint4 (&r)[U], const uint16_t* __restrict__ base, int64_t kvb, int c0, int gid,
                                          int t1) {
    constexpr int NG = kAttnPartThreads / 16;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = min(c0 + gid + NG * u, max(t1 - 1, 0));
        r[u] = *reinterpret_cast<const uint4*>(base + kvb + (int64_t)t * 128);
    }
}
// q.k of the chunk's keys (products exact in fp32, summed in f64, rounded once), the split's per-block
// maxima; the scores into sc (one-chunk splits) or the LDS score buffer
template <int U, bool ONE>
__device__ __forceinline__ void sdpa_scores(const uint4 (&kr)[U], const uint32_t (&qw)[4], int c0, int gid, int li, int t0,
                                            int t1, int cb0, float sm_scale, float (&mx)[3], float (&sc)[ONE ? U : 1],
                                            float* sc_lds) {
    constexpr int NG = kAttnPartThreads / 16;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t w[4] = {kr[u].x, kr[u].y, kr[u].z, kr[u].w};
        double dd = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dd += (double)(bf_lo(qw[i]) * bf_lo(w[i]));  // bf16 x bf16: exact in fp32
            dd += (double)(bf_hi(qw[i]) * bf_hi(w[i]));
        }
        const float sv = (float)group16_sum_d(dd) * sm_scale;
        const int t = c0 + gid + NG * u;
        const bool valid = t < t1;
        const bool in0 = t < 512 * (cb0 + 1), in1 = t < 512 * (cb0 + 2);
        mx[0] = (valid && in0) ? fmaxf(mx[0], sv) : mx[0];
        mx[1] = (valid && !in0 && in1) ? fmaxf(mx[1], sv) : mx[1];
        mx[2] = (valid && !in1) ? fmaxf(mx[2], sv) : mx[2];
        if constexpr (ONE) sc[u] = sv;
        else if (valid && li == 0) sc_lds[t - t0] = sv;
    }
}
// probabilities of the chunk's keys and their P.V: e = fexp_u20 / expf of (s - M_c) (vector part /
// tail of the key's 512-key block), l += e R, o += bf16(e) R v, R = the product of the block
// rescale factors between the key's block and the split's last one (1.0 in the last block)
// (the six block values by value: a struct passed by reference became a private array that the
// per-key selects indexed, in scratch -- or, under an occupancy attribute, in LDS, which stretched
// the launch's block dispatch over ~9 us)
template <int U, bool ONE>
__device__ __forceinline__ void sdpa_pv(const uint4 (&vr)[U], const float (&sc)[ONE ? U : 1], const float* sc_lds, int c0,
                                        int gid, int t0, int t1, int cb0, int Sb, float bm0, float bm1, float bm2,
                                        float br0, float br1, float br2, float& l, float (&o)[8]) {
    constexpr int NG = kAttnPartThreads / 16;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = c0 + gid + NG * u;
        if (t < t1) {
            float sv;
            if constexpr (ONE) sv = sc[u];
            else sv = sc_lds[t - t0];
            const bool in0 = t < 512 * (cb0 + 1), in1 = t < 512 * (cb0 + 2);
            const float Mc = in0 ? bm0 : (in1 ? bm1 : bm2);
            const float Rc = in0 ? br0 : (in1 ? br1 : br2);
            const int blk0 = t & ~511;
            const int vbnd = min(512, Sb - blk0) & ~15;  // the 16-wide vector part of the block
            const float x = sv - Mc;
            const float e = ((t - blk0) < vbnd) ? fexp_u20(x) : expf_rn(x);
            const float p = rbf(e) * Rc;
            l = fmaf(e, Rc, l);
            const uint32_t w[4] = {vr[u].x, vr[u].y, vr[u].z, vr[u].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                o[2 * i] = fmaf(p, bf_lo(w[i]), o[2 * i]);
                o[2 * i + 1] = fmaf(p, bf_hi(w[i]), o[2 * i + 1]);
            }
        }
    }
}

template <int U, bool ONE>
__device__ __forceinline__ void attn_sdpa_body(const uint16_t* __restrict__ q, int64_t q_sb, const uint16_t* __restrict__ K,
                                               const uint16_t* __restrict__ V, int64_t kv_sb, int64_t kv_sh, int Hq,
                                               int Hkv, int S, const int32_t* __restrict__ seq_lens, float sm_scale,
                                               int b0, uint64_t* __restrict__ xg, float2* __restrict__ ml_out,
                                               float* __restrict__ o_out, uint16_t* __restrict__ row_out,
                                               uint64_t* __restrict__ xo, unsigned* __restrict__ xep, int s, int hq,
                                               unsigned* __restrict__ err, int stall) {
    constexpr int NS = kAttnPartSplits1, D = 128, LP = 16, NG = kAttnPartThreads / LP, CH = U * NG;
    constexpr int NWV = kAttnPartThreads / 64;
    constexpr int DM = kSdpaMergeDims;  // split s merges dims DM s .. DM s + DM - 1
    static_assert(NS * DM == D && DM % 4 == 0 && DM < 64, "whole 4-dim pieces per merge range");
    const int b = b0 + (int)blockIdx.z;
    const int g = hq / (Hq / Hkv);
    const int gid = threadIdx.x / LP, li = threadIdx.x % LP, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int Sb = min(seq_lens[b], S);
    const int T = ((Sb + NS - 1) / NS + 15) / 16 * 16;
    const int t0 = s * T, t1 = min(t0 + T, Sb);
    const int cb0 = t0 >> 9;
    const int64_t bh = (int64_t)b * Hq + hq;
    WF_STAMP(0);
    // this launch's tag: the head's epoch word + 1, read before anything else (the word is advanced
    // by split 0 once every split has published its maxima, i.e. has read it)
    const unsigned ep = ld_sc1(xep + bh * kTailLine) + 1u;
    __shared__ float sc_lds[ONE ? 1 : kSdpaMaxT];
    __shared__ float red[NWV][3];
    __shared__ float blk_m[3], blk_r[3], fin_r;
    __shared__ float sm_l[NWV];
    __shared__ __attribute__((aligned(16))) float sm_o[NWV][D];

    const int64_t kvb = b * kv_sb + g * kv_sh + li * 8;
    const uint4 qv = *reinterpret_cast<const uint4*>(q + b * q_sb + (int64_t)hq * D + li * 8);
    const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w};
    float mx[3] = {-INFINITY, -INFINITY, -INFINITY};  // per 512-key block of the split (<= 3)
    float sc[ONE ? U : 1];
    uint4 vA[U], vB[ONE ? 1 : U];
    if (t0 < t1) {
        uint4 kA[U];
        sdpa_load<U>(kA, K, kvb, t0, gid, t1);
        if constexpr (ONE) {
            sdpa_load<U>(vA, V, kvb, t0, gid, t1);
            sdpa_scores<U, ONE>(kA, qw, t0, gid, li, t0, t1, cb0, sm_scale, mx, sc, sc_lds);
        } else {
            uint4 kB[U];
            for (int c0 = t0; c0 < t1; c0 += 2 * CH) {
                if (c0 + CH < t1) sdpa_load<U>(kB, K, kvb, c0 + CH, gid, t1);
                sdpa_scores<U, ONE>(kA, qw, c0, gid, li, t0, t1, cb0, sm_scale, mx, sc, sc_lds);
                if (c0 + 2 * CH < t1) sdpa_load<U>(kA, K, kvb, c0 + 2 * CH, gid, t1);
                if (c0 + CH < t1) sdpa_scores<U, ONE>(kB, qw, c0 + CH, gid, li, t0, t1, cb0, sm_scale, mx, sc, sc_lds);
            }
            sdpa_load<U>(vA, V, kvb, t0, gid, t1);  // V chunks 0 and 1 in flight across the exchange
            if (t0 + CH < t1) sdpa_load<U>(vB, V, kvb, t0 + CH, gid, t1);
        }
    }
    WF_STAMP(1);
    // ---- the exchange: per-block maxima of every split of this head ----
    // Each split publishes one 8-byte granule {max, epoch} per 512-key block it covers (a split spans
    // <= 3 blocks at T <= 1024) with an sc1 store; wave 0 polls the head's 3 NS granules with sc1
    // loads until every tag is this launch's epoch (MI355X_MICROARCH.md handoff-1to1: data-tagged
    // granules, no counter round trip). The epoch is the head's launch count, advanced by the
    // head's merging block after every split has passed its poll.
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
        const float w = wave_max(mx[jj]);
        if (lane == 0) red[wv][jj] = w;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(wv) == 0) {  // wave 0 (a scalar branch: no exec-masked loop)
        const unsigned want = stall ? ep + 1u : ep;  // test hook (wf_model_debug_stall_attention): a tag nobody stores
        float bmx[3];  // the block's maxima (constant LDS indices: uniform scalars)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
            bmx[jj] = red[0][jj];
#pragma unroll
            for (int w = 1; w < NWV; ++w) bmx[jj] = fmaxf(bmx[jj], red[w][jj]);
        }
        if (lane < 3) {
            const float m = lane == 0 ? bmx[0] : (lane == 1 ? bmx[1] : bmx[2]);
            st_sc1(xg + (bh * NS + s) * 3 + lane, ((uint64_t)ep << 32) | __float_as_uint(m));
        }
        // lanes 0 .. 3 NS - 1: split lane / 3, block cb0(split) + lane % 3
        const int sp = lane / 3, ent = lane - 3 * sp;
        uint64_t gv = ((uint64_t)ep << 32) | 0xff800000u;  // lanes past the granules: -inf, tagged
        int ok = 1;
        // (measured, not kept: two polls in flight; V loaded after the exchange or after the wave's
        // q.k instead of with K -- profiles/ab_attn_merge_r06.txt)
        for (int it = 0;; ++it) {
            if (lane < 3 * NS) gv = ld_sc1(xg + bh * NS * 3 + lane);
            if (__all((unsigned)(gv >> 32) == want)) break;
            if (it > WF_SDPA_SPIN) {  // a missing sibling ends in NaN outputs and the error word, never a hang
                ok = 0;
                if (lane == 0) attn_fail(err, WF_ATTN_ERR_SDPA);
                break;
            }
            __builtin_amdgcn_s_sleep(WF_SDPA_SLEEP);
        }
        // every split has published its maxima, so every split has read the epoch word: advance it
        if (s == 0 && lane == 0) st_sc1(xep + bh * kTailLine, ep);
        const float val = __uint_as_float((uint32_t)gv);
        const int blk = lane < 3 * NS ? ((sp * T) >> 9) + ent : -1;
        const int NB = (Sb + 511) >> 9;
        const int cb1 = max(t1 - 1, t0) >> 9;
        // prefix maxima, rescale factors and, for this split, the products of the factors after each
        // of its blocks up to its last one (blk_r) and after its last block (fin_r): uniform loop
        float M = -INFINITY, rr[3] = {1.f, 1.f, 1.f}, fin = 1.f;
        for (int c = 0; c < NB; ++c) {
            const float bmc = wave_max((blk == c) ? val : -INFINITY);
            const float Mn = fmaxf(M, bmc);
            const float r = (c == 0) ? 1.f : expf_rn(M - Mn);
            M = Mn;
            if (c > cb1) fin *= r;
#pragma unroll
            for (int jj = 0; jj < 3; ++jj)
                if (c > cb0 + jj && c <= cb1) rr[jj] *= r;
            if (lane == 0 && c >= cb0 && c < cb0 + 3) blk_m[c - cb0] = ok ? M : __uint_as_float(0x7fc00000u);
        }
        if (lane == 0) {
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) blk_r[jj] = rr[jj];
            fin_r = fin;
        }
    }
    __syncthreads();
    WF_STAMP(2);
    // ---- probabilities and P.V ----
    // block-uniform values read once into scalar registers (hipcc otherwise sank the LDS loads into
    // the per-key selects and built a table of LDS addresses in scratch)
    auto sload = [](const float& v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    const float bm0 = sload(blk_m[0]), bm1 = sload(blk_m[1]), bm2 = sload(blk_m[2]);
    const float br0 = sload(blk_r[0]), br1 = sload(blk_r[1]), br2 = sload(blk_r[2]);
    float l = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t0 < t1) {
        if constexpr (ONE) {
            sdpa_pv<U, ONE>(vA, sc, sc_lds, t0, gid, t0, t1, cb0, Sb, bm0, bm1, bm2, br0, br1, br2, l, o);
        } else {
            for (int c0 = t0; c0 < t1; c0 += 2 * CH) {
                sdpa_pv<U, ONE>(vA, sc, sc_lds, c0, gid, t0, t1, cb0, Sb, bm0, bm1, bm2, br0, br1, br2, l, o);
                if (c0 + 2 * CH < t1) sdpa_load<U>(vA, V, kvb, c0 + 2 * CH, gid, t1);
                if (c0 + CH < t1) {
                    sdpa_pv<U, ONE>(vB, sc, sc_lds, c0 + CH, gid, t0, t1, cb0, Sb, bm0, bm1, bm2, br0, br1, br2, l, o);
                    if (c0 + 3 * CH < t1) sdpa_load<U>(vB, V, kvb, c0 + 3 * CH, gid, t1);
                }
            }
        }
    }
    // ---- sum the lane groups (every record is in one frame: plain sums) ----
    auto sum16 = [](float v) __attribute__((always_inline)) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    };
    auto sum32 = [](float v) __attribute__((always_inline)) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    };
    l = sum32(sum16(l));
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = sum32(sum16(o[j]));
    if (lane < LP) {
        if (li == 0) sm_l[wv] = l;
        *reinterpret_cast<float4*>(&sm_o[wv][li * 8]) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(&sm_o[wv][li * 8 + 4]) = make_float4(o[4], o[5], o[6], o[7]);
    }
    __syncthreads();
    const float fr = sload(fin_r);
    // ---- records, and the merge as an all-to-all of tagged granules ----
    // Split s merges dims [DM s, DM s + DM) of the head. Every split publishes, for each target split
    // r, its DM dims of r's range and its l as 8-byte {value, tag} granules (slot (bh, r, s) of
    // kSdpaMergeSlot granules, one sc1 store per pair); wave 0 of split r polls the NS slots of its
    // own range and sums them in split order -- the operations (and order) of a single merging block,
    // without the drain, the arrival ticket and the last block's record reads.
    if (threadIdx.x < D / 4) {
        const int d = 4 * threadIdx.x;
        float ls = 0.f, os[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < NWV; ++w) {
            ls += sm_l[w];
            const float4 ov = *reinterpret_cast<const float4*>(&sm_o[w][d]);
            os[0] += ov.x; os[1] += ov.y; os[2] += ov.z; os[3] += ov.w;
        }
        ls *= fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) os[j] *= fr;
        const __amdgpu_buffer_rsrc_t rx = make_rsrc(xo);
        const int slot = (int)(((bh * NS + d / DM) * NS + s) * kSdpaMergeSlot) * 8;  // byte offset
        st16_sc1(rx, slot + 8 * (d % DM), make_uint4(__float_as_uint(os[0]), ep, __float_as_uint(os[1]), ep));
        st16_sc1(rx, slot + 8 * (d % DM) + 16, make_uint4(__float_as_uint(os[2]), ep, __float_as_uint(os[3]), ep));
        if (d % DM == 0) st_sc1(xo + slot / 8 + DM, ((uint64_t)ep << 32) | __float_as_uint(ls));
        // the records (the API's attention view): read by no kernel of this launch
        const int64_t rec = bh * NS + s;
        *reinterpret_cast<float4*>(o_out + part_o_off<NS>(bh, s, d)) = make_float4(os[0], os[1], os[2], os[3]);
        if (d == 0) *reinterpret_cast<float2*>(ml_out + rec) = make_float2(0.f, ls);
    }
    WF_STAMP(3);
    if (__builtin_amdgcn_readfirstlane(wv) != 0) return;
    // lane j < DM: dim DM s + j of every source split; lane DM: the sources' l
    const int64_t src = (bh * NS + s) * NS * kSdpaMergeSlot + min(lane, DM);
    uint64_t gv[NS];
    for (int it = 0;; ++it) {
        bool okl = true;
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            gv[u] = lane <= DM ? ld_sc1(xo + src + u * kSdpaMergeSlot) : ((uint64_t)ep << 32);
            okl = okl && (unsigned)(gv[u] >> 32) == ep;
        }
        if (__all(okl)) break;
        if (it > WF_SDPA_SPIN) {
            if (lane == 0) attn_fail(err, WF_ATTN_ERR_SDPA);
#pragma unroll
            for (int u = 0; u < NS; ++u) gv[u] = 0x7fc00000u;  // NaN row
            break;
        }
        __builtin_amdgcn_s_sleep(WF_SDPA_SLEEP);
    }
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < NS; ++u) acc += __uint_as_float((uint32_t)gv[u]);
    const float L = __shfl(acc, DM, 64);
    const float inv = 1.0f / L;
    if (lane < DM) row_out[bh * D + DM * s + lane] = f2bf(acc * inv);
    WF_STAMP(4);
}

__global__ __launch_bounds__(kAttnPartThreads) WF_SDPA_WPE void k_attn_sdpa(const uint16_t* __restrict__ q, int64_t q_sb,
                                                                const uint16_t* __restrict__ K,
                                                                const uint16_t* __restrict__ V, int64_t kv_sb,
                                                                int64_t kv_sh, int Hq, int Hkv, int S,
                                                                const int32_t* __restrict__ seq_lens, float sm_scale,
                                                                int b0, uint64_t* __restrict__ xg,
                                                                float2* __restrict__ ml_out, float* __restrict__ o_out,
                                                                uint16_t* __restrict__ row_out, uint64_t* __restrict__ xo,
                                                                unsigned* __restrict__ xep, unsigned* __restrict__ err,
                                                                int stall) {
    constexpr int NS = kAttnPartSplits1, NG = kAttnPartThreads / 16;
    const int s = blockIdx.x, hq = blockIdx.y;
    const int Sb = min(seq_lens[b0 + (int)blockIdx.z], S);
    const int T = ((Sb + NS - 1) / NS + 15) / 16 * 16;
    if (T <= kApUShort * NG)  // block-uniform: one load round holds the split
        attn_sdpa_body<kApUShort, true>(q, q_sb, K, V, kv_sb, kv_sh, Hq, Hkv, S, seq_lens, sm_scale, b0, xg, ml_out,
                                        o_out, row_out, xo, xep, s, hq, err, stall);
    else
        attn_sdpa_body<kApULong, false>(q, q_sb, K, V, kv_sb, kv_sh, Hq, Hkv, S, seq_lens, sm_scale, b0, xg, ml_out,
                                        o_out, row_out, xo, xep, s, hq, err, stall);
}

// ---------------------------------------------------------------------------------------------
// Fragment types and one-byte K/V widening shared by the batched decode attention
// (k_attn_sdpa_mfma): K / V caches in their tile layouts (wf_norm.h k_tile_off / v_tile_off), every
// fragment load one contiguous KiB per wave.
// ---------------------------------------------------------------------------------------------
#ifndef WF_ATTN_SPLIT2  // 0: one workgroup per (kv head, sequence) whatever the context
#define WF_ATTN_SPLIT2 1
#endif
constexpr bool kAttnSplit2 = WF_ATTN_SPLIT2;
typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef float v4f_t __attribute__((ext_vector_type(4)));
constexpr int kAttnMfmaMaxGrp = 8;
// FP8 (OCP e4m3fn) K/V caches: a fragment is 8 one-byte keys / dims (8 bytes per lane, 512
// contiguous bytes per wave-instruction), widened to bf16 in registers (exact: every e4m3 value is
// a bf16 value). The per-layer scales are folded into the score scale (K) and the partial records
// (V), so the arithmetic after the widening is the bf16 path's.
typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 fp8x8_to_bf16(uint2 r) {
    const v2bf_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(r.x, 1.0f, false);
    const v2bf_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(r.x, 1.0f, true);
    const v2bf_t c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(r.y, 1.0f, false);
    const v2bf_t d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(r.y, 1.0f, true);
    return make_uint4(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, c),
                      __builtin_bit_cast(uint32_t, d));
}
// int8 K/V caches (the reference's default KVCacheDtype.INT8, kv_cache/kv_cache.py:159-218, with a
// static per-layer scale): a fragment is 8 signed codes (8 bytes per lane), widened exactly -- each
// byte biased to unsigned (xor 0x80), v_cvt_f32_ubyteN, -128 (packed), then bf16 (|code| <= 127 is
// exact in bf16). Scales folded like FP8's.
#ifndef WF_I8_PK  // 0: the round-5 form (hipcc folds the -128 into an integer subtract: SDWA + v_cvt_f32_i32)
#define WF_I8_PK 1
#endif
__device__ __forceinline__ uint32_t i8x2_to_bf16(uint32_t u, int sh) {
    const float lo = (float)((u >> sh) & 0xffu) - 128.0f, hi = (float)((u >> (sh + 8)) & 0xffu) - 128.0f;
    return pk_bf16(lo, hi);
}
// four biased bytes -> floats (v_cvt_f32_ubyte0..3), -128 on pairs (v_pk_add_f32), packed to bf16
__device__ __forceinline__ uint2 i8x4_to_bf16_pk(uint32_t x) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a = {(float)(x & 0xffu), (float)((x >> 8) & 0xffu)};
    f2 b = {(float)((x >> 16) & 0xffu), (float)(x >> 24)};
    asm volatile("" : "+v"(a), "+v"(b));  // keep the conversions unsigned-byte (no integer -128 fold)
    const f2 m = {-128.f, -128.f};
    a += m;
    b += m;
    return make_uint2(pk_bf16(a.x, a.y), pk_bf16(b.x, b.y));
}
__device__ __forceinline__ uint4 i8x8_to_bf16(uint2 r) {
    const uint32_t x = r.x ^ 0x80808080u, y = r.y ^ 0x80808080u;
    if constexpr (WF_I8_PK) {
        const uint2 lo = i8x4_to_bf16_pk(x), hi = i8x4_to_bf16_pk(y);
        return make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
    return make_uint4(i8x2_to_bf16(x, 0), i8x2_to_bf16(x, 16), i8x2_to_bf16(y, 0), i8x2_to_bf16(y, 16));
}
// KVQ: K/V cache element type -- 0 bf16, 1 OCP e4m3fn, 2 int8 (include/wf_bitnet.h WF_KV_*)
template <int KVQ>
struct KvFrag {
    using T = uint4;  // 8 bf16
    __device__ static __forceinline__ T ld(const uint16_t* base, int64_t elem) { return kv_ld16(base + elem); }
    __device__ static __forceinline__ uint4 bf(const T& t) { return t; }
    // zero the keys >= lim of a V fragment (8 keys)
    __device__ static __forceinline__ T mask(const T& t, int lim) {
        if (lim >= 8) return t;
        uint32_t vm[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) vm[j] = (2 * j < lim ? 0xffffu : 0u) | (2 * j + 1 < lim ? 0xffff0000u : 0u);
        return make_uint4(t.x & vm[0], t.y & vm[1], t.z & vm[2], t.w & vm[3]);
    }
};
template <int KVQ>
struct KvFrag8 {
    using T = uint2;  // 8 one-byte codes
    __device__ static __forceinline__ T ld(const uint16_t* base, int64_t elem) {
        const uint2* p = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(base) + elem);
        if constexpr (WF_KV_NT) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
            return make_uint2(v.x, v.y);
        } else {
            return *p;
        }
    }
    __device__ static __forceinline__ uint4 bf(const T& t) {
        if constexpr (KVQ == 2) return i8x8_to_bf16(t);
        else return fp8x8_to_bf16(t);
    }
    __device__ static __forceinline__ T mask(const T& t, int lim) {
        if (lim >= 8) return t;
        const uint64_t m = lim <= 0 ? 0ull : (~0ull >> (8 * (8 - lim)));
        return make_uint2(t.x & (uint32_t)m, t.y & (uint32_t)(m >> 32));  // zero bytes: 0 in both codes
    }
};
template <>
struct KvFrag<1> : KvFrag8<1> {};
template <>
struct KvFrag<2> : KvFrag8<2> {};

// ---------------------------------------------------------------------------------------------
// Batched decode attention (batch >= 16, tile-layout K/V) with the reference's SDPA arithmetic
// (k_attn_sdpa's comment; oracle/wf_oracle.c orc_attention_sdpa_cpu_bf16): one block per (kv head
// g, sequence b) walks the sequence's 512-key blocks in order, exactly the CPU kernel's loop, so
// the running max needs no exchange between blocks of the launch. 4 waves; wave w takes tiles
// w, w + 4, w + 8, w + 12 (32 keys each) of every 512-key block, in two passes:
//   pass 1: K fragments -> QK on the bf16 matrix cores (A = K rows: tile tau, row 4 a + r <- key
//     base + 8 a + 4 tau + r; B = Q^T, lane quarter q4 takes dims 32 c + 8 q4 .. + 8 of MFMA c:
//     lane (head l16, quarter q4) then holds the scores of keys base + 8 q4 + 0..7, exactly the A
//     fragment of the P.V MFMA), the wave's per-head maximum;
//     the four waves' maxima meet in LDS (one barrier per block) -> M_c, r_c = expf(M_{c-1} - M_c);
//   pass 2: V fragments -> e = fexp_u20 / expf of (s - M_c) (vector part / tail of the block),
//     l = l r_c + sum e (unrounded), acc = acc r_c + bf16(e) . V (ONE bf16 MFMA term: P IS bf16).
// The fragment stream K(c, 0..3), V(c, 0..3), K(c + 1, 0..3) ... is double-buffered one tile ahead
// (a tile past the sequence loads nothing and computes nothing). The block writes the normalised
// bf16 attention row bf16(o * (1 / l)) of its group's heads into `row` [B][Hq * 128].
// ---------------------------------------------------------------------------------------------
template <int KV8, int GQ>
__global__ __launch_bounds__(256, 3) void k_attn_sdpa_mfma(const uint16_t* __restrict__ q, int64_t q_sb,
                                                          const uint16_t* __restrict__ K, const uint16_t* __restrict__ Vt,
                                                          int64_t kv_sb, int64_t kv_sh, int Hq, int Hkv, int S,
                                                          const int32_t* __restrict__ seq_lens, float sm_scale,
                                                          const int32_t* __restrict__ pt, int pps, int npages,
                                                          int64_t kv_pgs, float v_scale, uint16_t* __restrict__ row,
                                                          const int32_t* __restrict__ order, float2* __restrict__ rec_ml,
                                                          float* __restrict__ rec_o, unsigned* __restrict__ cnt,
                                                          unsigned* __restrict__ xep, uint64_t* __restrict__ xg,
                                                          unsigned* __restrict__ err) {
    constexpr int D = 128;
    using KF = KvFrag<KV8>;
    using FT = typename KF::T;
    // blocks in longest-context-first order (k_seq_order; any permutation is correct, the order only
    // balances ragged contexts over the CUs)
    const int g = blockIdx.x, b = order ? min(max(order[blockIdx.y], 0), (int)gridDim.y - 1) : (int)blockIdx.y;
    const int grp = Hq / Hkv, hq0 = g * grp;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q4 = lane >> 4;
    const int Sb = min(seq_lens[b], S);
    const int NB = (Sb + 511) >> 9;
    // gridDim.z == 2: a sequence of two or three 512-key blocks takes two workgroups, block 0 and
    // blocks 1 .. NB - 1 (5 kv heads x 128 sequences = 640 workgroups otherwise leave half the CUs 3
    // and half 2). Workgroup 1 needs M_0, the max of block 0, before its first probabilities:
    // workgroup 0 publishes it as epoch-tagged granules (k_attn_sdpa's exchange; all z = 0 workgroups
    // precede z = 1 in dispatch order, so workgroup 0 never waits on workgroup 1). Both store records
    // -- (M_0, l_0, o_0) and (R, l_1, o_1), R the product of workgroup 1's block rescale factors
    // r_1 r_2 ... (the factor the CPU loop's running sums carry block 0 by) -- and the second to finish
    // combines them: O = o_0 R + o_1, L = l_0 R + l_1.
    const int sp = blockIdx.z;
    // (two or three blocks only: at config-4 contexts a 7-block second workgroup became the tail,
    // 136.8 -> 138.7 us; at ctx 1024, three blocks, 67.9 -> 65.9 us)
    const bool two = gridDim.z == 2 && NB >= 2 && NB <= 3;
    if (sp == 1 && !two) return;  // whole workgroup
    const int c0 = two ? sp : 0, c1 = two ? (sp ? NB : 1) : NB;
    float Rp = 1.f;  // workgroup 1: product of its rescale factors
    const int64_t gb = (int64_t)b * Hkv + g;
    const unsigned ep = two ? ld_sc1(xep + gb * kTailLine) + 1u : 0u;  // this launch's tag
    __shared__ float sm_m0[kAttnMfmaMaxGrp], sm_mh[kAttnMfmaMaxGrp];
    __shared__ int sh_last;
    __shared__ float sm_mx[2][4][16];
    // the wave's scores of its 4 tiles of the block (LDS, not registers: three blocks per CU instead
    // of two); after the last block the same bytes hold the waves' output partials
    __shared__ __attribute__((aligned(16))) union {
        float x[4][4][8][64];
        float o[4][kAttnMfmaMaxGrp][D];
    } sm_u;
    __shared__ float sm_l[4][kAttnMfmaMaxGrp];
    const int64_t kvo = b * kv_sb + g * kv_sh + lane * 8;
    const int32_t* ptb = pt ? pt + (int64_t)b * pps : nullptr;
    WF_STAMP(0);

    // the q fragments (B operand: column = query head of the group) live in LDS, read per tile: 16
    // VGPRs fewer, three blocks per CU
    __shared__ __attribute__((aligned(16))) uint4 sm_q[4][64];
    {
        // GQ = 4: column l16 = head (l16 & 3) restricted to the lane quarter l16 >> 2 of every 32
        // dims, so each MFMA output is a sum of 8 products (below)
        const int hh = GQ == 4 ? (l16 & 3) : min(l16, grp - 1);
        const bool live = GQ == 4 ? (l16 >> 2) == q4 : l16 < grp;
        const uint16_t* qp = q + b * q_sb + (int64_t)(hq0 + hh) * D + 8 * q4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint4 t = *reinterpret_cast<const uint4*>(qp + 32 * c);
            if (!live) t = make_uint4(0, 0, 0, 0);
            if (wave == 0) sm_q[c][lane] = t;
        }
    }
    __syncthreads();
    // step s of block c: pass s >> 2 (0 = K, 1 = V), tile base 512 c + 32 (wave + 4 (s & 3))
    auto tbase = [&](int c, int s) { return 512 * c + 32 * (wave + 4 * (s & 3)); };
    auto load = [&](FT (&f)[8], int c, int s) {
        const int bs = tbase(c, s);
        const int64_t blk = ptb ? (int64_t)min(max(ptb[__builtin_amdgcn_readfirstlane(bs) >> 5], 0), npages - 1) * kv_pgs
                                : (int64_t)(bs >> 5) * 4096;
        const uint16_t* base = (s >> 2) ? Vt : K;
#pragma unroll
        for (int n = 0; n < 8; ++n) f[n] = KF::ld(base, kvo + blk + n * 512);
    };
    float m_run = -INFINITY, l_run = 0.f;  // per lane: head l16 (m), the lane's quarter of the sum (l)
    v4f_t acc[8];
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[n] = v4f_t{0.f, 0.f, 0.f, 0.f};
    FT fa[8], fb[8];
    if (c1 > c0 && tbase(c0, 0) < Sb) load(fa, c0, 0);
    for (int c = c0; c < c1; ++c) {
        const int nb = min(512, Sb - 512 * c), vbnd = nb & ~15;
        float wmx = -INFINITY;
        float mblk = -INFINITY, r = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            // the next step's fragments first (one tile ahead), into the other buffer
            {
                const int cn = s == 7 ? c + 1 : c, sn = (s + 1) & 7;
                if (cn < c1 && tbase(cn, sn) < Sb) {
                    if (s & 1) load(fa, cn, sn);
                    else load(fb, cn, sn);
                }
            }
            if (s == 4) {  // the block's maxima: every wave's pass 1 is done
                if (q4 == 0 && l16 < 16) sm_mx[c & 1][wave][l16] = wmx;
                if (two && sp == 1 && c == c0 && wave == 0 && lane < grp) {  // M_0 of head `lane` from workgroup 0
                    const uint64_t* gp = xg + gb * kAttnMfmaMaxGrp + lane;
                    uint64_t gv = ld_sc1(gp);
                    for (int it = 0; (unsigned)(gv >> 32) != ep; ++it) {
                        if (it > WF_SDPA_SPIN) {  // never in a valid launch: NaN and the error word, not a hang
                            gv = 0x7fc00000u;
                            attn_fail(err, WF_ATTN_ERR_SPLIT2);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        gv = ld_sc1(gp);
                    }
                    sm_m0[lane] = __uint_as_float((uint32_t)gv);
                }
                __syncthreads();
                if (two && sp == 1 && c == c0) m_run = sm_m0[l16 % grp];  // block 1 continues from block 0's max
                mblk = fmaxf(fmaxf(sm_mx[c & 1][0][l16], sm_mx[c & 1][1][l16]), fmaxf(sm_mx[c & 1][2][l16], sm_mx[c & 1][3][l16]));
                const float mn = fmaxf(m_run, mblk);
                r = (c == 0) ? 0.f : expf_rn(m_run - mn);
                Rp *= (c == 0) ? 1.f : r;
                m_run = mn;
                if (two && sp == 0 && wave == 0 && q4 == 0 && l16 < grp)
                    st_sc1(xg + gb * kAttnMfmaMaxGrp + l16, ((uint64_t)ep << 32) | __float_as_uint(mn));
                l_run *= r;
                if (c > 0) {
                    float ar[4];  // rescale of output row (head) 4 q4 + rr
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) ar[rr] = __shfl(r, 4 * q4 + rr, 64);
#pragma unroll
                    for (int n = 0; n < 8; ++n)
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) acc[n][rr] *= ar[rr];
                }
            }
            const int bs = tbase(c, s);
            if (bs >= Sb) continue;  // wave-uniform
            const FT (&f)[8] = (s & 1) ? fb : fa;
            const int i = s & 3;
            const int lim = Sb - bs - 8 * q4;  // valid keys among this lane's 8
            if (s < 4) {  // pass 1: scores
                // partial dots in separate accumulators, summed in f64 and rounded once: close to the
                // exactly rounded dot of the reference's GEMM. GQ = 4 (4 query heads per kv head) puts
                // the 12 idle B columns to work: column 4 c + h holds head h on dims 8 c .. 8 c + 7 of
                // each 32, so every MFMA output sums 8 products and the 16 partials of a score meet
                // in f64 (two row rotations); one fp32 accumulator chained through the four MFMAs
                // moved 1.6 % of the outputs at 4096 keys, four 32-product partials ~0.1 % on peaky
                // rows (tests/test_gpu_configs.py attention kernels)
#pragma unroll
                for (int tau = 0; tau < 2; ++tau) {
                    double dd[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc) {
                        const v4f_t pr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(v8s_t, KF::bf(f[tau * 4 + cc])), __builtin_bit_cast(v8s_t, sm_q[cc][lane]),
                            v4f_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
                        for (int r4 = 0; r4 < 4; ++r4) dd[r4] += (double)pr[r4];
                    }
                    if constexpr (GQ == 4) {  // lane l16 < 4: the sum of columns l16, +4, +8, +12
#pragma unroll
                        for (int r4 = 0; r4 < 4; ++r4) {
                            dd[r4] += dpp_d<DPP_ROW_ROR8>(dd[r4]);
                            dd[r4] += dpp_d<DPP_ROW_ROR4>(dd[r4]);
                        }
                    }
#pragma unroll
                    for (int r4 = 0; r4 < 4; ++r4) {
                        const int e = 4 * tau + r4;
                        const float xv = e < lim ? (float)dd[r4] * sm_scale : -INFINITY;
                        sm_u.x[wave][i][e][lane] = xv;
                        wmx = fmaxf(wmx, xv);
                    }
                }
                if (i == 3 || tbase(c, s + 1) >= Sb) {  // the wave's last tile of the block: its head maxima
                    wmx = fmaxf(wmx, __shfl_xor(wmx, 16, 64));
                    wmx = fmaxf(wmx, __shfl_xor(wmx, 32, 64));
                }
            } else {  // pass 2: probabilities and P.V
                const int j0 = bs - 512 * c + 8 * q4;  // the lane's first key within the block
                float p[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float xv = sm_u.x[wave][i][e][lane] - m_run;
                    const float ev = e < lim ? ((j0 + e) < vbnd ? fexp_u20(xv) : expf_rn(xv)) : 0.f;
                    l_run += ev;
                    p[e] = ev;
                }
                const v8s_t ph = __builtin_bit_cast(v8s_t, make_uint4(pk_bf16(p[0], p[1]), pk_bf16(p[2], p[3]),
                                                                      pk_bf16(p[4], p[5]), pk_bf16(p[6], p[7])));
#pragma unroll
                for (int n = 0; n < 8; ++n) {
                    const v8s_t vf = __builtin_bit_cast(v8s_t, KF::bf(KF::mask(f[n], lim)));
                    acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vf, acc[n], 0, 0, 0);
                }
            }
        }
    }
    WF_STAMP(1);
    __syncthreads();  // every wave is past its last score read: sm_u becomes the output partials
    l_run += __shfl_xor(l_run, 16, 64);
    l_run += __shfl_xor(l_run, 32, 64);
    if (q4 == 0 && l16 < grp) sm_l[wave][l16] = l_run;
    if (wave == 0 && q4 == 0 && l16 < grp) sm_mh[l16] = sp ? Rp : m_run;  // record field 0: M_0 / R
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
            if (4 * q4 + rr < grp) sm_u.o[wave][4 * q4 + rr][16 * n + l16] = acc[n][rr];
    __syncthreads();
    for (int idx = threadIdx.x; idx < grp * (D / 4); idx += 256) {
        const int h = idx / (D / 4), d = (idx % (D / 4)) * 4;
        float ls = 0.f, os[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            ls += sm_l[w][h];
            const float4 ov = *reinterpret_cast<const float4*>(&sm_u.o[w][h][d]);
            os[0] += ov.x; os[1] += ov.y; os[2] += ov.z; os[3] += ov.w;
        }
        if (two) {  // this block's record (frame M_sp), write-through for the combining workgroup
            const int64_t rec = (gb * 2 + sp) * grp + h;
            st16_sc1(make_rsrc(rec_o), (int)(4 * (rec * D + d)), __builtin_bit_cast(uint4, make_float4(os[0], os[1], os[2], os[3])));
            if (d == 0) st_sc1(reinterpret_cast<uint64_t*>(rec_ml) + rec, __builtin_bit_cast(uint64_t, make_float2(sm_mh[h], ls)));
            continue;
        }
        const float inv = 1.0f / ls;
        float o4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o4[k] = KV8 ? (os[k] * v_scale) * inv : os[k] * inv;
        *reinterpret_cast<uint2*>(row + (int64_t)b * Hq * D + (int64_t)(hq0 + h) * D + d) =
            make_uint2(pk_bf16(o4[0], o4[1]), pk_bf16(o4[2], o4[3]));
    }
    if (!two) {
        WF_STAMP(2);
        return;
    }
    // the second workgroup of the sequence to get here combines the two records
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* c = cnt + gb * kTailLine;
        const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sh_last = old == 1u;
        if (old == 1u) {  // both past the exchange: re-arm, advance the epoch
            st_sc1(c, 0u);
            st_sc1(xep + gb * kTailLine, ep);
        }
    }
    __syncthreads();
    if (!sh_last) return;
    const __amdgpu_buffer_rsrc_t rml = make_rsrc(rec_ml), ro = make_rsrc(rec_o);
    for (int idx = threadIdx.x; idx < grp * (D / 4); idx += 256) {
        const int h = idx / (D / 4), d = (idx % (D / 4)) * 4;
        const int64_t r0 = (gb * 2) * grp + h, r1 = (gb * 2 + 1) * grp + h;
        const uint4 m0 = ld16_sc1(rml, (int)(8 * (r0 & ~1)));  // (M, l) pairs of two heads
        const uint4 m1 = ld16_sc1(rml, (int)(8 * (r1 & ~1)));
        const float4 o0 = __builtin_bit_cast(float4, ld16_sc1(ro, (int)(4 * (r0 * D + d))));
        const float4 o1 = __builtin_bit_cast(float4, ld16_sc1(ro, (int)(4 * (r1 * D + d))));
        const float L0 = __uint_as_float((r0 & 1) ? m0.w : m0.y);
        const float rr = __uint_as_float((r1 & 1) ? m1.z : m1.x), L1 = __uint_as_float((r1 & 1) ? m1.w : m1.y);
        const float L = L0 * rr + L1;
        const float os[4] = {o0.x * rr + o1.x, o0.y * rr + o1.y, o0.z * rr + o1.z, o0.w * rr + o1.w};
        const float inv = 1.0f / L;
        float o4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o4[k] = KV8 ? (os[k] * v_scale) * inv : os[k] * inv;
        *reinterpret_cast<uint2*>(row + (int64_t)b * Hq * D + (int64_t)(hq0 + h) * D + d) =
            make_uint2(pk_bf16(o4[0], o4[1]), pk_bf16(o4[2], o4[3]));
    }
    WF_STAMP(2);
}

// The sequences of a batch by decreasing context (ties by index): one 1024-thread block, bitonic sort
// of (length, index) keys in LDS, B <= 2048 (longer batches keep the identity order). Launched once
// per decode step before the first layer's batched attention; every layer uses the order.
__global__ __launch_bounds__(1024) void k_seq_order(const int32_t* __restrict__ seq_lens, int B, int S,
                                                    int32_t* __restrict__ order) {
    __shared__ uint32_t key[2048];
    int n = 2;  // the smallest power of two >= B: log2(n) (log2(n) + 1) / 2 barrier steps (28 at B = 128, not 55)
    while (n < B) n <<= 1;
    for (int i = threadIdx.x; i < n; i += 1024) {
        const uint32_t len = i < B ? (uint32_t)min(max(seq_lens[i], 0), S) : 0u;
        // descending length = ascending (~len); pads (len 0, index >= B) sort last
        key[i] = i < B ? ((~len & 0xffffu) << 16) | (uint32_t)i : 0xffff0000u | (uint32_t)i;
    }
    __syncthreads();
    for (int k = 2; k <= n; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += 1024) {
                const int p = i ^ j;
                if (p > i) {
                    const uint32_t a = key[i], c = key[p];
                    const bool up = (i & k) == 0;
                    if ((a > c) == up) { key[i] = c; key[p] = a; }
                }
            }
            __syncthreads();
        }
    for (int i = threadIdx.x; i < B; i += 1024) order[i] = (int32_t)(key[i] & 0xffffu);
}

int seq_order(const int32_t* seq_lens, int B, int S, int32_t* order, hipStream_t st) {
    if (B > 2048 || S > 65535) return WF_OK;  // identity order stays (set at model creation)
    hipLaunchKernelGGL(k_seq_order, dim3(1), dim3(1024), 0, st, seq_lens, B, S, order);
    return check_launch("seq_order");
}

// ---------------------------------------------------------------------------------------------
// Prefill (causal) attention on the tile-layout K/V caches, after the prefill QKV GEMM has written
// the prompt's K/V rows: query row m (a prompt token of KV slot row_slot[m] at position
// row_pos[m]) attends to keys [0, row_pos[m]] of its slot, with the reference's SDPA arithmetic
// (k_attn_prefill_sdpa below; every K/V element type, round 6 -- the round-1..5 row-split
// exact-softmax kernel k_attn_prefill that one-byte caches took is gone).
// ---------------------------------------------------------------------------------------------
constexpr int kPfMaxTiles = 1024;  // 32-key tiles per sequence (max_seq <= 32768; page ids in LDS)

// Prefill attention on 32 x 32 bf16 matrix cores (k_attn_prefill_sdpa, the default for bf16 K/V):
// block = one row group of kPrefillRowGroup = 32 consecutive rows of one slot x kv head g; wave w
// takes tokens 8 w .. 8 w + 7 x the group's 4 query heads = 32 query columns (column c = token
// 8 w + c / 4, head c % 4). K/V tiles (32 keys) are staged once per block in a 4 x 16 KiB LDS ring by
// LDS-DMA, each wave a quarter, P - 2 stages in flight beyond the one being read:
//   S^T (32 keys x 32 queries) = K . Q^T: 8 v_mfma_f32_32x32x16_bf16 (K fragments = 16 bytes of one
//       key's 8 dims, ds_read_b128; Q^T fragments in registers for the whole key range); lane (c, h)
//       holds keys (j & 7) + 8 h + 16 (j >> 3) of column c, so a column's max / sum needs one
//       v_permlane32_swap;
//   O^T (128 dims x 32 queries) += V^T . P^T: P^T's fragments are the score lanes as they stand
//       (the QK MFMA takes the keys permuted so that k-slot i of lane half h is key 16 s + 8 h + i),
//       V^T's fragments one 16-byte ds_read of the V tile layout each.
// Per-column causal limit (masking only where a tile crosses it), V rows past the block's last
// position zeroed. A column's result depends only on its own key range, so chunked prefill stays
// bit-exact.
constexpr int kFaStages = 4;  // 64 KiB ring + page ids: two blocks per CU
typedef __bf16 v8bf_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));
__device__ __forceinline__ float swap32_max(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap32_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Prefill attention with the reference's SDPA arithmetic (k_attn_sdpa's comment): the decode loop
// the reference runs for a prompt computes each position's attention over keys [0, pos] in 512-key
// blocks with a running max (layout above; XCD-chunked block order), per 512-key block in two passes
// over its tiles:
//   pass 1 (ring stages of TWO tiles' K): S^T = K . Q^T (two 64-dim MFMA chains), the column's block
//     maximum (causal limit per column);
//   then M_c = max(M_{c-1}, block max), r = expf(M_{c-1} - M_c) rescales the column's O^T and l;
//   pass 2 (stages of one tile's K + V): the same S^T again, e = fexp_u20 / expf of (s - M_c) (the
//     16-key vector part / the tail of the column's block), l += e, O^T += V^T . bf16(e)^T (one MFMA
//     term per k-step: P is bf16, 24 instead of 32 MFMAs per tile).
// Every stage is 16 KiB and four 1-KiB DMAs per wave (bf16 K/V). One-byte K/V (KV8 = 1 e4m3, 2 int8;
// kv_cache tile layouts with one byte per element): the same stages at half the bytes (two 1-KiB
// DMAs per wave), every K / V^T fragment 8 codes widened to bf16 in registers exactly as the decode
// kernels do (KvFrag<KV8>); the K scale is folded into `scale`, the V scale multiplies the output
// (k_attn_sdpa_mfma's arithmetic), so a prompt and its decode steps share the SDPA semantics.
// F64: q.k as eight zero-C 16-product MFMA partials summed in f64 in both passes (study: 109 vs 307
// of 911360 outputs off the oracle; 2.7x the kernel time on the round-6 build, 441 -> 1,178 us).
template <int KV8, bool F64>
__global__ __launch_bounds__(256, 2) void k_attn_prefill_sdpa(const uint16_t* __restrict__ q, int64_t q_rs,
                                                              const uint16_t* __restrict__ K,
                                                              const uint16_t* __restrict__ Vt, int64_t kv_sb,
                                                              int64_t kv_sh, const int32_t* __restrict__ row_pos,
                                                              const int32_t* __restrict__ row_slot, int M,
                                                              float scale, const int32_t* __restrict__ pt, int pps,
                                                              int npages, int64_t kv_pgs, uint16_t* __restrict__ out,
                                                              int64_t o_rs, int xchunk, float v_scale) {
    constexpr int D = 128, P = kFaStages;
    constexpr int kSlot = 16384;
    constexpr int EB = KV8 ? 1 : 2;            // bytes per K / V element
    constexpr int NDMA = 2 * EB;               // 1-KiB DMAs per wave per stage (16 KiB bf16, 8 KiB one-byte)
    constexpr int TB = 4096 * EB;              // bytes of one 32-key K or V tile
    using KF = KvFrag<KV8>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[P * kSlot];
    __shared__ int s_page[kPfMaxTiles];
    const int nrb = M / 32;
    int g, rbi;
    if (xchunk > 0) {
        const int b = blockIdx.x, item = (b & 7) * xchunk + (xchunk - 1 - (b >> 3));
        g = item / nrb;
        rbi = item - g * nrb;
    } else {
        g = blockIdx.y;
        rbi = nrb - 1 - (int)blockIdx.x;
    }
    const int hq0 = g * 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
    const int rb = rbi * 32;
    const int slot = __builtin_amdgcn_readfirstlane(row_slot[rb]);
    const int qrow = rb + 8 * wave + (c >> 2);
    const int lim_q = row_pos[qrow] + 1;  // keys [0, lim_q) of column c
    int lim_b = 0;
    for (int t = 0; t < 32; ++t) lim_b = max(lim_b, row_pos[rb + t] + 1);
    lim_b = __builtin_amdgcn_readfirstlane(min(lim_b, 32 * min(pps, kPfMaxTiles)));
    v8bf_t qf[8];  // Q^T fragments: column c, dims 16 s + 8 h .. + 7
    {
        const uint16_t* qp = q + (int64_t)qrow * q_rs + (int64_t)(hq0 + (c & 3)) * D + 8 * h;
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) qf[s2] = __builtin_bit_cast(v8bf_t, *reinterpret_cast<const uint4*>(qp + 16 * s2));
    }
#pragma unroll
    for (int s2 = 0; s2 < 8; ++s2) asm volatile("" : "+v"(qf[s2]));
    const int ntiles = (lim_b + 31) >> 5;
    const int NB = (ntiles + 15) >> 4;
    // (element offsets; one-byte caches index bytes, as the decode kernels)
    const uint8_t* Kg = reinterpret_cast<const uint8_t*>(K) + ((pt ? 0 : (int64_t)slot * kv_sb) + g * kv_sh) * EB + lane * 16;
    const uint8_t* Vg = reinterpret_cast<const uint8_t*>(Vt) + ((pt ? 0 : (int64_t)slot * kv_sb) + g * kv_sh) * EB + lane * 16;
    if (pt) {
        for (int t = threadIdx.x; t < ntiles; t += 256) s_page[t] = min(max(pt[(int64_t)slot * pps + t], 0), npages - 1);
        __syncthreads();
    }
    // stage i -> (block, pass, tiles): a full block has 8 pass-1 stages (two tiles' K each) then 16
    // pass-2 stages (one tile's K + V); the last block s1 = ceil(nt / 2) + nt
    const int nt_last = ntiles - 16 * (NB - 1), s1_last = (nt_last + 1) >> 1;
    const int nstages = 24 * (NB - 1) + s1_last + nt_last;
    auto stage_of = [=](int i, int& cb, int& pass, int& ta, int& tb) __attribute__((always_inline)) {
        cb = min(i / 24, NB - 1);
        const int j = i - 24 * cb;
        const int nt = cb == NB - 1 ? nt_last : 16, s1 = (nt + 1) >> 1;
        if (j < s1) {
            pass = 1;
            ta = 16 * cb + 2 * j;
            tb = min(ta + 1, 16 * cb + nt - 1);
        } else {
            pass = 2;
            ta = tb = 16 * cb + (j - s1);
        }
    };
    auto issue = [=](int i) __attribute__((always_inline)) {
        int cb, pass, ta, tb;
        stage_of(i, cb, pass, ta, tb);
        const int64_t ba = (pt ? (int64_t)s_page[ta] * kv_pgs : (int64_t)ta * 4096) * EB;
        const int64_t bb = (pt ? (int64_t)s_page[tb] * kv_pgs : (int64_t)tb * 4096) * EB;
        uint8_t* st = ring + (i % P) * kSlot;
        const uint8_t* second = pass == 1 ? Kg + bb : Vg + bb;
        constexpr int HALF = 2 * NDMA;  // KiB of the stage's first tile (4 waves x NDMA KiB per stage)
#pragma unroll
        for (int jj = 0; jj < NDMA; ++jj) {
            const int j = wave * NDMA + jj;
            glds16_asm(j < HALF ? Kg + ba + j * 1024 : second + (j - HALF) * 1024, st + j * 1024);
        }
    };
    const int o = (c & ~12) | ((c & 4) << 1) | ((c & 8) >> 1);
    const int koff = ((((o >> 2) & 1) * 16 + h) * 16 + 4 * (o >> 3) + (o & 3)) * 8 * EB;
    // S^T of one tile, raw dots (unscaled): two 64-dim MFMA accumulator chains and one fp32 add.
    // Measured against the oracle on the same caches (tests/test_gpu_configs.py
    // test_prefill_attention_vs_oracle_sdpa; 2 x 2048 rows, 911360 sampled outputs): these chains
    // 307 off and 54 of 2048 layer-1 positions > 1e-3 in test_prefill_8x2048_full_width_vs_oracle;
    // 8 zero-C partials in a pairwise fp32 tree 292 (+80 us per layer); the 8 partials summed in f64
    // in pass 2 only 274 / 54, in pass 1 only 192 / 58, in both passes 109 / 27 (the batched decode
    // kernel's level: 11 positions) at +30 % kernel time and 216 B of scratch. The matrix cores align
    // each 8-product group to its largest product and truncate (tools/ubench/mfma_round.hip), and
    // every fp32 partial sum rounds; the block max M_c enters every probability (l is summed from
    // the unrounded e, P.V from the rounded P), so pass 1 needs the precision as much as pass 2.
    auto kfrag = [=](const uint8_t* p) __attribute__((always_inline)) {  // 8 keys' or dims' bf16 values
        if constexpr (KV8) return KF::bf(*reinterpret_cast<const uint2*>(p));
        else return *reinterpret_cast<const uint4*>(p);
    };
    auto qk = [=](const uint8_t* st, float (&x)[16]) __attribute__((always_inline)) {
        uint4 kf[8];
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2) kf[s2] = kfrag(st + koff + s2 * 256 * EB);
        if constexpr (F64) {
            double dd[16];
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2) {
                const v16f_t pr = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf_t, kf[s2]), qf[s2],
                                                                          v16f_t{}, 0, 0, 0);
#pragma unroll
                for (int e = 0; e < 16; ++e) dd[e] = s2 ? dd[e] + (double)pr[e] : (double)pr[e];
            }
#pragma unroll
            for (int e = 0; e < 16; ++e) x[e] = (float)dd[e];
        } else {
            v16f_t a0 = {}, a1 = {};
#pragma unroll
            for (int s2 = 0; s2 < 8; s2 += 2) {
                a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf_t, kf[s2]), qf[s2], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf_t, kf[s2 + 1]), qf[s2 + 1], a1, 0, 0, 0);
            }
            const v16f_t t = a0 + a1;
#pragma unroll
            for (int e = 0; e < 16; ++e) x[e] = t[e];
        }
    };
    float m_run = -INFINITY, l_run = 0.f, bmax = -INFINITY;
    int vmin = 0;
    const int lim_lo = (int)-wave_max((float)-lim_q);  // the wave's smallest causal limit
    v16f_t oacc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) oacc[mt][e] = 0.f;
#pragma unroll
    for (int i = 0; i < P - 1; ++i)
        if (i < nstages) issue(i);
    auto wait_through = [=](int i, int last_issued) __attribute__((always_inline)) {
        const int pending = min(nstages - 1, last_issued) - i;
        if (pending <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (NDMA == 2) {
            if (pending == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else if (pending == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else if (pending == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (pending == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    // one loop per pass of each block (a single stage loop with a pass switch made the register
    // allocator copy the 64 O accumulators at every stage)
    int i = 0;
    for (int cb = 0; cb < NB; ++cb) {
        const int nt = cb == NB - 1 ? nt_last : 16, s1 = (nt + 1) >> 1, blk0 = 512 * cb;
        for (int jj = 0; jj < s1; ++jj, ++i) {
            wait_through(i, i + P - 2);  // stage i landed, and everyone is done with stage i - 1's slot
            if (i + P - 1 < nstages) issue(i + P - 1);
            const uint8_t* st = ring + (i % P) * kSlot;
            const int ta = 16 * cb + 2 * jj, tb = min(ta + 1, 16 * cb + nt - 1);
            // this column's maximum over its keys of the stage's tiles
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int t = u ? tb : ta;
                if (u && tb == ta) break;  // wave-uniform
                if (32 * t >= lim_b) break;
                float x[16];
                qk(st + u * TB, x);
                if (32 * t + 32 <= lim_lo) {  // below every column's limit (wave-uniform): no masks
#pragma unroll
                    for (int j = 0; j < 16; ++j) bmax = fmaxf(bmax, x[j]);
                } else {
                    const int lim = lim_q - 32 * t - 8 * h;
#pragma unroll
                    for (int j = 0; j < 16; ++j)
                        if ((j & 7) + 16 * (j >> 3) < lim) bmax = fmaxf(bmax, x[j]);
                }
            }
        }
        {  // M_c, rescale O and l (the max of the raw dots, scaled once: rounding a product is monotone)
            const float mn = fmaxf(m_run, swap32_max(bmax) * scale);
            vmin = (int)-wave_max((float)-(min(512, lim_q - blk0) & ~15));  // the wave's smallest vector part
            const float r = expf_rn(m_run - mn);  // 0 before the first block, 1 if no key of it
            m_run = mn;
            bmax = -INFINITY;
            l_run *= r;
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int e = 0; e < 16; ++e) oacc[mt][e] *= r;
        }
        for (int jj = 0; jj < nt; ++jj, ++i) {
            wait_through(i, i + P - 2);
            if (i + P - 1 < nstages) issue(i + P - 1);
            const uint8_t* st = ring + (i % P) * kSlot;
            const int bs = 32 * (16 * cb + jj);
            if (bs >= lim_b) continue;  // wave-uniform (the block's tiles past the group's last row)
                // V^T fragments (dim 32 mt + c, keys 16 s + 8 h + 0..7): issued first (one-byte caches:
                // the raw codes, masked and widened at their MFMA)
                uint4 vv[4][2];
                uint2 vc[KV8 ? 4 : 1][KV8 ? 2 : 1];
    #pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    const int d = 32 * mt + c, n = d >> 4, l = d & 15;
    #pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const uint8_t* vp = st + TB + ((n * 4 + 2 * s2 + h) * 16 + l) * 8 * EB;
                        if constexpr (KV8) vc[mt][s2] = *reinterpret_cast<const uint2*>(vp);
                        else vv[mt][s2] = *reinterpret_cast<const uint4*>(vp);
                    }
                }
                float x[16];
                qk(st, x);
                const int lim = lim_q - bs - 8 * h;
                const int nbc = min(512, lim_q - blk0), vbnd = nbc & ~15;  // the column's block: vector part
                uint32_t pk[8];
                // every key of the tile below every column's causal limit and inside its block's 16-wide
                // vector part (the common case): fexp_u20 only, no per-key bounds
                // the lane's 16 exponentials of the tile summed as a pairwise tree, then into l: 16
                // sequential adds per 512-key block instead of 256 (the one long fp32 chain of the kernel;
                // it moved 2x the decode kernel's share of outputs off the oracle)
                float ee[16];
                if (bs - blk0 + 32 <= vmin) {  // packed fp32 pairs (v_pk_mul / v_pk_add / v_pk_fma)
                    const f32x2_t sc2 = {scale, scale}, m2 = {m_run, m_run};
    #pragma unroll
                    for (int j = 0; j < 16; j += 2) {
                        const f32x2_t e2 = fexp_u20_pk(f32x2_t{x[j], x[j + 1]} * sc2 - m2);
                        ee[j] = e2.x;
                        ee[j + 1] = e2.y;
                    }
                } else {
    #pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const int kk = (j & 7) + 8 * h + 16 * (j >> 3);  // key within the tile
                        const int kb = bs - blk0 + kk;                   // key within the block
                        const float xv = x[j] * scale - m_run;
                        ee[j] = kk < lim + 8 * h ? (kb < vbnd ? fexp_u20(xv) : expf_rn(xv)) : 0.f;
                    }
                }
    #pragma unroll
                for (int j = 0; j < 16; j += 2) pk[j >> 1] = pk_bf16(ee[j], ee[j + 1]);
    #pragma unroll
                for (int w2 = 8; w2 >= 1; w2 >>= 1)
    #pragma unroll
                    for (int j = 0; j < w2; ++j) ee[j] += ee[j + w2];
                l_run += ee[0];
                uint4 pu0 = make_uint4(pk[0], pk[1], pk[2], pk[3]), pu1 = make_uint4(pk[4], pk[5], pk[6], pk[7]);
                reg_fence(pu0);  // packed once (hipcc otherwise re-packed P before every P.V MFMA)
                reg_fence(pu1);
                const v8bf_t pb0 = __builtin_bit_cast(v8bf_t, pu0), pb1 = __builtin_bit_cast(v8bf_t, pu1);
                const int limv = lim_b - bs - 8 * h;  // V keys past the block's last position: zero (stale)
                const bool vtail = lim_b - bs < 40;   // wave-uniform: some lane's V keys cross the block end
    #pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
    #pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        uint4 a;
                        if constexpr (KV8) {
                            a = KF::bf(vtail ? KF::mask(vc[mt][s2], limv - 16 * s2) : vc[mt][s2]);
                        } else {
                            a = vv[mt][s2];
                            if (vtail) {
                                const int k0 = 16 * s2;
                                a.x &= (k0 < limv ? 0xffffu : 0u) | (k0 + 1 < limv ? 0xffff0000u : 0u);
                                a.y &= (k0 + 2 < limv ? 0xffffu : 0u) | (k0 + 3 < limv ? 0xffff0000u : 0u);
                                a.z &= (k0 + 4 < limv ? 0xffffu : 0u) | (k0 + 5 < limv ? 0xffff0000u : 0u);
                                a.w &= (k0 + 6 < limv ? 0xffffu : 0u) | (k0 + 7 < limv ? 0xffff0000u : 0u);
                            }
                        }
                        oacc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf_t, a), s2 ? pb1 : pb0,
                                                                           oacc[mt], 0, 0, 0);
                    }
                }

        }
    }
    const float inv = 1.0f / swap32_sum(l_run);
    if constexpr (KV8 != 0) {  // the V scale on the unnormalised sums, then 1 / l (k_attn_sdpa_mfma's order)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int e = 0; e < 16; ++e) oacc[mt][e] *= v_scale;
    }
    if (qrow < M) {
        uint16_t* orow = out + (int64_t)qrow * o_rs + (int64_t)(hq0 + (c & 3)) * D;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int u = 0; u < 4; ++u)  // dims 32 mt + 8 u + 4 h .. + 3
                *reinterpret_cast<uint2*>(orow + 32 * mt + 8 * u + 4 * h) =
                    make_uint2(pk_bf16(oacc[mt][4 * u] * inv, oacc[mt][4 * u + 1] * inv),
                               pk_bf16(oacc[mt][4 * u + 2] * inv, oacc[mt][4 * u + 3] * inv));
    }
}

// Contract of prefill_attention, checked by wf_model_prefill before its first launch (so a refused
// call leaves the cache untouched).
int prefill_attention_check(int Hq, int Hkv, int pps) {
    if (Hq != 4 * Hkv) {
        set_error("prefill_attention: GQA group %d != 4 not supported", Hq / Hkv);
        return WF_EINVAL;
    }
    if (pps > kPfMaxTiles) {
        set_error("prefill_attention: max_seq %d > %d keys", 32 * pps, 32 * kPfMaxTiles);
        return WF_EINVAL;
    }
    return WF_OK;
}

// k_attn_prefill_sdpa for every K/V element type (bf16, e4m3, int8), its blocks in XCD-chunked order
// when the items split evenly over the 8 XCDs (each XCD streams one (slot, kv head) K/V at a time
// from its own L2: 333 -> 250 us per layer at 8 x 2048). Rows come in aligned groups of 32 of one slot
// (wf_model_prefill checks M % kPrefillRowGroup == 0).
#ifndef WF_PF_QK_F64  // study: q.k partials in f64 in both passes (round 6, same box: 441 -> 1,178 us
#define WF_PF_QK_F64 0   // per layer; 307 -> 109 sampled outputs, 54 -> 27 layer-1 positions off the oracle)
#endif
int prefill_attention(const uint16_t* q, int64_t q_rs, const uint16_t* k, const uint16_t* v, int64_t kv_sb,
                      int64_t kv_sh, int Hq, int Hkv, const int32_t* row_pos, const int32_t* row_slot, int M,
                      float sm_scale, const int32_t* pt, int pps, int npages, int64_t kv_pgs, uint16_t* out,
                      int64_t o_rs, hipStream_t st, int kv8, float k_scale, float v_scale) {
    if (int rc = prefill_attention_check(Hq, Hkv, pps)) return rc;
    if (M % 32 != 0) {
        set_error("prefill_attention: rows %d not a multiple of 32", M);
        return WF_EINVAL;
    }
    constexpr bool F = WF_PF_QK_F64;
    const int items = (M / 32) * Hkv, xchunk = items % 8 == 0 ? items / 8 : 0;
    const dim3 grid = xchunk ? dim3(items) : dim3(M / 32, Hkv);
    auto kern = kv8 == 2 ? k_attn_prefill_sdpa<2, F> : kv8 == 1 ? k_attn_prefill_sdpa<1, F> : k_attn_prefill_sdpa<0, F>;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, q, q_rs, k, v, kv_sb, kv_sh, row_pos, row_slot, M,
                       kv8 ? sm_scale * k_scale : sm_scale, pt, pps, npages, kv_pgs, out, o_rs, xchunk,
                       kv8 ? v_scale : 1.0f);
    return check_launch("prefill_attention");
}

int decode_attention_partials(const uint16_t* q, int64_t q_sb, const uint16_t* k, const uint16_t* v, int64_t kv_sb,
                              int64_t kv_sh, int B, int Hq, int Hkv, int S, const int32_t* seq_lens, float sm_scale,
                              float2* ml, float* o, hipStream_t st, bool kv_tiled, const int32_t* pt, int pps,
                              int npages, int64_t kv_pgs, int kv8, float k_scale, float v_scale,
                              uint16_t* merged_row, unsigned* merge_cnt, uint64_t* xmax, const int32_t* order,
                              const SdpaBufs* sb) {
    const int grp = Hq / Hkv;
    if (grp > 8) {
        set_error("decode_attention_partials: GQA group %d > 8", grp);
        return WF_EINVAL;
    }
    if (B < 16 || !kv_tiled) {
        // the reference's SDPA semantics (k_attn_sdpa): one block per (split, query head, sequence),
        // the head's records merged into the bf16 row merged_row in the launch
        if (!merged_row || !merge_cnt || !xmax || pt) {
            set_error("decode_attention_partials: batch < 16 / untiled caches need the merged-row, arrival and exchange buffers, no page table");
            return WF_EINVAL;
        }
        if (S > kSdpaMaxSeq) {
            set_error("decode_attention_partials: max_seq %d > %d at batch < 16 / untiled caches", S, kSdpaMaxSeq);
            return WF_EINVAL;
        }
        // every split of a head polls its siblings: a launch holds only blocks the chip keeps resident
        // at once (half the occupancy API's count), whole sequences per launch
        static int cap = 0;
        if (!cap) {
            int dev = 0, ncu = 0, per = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_attn_sdpa, kAttnPartThreads, 0) != hipSuccess) {
                set_error("decode_attention_partials: occupancy query failed");
                return WF_EHIP;
            }
            cap = std::max(1, per * ncu / 2);
        }
        const int per_seq = kAttnPartSplits1 * Hq;
        if (per_seq > cap) {
            set_error("decode_attention_partials: %d blocks per sequence exceed the resident bound %d", per_seq, cap);
            return WF_EINVAL;
        }
        const int chunk = std::max(1, cap / per_seq);
        unsigned* xep = merge_cnt + (int64_t)B * Hq * kTailLine;  // per-head launch epochs
        uint64_t* xo = xmax + sdpa_xmax_granules(B, Hq);             // merge granules
        for (int b0 = 0; b0 < B; b0 += chunk) {
            hipLaunchKernelGGL(k_attn_sdpa, dim3(kAttnPartSplits1, Hq, std::min(chunk, B - b0)), dim3(kAttnPartThreads), 0, st,
                               q, q_sb, k, v, kv_sb, kv_sh, Hq, Hkv, S, seq_lens, sm_scale, b0, xmax, ml, o, merged_row,
                               xo, xep, sb ? sb->err : nullptr, sb ? sb->stall : 0);
            if (int rc = check_launch("decode_attention_partials")) return rc;
        }
        return WF_OK;
    }
    // batched, tile-layout caches: one block per (kv head, sequence) walking its 512-key blocks in
    // order (k_attn_sdpa_mfma), the normalised bf16 rows into merged_row
    if (S % 32 != 0) {
        set_error("decode_attention_partials: tiled K/V need S %% 32 == 0 (S=%d)", S);
        return WF_EINVAL;
    }
    if (!merged_row || grp > kAttnMfmaMaxGrp) {
        set_error("decode_attention_partials: batched attention needs the merged-row buffer and a GQA group <= %d",
                  kAttnMfmaMaxGrp);
        return WF_EINVAL;
    }
    if (kAttnSplit2 && (!merge_cnt || !xmax)) {
        set_error("decode_attention_partials: batched attention needs the arrival and exchange buffers");
        return WF_EINVAL;
    }
    const dim3 grid(Hkv, B, kAttnSplit2 ? 2 : 1);
    const bool g4 = Hq == 4 * Hkv;
    const float ss = kv8 ? sm_scale * k_scale : sm_scale, vs = kv8 ? v_scale : 1.0f;
    auto kern = kv8 == 2 ? (g4 ? k_attn_sdpa_mfma<2, 4> : k_attn_sdpa_mfma<2, 0>)
              : kv8      ? (g4 ? k_attn_sdpa_mfma<1, 4> : k_attn_sdpa_mfma<1, 0>)
                         : (g4 ? k_attn_sdpa_mfma<0, 4> : k_attn_sdpa_mfma<0, 0>);
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, q, q_sb, k, v, kv_sb, kv_sh, Hq, Hkv, S, seq_lens, ss, pt, pps,
                       npages, kv_pgs, vs, merged_row, order, ml, o, merge_cnt, merge_cnt + (int64_t)B * Hq * kTailLine,
                       xmax, sb ? sb->err : nullptr);
    return check_launch("decode_attention_partials");
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

// The same scatter / gather on the decode engine's own paged pool (the pool wf_model_desc.page_table
// addresses): page = 32 tokens of every kv head in the K / V tile layouts (wf_norm.h k_tile_off /
// v_tile_off), token row t of k / v ([T][H * D]) at page pages[t], slot slots[t] < 32 -- the
// reference's slot_indices (tests/test_kv_cache_cpp.py:80-126). One block per (token, K | V).
__global__ void k_kv_tile_copy(uint16_t* __restrict__ kpool, uint16_t* __restrict__ vpool, const uint16_t* __restrict__ src_k,
                               const uint16_t* __restrict__ src_v, uint16_t* __restrict__ dst_k, uint16_t* __restrict__ dst_v,
                               const int32_t* __restrict__ pages, const int32_t* __restrict__ slots, int P, int H, int scatter,
                               int32_t* __restrict__ bad) {
    constexpr int D = 128;
    const int t = blockIdx.x, kv = blockIdx.y;
    const int page = pages[t], o = slots[t];
    if (page < 0 || page >= P || o < 0 || o >= 32) {
        if (threadIdx.x == 0 && kv == 0 && bad) atomicAdd(bad, 1);
        return;
    }
    uint16_t* pool = (kv ? vpool : kpool) + (int64_t)page * H * 32 * D;
    for (int e = threadIdx.x; e < H * D; e += blockDim.x) {
        const int h = e / D, d = e - h * D;
        const int64_t off = (int64_t)h * 32 * D + (kv ? v_tile_off(o, d) : k_tile_off(o, d));
        if (scatter) pool[off] = (kv ? src_v : src_k)[(int64_t)t * H * D + e];
        else (kv ? dst_v : dst_k)[(int64_t)t * H * D + e] = pool[off];
    }
}

struct AttnArgs {
    const void* q; int qdt; int64_t q_sb, q_sh;
    const void* k; const void* v; int64_t kv_sb, kv_sh, kv_st; float ks, vs;
    int Hq, Hkv, S; const int32_t* sl; float sm; int NS; unsigned* cnt; float* part;
    void* out; int odt; int64_t o_sb, o_sh;
};

template <int D, int G, int KVDT>
static void launch_attn(dim3 grid, hipStream_t st, const AttnArgs& a) {
    hipLaunchKernelGGL((k_attn_split<D, G, KVDT>), grid, dim3(kAttnThreads), 0, st, a.q, a.qdt, a.q_sb, a.q_sh, a.k,
                       a.v, a.kv_sb, a.kv_sh, a.kv_st, a.ks, a.vs, a.Hq, a.Hkv, a.S, a.sl, a.sm, a.NS, a.cnt, a.part,
                       a.out, a.odt, a.o_sb, a.o_sh);
}

template <int D, int G>
static int dispatch_kvdt(int kvdt, dim3 grid, hipStream_t st, const AttnArgs& a) {
    switch (kvdt) {
        case DT_BF16: launch_attn<D, G, DT_BF16>(grid, st, a); return 0;
        case DT_F16: launch_attn<D, G, DT_F16>(grid, st, a); return 0;
        case DT_F32: launch_attn<D, G, DT_F32>(grid, st, a); return 0;
        case DT_I8: launch_attn<D, G, DT_I8>(grid, st, a); return 0;
    }
    return 1;
}

template <int D>
static int dispatch_g(int grp, int kvdt, dim3 grid, hipStream_t st, const AttnArgs& a) {
    if (grp == 1) return dispatch_kvdt<D, 1>(kvdt, grid, st, a);
    if (grp == 2) return dispatch_kvdt<D, 2>(kvdt, grid, st, a);
    if (grp <= 4) return dispatch_kvdt<D, 4>(kvdt, grid, st, a);
    if (grp <= 8) return dispatch_kvdt<D, 8>(kvdt, grid, st, a);
    return 1;
}

// ws = [tickets: B*Hkv uint32, 256-B aligned block][partials: B*Hq*NS*(D+2) f32]. The tickets must
// be zero before the first launch; every launch leaves them zero again.
int decode_attention_impl(const void* q, int q_dtype, int64_t q_sb, int64_t q_sh, const void* k, const void* v,
                          int kv_dtype, int64_t kv_sb, int64_t kv_sh, int64_t kv_st, float k_scale, float v_scale, int B,
                          int Hq, int Hkv, int D, int S, const int32_t* seq_lens, float sm_scale, void* out,
                          int out_dtype, int64_t o_sb, int64_t o_sh, void* ws, hipStream_t st) {
    WF_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128, "decode_attention: head_dim %d unsupported", D);
    const int NS = attn_splits(D, S);
    WF_REQUIRE(NS <= kAttnMaxSplits, "decode_attention: S=%d exceeds %d keys", S, kAttnMaxSplits * attn_split_len(D));
    WF_REQUIRE((int64_t)B * Hq * NS * attn_rec_floats(D) * 4 < 0x7fffffff, "decode_attention: workspace > 2 GiB");
    AttnArgs a{q, q_dtype, q_sb, q_sh, k, v, kv_sb, kv_sh, kv_st, k_scale, v_scale, Hq, Hkv, S, seq_lens, sm_scale, NS,
               reinterpret_cast<unsigned*>(ws),
               reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(ws) + attn_cnt_bytes(B, Hkv)), out, out_dtype,
               o_sb, o_sh};
    const dim3 grid(NS, Hkv, B);
    const int grp = Hq / Hkv;
    int bad = 1;
    switch (D) {
        case 16: bad = dispatch_g<16>(grp, kv_dtype, grid, st, a); break;
        case 32: bad = dispatch_g<32>(grp, kv_dtype, grid, st, a); break;
        case 64: bad = dispatch_g<64>(grp, kv_dtype, grid, st, a); break;
        case 128: bad = dispatch_g<128>(grp, kv_dtype, grid, st, a); break;
    }
    WF_REQUIRE(!bad, "decode_attention: unsupported D=%d / group=%d / kv dtype=%d", D, grp, kv_dtype);
    return check_launch("decode_attention");
}

}  // namespace wf

WF_STAMP_READER(wf_debug_stamps_attn)

using namespace wf;

extern "C" {

int64_t wf_decode_attention_ws_bytes(int B, int Hq, int D, int S) {
    if (D <= 0 || D % 8) return 0;
    return attn_cnt_bytes(B, Hq) + (int64_t)B * Hq * attn_splits(D, S) * attn_rec_floats(D) * (int64_t)sizeof(float);
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
    WF_HIP(hipMemsetAsync(ws, 0, attn_cnt_bytes(B, Hkv), as_stream(stream)));  // tickets (graph-capturable)
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

static int kv_tile_common(void* kpool, void* vpool, int num_pages, int H, int D, const void* k, const void* v, void* ko,
                          void* vo, const int32_t* pages, const int32_t* slots, int T, int32_t* bad, int scatter,
                          void* stream) {
    WF_REQUIRE(kpool && vpool && pages && slots && T >= 0 && num_pages > 0 && H > 0, "kv_tiles: bad arguments");
    WF_REQUIRE(D == 128, "kv_tiles: the engine pool's tile layouts need head_dim 128 (got %d)", D);
    if (T == 0) return WF_OK;
    hipLaunchKernelGGL(k_kv_tile_copy, dim3(T, 2), dim3(256), 0, as_stream(stream), (uint16_t*)kpool, (uint16_t*)vpool,
                       (const uint16_t*)k, (const uint16_t*)v, (uint16_t*)ko, (uint16_t*)vo, pages, slots, num_pages, H,
                       scatter, bad);
    return check_launch("kv_tile_copy");
}

int wf_kv_scatter_tiles(void* k_pool, void* v_pool, int num_pages, int H, int D, const uint16_t* k, const uint16_t* v,
                        const int32_t* pages, const int32_t* slots, int T, int32_t* bad, void* stream) {
    WF_REQUIRE(k && v, "kv_scatter_tiles: null k/v");
    return kv_tile_common(k_pool, v_pool, num_pages, H, D, k, v, nullptr, nullptr, pages, slots, T, bad, 1, stream);
}

int wf_kv_gather_tiles(const void* k_pool, const void* v_pool, int num_pages, int H, int D, uint16_t* k_out,
                       uint16_t* v_out, const int32_t* pages, const int32_t* slots, int T, int32_t* bad, void* stream) {
    WF_REQUIRE(k_out && v_out, "kv_gather_tiles: null outputs");
    return kv_tile_common(const_cast<void*>(k_pool), const_cast<void*>(v_pool), num_pages, H, D, nullptr, nullptr, k_out,
                          v_out, pages, slots, T, bad, 0, stream);
}

int wf_kv_gather(const void* pool, int elem_bytes, int max_pages, int L, int H, int D, void* k_out, void* v_out,
                 const int32_t* pages, int T, int layer, int32_t* bad, void* stream) {
    WF_REQUIRE(k_out && v_out, "kv_gather: null outputs");
    return kv_page_common((uint8_t*)pool, elem_bytes, max_pages, L, H, D, nullptr, nullptr, k_out, v_out, pages, T,
                          layer, bad, 0, stream);
}

}  // extern "C"
