// wf_norm.h -- block-level RMSNorm + int8 activation quantizer, the in-launch hand-off helpers
// (launch tickets) and the diagnostic stamp facility of the fused decode step (gfx950).
//
// At batch 1 every GEMV block normalises + quantises its input row itself, straight into its LDS
// activation image, while its first weight chunks are in flight (k_gemv's prologue); at larger
// batch one k_rownorm launch does it once per row. Hand-off protocol of the launch tickets
// (MI355X_MICROARCH.md, Valid forms row 1): every block stores write-through (sc1), drains
// (s_waitcnt vmcnt(0)) in every storing wave, meets at a barrier, one lane bumps an agent-scope
// ticket; the block whose add returns n-1 reads with sc1 loads and re-arms the ticket.
#pragma once
#include "wf_device.h"

namespace wf {

template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_sc1(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
// 16-byte write-through store / L1-bypassing load (aux 16 = sc1 on gfx950)
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, uint4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, byte_off, 0, 16);
}
__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}

// Producer side of the launch ticket: all of this block's sc1 stores must be issued before the
// call. Arrivals are spread over kTicketShards counters, each on its own 128-byte line (memory-side
// atomics serialise per LINE at ~88 per us: 501 LM-head arrivals on 32 shards packed into one line
// queued for ~6 us, the median block's arrival in the in-graph stamps); the last arriver of each
// shard re-arms its shard and relays to the top counter (a line of its own). Returns true in exactly
// one block of the launch (the last arriver), which must call ticket_rearm() when done. `t` points
// at kTicketWords words.
#ifndef WF_TICKET_LINE  // study: 1 = the shards packed into one line (round 5)
#define WF_TICKET_LINE 32
#endif
constexpr int kTicketShards = 32;
constexpr int kTicketLine = WF_TICKET_LINE;  // words between shards
constexpr int kTicketWords = (kTicketShards + 1) * 32;  // words reserved per ticket (256-byte multiple)

// `idx` in [0, n_blocks) names the arriving block within the ticket's arrival set.
__device__ __forceinline__ bool ticket_arrive(unsigned* t, unsigned n_blocks, unsigned idx, int* sh_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned bid = idx;
        const unsigned nsh = n_blocks < (unsigned)kTicketShards ? n_blocks : (unsigned)kTicketShards;
        const unsigned sh = bid % nsh;
        const unsigned members = (n_blocks - sh + nsh - 1) / nsh;  // blocks with bid % nsh == sh
        bool last = false;
        unsigned* ws = t + sh * kTicketLine;
        const unsigned old = __hip_atomic_fetch_add(ws, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == members - 1u) {
            st_sc1(ws, 0u);  // every member of this shard has arrived: re-arm it
            const unsigned top =
                __hip_atomic_fetch_add(t + kTicketShards * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (top == nsh - 1u);
        }
        *sh_flag = last;
    }
    __syncthreads();
    return *sh_flag != 0;
}
__device__ __forceinline__ unsigned linear_block_id() {
    return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
__device__ __forceinline__ void ticket_rearm(unsigned* t) {
    if (threadIdx.x == 0) st_sc1(t + kTicketShards * 32, 0u);
}

// Diagnostic build only (make stamps -> lib/libwfbitnet_stamps.so): thread 0 of every block records
// the 100 MHz wall clock (s_memrealtime) at named points; read back with wf_debug_stamps_<tu>().
// In the product build WF_STAMP compiles to nothing.
#ifdef WF_STAMPS
constexpr int kStampSlots = 80;  // 4 waves x 16 realtime slots + 16 shader-clock slots
constexpr int kStampBlocks = 16384;
// hidden visibility: PC-relative address (no GOT load per stamp); row = the op's base + linear block id
__attribute__((visibility("hidden"))) static __device__ unsigned long long g_stamps[kStampBlocks * kStampSlots];
// slot i of wave w lives at column 16 w + i; wave 0 also records the shader clock (s_memtime) of
// slot i in column 64 + i (clock rate = d(memtime) / d(memrealtime) * 100 MHz)
// WF_STAMPS_EVEN: record the even waves 0, 2, 4, 6 (columns 0, 16, 32, 48) instead of waves 0..3
#ifdef WF_STAMPS_EVEN
#define WF_STAMP_WAVE_OK ((threadIdx.x >> 6) % 2 == 0 && threadIdx.x < 512)
#define WF_STAMP_COL (16 * ((threadIdx.x >> 6) >> 1))
#else
#define WF_STAMP_WAVE_OK (threadIdx.x < 256)
#define WF_STAMP_COL (16 * (threadIdx.x >> 6))
#endif
// a kernel may move its rows with WF_STAMP_BASE(v) (e.g. one region per decode op, so a graph
// replay of the whole step keeps every op's stamps of the last layer)
constexpr unsigned wf_stamp_base = 0;
#define WF_STAMP_BASE(v) constexpr unsigned wf_stamp_base = (v)
#define WF_STAMP(i)                                                                                 \
    do {                                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        if ((threadIdx.x & 63) == 0 && WF_STAMP_WAVE_OK) {                                          \
            const unsigned sb_ = wf_stamp_base + blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); \
            if (sb_ < (unsigned)::wf::kStampBlocks) {                                                \
                unsigned long long* row_ = ::wf::g_stamps + (size_t)sb_ * ::wf::kStampSlots;          \
                row_[WF_STAMP_COL + (i)] = __builtin_amdgcn_s_memrealtime();                         \
                if (threadIdx.x == 0) row_[64 + (i)] = __builtin_amdgcn_s_memtime();                  \
            }                                                                                       \
        }                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                          \
    } while (0)
// stamp after draining this wave's outstanding loads (when its data has landed)
#define WF_STAMP_DRAIN(i)                                   \
    do {                                                    \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   \
        WF_STAMP(i);                                        \
    } while (0)
#define WF_STAMP_READER(NAME)                                                                     \
    extern "C" int NAME(void* host, int n_words, int reset) {                                     \
        const size_t nb = sizeof(unsigned long long) * (size_t)::wf::kStampBlocks * ::wf::kStampSlots; \
        if (reset) return (int)hipMemset(::wf::g_stamps_addr(), 0, nb);                           \
        size_t b = sizeof(unsigned long long) * (size_t)n_words;                                   \
        if (b > nb) b = nb;                                                                        \
        return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(::wf::g_stamps), b, 0, hipMemcpyDeviceToHost); \
    }
inline void* g_stamps_addr() {
    void* p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps));
    return p;
}
#else
#define WF_STAMP_BASE(v)
#define WF_STAMP(i) \
    do {            \
    } while (0)
#define WF_STAMP_DRAIN(i) \
    do {                  \
    } while (0)
#define WF_STAMP_READER(NAME)
#endif

// ---------------------------------------------------------------------------------------------
// rms_norm -> int8 activation quantizer for one row, NT threads (256 or 512), 8-element pieces
// (p = threadIdx.x + NT * i, i < PPT). Float sequence of the reference
// (scripts/direct_inference_full.py:181-184, tests/test_bitnet_core.py:139-146):
//   r = bf16(1 / sqrt(mean(x^2) + eps)); y = bf16(bf16(x * r) * w)
//   s = double(max|y|) / 127 (1/127 if max < 1e-6); q = clamp(rne(y / float(s)), -128, 127)
// Loads are issued unconditionally (clamped index, masked in the arithmetic) so the caller can
// put its own loads behind them and hipcc counts vmcnt exactly.
// ---------------------------------------------------------------------------------------------

// Register fence: the value must exist here and nothing computed from it can move above this point
// (hipcc otherwise hoists the input-stage math above a later weight stream, delaying its issue).
__device__ __forceinline__ void reg_fence(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void reg_fence(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

template <int PPT, int NT>
struct NormRow {
    uint4 x[PPT], w[PPT];
    __device__ __forceinline__ void issue(const uint16_t* __restrict__ xrow, const uint16_t* __restrict__ nw, int K) {
        const int npk = K >> 3;
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            const int p = min((int)threadIdx.x + NT * i, npk - 1);
            x[i] = *reinterpret_cast<const uint4*>(xrow + 8 * p);
            w[i] = *reinterpret_cast<const uint4*>(nw + 8 * p);
        }
    }
    // the row only (no norm: BitNetLinear)
    __device__ __forceinline__ void issue_x(const uint16_t* __restrict__ xrow, int K) {
        const int npk = K >> 3;
#pragma unroll
        for (int i = 0; i < PPT; ++i) x[i] = *reinterpret_cast<const uint4*>(xrow + 8 * min((int)threadIdx.x + NT * i, npk - 1));
    }
    // norm weight only (the row itself is computed in registers)
    __device__ __forceinline__ void issue_w(const uint16_t* __restrict__ nw, int K) {
        const int npk = K >> 3;
#pragma unroll
        for (int i = 0; i < PPT; ++i) w[i] = *reinterpret_cast<const uint4*>(nw + 8 * min((int)threadIdx.x + NT * i, npk - 1));
    }
    __device__ __forceinline__ void fence(bool with_x = true, bool with_w = true) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
            if (with_x) reg_fence(x[i]);
            if (with_w) reg_fence(w[i]);
        }
    }
};

// bf16 pieces of `r.x` -> floats (0 for pieces >= K/8)
template <int PPT, int NT>
__device__ __forceinline__ void unpack_row(const NormRow<PPT, NT>& r, int K, float (&y)[PPT][8]) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const bool valid = (int)threadIdx.x + NT * i < (K >> 3);
        const uint32_t w4[4] = {r.x[i].x, r.x[i].y, r.x[i].z, r.x[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            y[i][2 * j] = valid ? bf_lo(w4[j]) : 0.f;
            y[i][2 * j + 1] = valid ? bf_hi(w4[j]) : 0.f;
        }
    }
}

// Normalises the row held in `y` (x values, 0 for pieces >= K/8) in place with the norm weight in
// `r.w`; returns the quantizer's float scale. `red` = 2 * NT / 64 floats of LDS (two barriers
// inside). The cross-wave sum order is a fixed tree, so kernels with the same NT agree bit for bit.
template <int W>
__device__ __forceinline__ float tree_sum(const float* r) {
    if constexpr (W == 1) return r[0];
    else return tree_sum<W / 2>(r) + tree_sum<W / 2>(r + W / 2);
}
template <int PPT, int NT, unsigned wf_stamp_base = 0>
__device__ __forceinline__ float norm_core(const NormRow<PPT, NT>& r, int K, float eps, float (&y)[PPT][8], float* red,
                                           bool want_scale = true) {
    constexpr int NW = NT / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float fK = (float)K, invK = 1.0f / fK;  // off the reduction chain
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) ss = fmaf(y[i][j], y[i][j], ss);
    WF_STAMP(8);
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    WF_STAMP(9);
    ss = tree_sum<NW>(red);
    const float rr = rms_factor(div_rn(ss, fK, invK) + eps);  // == rbf(1 / sqrtf(ss / K + eps))
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const uint32_t n4[4] = {r.w[i].x, r.w[i].y, r.w[i].z, r.w[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t a = pk_bf16(y[i][2 * j] * rr, y[i][2 * j + 1] * rr);
            const uint32_t b = pk_bf16(bf_lo(a) * bf_lo(n4[j]), bf_hi(a) * bf_hi(n4[j]));
            y[i][2 * j] = bf_lo(b);
            y[i][2 * j + 1] = bf_hi(b);
            mx = fmaxf(mx, fmaxf(fabsf(y[i][2 * j]), fabsf(y[i][2 * j + 1])));
        }
    }
    if (!want_scale) return 0.f;
    WF_STAMP(10);
    mx = wave_max(mx);
    if (lane == 0) red[NW + wave] = mx;
    __syncthreads();
    WF_STAMP(11);
    mx = red[NW];
#pragma unroll
    for (int i = 1; i < NW; ++i) mx = fmaxf(mx, red[NW + i]);
    return act_scale_f(mx);
}
// Activation scale of a row without normalisation (BitNetLinear's own quantizer,
// scripts/direct_inference_full.py:196): s = double(max|x|)/127. `red` as norm_core.
template <int PPT, int NT>
__device__ __forceinline__ float absmax_scale(const float (&y)[PPT][8], float* red) {
    constexpr int NW = NT / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < PPT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(y[i][j]));
    mx = wave_max(mx);
    if (lane == 0) red[NW + wave] = mx;
    __syncthreads();
    mx = red[NW];
#pragma unroll
    for (int i = 1; i < NW; ++i) mx = fmaxf(mx, red[NW + i]);
    return act_scale_f(mx);
}

// unpack_row + norm_core
template <int PPT, int NT, unsigned wf_stamp_base = 0>
__device__ __forceinline__ float norm_row(const NormRow<PPT, NT>& r, int K, float eps, float (&y)[PPT][8], float* red,
                                          bool want_scale = true) {
    unpack_row(r, K, y);
    return norm_core<PPT, NT, wf_stamp_base>(r, K, eps, y, red, want_scale);
}

// 256 threads replaying the 512-thread norm_core (the batch-1 / k_rownorm reduction tree, so the
// codes are bit-identical): thread t holds pieces t + 256 i (NormRow<PPT2, 256>).
template <int PPT2>
__device__ __forceinline__ float norm_core_e512(const NormRow<PPT2, 256>& r, int K, float eps, float (&y)[PPT2][8],
                                                float* red) {
    // 256 threads replaying the 512-thread norm_core: virtual thread t + 256 j owns pieces 2 i + j
    static_assert(PPT2 % 2 == 0, "two virtual threads per lane");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float ss[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PPT2 / 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) ss[j] = fmaf(y[2 * i + j][e], y[2 * i + j][e], ss[j]);
    ss[0] = wave_sum(ss[0]);
    ss[1] = wave_sum(ss[1]);
    if (lane == 0) {
        red[wave] = ss[0];
        red[wave + 4] = ss[1];
    }
    __syncthreads();
    const float rr = rms_factor(div_rn(tree_sum<8>(red), (float)K, 1.0f / (float)K) + eps);
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < PPT2; ++i) {
        const uint32_t n4[4] = {r.w[i].x, r.w[i].y, r.w[i].z, r.w[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t a = pk_bf16(y[i][2 * j] * rr, y[i][2 * j + 1] * rr);
            const uint32_t b = pk_bf16(bf_lo(a) * bf_lo(n4[j]), bf_hi(a) * bf_hi(n4[j]));
            y[i][2 * j] = bf_lo(b);
            y[i][2 * j + 1] = bf_hi(b);
            mx = fmaxf(mx, fmaxf(fabsf(y[i][2 * j]), fabsf(y[i][2 * j + 1])));
        }
    }
    mx = wave_max(mx);
    if (lane == 0) red[8 + wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[8], red[9]), fmaxf(red[10], red[11]));
    return act_scale_f(mx);
}

// Quantizes the normalised pieces; piece p (< npad = padded K / 8) goes to dst + off(p). Returns
// this thread's code sum (the caller reduces it).
template <int PPT, int NT, class Off, unsigned wf_stamp_base = 0>
__device__ __forceinline__ int quant_row(const float (&y)[PPT][8], float sf, int npad, int8_t* dst, Off off) {
    const float inv = rcp_1ulp(sf);
    int asum = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int p = (int)threadIdx.x + NT * i;
        const uint2 q = quant8(y[i], sf, inv, asum);
        if (p < npad) *reinterpret_cast<uint2*>(dst + off(p)) = q;
    }
    WF_STAMP(12);
    return asum;
}

// quant_row into the matrix-core tile layout of the batched GEMM's activation codes: row `row`,
// I2_S block kb, half h, lane l16 + 16q holds 16 codes at [4g + jj] = code of
// k = 128 kb + 16 h + 4 q + jj + 32 g  (the permutation the WF_FMT_I2S_MFMA weight dwords decode to).
__device__ __forceinline__ int64_t tile_code_pos(int row, int k, int nkb) {
    const int o = k & 127;
    return ((((int64_t)(row >> 4) * nkb + (k >> 7)) * 2 + ((o >> 4) & 1)) << 10) +
           (((row & 15) + 16 * ((o & 15) >> 2)) << 4) + 4 * (o >> 5);
}
template <int PPT, int NT>
__device__ __forceinline__ int quant_row_tiled(const float (&y)[PPT][8], float sf, int npad, int8_t* base, int row,
                                               int nkb) {
    const float inv = rcp_1ulp(sf);
    int asum = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int p = (int)threadIdx.x + NT * i;
        const uint2 q = quant8(y[i], sf, inv, asum);
        if (p < npad) {
            *reinterpret_cast<uint32_t*>(base + tile_code_pos(row, 8 * p, nkb)) = q.x;
            *reinterpret_cast<uint32_t*>(base + tile_code_pos(row, 8 * p + 4, nkb)) = q.y;
        }
    }
    return asum;
}

// bf16 matrix-core fragment layout of a [rows][H] operand (16 x 32 fragments): element offset of
// the 8-element piece p (k = 8p) of row r. Fragment (row tile, k-step s) = 64 lanes x 8 elements,
// lane l16 + 16q = row 16 rt + l16, k = 32 s + 8 q: one contiguous KiB per wave-instruction.
__device__ __forceinline__ int64_t bf_tile_off(int r, int p, int H) {
    return ((((int64_t)(r >> 4) * (H >> 5) + (p >> 2)) << 6) + (r & 15) + 16 * (p & 3)) << 3;
}

// (WF_SPLITS / WF_SPLITS1: study builds only, tools/build_variant.sh; the library uses the defaults)
#ifndef WF_SPLITS
#define WF_SPLITS 4
#endif
#ifndef WF_SPLITS1
#define WF_SPLITS1 8
#endif
constexpr int kAttnPartSplits = WF_SPLITS;    // records per (sequence, query head): batched decode (B >= 16)
constexpr int kAttnPartSplits1 = WF_SPLITS1;  // batch < 16 (16 measured: attention 5.70 -> 5.63 us, O input 6.01 -> 7.27 us)
constexpr int kAttnPartSplitsMax = 16;
// k_attn_sdpa's exchange buffer (the model's attn_xmax): the split maxima [B][Hq][splits][3], then the
// merge granules [B][Hq][target split][source split][kSdpaMergeSlot] (the target's 128 / splits dims
// + l, padded to 16-byte pairs)
constexpr int kSdpaMergeDims = 128 / kAttnPartSplits1;
constexpr int kSdpaMergeSlot = (kSdpaMergeDims + 2) & ~1;
inline int64_t sdpa_xmax_granules(int B, int Hq) { return 3LL * B * Hq * kAttnPartSplits1; }
inline int64_t sdpa_xbuf_granules(int B, int Hq) {
    return sdpa_xmax_granules(B, Hq) + (int64_t)B * Hq * kAttnPartSplits1 * kAttnPartSplits1 * kSdpaMergeSlot;
}
static_assert(kAttnPartSplits <= kAttnPartSplitsMax && kAttnPartSplits1 <= kAttnPartSplitsMax,
              "part_ml / part_o are sized for kAttnPartSplitsMax records per (sequence, head)");
static_assert(kAttnPartSplits % 4 == 0 && kAttnPartSplits1 % 2 == 0, "record counts: whole 4-wave blocks / pairs");
// Float offset of element d of split s's unnormalised o in the decode-attention partials of (b, h)
// (bh = b * Hq + h; head_dim 128): [bh][split][half = (d >> 2) & 1][d >> 3][4] (include/wf_bitnet.h
// wf_attn_records; k_attn_sdpa's writers and merging block address 4-float slots of it). (m, l)
// records stay [bh][split].
template <int NS = kAttnPartSplits>
__device__ __forceinline__ int64_t part_o_off(int64_t bh, int s, int d) {
    return ((bh * NS + s) * 2 + ((d >> 2) & 1)) * 64 + (d >> 3) * 4 + (d & 3);
}
constexpr int kPrefillRowGroup = WF_PREFILL_ROW_GROUP;  // prefill rows per slot-uniform group (include/wf_bitnet.h)

// Matrix-core tile layouts of the K / V caches (batched decode; head_dim 128, S % 32 == 0), element
// offsets within one (sequence, kv head) slab of S x 128 bf16. Key position t = 32 blk + o:
//   K: [blk][tau 2][dg 16][row 16][8 dims], row = 4 (o >> 3) + (o & 3), tau = (o >> 2) & 1, dg = d >> 3
//      -> the QK MFMA's A fragment (lane = row + 16 q, dims 32 c + 8 q) of key tile tau, step c, is
//      one contiguous KiB;
//   V: [blk][n 8][q 4][l 16][8 keys], n = d >> 4, l = d & 15, q = o >> 3 -> the P.V MFMA's B
//      fragment (lane = l + 16 q, keys 8 q .. +8 of dims 16 n + l) is one contiguous KiB.
__device__ __forceinline__ int64_t k_tile_off(int t, int d) {
    const int blk = t >> 5, o = t & 31;
    return ((((int64_t)blk * 2 + ((o >> 2) & 1)) * 16 + (d >> 3)) * 16 + 4 * (o >> 3) + (o & 3)) * 8 + (d & 7);
}
__device__ __forceinline__ int64_t v_tile_off(int t, int d) {
    const int blk = t >> 5, o = t & 31;
    return ((((int64_t)blk * 8 + (d >> 4)) * 4 + (o >> 3)) * 16 + (d & 15)) * 8 + (o & 7);
}

// one 128-byte line per arrival counter (memory-side atomics and polls on one line serialise)
constexpr int kTailLine = 32;  // one 128-byte line per counter

// Batch-1 GEMV prologue (k_gemv PPT > 0: NormRow + norm_core + quant_row) is VALU-issue /
// dependency-latency bound, not memory-bound (in-graph stamps, tools/stamps_graph.py). Measured
// and not kept (round 3): all of it on one wave per SIMD (QKV input image 2.64 -> 3.16 us: a lone
// wave issues a dependent chain at ~8 cycles per instruction); data-less waves skipping the
// elementwise work plus packed-bf16 maxima (QKV 4.59 -> 4.90 us, gate/up 5.91 -> 6.13 us per
// layer in the same-box graph A/B: the extra barrier and branches cost more than they saved).

}  // namespace wf
