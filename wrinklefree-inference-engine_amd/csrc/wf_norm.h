// wf_norm.h -- block-level RMSNorm + int8 activation quantizer and the in-launch hand-off helpers
// used by the fused decode step (gfx950).
//
// The decode step runs each op's "rms_norm -> quantize" exactly once per token: the LAST block of
// the producing kernel (per-launch ticket) normalises the full output vector and publishes
// int8 codes + scale + code sum for the consumer GEMV, which then only stages the int8 image.
// Hand-off protocol (MI355X_MICROARCH.md, Valid forms row 1): every block stores its slice of the
// vector write-through (sc1), drains (s_waitcnt vmcnt(0)) in every storing wave, meets at a
// barrier, one lane bumps an agent-scope ticket; the block whose add returns n-1 reads the vector
// with sc1 loads, computes, and re-arms the ticket for the next launch.
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
// call. Arrivals are spread over kTicketShards counters (one word takes ~88 atomics/us, so 800+
// arrivals on one word would serialise for ~10 us); the last arriver of each shard re-arms its shard
// and relays to the top counter. Returns true in exactly one block of the launch (the last
// arriver), which must call ticket_rearm() when done. `t` points at kTicketShards + 1 words.
constexpr int kTicketShards = 32;
constexpr int kTicketWords = 64;  // words reserved per ticket (>= kTicketShards + 1, 256-byte aligned)

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
        const unsigned old = __hip_atomic_fetch_add(t + sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == members - 1u) {
            st_sc1(t + sh, 0u);  // every member of this shard has arrived: re-arm it
            const unsigned top =
                __hip_atomic_fetch_add(t + kTicketShards, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    if (threadIdx.x == 0) st_sc1(t + kTicketShards, 0u);
}

// Where a normalised row goes: int8 codes + float scale + exact code sum (for the next ternary
// GEMV), or bf16 (final norm feeding the LM head).
struct NormOut {
    int8_t* q8;      // [K] int8, or nullptr
    float* sf;       // float(s), s = double(max|y|)/127
    int* asum;       // sum of the codes
    uint16_t* y16;   // [K] bf16 normalised row (final norm), or nullptr
};

constexpr int kNormMaxPieces = 4;  // 8-element pieces per thread: K <= 4 * 8 * 256 = 8192

// One block (256 threads) normalises one row: y = bf16(bf16(x * r) * w), r = bf16(1/sqrt(mean(x^2)
// + eps)) (scripts/direct_inference_full.py:181-184), then q = clamp(rne(y / float(s)), -128, 127)
// with s = max|y| / 127 in double (tests/test_bitnet_core.py:139-146). `red` >= 48 floats of LDS.
// SC1: read x with sc1 loads (x was written by other blocks of this launch).
template <bool SC1>
__device__ void norm_quant_row(const uint16_t* __restrict__ x, const uint16_t* __restrict__ nw, int K, float eps,
                               NormOut o, float* red) {
    const int nwv = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int np = K / 8;
    uint4 xr[kNormMaxPieces], wr[kNormMaxPieces];
    __amdgpu_buffer_rsrc_t rs = make_rsrc(x);
#pragma unroll
    for (int i = 0; i < kNormMaxPieces; ++i) {
        const int p = threadIdx.x + i * blockDim.x;
        xr[i] = make_uint4(0, 0, 0, 0);
        wr[i] = make_uint4(0, 0, 0, 0);
        if (p < np) {
            xr[i] = SC1 ? ld16_sc1(rs, p * 16) : *reinterpret_cast<const uint4*>(x + 8 * p);
            wr[i] = *reinterpret_cast<const uint4*>(nw + 8 * p);
        }
    }
    float xv[kNormMaxPieces][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < kNormMaxPieces; ++i) {
        const uint32_t w4[4] = {xr[i].x, xr[i].y, xr[i].z, xr[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xv[i][2 * j] = __uint_as_float(w4[j] << 16);
            xv[i][2 * j + 1] = __uint_as_float(w4[j] & 0xffff0000u);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss = fmaf(xv[i][j], xv[i][j], ss);
    }
    ss = wave_sum(ss);
    if (lane == 0) red[wave] = ss;
    __syncthreads();
    ss = red[0];
    for (int i = 1; i < nwv; ++i) ss += red[i];
    const float r = rbf(1.0f / sqrtf(ss / (float)K + eps));
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < kNormMaxPieces; ++i) {
        const uint32_t n4[4] = {wr[i].x, wr[i].y, wr[i].z, wr[i].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float wv = (j & 1) ? __uint_as_float(n4[j >> 1] & 0xffff0000u) : __uint_as_float(n4[j >> 1] << 16);
            xv[i][j] = rbf(rbf(xv[i][j] * r) * wv);
            mx = fmaxf(mx, fabsf(xv[i][j]));
        }
    }
    if (o.y16) {  // final norm: bf16 row out, no quantization
#pragma unroll
        for (int i = 0; i < kNormMaxPieces; ++i) {
            const int p = threadIdx.x + i * blockDim.x;
            if (p < np) {
                uint32_t pk[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) pk[j] = (uint32_t)f2bf(xv[i][2 * j]) | ((uint32_t)f2bf(xv[i][2 * j + 1]) << 16);
                *reinterpret_cast<uint4*>(o.y16 + 8 * p) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            }
        }
        __syncthreads();  // red[] is reused by the caller's next row
        return;
    }
    mx = wave_max(mx);
    if (lane == 0) red[16 + wave] = mx;
    __syncthreads();
    mx = red[16];
    for (int i = 1; i < nwv; ++i) mx = fmaxf(mx, red[16 + i]);
    const float sf = (float)act_scale_from_max(mx);
    int asum = 0;
#pragma unroll
    for (int i = 0; i < kNormMaxPieces; ++i) {
        const int p = threadIdx.x + i * blockDim.x;
        if (p < np) {
            uint32_t pk[2] = {0u, 0u};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int8_t q = quant_one(xv[i][j], sf);
                asum += q;
                pk[j >> 2] |= (uint32_t)(uint8_t)q << (8 * (j & 3));
            }
            *reinterpret_cast<uint2*>(o.q8 + 8 * p) = make_uint2(pk[0], pk[1]);
        }
    }
    asum = wave_sum_i(asum);
    int* redi = reinterpret_cast<int*>(red + 32);
    if (lane == 0) redi[wave] = asum;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < nwv; ++i) t += redi[i];
        *o.asum = t;
        *o.sf = sf;
    }
}

}  // namespace wf
