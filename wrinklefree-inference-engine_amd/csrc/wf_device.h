// wf_device.h -- gfx950 device helpers shared by the BitNet HIP kernels.
//
// Wave = 64 lanes (CDNA4). Packed-weight formats:
//   I2S : the reference's blocked 2-bit layout (cache/bitnet_converter.py:26-77), [N][K/4] bytes.
//         A 16-byte chunk c of a row = half h=c&1 of 128-wide block b=c>>1; byte j holds
//         enc(w[128b+16h+j]) << 6 | enc(w[+32]) << 4 | enc(w[+64]) << 2 | enc(w[+96]).
//   TQ  : the build's ~1.6-bit format (5 trits/byte, base 3; oracle/wf_oracle.c pack_tq), [N][C*16]
//         bytes with C = ceil(K/80); chunk c, byte j, digit i <-> weight 80c + 16i + j.
// Both store enc = w + 1 in {0,1,2}; the kernels accumulate sum(enc * a) exactly in int32, which is
// the raw sgl-kernel semantics (tests/test_bitnet_core.py:149-167).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wf {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// bf16 <-> f32 (bit exact, round-to-nearest-even like torch .to(bfloat16); NaN stays NaN).
// gfx950 converts in hardware (v_cvt_pk_bf16_f32): no per-element branch for the NaN case.
// ---------------------------------------------------------------------------------------------
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
// two floats -> packed bf16x2 (lo in bits 0..15), one instruction
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
    const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// dtype codes shared with include/wf_bitnet.h
enum { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2, DT_I8 = 3, DT_U8 = 4 };

__device__ __forceinline__ float load_as_f32(const void* p, int64_t i, int dt) {
    if (dt == DT_F32) return ((const float*)p)[i];
    if (dt == DT_BF16) return bf2f(((const uint16_t*)p)[i]);
    return h2f(((const uint16_t*)p)[i]);
}
__device__ __forceinline__ void store_from_f32(void* p, int64_t i, int dt, float v) {
    if (dt == DT_F32) ((float*)p)[i] = v;
    else if (dt == DT_BF16) ((uint16_t*)p)[i] = f2bf(v);
    else ((uint16_t*)p)[i] = f2h(v);
}

// ---------------------------------------------------------------------------------------------
// wave / lane-group reductions (wave64) on DPP: quad_perm, row_half_mirror and row_mirror combine
// lanes inside a 16-lane row (every lane ends with the same bits: each step adds two equal-order
// partials), row_bcast:15/31 carry rows into lane 63 for a full-wave result (then v_readlane).
// ~8 cycles per step instead of an LDS-latency ds_bpermute per step.
// ---------------------------------------------------------------------------------------------
enum : int { DPP_QP_1032 = 0xB1, DPP_QP_2301 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140,
             DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143, DPP_ROW_ROR8 = 0x128, DPP_ROW_ROR4 = 0x124 };
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i(int v, int old = 0) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v, float old = 0.f) {
    return __int_as_float(dpp_i<CTRL, ROW_MASK>(__float_as_int(v), __float_as_int(old)));
}
template <int CTRL, int ROW_MASK = 0xF, class T>
__device__ __forceinline__ T dpp_cast(T v, T old = T(0)) {
    if constexpr (__is_same(T, float)) return dpp_f<CTRL, ROW_MASK>(v, old);
    else return dpp_i<CTRL, ROW_MASK>(v, old);
}
// 4 x 4 transpose of bf16 values inside each lane quad: lane qi holds y[r] = M[qi][r] (float,
// bf16-representable); returns row qi of M^T packed as bf16 pairs: (M[0][qi], M[1][qi]),
// (M[2][qi], M[3][qi]). Two DPP exchanges: 2 x 2 blocks across lanes qi ^ 2, then 16-bit halves
// across lanes qi ^ 1 (v_perm_b32 selects the halves).
__device__ __forceinline__ uint2 quad_transpose_pk(uint32_t A, uint32_t B, int qi);
__device__ __forceinline__ uint2 quad_transpose_bf16(const float (&y)[4], int qi) {
    return quad_transpose_pk(pk_bf16(y[0], y[1]), pk_bf16(y[2], y[3]), qi);
}
// the same on the packed pairs A = (y0, y1), B = (y2, y3)
__device__ __forceinline__ uint2 quad_transpose_pk(uint32_t A, uint32_t B, int qi) {
    const bool hi2 = qi & 2, odd = qi & 1;
    // own = (M[qi][r0], M[qi][r0 + 1]), other = (M[qi ^ 2][r0], M[qi ^ 2][r0 + 1]), r0 = qi & 2
    const uint32_t own = hi2 ? B : A;
    const uint32_t other = (uint32_t)dpp_i<DPP_QP_2301>((int)(hi2 ? A : B));
    const uint32_t lo = __builtin_amdgcn_perm(other, own, 0x05040100u);  // (own.lo, other.lo)
    const uint32_t hi = __builtin_amdgcn_perm(other, own, 0x07060302u);  // (own.hi, other.hi)
    // even lanes keep the low halves (row qi = r0), odd ones the high halves (row r0 + 1)
    const uint32_t keep = odd ? hi : lo;
    const uint32_t got = (uint32_t)dpp_i<DPP_QP_1032>((int)(odd ? lo : hi));
    // keep = (M[qi][qi], M[qi ^ 2][qi]), got = (M[qi ^ 1][qi], M[qi ^ 3][qi])
    const uint32_t x = odd ? got : keep;  // (M[qi & 2][qi], M[(qi & 2) ^ 2][qi])
    const uint32_t z = odd ? keep : got;  // (M[(qi & 2) | 1][qi], M[((qi & 2) | 1) ^ 2][qi])
    const uint32_t p01 = __builtin_amdgcn_perm(z, x, 0x05040100u), p23 = __builtin_amdgcn_perm(z, x, 0x07060302u);
    return hi2 ? make_uint2(p23, p01) : make_uint2(p01, p23);
}

// Two rows of one 16 x 16 accumulator column through the reference correction
// (direct_inference_full.py:201-208: fl32(fl32(S ws) - fl32(ws asum)) * s) on the packed-fp32 VALU
// (v_pk_mul_f32 / v_pk_add_f32 round each lane like the scalar ops), returned as a bf16 pair.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t corrected_pk(int s0, int s1, float ws, int a0, int a1, float f0, float f1) {
    const f32x2_t W = {ws, ws};
    const f32x2_t u = (f32x2_t{(float)s0, (float)s1} * W - W * f32x2_t{(float)a0, (float)a1}) * f32x2_t{f0, f1};
    return pk_bf16(u.x, u.y);
}

// bf16(a + b) for two packed bf16 pairs (the residual add bf16(resid + bf16(o)))
__device__ __forceinline__ uint32_t bf16_add_pk(uint32_t a, uint32_t b) {
    const f32x2_t s = f32x2_t{bf_lo(a), bf_hi(a)} + f32x2_t{bf_lo(b), bf_hi(b)};
    return pk_bf16(s.x, s.y);
}
// RoPE on a packed bf16 pair of each half: y1 = bf16(bf16(x1 c) - bf16(x2 s)), y2 = bf16(bf16(x1 s) +
// bf16(x2 c)) (scripts/direct_inference_full.py:58-70, bf16 tensor ops)
__device__ __forceinline__ void rope_pk(uint32_t x1, uint32_t x2, uint32_t c, uint32_t s, uint32_t& y1, uint32_t& y2) {
    const f32x2_t a = {bf_lo(x1), bf_hi(x1)}, b = {bf_lo(x2), bf_hi(x2)};
    const f32x2_t cc = {bf_lo(c), bf_hi(c)}, ss = {bf_lo(s), bf_hi(s)};
    const f32x2_t ac = a * cc, bs = b * ss, as = a * ss, bc = b * cc;
    const uint32_t pac = pk_bf16(ac.x, ac.y), pbs = pk_bf16(bs.x, bs.y), pas = pk_bf16(as.x, as.y), pbc = pk_bf16(bc.x, bc.y);
    const f32x2_t d = f32x2_t{bf_lo(pac), bf_hi(pac)} - f32x2_t{bf_lo(pbs), bf_hi(pbs)};
    const f32x2_t u = f32x2_t{bf_lo(pas), bf_hi(pas)} + f32x2_t{bf_lo(pbc), bf_hi(pbc)};
    y1 = pk_bf16(d.x, d.y);
    y2 = pk_bf16(u.x, u.y);
}

struct OpAdd {
    template <class T> __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
    __device__ __forceinline__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
// Reduce over aligned groups of G lanes (G in 1..64); every lane of the group gets the result.
template <int G, class T, class Op>
__device__ __forceinline__ T group_reduce(T v, Op op) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "group size");
    if constexpr (G >= 2) v = op(v, dpp_cast<DPP_QP_1032>(v));
    if constexpr (G >= 4) v = op(v, dpp_cast<DPP_QP_2301>(v));
    if constexpr (G >= 8) v = op(v, dpp_cast<DPP_HALF_MIRROR>(v));
    if constexpr (G >= 16) v = op(v, dpp_cast<DPP_MIRROR>(v));
    if constexpr (G >= 32) v = op(v, __shfl_xor(v, 16, 64));
    if constexpr (G >= 64) v = op(v, __shfl_xor(v, 32, 64));
    return v;
}
// Full-wave reduction, result uniform (scalar) in every lane: rows -> lane 63 -> readlane.
template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op, T ident) {
    v = group_reduce<16>(v, op);
    v = op(v, dpp_cast<DPP_BCAST15, 0xA>(v, ident));
    v = op(v, dpp_cast<DPP_BCAST31, 0xC>(v, ident));
    if constexpr (sizeof(T) == 4 && __is_same(T, float))
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
    else
        return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ float wave_max(float v) { return wave_reduce(v, OpMax{}, -INFINITY); }
__device__ __forceinline__ float wave_sum(float v) { return wave_reduce(v, OpAdd{}, 0.f); }
__device__ __forceinline__ int wave_sum_i(int v) { return wave_reduce(v, OpAdd{}, 0); }
// Reduce across the 16 lanes of a 16-lane group.
__device__ __forceinline__ int group16_sum_i(int v) { return group_reduce<16>(v, OpAdd{}); }

// Block-wide reductions over blockDim.x (multiple of 64, <= 1024). `red` is >= 16 floats of LDS.
__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, red[i]);
    return r;
}
// Deterministic fixed-order sum (per-wave tree, then waves in order).
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; ++i) r += red[i];
    return r;
}
__device__ __forceinline__ int block_sum_i(int v, int* red) {
    v = wave_sum_i(v);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int r = red[0];
    for (int i = 1; i < nw; ++i) r += red[i];
    return r;
}

// ---------------------------------------------------------------------------------------------
// Activation quantization (tests/test_bitnet_core.py:139-146): s = double(m)/127 (m -> 1 if
// m < 1e-6); q = clamp(rne(x / float(s)), -128, 127). Division is IEEE (hipcc's default
// correctly-rounded fp32 divide), rint() is round-half-even.
// ---------------------------------------------------------------------------------------------
// sum of the four signed bytes of `a` (+ c)
__device__ __forceinline__ int sdot4_ones(uint32_t a, int c) { return __builtin_amdgcn_sdot4((int)a, 0x01010101, c, false); }
__device__ __forceinline__ double act_scale_from_max(float m) {
    double md = (double)m;
    if (md < 1e-6) md = 1.0;
    return md / 127.0;
}
__device__ __forceinline__ int8_t quant_one(float x, float sf) {
    float v = rintf(x / sf);
    v = fminf(fmaxf(v, -128.f), 127.f);
    return (int8_t)(int)v;
}

// Correctly rounded quotient without the IEEE divide sequence (Markstein): given yb within 1 ulp of
// 1/b (RN(1/b) for the 1/K use), q = RN(a*yb) is within an ulp of a/b, the fma remainder
// r = a - q*b is exact, and RN(q + r*yb) = RN(a/b) for finite a/b clear of over/underflow.
// Checked on the host against the IEEE divide: 1.2e8 random a for K in {128 .. 6912}, every
// positive bf16 numerator over 127, 1.8e8 quantizer cases incl. constructed half-integer ties, with
// yb exact and +-1 ulp (round 4; tools/check_fast_arith.c).
__device__ __forceinline__ float div_rn(float a, float b, float yb) {
    const float q = a * yb;
    const float r = fmaf(-q, b, a);
    return fmaf(r, yb, q);
}
// 1/b within 1 ulp (v_rcp_f32 + one Newton step; b normal)
__device__ __forceinline__ float rcp_1ulp(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return fmaf(fmaf(-b, y0, 1.0f), y0, y0);
}
// (float)act_scale_from_max(m) in fp32: float(double(m) / 127) == RN_f32(m / 127) (the double
// rounding cannot bite: m / 127 has a 7-bit period, so bits 25..53 are never a midpoint pattern),
// and double(m) < 1e-6 <=> m <= float(1e-6) = 9.99999997e-07f.
__device__ __forceinline__ float act_scale_f(float m) {
    if (m <= 9.99999997e-07f) return 1.0f / 127.0f;
    return div_rn(m, 127.0f, 1.0f / 127.0f);
}
// rbf(1 / sqrtf(v)) (IEEE sqrt, IEEE divide, bf16 RNE: the rms_norm factor of
// scripts/direct_inference_full.py:181-184 as the oracle computes it). v_rsq_f32 is within 1 ulp
// of 1/sqrt(v) and the two-rounding reference within 1.5 ulp, so their bf16 roundings agree unless
// the fp32 value sits within a few ulps of a bf16 midpoint: there (p ~ 2e-3, wave-uniform: v is
// the same in every lane) the exact sequence runs.
__device__ __forceinline__ float rms_factor(float v) {
    const float a = __builtin_amdgcn_rsqf(v);
    const uint32_t lo = __float_as_uint(a) & 0xffffu;
    if (lo - (0x8000u - 64u) < 128u) return rbf(1.0f / sqrtf(v));
    return rbf(a);
}
// Eight codes at once, bit-identical to quant_one: rne(RN(x / s)) -- the reference divides in
// fp32 (tests/test_bitnet_core.py:144: (activations / scale).round()), so the quotient is rounded
// to fp32 BEFORE the round-to-integer (x / s a hair below k + 1/2 can round up to k + 1/2 and then
// to even). RN(x / s) by div_rn (inv = 1/s within 1 ulp), then + 1.5 * 2^23 rounds it to the
// integer (RNE) in the add and leaves the code in the low byte. No clamp: s = max|x| / 127 bounds
// |x / s| by 127 (1 + 2^-23). Branch-free (the former form re-divided near-ties under a branch per
// element). Returns the 8 codes packed little-endian; adds them to `asum`.
__device__ __forceinline__ uint2 quant8(const float (&x)[8], float sf, float inv, int& asum) {
    constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23
    uint32_t b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = __float_as_uint(div_rn(x[j], sf, inv) + kMagic);
    const uint32_t lo = __builtin_amdgcn_perm(b[1], b[0], 0x0c0c0400u) | __builtin_amdgcn_perm(b[3], b[2], 0x04000c0cu);
    const uint32_t hi = __builtin_amdgcn_perm(b[5], b[4], 0x0c0c0400u) | __builtin_amdgcn_perm(b[7], b[6], 0x04000c0cu);
    asum = sdot4_ones(lo, sdot4_ones(hi, asum));
    return make_uint2(lo, hi);
}

// quant8 of eight packed bf16 values on fp32 pairs: v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32
// round each lane exactly as the scalar ops do, so the codes and the sum are quant8's.
__device__ __forceinline__ uint2 quant8_bf16x8(uint4 v, float sf, float inv, int& asum) {
    const f32x2_t S = {sf, sf}, I = {inv, inv}, G = {12582912.0f, 12582912.0f};
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t b[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const f32x2_t x = {bf_lo(w[e]), bf_hi(w[e])};
        const f32x2_t q = x * I;
        const f32x2_t r = __builtin_elementwise_fma(-q, S, x);
        const f32x2_t d = __builtin_elementwise_fma(r, I, q) + G;
        b[2 * e] = __float_as_uint(d.x);
        b[2 * e + 1] = __float_as_uint(d.y);
    }
    const uint32_t lo = __builtin_amdgcn_perm(b[1], b[0], 0x0c0c0400u) | __builtin_amdgcn_perm(b[3], b[2], 0x04000c0cu);
    const uint32_t hi = __builtin_amdgcn_perm(b[5], b[4], 0x0c0c0400u) | __builtin_amdgcn_perm(b[7], b[6], 0x04000c0cu);
    asum = sdot4_ones(lo, sdot4_ones(hi, asum));
    return make_uint2(lo, hi);
}

// ---------------------------------------------------------------------------------------------
// Packed-weight formats and their LDS activation images.
//
// The GEMV kernels put 16 lanes on one weight row; lane `sub` (0..15) takes chunks c = sub + 16*i.
// The activation image in LDS is laid out so that, for a fixed (i, group g), the 16 lanes' 16-byte
// activation pieces are one contiguous 256-byte bank row -> every ds_read_b128 is conflict-free
// (the other 48 lanes of the wave read the same addresses: broadcast).
// ---------------------------------------------------------------------------------------------
struct FmtI2S {
    static constexpr int kGroups = 4;   // 16-byte activation pieces per chunk
    static constexpr int kChunkW = 64;  // weights per 16-byte chunk
    __host__ __device__ static int64_t row_bytes(int K) { return K / 4; }
    __host__ __device__ static int chunks(int K) { return K / 64; }
    __host__ __device__ static int k_pad(int K) { return K; }
    // LDS byte offset of activation element k.
    __device__ static __forceinline__ int lds_off(int k) {
        const int b = k >> 7, r = k & 127, g = r >> 5, t = r & 31, h = t >> 4, j = t & 15;
        const int c = 2 * b + h;
        return (((c >> 4) * 4 + g) << 8) + ((c & 15) << 4) + j;
    }
};

struct FmtTQ {
    static constexpr int kGroups = 5;
    static constexpr int kChunkW = 80;
    __host__ __device__ static int chunks(int K) { return (K + 79) / 80; }
    __host__ __device__ static int64_t row_bytes(int K) { return (int64_t)chunks(K) * 16; }
    __host__ __device__ static int k_pad(int K) { return chunks(K) * 80; }
    __device__ static __forceinline__ int lds_off(int k) {
        const int c = k / 80, r = k - c * 80, g = r >> 4, j = r & 15;
        return (((c >> 4) * 5 + g) << 8) + ((c & 15) << 4) + j;
    }
};

// LDS bytes for one activation row image of K elements (rounded to whole 16-chunk stripes).
template <class F>
__host__ __device__ constexpr int lds_image_bytes(int K) {
    return ((F::chunks(K) + 15) / 16) * F::kGroups * 256;
}

__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// Per-chunk decode: fill `e[g][t]` = 4 enc bytes (one dword) of group g, dword t, for the chunk.
// I2S: group g of dword t = (d_t >> (6 - 2g)) & 0x03030303.
__device__ __forceinline__ void decode_i2s(const uint4 w, uint32_t (&e)[4][4]) {
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
    constexpr uint32_t M = 0x03030303u;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        e[0][t] = (d[t] >> 6) & M;
        e[1][t] = (d[t] >> 4) & M;
        e[2][t] = (d[t] >> 2) & M;
        e[3][t] = d[t] & M;
    }
}

// TQ: bytes hold q; digit i = ((q*3^i mod 256)*3) >> 8. Even/odd bytes ride in 16-bit lanes so
// one 24-bit multiply by 3 advances two bytes per register; the digit is the high byte of
// each 16-bit lane (3*255 < 768 -> {0,1,2}), the low byte is the next q.
__device__ __forceinline__ void decode_tq(const uint4 w, uint32_t (&e)[5][4]) {
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#ifndef WF_TQ_PERM  // study: 0 = the shift / mask / and-or digit pick on 32-bit lanes (37 VALU per word)
#define WF_TQ_PERM 2  // 1 = v_perm digit pick (25); 2 = + E and O multiplied as one 64-bit pair (20)
#endif
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        uint32_t E = d[t] & 0x00ff00ffu;
        uint32_t O = (d[t] >> 8) & 0x00ff00ffu;
        if constexpr (WF_TQ_PERM == 2) {
            // {E, O} as one 64-bit value: 3 x every 16-bit lane in one v_lshl_add_u64 (lanes <= 765: no
            // carry crosses a lane), the digit bytes {YE.b1, YO.b1, YE.b3, YO.b3} in one v_perm_b32
            uint64_t eo = ((uint64_t)O << 32) | E;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                uint64_t y;
                asm("v_lshl_add_u64 %0, %1, 1, %1" : "=v"(y) : "v"(eo));
                e[i][t] = __builtin_amdgcn_perm((uint32_t)(y >> 32), (uint32_t)y, 0x07030501u);
                eo = y & 0x00ff00ff00ff00ffull;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const uint32_t YE = (E << 1) + E;  // v_lshl_add_u32
                const uint32_t YO = (O << 1) + O;
                if constexpr (WF_TQ_PERM == 1) e[i][t] = __builtin_amdgcn_perm(YO, YE, 0x07030501u);
                else e[i][t] = ((YE >> 8) & 0x00ff00ffu) | (YO & 0xff00ff00u);
                E = YE & 0x00ff00ffu;
                O = YO & 0x00ff00ffu;
            }
        }
    }
}

template <class F>
struct Decoded;
template <class F>
struct DotAcc;
template <>
struct Decoded<FmtTQ> {
    uint32_t e[5][4];
    __device__ __forceinline__ void load(const uint4 w) { decode_tq(w, e); }
};
template <>
struct DotAcc<FmtTQ> {
    int s[1];
    __device__ __forceinline__ DotAcc() : s{0} {}
    __device__ __forceinline__ int total() const { return s[0]; }
};
// I2S, the GEMV form: the 2-bit field of group g is masked in place (d & 0x30303030 = 16 x code,
// d & 0x0c0c0c0c = 4 x code, d & 0x03030303 = code; group 0's top field is shifted once, 32 x code
// <= 64 stays a positive int8), 5 VALU per dword instead of 7 for shift + mask per group; each group
// accumulates on its own (four independent dot4 chains per chunk instead of one of 16) and its scale
// is divided out once at the end (DotAcc::total, exact). Same-box graph A/B against the round-2
// decode (shift + mask per group, one accumulator): equal batch-1 step time (1045 vs 1040 tok/s).
template <>
struct Decoded<FmtI2S> {
    uint32_t e[4][4];
    __device__ __forceinline__ void load(const uint4 w) {
        const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            e[0][t] = (d[t] >> 1) & 0x60606060u;
            e[1][t] = d[t] & 0x30303030u;
            e[2][t] = d[t] & 0x0c0c0c0cu;
            e[3][t] = d[t] & 0x03030303u;
        }
    }
};
template <>
struct DotAcc<FmtI2S> {
    int s[4];
    __device__ __forceinline__ DotAcc() : s{0, 0, 0, 0} {}
    __device__ __forceinline__ int total() const { return s[3] + (s[2] >> 2) + (s[1] >> 4) + (s[0] >> 5); }
};

// sum_g,t dot4(e[g][t], act[g][t]) with act read from the LDS image at stripe base `abase`
// (abase = image + (i*G)*256 + sub*16; group g adds g*256).
template <class F>
__device__ __forceinline__ void chunk_dot(const Decoded<F>& dw, const int8_t* abase, DotAcc<F>& acc) {
#pragma unroll
    for (int g = 0; g < F::kGroups; ++g) {
        const uint4 a = *reinterpret_cast<const uint4*>(abase + g * 256);
        int& r = acc.s[__is_same(F, FmtI2S) ? g : 0];
        r = sdot4(dw.e[g][0], a.x, r);
        r = sdot4(dw.e[g][1], a.y, r);
        r = sdot4(dw.e[g][2], a.z, r);
        r = sdot4(dw.e[g][3], a.w, r);
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg_nt(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

}  // namespace wf
