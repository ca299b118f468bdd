// wf_msb.hip -- the SGLang BitNet linear method on the MSB-interleaved 2-bit layout
// (sglang_backend/bitnet_quantization.py:69-409): ternarisation + packing,
// dequantisation, and the linear itself computed straight from the packed bytes.
//
// Layout (bitnet_quantization.py:99-105 / :128-133): byte j of row n holds
//   code(w[n,4j]) << 6 | code(w[n,4j+1]) << 4 | code(w[n,4j+2]) << 2 | code(w[n,4j+3]),
// code = w + 1 in {0,1,2}. The reference dequantises once to bf16 and runs x @ W^T; here the
// small-M linear reads the 2-bit bytes (8x fewer HBM bytes than the cached bf16 matrix) and turns
// codes into bf16/fp16 +-1/0 pairs in registers with byte permutes, accumulating with
// v_dot2c_f32_{bf16,f16}. Algorithmic bytes per launch = N*K/4 + M*K*2 + M*N*2 (HBM-bound).
#include <hip/hip_runtime.h>

#include "wf_common.h"
#include "wf_device.h"

namespace wf {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

// -------------------------------------------------------------------------------------------
// quantize_to_bitnet (bitnet_quantization.py:69-109): normalized = w / scale in the weight's dtype
// (torch CPU: fp32 true division by float(scale), rounded to the tensor dtype), code 2 if > 0.5,
// 0 if < -0.5, 1 if within [-0.5, 0.5]; a NaN stays at the zeros_like initial value (code 0).
// One thread per output byte (4 consecutive k).
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ternary_code(float w, float s, int dt) {
    float v = w / s;
    if (dt == DT_BF16) v = rbf(v);
    else if (dt == DT_F16) v = h2f(f2h(v));
    if (v > 0.5f) return 2u;
    if (v < -0.5f) return 0u;
    return (v >= -0.5f && v <= 0.5f) ? 1u : 0u;
}

__global__ void k_msb_ternarize(const void* __restrict__ w, int dt, int64_t nbytes, float s, uint8_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t b = 0;
#pragma unroll
        for (int p = 0; p < 4; ++p) b |= ternary_code(load_as_f32(w, 4 * i + p, dt), s, dt) << (6 - 2 * p);
        out[i] = (uint8_t)b;
    }
}

// dequantize_bitnet (bitnet_quantization.py:211-252; reference twin :115-137): value = (code - 1)
// as fp32 times float(scale), then the caller's dtype. One thread per packed dword (16 outputs).
__global__ void k_msb_dequant(const uint32_t* __restrict__ p, int64_t ndw, float s, void* __restrict__ out, int odt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ndw; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t w = p[i];
        float v[16];
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[4 * b + q] = (float)(int)(((w >> (8 * b + 6 - 2 * q)) & 3u) - 1u) * s;
        if (odt == DT_F32) {
            float4* o = reinterpret_cast<float4*>(out) + 4 * i;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
        } else {
            uint32_t h[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                h[j] = odt == DT_BF16 ? ((uint32_t)f2bf(v[2 * j]) | ((uint32_t)f2bf(v[2 * j + 1]) << 16))
                                      : ((uint32_t)f2h(v[2 * j]) | ((uint32_t)f2h(v[2 * j + 1]) << 16));
            uint4* o = reinterpret_cast<uint4*>(out) + 2 * i;
            o[0] = make_uint4(h[0], h[1], h[2], h[3]);
            o[1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
    }
}

// -------------------------------------------------------------------------------------------
// Small-M linear: y[m,n] = rnd(rnd(ws * sum_k (code-1) x[m,k]) + bias[n]), ws = the weight
// scale rounded to the compute dtype (the reference multiplies bf16(+-scale) weights).
//
// Block = 256 threads; G lanes own one weight row (256/G rows per block). A row is K/64 chunks of
// 16 bytes (64 weights); lane `sub` of the group loads chunks sub, sub+G, ... all in flight.
// Within a weight dword (bytes j..j+3 -> k = 4j..4j+15), bit-pair p of every byte is the code of
// k = 4j + 4b + p; (w >> (6-2p)) & 0x03030303 puts the 4 codes in byte lanes, a v_perm_b32 against
// a 3-entry byte table turns them into the high (and, for bf16, low) bytes of +-1/0, and two more
// permutes interleave them into two bf16/f16 pairs: (k+p, k+4+p) and (k+8+p, k+12+p).
// The activation image in LDS holds x in exactly that pair order: piece r (16 bytes) of chunk c =
// the 4 pairs {(p, 4+p) if r even, (8+p, 12+p) if odd} of dword r/2, p = 0..3, stored at
// ((c/16)*8 + r)*256 + (c%16)*16 so the 16 lanes reading one piece of consecutive chunks hit one
// contiguous 256-byte bank row (the other rows of the wave broadcast).
// -------------------------------------------------------------------------------------------
int launch_absmax(const void* x, int dt, int64_t n, float* out, hipStream_t st);  // wf_gemv.hip

constexpr int kMsbMaxMB = 4;
constexpr int kMsbMaxLds = 65536;  // activation images per launch (default dynamic-LDS limit)
constexpr int kMsbMaxCPL = 8;  // chunks per lane: K <= 8 * 32 * 64 = 16384

__host__ __device__ constexpr int msb_img_bytes(int K) { return ((K / 64 + 15) / 16) * 16 * 128; }

__device__ __forceinline__ int msb_piece_off(int c, int r) { return (((c >> 4) * 8 + r) << 8) + ((c & 15) << 4); }

template <bool BF>
__device__ __forceinline__ float dot2(uint32_t w, uint32_t x, float acc) {
    if constexpr (BF) return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, w), __builtin_bit_cast(bf16x2_t, x), acc, false);
    else return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, w), __builtin_bit_cast(f16x2_t, x), acc, false);
}

template <bool BF, int G, int MB, int CPL>
__global__ __launch_bounds__(256) void k_msb_linear(const uint8_t* __restrict__ W, const uint16_t* __restrict__ X,
                                                    int64_t ldx, int M, int N, int K, float ws,
                                                    const uint16_t* __restrict__ bias, uint16_t* __restrict__ Y,
                                                    int64_t ldy) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int nch = K / 64, img = msb_img_bytes(K);
    // stage x rows in pair order: one work item = (row m, chunk c, dword d) -> pieces 2d, 2d+1
    for (int it = threadIdx.x; it < MB * nch * 4; it += blockDim.x) {
        const int m = it / (nch * 4), rem = it - m * nch * 4, c = rem >> 2, d = rem & 3;
        uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
        if (m < M) {
            const uint4* src = reinterpret_cast<const uint4*>(X + (int64_t)m * ldx + 64 * c + 16 * d);
            a = src[0];
            b = src[1];
        }
        // a = x[0..7], b = x[8..15] (two per dword); pair (p, 4+p) and (8+p, 12+p)
        const uint4 p0 = make_uint4(__builtin_amdgcn_perm(a.z, a.x, 0x05040100), __builtin_amdgcn_perm(a.z, a.x, 0x07060302),
                                    __builtin_amdgcn_perm(a.w, a.y, 0x05040100), __builtin_amdgcn_perm(a.w, a.y, 0x07060302));
        const uint4 p1 = make_uint4(__builtin_amdgcn_perm(b.z, b.x, 0x05040100), __builtin_amdgcn_perm(b.z, b.x, 0x07060302),
                                    __builtin_amdgcn_perm(b.w, b.y, 0x05040100), __builtin_amdgcn_perm(b.w, b.y, 0x07060302));
        uint8_t* base = smem + m * img;
        *reinterpret_cast<uint4*>(base + msb_piece_off(c, 2 * d)) = p0;
        *reinterpret_cast<uint4*>(base + msb_piece_off(c, 2 * d + 1)) = p1;
    }

    const int lane = threadIdx.x & 63, sub = lane & (G - 1);
    const int n = blockIdx.x * (256 / G) + (threadIdx.x / G);
    const int nc = n < N ? n : N - 1;
    const uint8_t* wrow = W + (int64_t)nc * (K / 4);
    uint4 wv[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        const int c = sub + G * i;
        // chunks past the row end read as code 1 (weight 0)
        wv[i] = c < nch ? ldg_nt(wrow + 16 * c) : make_uint4(0x55555555u, 0x55555555u, 0x55555555u, 0x55555555u);
    }
    __syncthreads();

    // byte c: high byte of (c - 1); code 3 (never written by the packer) is +2 like dequantize_bitnet
    constexpr uint32_t LUT_HI = BF ? 0x403F00BFu : 0x403C00BCu;
    constexpr uint32_t LUT_LO = BF ? 0x00800080u : 0u;
    float acc[MB][2];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m][0] = acc[m][1] = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
        const int c = sub + G * i;
        if (c >= nch) break;
        const uint32_t wd[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            uint32_t pr[2][4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const uint32_t codes = (wd[d] >> (6 - 2 * p)) & 0x03030303u;
                const uint32_t hi = __builtin_amdgcn_perm(0u, LUT_HI, codes);
                if constexpr (BF) {
                    const uint32_t lo = __builtin_amdgcn_perm(0u, LUT_LO, codes);
                    pr[0][p] = __builtin_amdgcn_perm(hi, lo, 0x05010400);
                    pr[1][p] = __builtin_amdgcn_perm(hi, lo, 0x07030602);
                } else {
                    pr[0][p] = __builtin_amdgcn_perm(hi, 0u, 0x050C040C);
                    pr[1][p] = __builtin_amdgcn_perm(hi, 0u, 0x070C060C);
                }
            }
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const uint8_t* base = smem + m * img;
                const uint4 x0 = *reinterpret_cast<const uint4*>(base + msb_piece_off(c, 2 * d));
                const uint4 x1 = *reinterpret_cast<const uint4*>(base + msb_piece_off(c, 2 * d + 1));
                acc[m][0] = dot2<BF>(pr[0][0], x0.x, acc[m][0]);
                acc[m][1] = dot2<BF>(pr[0][1], x0.y, acc[m][1]);
                acc[m][0] = dot2<BF>(pr[0][2], x0.z, acc[m][0]);
                acc[m][1] = dot2<BF>(pr[0][3], x0.w, acc[m][1]);
                acc[m][0] = dot2<BF>(pr[1][0], x1.x, acc[m][0]);
                acc[m][1] = dot2<BF>(pr[1][1], x1.y, acc[m][1]);
                acc[m][0] = dot2<BF>(pr[1][2], x1.z, acc[m][0]);
                acc[m][1] = dot2<BF>(pr[1][3], x1.w, acc[m][1]);
            }
        }
    }
    float bv = 0.f;
    if (bias != nullptr) bv = BF ? bf2f(bias[nc]) : h2f(bias[nc]);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        const float s = group_reduce<G>(acc[m][0] + acc[m][1], OpAdd{});
        if (sub == 0 && n < N && m < M) {
            float y = s * ws;
            y = BF ? rbf(y) : h2f(f2h(y));
            if (bias != nullptr) y = y + bv;
            Y[(int64_t)m * ldy + n] = BF ? f2bf(y) : f2h(y);
        }
    }
}

template <bool BF, int G, int MB>
static void launch_msb(const uint8_t* w, const uint16_t* x, int64_t ldx, int M, int N, int K, float ws,
                       const uint16_t* bias, uint16_t* y, int64_t ldy, hipStream_t st) {
    const int rows = 256 / G;
    const size_t lds = (size_t)MB * msb_img_bytes(K);
    hipLaunchKernelGGL((k_msb_linear<BF, G, MB, kMsbMaxCPL>), dim3((N + rows - 1) / rows), dim3(256), lds, st, w, x,
                       ldx, M, N, K, ws, bias, y, ldy);
}

template <bool BF, int G>
static void launch_msb_mb(const uint8_t* w, const uint16_t* x, int64_t ldx, int M, int N, int K, float ws,
                          const uint16_t* bias, uint16_t* y, int64_t ldy, hipStream_t st) {
    if (M == 1) launch_msb<BF, G, 1>(w, x, ldx, M, N, K, ws, bias, y, ldy, st);
    else if (M == 2) launch_msb<BF, G, 2>(w, x, ldx, M, N, K, ws, bias, y, ldy, st);
    else launch_msb<BF, G, 4>(w, x, ldx, M, N, K, ws, bias, y, ldy, st);
}

}  // namespace wf

using namespace wf;

extern "C" int wf_absmax(const void* x, int dtype, int64_t n, float* out, void* stream) {
    WF_REQUIRE(x && out, "wf_absmax: null pointer");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "wf_absmax: dtype must be f32/bf16/f16");
    WF_REQUIRE(n >= 0, "wf_absmax: n < 0");
    hipStream_t st = as_stream(stream);
    WF_HIP(hipMemsetAsync(out, 0, sizeof(float), st));
    if (n == 0) return WF_OK;
    return launch_absmax(x, dtype, n, out, st);
}

extern "C" int wf_msb_ternarize(const void* w, int dtype, int N, int K, float scale, uint8_t* out, void* stream) {
    WF_REQUIRE(w && out, "wf_msb_ternarize: null pointer");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "wf_msb_ternarize: dtype must be f32/bf16/f16");
    WF_REQUIRE(N >= 0 && K > 0 && K % 4 == 0, "wf_msb_ternarize: K (%d) must be a positive multiple of 4", K);
    WF_REQUIRE(scale > 0.f, "wf_msb_ternarize: scale must be > 0");
    const int64_t nb = (int64_t)N * (K / 4);
    if (nb == 0) return WF_OK;
    int64_t blocks = (nb + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_msb_ternarize, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), w, dtype, nb, scale, out);
    return check_launch("k_msb_ternarize");
}

extern "C" int wf_msb_dequant(const uint8_t* packed, int N, int K, float scale, void* out, int out_dtype, void* stream) {
    WF_REQUIRE(packed && out, "wf_msb_dequant: null pointer");
    WF_REQUIRE(out_dtype == WF_F32 || out_dtype == WF_BF16 || out_dtype == WF_F16, "wf_msb_dequant: bad out dtype");
    WF_REQUIRE(N >= 0 && K > 0 && K % 16 == 0, "wf_msb_dequant: K (%d) must be a positive multiple of 16", K);
    WF_REQUIRE(aligned16(packed) && aligned16(out), "wf_msb_dequant: pointers must be 16-byte aligned");
    const int64_t ndw = (int64_t)N * (K / 16);
    if (ndw == 0) return WF_OK;
    int64_t blocks = (ndw + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_msb_dequant, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const uint32_t*>(packed), ndw, scale, out, out_dtype);
    return check_launch("k_msb_dequant");
}

extern "C" int wf_msb_linear(const uint8_t* w, float scale, const void* x, int x_dtype, int64_t ldx, int M, int N,
                             int K, const void* bias, void* y, int64_t ldy, void* stream) {
    WF_REQUIRE(w && x && y, "wf_msb_linear: null pointer");
    WF_REQUIRE(x_dtype == WF_BF16 || x_dtype == WF_F16, "wf_msb_linear: x dtype must be bf16 or f16");
    WF_REQUIRE(M >= 0 && N > 0 && K > 0, "wf_msb_linear: bad shape");
    if (K % 64 != 0 || K > kMsbMaxCPL * 32 * 64) {
        set_error("wf_msb_linear: K=%d unsupported (K %% 64 == 0 and K <= %d)", K, kMsbMaxCPL * 32 * 64);
        return WF_ENOTSUP;
    }
    WF_REQUIRE(ldx >= K && ldx % 8 == 0 && ldy >= N, "wf_msb_linear: bad strides");
    WF_REQUIRE(aligned16(x) && aligned16(w), "wf_msb_linear: x and w must be 16-byte aligned");
    if (M == 0) return WF_OK;
    hipStream_t st = as_stream(stream);
    const bool bf = x_dtype == WF_BF16;
    // the weight scale as the reference's weight tensor holds it: fp32 -> compute dtype
    const float ws = bf ? (float)(__bf16)scale : (float)(_Float16)scale;
    const int nch = K / 64;
    const auto* xb = static_cast<const uint16_t*>(x);
    const auto* bb = static_cast<const uint16_t*>(bias);
    auto* yb = static_cast<uint16_t*>(y);
    int mb = kMsbMaxLds / msb_img_bytes(K);
    if (mb > kMsbMaxMB) mb = kMsbMaxMB;
    for (int m0 = 0; m0 < M; m0 += mb) {
        const int mr = M - m0 < mb ? M - m0 : mb;
        const uint16_t* xm = xb + (int64_t)m0 * ldx;
        uint16_t* ym = yb + (int64_t)m0 * ldy;
        const bool g32 = nch > 16 * kMsbMaxCPL || nch >= 64;
        if (bf) {
            if (g32) launch_msb_mb<true, 32>(w, xm, ldx, mr, N, K, ws, bb, ym, ldy, st);
            else launch_msb_mb<true, 16>(w, xm, ldx, mr, N, K, ws, bb, ym, ldy, st);
        } else {
            if (g32) launch_msb_mb<false, 32>(w, xm, ldx, mr, N, K, ws, bb, ym, ldy, st);
            else launch_msb_mb<false, 16>(w, xm, ldx, mr, N, K, ws, bb, ym, ldy, st);
        }
        const int rc = check_launch("k_msb_linear");
        if (rc != WF_OK) return rc;
    }
    return WF_OK;
}
