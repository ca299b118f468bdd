// wf_gemv.hip -- raw ternary GEMV/GEMM (sgl-kernel drop-in), activation quantizers and load-time
// weight-format kernels for gfx950.
//
// Roofline: the decode GEMV is HBM-bound. Algorithmic bytes per call = W_bytes + M*K + 4*M*N
// (scripts/benchmark_kernels.py:61-66), W_bytes = N*K/4 (I2S) or N*ceil(K/80)*16 (TQ).
#include <hip/hip_runtime.h>

#include <string.h>

#include "wf_common.h"
#include "wf_device.h"
#include "wf_norm.h"  // stamps (diagnostic build)
#include "wf_small.h"

namespace wf {

int launch_tgemm_mfma(const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K, float* y,
                      int64_t ldy, hipStream_t st);
constexpr int kMfmaMinM = 16;  // rows from which the int8-MFMA GEMM beats the VALU dot4 stream

static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// =============================================================================================
// Ternary GEMV / small-M GEMM.
// Block = 256 threads = 4 waves; a block owns 16 weight rows (4 per wave, 16 lanes per row) and
// MB activation rows. Each lane streams 16-byte chunks c = sub + 16*i of its row with U loads in
// flight, decodes trits in registers and accumulates sum(enc*a) with v_dot4_i32_i8 against the
// LDS activation image (conflict-free layout, see wf_device.h). The 16 lanes of a row reduce
// with 4 xor-shuffles; the epilogue is float(sum) * scale (bit-exact with the oracle).
// =============================================================================================
constexpr int kRowsPerBlock = 16;
constexpr int kUnroll = 4;

template <class F>
__device__ __forceinline__ void stage_activation_rows(int8_t* smem, int img, const int8_t* A, int64_t lda, int rows,
                                                      int MBcap, int K) {
    const int pieces = F::k_pad(K) / 16;
    for (int idx = threadIdx.x; idx < MBcap * pieces; idx += blockDim.x) {
        const int m = idx / pieces, p = idx - m * pieces;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (m < rows && p * 16 < K) v = *reinterpret_cast<const uint4*>(A + (int64_t)m * lda + p * 16);
        *reinterpret_cast<uint4*>(smem + m * img + F::lds_off(p * 16)) = v;
    }
}

template <class F, int MB>
__global__ __launch_bounds__(256) void k_ternary_gemm(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                      int64_t lda, float scale, int M, int N, int K,
                                                      float* __restrict__ Y, int64_t ldy) {
    extern __shared__ __attribute__((aligned(16))) int8_t smem[];
    const int img = lds_image_bytes<F>(K);
    const int m0 = blockIdx.y * MB;
    const int mrows = min(MB, M - m0);
    stage_activation_rows<F>(smem, img, A + (int64_t)m0 * lda, lda, mrows, MB, K);
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 15;
    const int row = blockIdx.x * kRowsPerBlock + wave * 4 + (lane >> 4);
    const int C = F::chunks(K);
    DotAcc<F> dacc[MB];
    if (row < N) {
        const uint8_t* wr = W + (int64_t)row * F::row_bytes(K) + sub * 16;
        for (int c0 = 0; c0 < C; c0 += 16 * kUnroll) {
            uint4 w[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int c = c0 + 16 * u + sub;
                w[u] = (c < C) ? ldg_nt(wr + (int64_t)(c0 + 16 * u) * 16) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int c = c0 + 16 * u + sub;
                if (c < C) {
                    Decoded<F> d;
                    d.load(w[u]);
                    const int8_t* ab = smem + ((c >> 4) * F::kGroups) * 256 + sub * 16;
#pragma unroll
                    for (int m = 0; m < MB; ++m) chunk_dot<F>(d, ab + m * img, dacc[m]);
                }
            }
        }
    }
    int acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) acc[m] = group16_sum_i(dacc[m].total());
    if (row < N && sub == 0) {
#pragma unroll
        for (int m = 0; m < MB; ++m)
            if (m < mrows) Y[(int64_t)(m0 + m) * ldy + row] = (float)acc[m] * scale;
    }
}

// ---------------------------------------------------------------------------------------------
// Standalone GEMV (M = 1; sgl_kernel bitnet_gemv, scripts/benchmark_kernels.py:40-66): a memory-
// latency problem -- 0.4-4.5 MB per call, i.e. 1.6-17 KB per CU -- so every byte of the matrix is
// in flight at once and as many CUs as possible take part. One wave per weight row (lane l takes
// chunks l + 64 j), NW waves per block. Issue order: the activation pieces (L2-resident), then every weight chunk of
// the lane (nt), then the activation image goes to LDS (conflict-free stripes, wf_device.h) behind
// one barrier that the weight latency hides. Each wave sums its lanes with DPP; the W wave partials
// of a row meet in LDS in wave order. Integer sums: bit-exact with any split.
// ---------------------------------------------------------------------------------------------
constexpr int kGemvMaxPieces = 2;  // 16-byte activation pieces per thread: K_pad <= 8192
template <class F, int NW, int J>
__global__ __launch_bounds__(NW * 64) void k_gemv_rows(const uint8_t* __restrict__ Wt, const int8_t* __restrict__ A,
                                                       float scale, int N, int K, float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) int8_t smem[];
    constexpr int NT = NW * 64, MAXP = (8192 / 16 + NT - 1) / NT;  // activation pieces per thread
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    WF_STAMP(0);
    const int row = blockIdx.x * NW + wave;
    const int C = F::chunks(K);
    const int pieces = F::k_pad(K) / 16;
    uint4 apre[MAXP];
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
        const int p = min((int)threadIdx.x + NT * i, pieces - 1), pk = min(p, K / 16 - 1);
        apre[i] = *reinterpret_cast<const uint4*>(A + 16 * pk);  // pieces >= K/16: zeroed below
    }
    const uint8_t* wr = Wt + (int64_t)min(row, N - 1) * F::row_bytes(K);
    uint4 wv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) wv[j] = ldg_nt(wr + (int64_t)min(lane + 64 * j, C - 1) * 16);
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
        const int p = (int)threadIdx.x + NT * i;
        if (p < pieces)
            *reinterpret_cast<uint4*>(smem + F::lds_off(16 * p)) = 16 * p < K ? apre[i] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    DotAcc<F> dacc;
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int c = lane + 64 * j;
        if (c < C) {
            Decoded<F> d;
            d.load(wv[j]);
            chunk_dot<F>(d, smem + ((c >> 4) * F::kGroups) * 256 + (c & 15) * 16, dacc);
        }
    }
    const int acc = wave_sum_i(dacc.total());
    if (lane == 0 && row < N) Y[row] = (float)acc * scale;
#ifdef WF_STAMPS
    __syncthreads();  // stamps build: waves 0-3 stamp, so the exit is taken once every wave is done
#endif
    WF_STAMP(1);
}


template <class F>
static int launch_gemv_rows(const uint8_t* w, const int8_t* a, float scale, int N, int K, float* y, hipStream_t st) {
    // one wave per row; NW rows (waves) per block share one LDS activation image. Measured (graph
    // replay, same box, tools/gemv_bench.py, profiles/gemv_ab_r03.txt): splitting rows over 2-4 waves
    // to reach >= 1024 blocks was slower (q/o 2.91 -> 2.49 us, k/v 2.56 -> 2.18, down 3.27 -> 3.17
    // with one wave per row); 8 rows per block helps only q/o (2.48 -> 2.43 us); 16 rows for gate|up
    // (3.08 -> 3.20) and 2 rows for k/v (2.18 -> 2.40) lost.
    const int J = (F::chunks(K) + 63) / 64;
#ifdef WF_GEMV_WAVES
    const int NW = WF_GEMV_WAVES;
#else
    const int NW = (N >= 2048 && N < 4096 && J == 1) ? 8 : 4;
#endif
    const int img = lds_image_bytes<F>(K);
    const dim3 grid((N + NW - 1) / NW);
#define WF_GR(NWV, JV) hipLaunchKernelGGL((k_gemv_rows<F, NWV, JV>), grid, dim3(NWV * 64), (size_t)img, st, w, a, scale, N, K, y)
#define WF_GRJ(NWV)            \
    if (J == 1) WF_GR(NWV, 1); \
    else WF_GR(NWV, 2);
    if (NW == 8) { WF_GRJ(8) }
    else { WF_GRJ(4) }
#undef WF_GRJ
#undef WF_GR
    return check_launch("gemv_rows");
}

template <class F>
static int launch_ternary_gemm(const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K,
                               float* y, int64_t ldy, hipStream_t st) {
    // GEMV with K_pad <= 8192 and at most 2 chunks per lane: the wave-per-row kernel
    if (M == 1 && F::k_pad(K) <= 256 * 16 * kGemvMaxPieces && F::chunks(K) <= 128)
        return launch_gemv_rows<F>(w, a, scale, N, K, y, st);
    const int img = lds_image_bytes<F>(K);
    const dim3 block(256);
    const int gx = (N + kRowsPerBlock - 1) / kRowsPerBlock;
#define WF_GEMM_CASE(MBV)                                                                                  \
    {                                                                                                      \
        const dim3 grid(gx, (M + MBV - 1) / MBV);                                                          \
        hipLaunchKernelGGL((k_ternary_gemm<F, MBV>), grid, block, (size_t)img * MBV, st, w, a, lda, scale, \
                           M, N, K, y, ldy);                                                               \
    }
    if (M == 1) WF_GEMM_CASE(1)
    else if (M == 2) WF_GEMM_CASE(2)
    else if (M <= 4) WF_GEMM_CASE(4)
    else WF_GEMM_CASE(8)
#undef WF_GEMM_CASE
    return check_launch("ternary_gemm");
}

// Small-M GEMM (2 <= M <= kSmallMaxM): wf_small.h.
// fp32 output of the raw GEMM: Y = float(sum) * scale (the small-M kernel's epilogue)
struct EpiRawSmall {
    float* Y;
    int64_t ldy;
    float scale;
    int M, N;
    __device__ __forceinline__ void apply(int r0, int c0, const v4i_t& acc, int l16, int q) const {
        const int n = c0 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r0 + 4 * q + r;
            if (m < M && n < N) Y[(int64_t)m * ldy + n] = (float)acc[r] * scale;
        }
    }
};

// kernels/native.py:27-65: signed LSB-layout dot. Simple, correctness-first (not on the hot path:
// the reference's own fast path is sgl-kernel's blocked layout above).
__global__ __launch_bounds__(256) void k_lsb_gemm(const uint8_t* __restrict__ W, const int8_t* __restrict__ A,
                                                  float scale, int M, int N, int K, float* __restrict__ Y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int m = blockIdx.y;
    if (row >= N) return;
    const uint8_t* wr = W + (int64_t)row * (K / 4);
    const int8_t* ar = A + (int64_t)m * K;
    int acc = 0;
    for (int j = lane; j < K / 4; j += 64) {
        const uint32_t b = wr[j];
        const uint32_t e = (b & 3u) | (((b >> 2) & 3u) << 8) | (((b >> 4) & 3u) << 16) | (((b >> 6) & 3u) << 24);
        const uint32_t av = *reinterpret_cast<const uint32_t*>(ar + 4 * j);
        // sum (e-1)*a = sum e*a - sum a
        acc = sdot4(e, av, acc);
        acc -= (int)(int8_t)(av) + (int)(int8_t)(av >> 8) + (int)(int8_t)(av >> 16) + (int)(int8_t)(av >> 24);
    }
    acc = wave_sum_i(acc);
    if (lane == 0) Y[(int64_t)m * N + row] = (float)acc * scale;
}

// =============================================================================================
// Activation quantizers.
// =============================================================================================
__global__ __launch_bounds__(256) void k_absmax(const void* __restrict__ x, int dt, int64_t n,
                                                unsigned* __restrict__ out) {
    __shared__ float red[16];
    float m = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(load_as_f32(x, i, dt)));
    m = block_max(m, red);
    if (threadIdx.x == 0) atomicMax(out, __float_as_uint(m));  // |x| >= 0: uint order == float order
}

// mode 0: activation quantizer (x / float(m/127), clamp [-128,127]); mode 1: truncating numpy
// variant (kernels/native.py:253-255); mode 2: KV int8 (x * float(127/m), clamp [-127,127]).
__global__ __launch_bounds__(256) void k_quant_apply(const void* __restrict__ x, int dt, int64_t n,
                                                     const float* __restrict__ mx, int8_t* __restrict__ q, int mode) {
    const float m = *mx;
    float sf;
    if (mode == 0) sf = (float)act_scale_from_max(m);
    else if (mode == 1) sf = (m > 1e-6f) ? (float)((double)m / 127.0) : 1.0f;
    else sf = (float)(127.0 / ((double)m < 1e-6 ? 1.0 : (double)m));
    if (mode == 0) {  // 8 codes per thread through quant8 (the decode step's quantizer), scalar tail
        const float inv = 1.0f / sf;
        const int64_t n8 = n / 8;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = load_as_f32(x, 8 * i + j, dt);
            int dummy = 0;
            const uint2 pk = quant8(v, sf, inv, dummy);
#pragma unroll
            for (int j = 0; j < 8; ++j) q[8 * i + j] = (int8_t)(((j < 4 ? pk.x : pk.y) >> (8 * (j & 3))) & 0xff);
        }
        for (int64_t i = 8 * n8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
            q[i] = quant_one(load_as_f32(x, i, dt), sf);
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = load_as_f32(x, i, dt);
        int8_t r;
        if (mode == 0) r = quant_one(v, sf);
        else if (mode == 1) r = (int8_t)(int)fminf(fmaxf(v / sf, -128.f), 127.f);
        else r = (int8_t)(int)fminf(fmaxf(rintf(v * sf), -127.f), 127.f);
        q[i] = r;
    }
}

__global__ __launch_bounds__(256) void k_quant_rows(const void* __restrict__ x, int dt, int K,
                                                    int8_t* __restrict__ q, float* __restrict__ row_max) {
    __shared__ float red[16];
    const int64_t base = (int64_t)blockIdx.x * K;
    float m = 0.f;
    for (int k = threadIdx.x; k < K; k += blockDim.x) m = fmaxf(m, fabsf(load_as_f32(x, base + k, dt)));
    m = block_max(m, red);
    const float sf = (float)act_scale_from_max(m);
    for (int k = threadIdx.x; k < K; k += blockDim.x) q[base + k] = quant_one(load_as_f32(x, base + k, dt), sf);
    if (threadIdx.x == 0) row_max[blockIdx.x] = m;
}

__global__ void k_kv_dequant(const int8_t* __restrict__ q, int64_t n, const float* __restrict__ scale,
                             void* __restrict__ out, int odt) {
    const float s = *scale;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // kv_cache.py:226-228: tensor.to(float32) * scale -> .to(bfloat16)
        store_from_f32(out, i, odt, rbf((float)q[i] * s));
    }
}

// =============================================================================================
// Load-time weight formats.
// =============================================================================================
// cache/bitnet_converter.py:26-77 for K % 128 == 0: one thread per output byte.
__global__ void k_pack_i2s(const void* __restrict__ w, int dt, int N, int K, uint8_t* __restrict__ out) {
    const int64_t nb = (int64_t)N * (K / 4);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = i / (K / 4);
        const int j = (int)(i - n * (K / 4));
        const int b = j >> 5, k = j & 31;
        const int64_t base = n * K + b * 128 + k;
        uint32_t v = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float t = rintf(load_as_f32(w, base + 32 * g, dt));
            t = fminf(fmaxf(t, -1.f), 1.f);
            v |= (uint32_t)((int)t + 1) << (6 - 2 * g);
        }
        out[i] = (uint8_t)v;
    }
}

// HF [N/4, K] (tests/test_bitnet_core.py:21-53: packed row r bits 2i -> out row i*(N/4)+r) -> I2S.
// The invalid HF code 3 unpacks to +2 in the reference; round(2).clamp(-1,1) then packs it as +1.
__global__ void k_hf_to_i2s(const uint8_t* __restrict__ hf, int Np, int K, uint8_t* __restrict__ out) {
    const int N = Np * 4;
    const int64_t nb = (int64_t)N * (K / 4);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = i / (K / 4);
        const int j = (int)(i - n * (K / 4));
        const int b = j >> 5, k = j & 31;
        const int ii = (int)(n / Np), r = (int)(n - (int64_t)ii * Np);
        uint32_t v = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            uint32_t e = (hf[(int64_t)r * K + b * 128 + k + 32 * g] >> (2 * ii)) & 3u;
            if (e > 2u) e = 2u;
            v |= e << (6 - 2 * g);
        }
        out[i] = (uint8_t)v;
    }
}

// I2S -> TQ: one thread per TQ byte (digit i of byte j of chunk c = weight 80c + 16i + j).
// I2_S <-> matrix-core tiles (include/wf_bitnet.h WF_FMT_I2S_MFMA), one thread per dword.
__global__ void k_i2s_mfma(const uint8_t* __restrict__ in, int N, int K, uint8_t* __restrict__ out, int fwd) {
    const int nkb = K >> 7;
    const int64_t nd = (int64_t)N * K / 16;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nd; t += (int64_t)gridDim.x * blockDim.x) {
        const int h = (int)(t & 1), lane = (int)((t >> 1) & 63);
        const int64_t blk = t >> 7;  // ct * nkb + kb
        const int kb = (int)(blk % nkb);
        const int64_t ct = blk / nkb;
        const int64_t n = ct * 16 + (lane & 15);
        const int64_t src = n * (K / 4) + 32 * kb + 16 * h + 4 * (lane >> 4);
        if (fwd) reinterpret_cast<uint32_t*>(out)[t] = *reinterpret_cast<const uint32_t*>(in + src);
        else *reinterpret_cast<uint32_t*>(out + src) = reinterpret_cast<const uint32_t*>(in)[t];
    }
}

__global__ void k_i2s_to_tq(const uint8_t* __restrict__ in, int N, int K, uint8_t* __restrict__ out) {
    const int C = FmtTQ::chunks(K);
    const int64_t nb = (int64_t)N * C * 16;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = i / (C * 16);
        const int rem = (int)(i - n * C * 16), c = rem >> 4, j = rem & 15;
        const uint8_t* row = in + n * (K / 4);
        int v = 0;
#pragma unroll
        for (int d = 0; d < 5; ++d) {
            const int k = 80 * c + 16 * d + j;
            int e = 1;
            if (k < K) {
                const int b = k >> 7, r = k & 127, g = r >> 5, jj = r & 31;
                e = (row[b * 32 + jj] >> (6 - 2 * g)) & 3;
            }
            v = v * 3 + e;
        }
        out[i] = (uint8_t)((v * 256 + 242) / 243);
    }
}

// TQ -> I2S: one thread per I2S byte.
__global__ void k_tq_to_i2s(const uint8_t* __restrict__ in, int N, int K, uint8_t* __restrict__ out) {
    const int C = FmtTQ::chunks(K);
    const int64_t nb = (int64_t)N * (K / 4);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n = i / (K / 4);
        const int jb = (int)(i - n * (K / 4));
        const int b = jb >> 5, jj = jb & 31;
        uint32_t v = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int k = b * 128 + 32 * g + jj;
            const int c = k / 80, r = k - c * 80, d = r >> 4, j = r & 15;
            uint32_t q = in[n * C * 16 + c * 16 + j];
            for (int s = 0; s < d; ++s) q = (q * 3u) & 0xffu;
            v |= ((q * 3u) >> 8) << (6 - 2 * g);
        }
        out[i] = (uint8_t)v;
    }
}

static inline int grid_for(int64_t n, int per = 256, int cap = 4096) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

}  // namespace wf

WF_STAMP_READER(wf_debug_stamps_gemv)

using namespace wf;

namespace wf {
int launch_absmax(const void* x, int dt, int64_t n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_absmax, dim3(grid_for(n, 256, 2048)), dim3(256), 0, st, x, dt, n, reinterpret_cast<unsigned*>(out));
    return check_launch("absmax");
}
}  // namespace wf

extern "C" {

const char* wf_last_error(void) { return wf::g_err; }
int wf_abi_version(void) { return 1; }

int wf_check_kernel_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

int wf_bitnet_gemm_ex(int fmt, const uint8_t* w, const int8_t* a, int64_t lda, float scale, int M, int N, int K,
                      float* y, int64_t ldy, void* stream) {
    WF_REQUIRE(w && a && y, "bitnet_gemm: null pointer");
    WF_REQUIRE(M > 0 && N > 0 && K > 0, "bitnet_gemm: bad shape M=%d N=%d K=%d", M, N, K);
    WF_REQUIRE(K % 128 == 0, "bitnet_gemm: in_features (%d) must be a multiple of BITNET_BLOCK_SIZE=128", K);
    WF_REQUIRE(lda >= K && lda % 16 == 0 && aligned16(a) && aligned16(w), "bitnet_gemm: activations/weights must be 16-byte aligned rows");
    WF_REQUIRE(ldy >= N, "bitnet_gemm: bad ldy");
    hipStream_t st = as_stream(stream);
    // batched rows go to the matrix cores (wf_mfma.hip); GEMV / small M stream on the VALU
#ifndef WF_GEMM_SMALL  // study: 0 = M 2..64 on the VALU stream / 128 x 64 LDS-DMA tiles as before
#define WF_GEMM_SMALL 1
#endif
    if (WF_GEMM_SMALL && fmt == WF_FMT_I2S && gemm_small_ok(M, N) && K >= 16)
        return launch_gemm_small_mfma(w, a, lda, M, N, K, EpiRawSmall{y, ldy, scale, M, N}, st), check_launch("gemm_small_mfma");
    if (fmt == WF_FMT_I2S && M >= kMfmaMinM) return launch_tgemm_mfma(w, a, lda, scale, M, N, K, y, ldy, st);
    if (fmt == WF_FMT_I2S) return launch_ternary_gemm<FmtI2S>(w, a, lda, scale, M, N, K, y, ldy, st);
    if (fmt == WF_FMT_TQ) return launch_ternary_gemm<FmtTQ>(w, a, lda, scale, M, N, K, y, ldy, st);
    WF_REQUIRE(false, "bitnet_gemm: unknown weight format %d", fmt);
}

int wf_bitnet_gemv(const uint8_t* w, const int8_t* a, float scale, int N, int K, float* y, void* stream) {
    return wf_bitnet_gemm_ex(WF_FMT_I2S, w, a, K, scale, 1, N, K, y, N, stream);
}

int wf_bitnet_gemm(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y, void* stream) {
    return wf_bitnet_gemm_ex(WF_FMT_I2S, w, a, K, scale, M, N, K, y, N, stream);
}

int wf_bitnet_gemm_lsb(const uint8_t* w, const int8_t* a, float scale, int M, int N, int K, float* y, void* stream) {
    WF_REQUIRE(w && a && y && M > 0 && N > 0 && K > 0 && K % 4 == 0, "gemm_lsb: bad arguments");
    WF_REQUIRE(((uintptr_t)a & 3u) == 0, "gemm_lsb: activations must be 4-byte aligned");
    hipLaunchKernelGGL(k_lsb_gemm, dim3((N + 3) / 4, M), dim3(256), 0, as_stream(stream), w, a, scale, M, N, K, y);
    return check_launch("gemm_lsb");
}

static int quant_common(const void* x, int dtype, int64_t n, int8_t* q, float* absmax, void* stream, int mode) {
    WF_REQUIRE(x && q && absmax && n > 0, "quantize: bad arguments");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "quantize: unsupported dtype %d", dtype);
    hipStream_t st = as_stream(stream);
    WF_HIP(hipMemsetAsync(absmax, 0, sizeof(float), st));
    const int g = grid_for(n, 256, 2048);
    hipLaunchKernelGGL(k_absmax, dim3(g), dim3(256), 0, st, x, dtype, n, reinterpret_cast<unsigned*>(absmax));
    hipLaunchKernelGGL(k_quant_apply, dim3(g), dim3(256), 0, st, x, dtype, n, absmax, q, mode);
    return check_launch("quantize");
}

int wf_quantize_i8(const void* x, int dtype, int64_t n, int8_t* q, float* absmax, void* stream) {
    return quant_common(x, dtype, n, q, absmax, stream, 0);
}
int wf_quantize_i8_trunc(const void* x, int dtype, int64_t n, int8_t* q, float* absmax, void* stream) {
    return quant_common(x, dtype, n, q, absmax, stream, 1);
}

int wf_quantize_i8_rows(const void* x, int dtype, int M, int K, int8_t* q, float* row_absmax, void* stream) {
    WF_REQUIRE(x && q && row_absmax && M > 0 && K > 0, "quantize_rows: bad arguments");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "quantize_rows: unsupported dtype %d", dtype);
    hipLaunchKernelGGL(k_quant_rows, dim3(M), dim3(256), 0, as_stream(stream), x, dtype, K, q, row_absmax);
    return check_launch("quantize_rows");
}

int wf_kv_quant_i8(const void* x, int dtype, int64_t n, const float* absmax, int8_t* q, void* stream) {
    WF_REQUIRE(x && q && absmax && n > 0, "kv_quant: bad arguments");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "kv_quant: unsupported dtype %d", dtype);
    hipLaunchKernelGGL(k_quant_apply, dim3(grid_for(n, 256, 2048)), dim3(256), 0, as_stream(stream), x, dtype, n,
                       absmax, q, 2);
    return check_launch("kv_quant");
}

int wf_kv_dequant_i8(const int8_t* q, int64_t n, const float* scale, void* out, int out_dtype, void* stream) {
    WF_REQUIRE(q && scale && out && n > 0, "kv_dequant: bad arguments");
    WF_REQUIRE(out_dtype == WF_F32 || out_dtype == WF_BF16 || out_dtype == WF_F16, "kv_dequant: bad dtype");
    hipLaunchKernelGGL(k_kv_dequant, dim3(grid_for(n, 256, 2048)), dim3(256), 0, as_stream(stream), q, n, scale, out,
                       out_dtype);
    return check_launch("kv_dequant");
}

int wf_pack_i2s(const void* w, int dtype, int N, int K, uint8_t* out, void* stream) {
    WF_REQUIRE(w && out && N > 0 && K > 0 && K % 128 == 0, "pack_i2s: bad arguments (K %% 128 == 0 required)");
    WF_REQUIRE(dtype == WF_F32 || dtype == WF_BF16 || dtype == WF_F16, "pack_i2s: unsupported dtype %d", dtype);
    hipLaunchKernelGGL(k_pack_i2s, dim3(grid_for((int64_t)N * K / 4)), dim3(256), 0, as_stream(stream), w, dtype, N,
                       K, out);
    return check_launch("pack_i2s");
}

int wf_hf_to_i2s(const uint8_t* hf, int Np, int K, uint8_t* out, void* stream) {
    WF_REQUIRE(hf && out && Np > 0 && K > 0 && K % 128 == 0, "hf_to_i2s: bad arguments (K %% 128 == 0 required)");
    hipLaunchKernelGGL(k_hf_to_i2s, dim3(grid_for((int64_t)Np * K)), dim3(256), 0, as_stream(stream), hf, Np, K, out);
    return check_launch("hf_to_i2s");
}

int64_t wf_tq_row_bytes(int K) { return FmtTQ::row_bytes(K); }

int wf_i2s_to_mfma(const uint8_t* i2s, int N, int K, uint8_t* out, void* stream) {
    WF_REQUIRE(i2s && out && N > 0 && N % 16 == 0 && K > 0 && K % 128 == 0, "i2s_to_mfma: bad arguments");
    hipLaunchKernelGGL(k_i2s_mfma, dim3(grid_for((int64_t)N * K / 16)), dim3(256), 0, as_stream(stream), i2s, N, K, out, 1);
    return check_launch("i2s_to_mfma");
}

int wf_mfma_to_i2s(const uint8_t* mf, int N, int K, uint8_t* i2s, void* stream) {
    WF_REQUIRE(i2s && mf && N > 0 && N % 16 == 0 && K > 0 && K % 128 == 0, "mfma_to_i2s: bad arguments");
    hipLaunchKernelGGL(k_i2s_mfma, dim3(grid_for((int64_t)N * K / 16)), dim3(256), 0, as_stream(stream), mf, N, K, i2s, 0);
    return check_launch("mfma_to_i2s");
}

int wf_i2s_to_tq(const uint8_t* i2s, int N, int K, uint8_t* tq, void* stream) {
    WF_REQUIRE(i2s && tq && N > 0 && K > 0 && K % 128 == 0, "i2s_to_tq: bad arguments");
    hipLaunchKernelGGL(k_i2s_to_tq, dim3(grid_for((int64_t)N * FmtTQ::row_bytes(K))), dim3(256), 0,
                       as_stream(stream), i2s, N, K, tq);
    return check_launch("i2s_to_tq");
}

int wf_tq_to_i2s(const uint8_t* tq, int N, int K, uint8_t* i2s, void* stream) {
    WF_REQUIRE(i2s && tq && N > 0 && K > 0 && K % 128 == 0, "tq_to_i2s: bad arguments");
    hipLaunchKernelGGL(k_tq_to_i2s, dim3(grid_for((int64_t)N * K / 4)), dim3(256), 0, as_stream(stream), tq, N, K,
                       i2s);
    return check_launch("tq_to_i2s");
}

}  // extern "C"
