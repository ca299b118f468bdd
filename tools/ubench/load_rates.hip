// Micro-benchmark: per-CU global-load throughput on gfx950 for the fragment access patterns of the
// batched decode GEMM / attention (one 512-thread block per CU, every CU loading at once).
// Patterns (per wave-instruction, lane = (l16 = lane & 15, q = lane >> 4)):
//   0 contig  : 1 KiB contiguous (dwordx4 per lane)
//   1 rows64  : 16 rows x 64 contiguous bytes (dwordx4), A fragment with a permuted code layout
//   2 rows16x4: 16 rows x four 16-byte pieces at a 32-byte stride (dwordx4), the I2_S A fragment
//   3 dup4    : 16 rows x 16 bytes, each read by the 4 lanes q (dwordx4), the I2_S B fragment
//   4 dword16 : 16 rows x 16 bytes as 4 dwords (lane q reads bytes 4q..4q+3), B fragment permuted
// Source: "l2" = every block reads the same 2.5 MiB region (L2 / MALL hits after first touch),
// "hbm" = each block its own region of a 1 GiB buffer.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/load_rates.hip -o tools/ubench/load_rates
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

constexpr int NT = 512, NI = 16;  // loads in flight per wave per round
constexpr int64_t kRowStride = 2560;

template <int P>
__device__ __forceinline__ int64_t addr(int wave, int lane, int i, int r) {
    const int l16 = lane & 15, q = lane >> 4;
    const int64_t step = (int64_t)(r * 8 + wave) * NI + i;  // distinct per (round, wave, i)
    if (P == 0) return step * 1024 + lane * 16;
    const int64_t row = (step % 64) * 16 + l16;               // 1024 rows
    const int64_t col = (step / 64) * 64;                     // next 64-byte column band
    if (P == 1) return row * kRowStride + (col % kRowStride) + q * 16;
    if (P == 2) return row * kRowStride + ((step / 64) * 128 % kRowStride) + 32 * q + 16 * (i & 1);
    if (P == 3) return row * kRowStride + (col % kRowStride);
    return row * kRowStride + (col % kRowStride) + 4 * q;
}

template <int P>
__global__ __launch_bounds__(NT) void k(const uint8_t* __restrict__ buf, int64_t region, int shared, int rounds,
                                        unsigned* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint8_t* base = buf + (shared ? 0 : (int64_t)blockIdx.x * region);
    unsigned x = 0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rounds; ++r) {
        if (P == 4) {
            unsigned v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) v[i] = *reinterpret_cast<const unsigned*>(base + (addr<P>(wave, lane, i, r) % region & ~3ll));
#pragma unroll
            for (int i = 0; i < NI; ++i) x ^= v[i];
        } else {
            uint4 v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) v[i] = *reinterpret_cast<const uint4*>(base + (addr<P>(wave, lane, i, r) % region & ~15ll));
#pragma unroll
            for (int i = 0; i < NI; ++i) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (x == 0x12345678u) out[0] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
    const int nblk = 256, rounds = argc > 1 ? atoi(argv[1]) : 8;
    const int64_t region = 1024 * kRowStride;  // 2.5 MiB
    uint8_t* buf;
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&buf, region * nblk);
    hipMemset(buf, 1, region * nblk);
    hipMalloc(&out, 64);
    hipMalloc(&cyc, 8 * nblk);
    unsigned long long h[256];
    const char* names[] = {"contig", "rows64", "rows16x4", "dup4", "dword16"};
    for (int shared = 1; shared >= 0; --shared) {
        for (int p = 0; p < 5; ++p) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                switch (p) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(nblk), dim3(NT), 0, 0, buf, region, shared, rounds, out, cyc); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(nblk), dim3(NT), 0, 0, buf, region, shared, rounds, out, cyc); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(nblk), dim3(NT), 0, 0, buf, region, shared, rounds, out, cyc); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(nblk), dim3(NT), 0, 0, buf, region, shared, rounds, out, cyc); break;
                    default: hipLaunchKernelGGL(k<4>, dim3(nblk), dim3(NT), 0, 0, buf, region, shared, rounds, out, cyc); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            hipMemcpy(h, cyc, 8 * nblk, hipMemcpyDeviceToHost);
            double mean = 0;
            for (int b = 0; b < nblk; ++b) mean += h[b];
            mean /= nblk;
            const double lane_bytes = (double)rounds * 8 * NI * 64 * (p == 4 ? 4 : 16);
            printf("%-4s %-9s lane-bytes/block %8.0f KiB  cycles/block %8.0f  lane-B/clk/CU %6.1f  kernel %.1f us\n",
                   shared ? "l2" : "hbm", names[p], lane_bytes / 1024, mean, lane_bytes / mean, best * 1000);
        }
    }
    return 0;
}
