// Micro-benchmark of in-block synchronisation costs on gfx950 (256-thread blocks): barrier, DPP
// wave reduction, block reduction through LDS, and a diagnostic stamp. Prints shader cycles per
// operation (s_memtime) measured by wave 0 of block 0.  hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../wrinklefree-inference-engine_amd/csrc/wf_device.h"

using namespace wf;
constexpr int R = 64;

__device__ __forceinline__ unsigned long long clk() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ __launch_bounds__(256) void k(float* out, unsigned long long* cyc, float seed) {
    __shared__ float red[8];
    float v = seed * threadIdx.x;
    unsigned long long t[6];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
    t[0] = clk();
    for (int i = 0; i < R; ++i) { __syncthreads(); }
    __builtin_amdgcn_sched_barrier(0);
    t[1] = clk();
    for (int i = 0; i < R; ++i) { v = wave_sum(v) * 1e-3f + seed; }
    __builtin_amdgcn_sched_barrier(0);
    t[2] = clk();
    for (int i = 0; i < R; ++i) {
        float s = wave_sum(v);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        v = ((red[0] + red[1]) + (red[2] + red[3])) * 1e-3f + seed;
        __syncthreads();
    }
    __builtin_amdgcn_sched_barrier(0);
    t[3] = clk();
    for (int i = 0; i < R; ++i) {
        unsigned long long r = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) cyc[64 + i] = r;
    }
    __builtin_amdgcn_sched_barrier(0);
    t[4] = clk();
    for (int i = 0; i < R; ++i) v = fmaf(v, 1.0001f, seed);  // dependent VALU chain
    __builtin_amdgcn_sched_barrier(0);
    t[5] = clk();
    out[blockIdx.x * 256 + threadIdx.x] = v;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        for (int i = 0; i < 5; ++i) cyc[i] = t[i + 1] - t[i];
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 4 << 20);
    hipMalloc(&cyc, 4096);
    const char* names[5] = {"barrier", "wave_sum(DPP)", "block_sum(DPP+LDS+2 barriers)", "memrealtime+store", "dependent fma"};
    for (int grid : {1, 256, 1024}) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, cyc, 1.0f);
        hipDeviceSynchronize();
        unsigned long long h[5];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("grid %4d:", grid);
        for (int i = 0; i < 5; ++i) printf("  %s %.1f", names[i], (double)h[i] / R);
        printf("  (cycles per op)\n");
    }
    return 0;
}
