// Which XCD runs which workgroup: every block stores its XCC_ID (s_getreg HW_REG_XCC_ID) so the host
// can check the round-robin assumption (block b on XCD b % 8) for 1-D and 3-D grids.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/xcd_map.hip -o tools/ubench/xcd_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(int* out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(id));
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (threadIdx.x == 0) out[lin] = (int)id;
}
int main() {
    int* d;
    hipMalloc(&d, 4 * 4096);
    const dim3 grids[] = {dim3(192), dim3(8, 20, 1), dim3(192, 1, 2), dim3(160), dim3(640)};
    for (const dim3& g : grids) {
        const int n = g.x * g.y * g.z;
        hipMemset(d, 0xff, 4 * n);
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k, g, dim3(256), 0, 0, d);
            std::vector<int> h(n);
            hipMemcpy(h.data(), d, 4 * n, hipMemcpyDeviceToHost);
            int match = 0;
            for (int i = 0; i < n; ++i) match += (h[i] == i % 8);
            printf("grid (%u,%u,%u) rep %d: %d / %d blocks on XCD (linear id %% 8); first 24:", g.x, g.y, g.z, rep, match, n);
            for (int i = 0; i < 24 && i < n; ++i) printf(" %d", h[i]);
            printf("\n");
        }
    }
    return 0;
}
