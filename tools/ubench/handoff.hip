// One-to-one hand-off latency between two workgroups on the same XCD (block 0 -> block 8) and on two
// XCDs (block 0 -> block 1), per store / load flavour. Block 0 stamps, stores a tagged word; the
// consumer polls (bounded) and stamps when it sees the tag. Prints the median latency (100 MHz
// s_memrealtime ticks -> us) over repetitions and whether the tag was seen.
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/handoff.hip -o tools/ubench/handoff
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7fffffff, 0x00020000);
}
template <int SF, int LF>
__global__ void k(unsigned* flag, unsigned long long* t, int consumer, unsigned tag) {
    if (threadIdx.x != 0) return;
    const __amdgpu_buffer_rsrc_t r = rs(flag);
    if (blockIdx.x == 0) {
        __builtin_amdgcn_s_sleep(127);  // let the consumer start polling
        __builtin_amdgcn_s_sleep(127);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        if (SF == 0) __hip_atomic_store(flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
        else __builtin_amdgcn_raw_buffer_store_b32(tag, r, 0, 0, SF);  // aux flavour
        t[0] = t0;
    } else if ((int)blockIdx.x == consumer) {
        unsigned v = 0;
        int it = 0;
        for (; it < (1 << 20); ++it) {
            if (LF == 100) {
                v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
            } else if (LF == 101) {
                asm volatile("buffer_inv sc0" ::: "memory");
                v = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0);
            } else {
                v = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, LF);
            }
            if (v == tag) break;
        }
        t[1] = __builtin_amdgcn_s_memrealtime();
        t[2] = (unsigned long long)it;
        t[3] = v == tag;
    }
}
template <int SF, int LF>
void run(const char* name, unsigned* flag, unsigned long long* t) {
    for (int consumer : {8, 1}) {
        std::vector<double> us;
        int seen = 0;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipMemset(flag, 0, 4);
            hipLaunchKernelGGL((k<SF, LF>), dim3(16), dim3(64), 0, 0, flag, t, consumer, 1000u + rep);
            unsigned long long h[4];
            (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
            seen += (int)h[3];
            if (h[3]) us.push_back((double)(h[1] - h[0]) / 100.0);
        }
        std::sort(us.begin(), us.end());
        printf("%-28s %s: seen %2d/20, median %.3f us\n", name, consumer == 8 ? "same XCD " : "other XCD", seen,
               us.empty() ? -1.0 : us[us.size() / 2]);
    }
}
int main() {
    unsigned* flag;
    unsigned long long* t;
    (void)hipMalloc(&flag, 256);
    (void)hipMalloc(&t, 64);
    run<0, 100>("store sc1 / load sc1", flag, t);
    run<0, 1>("store sc1 / load sc0", flag, t);
    run<0, 2>("store sc1 / load nt", flag, t);
    run<0, 3>("store sc1 / load sc0|nt", flag, t);
    run<0, 101>("store sc1 / inv sc0+load", flag, t);
    run<1, 1>("store sc0 / load sc0", flag, t);
    run<1, 101>("store sc0 / inv sc0+load", flag, t);
    run<16, 1>("store aux16 / load sc0", flag, t);
    return 0;
}
