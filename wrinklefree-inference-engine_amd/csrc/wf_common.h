// wf_common.h -- host-side helpers for the C-ABI entry points (status codes, error text, launch
// checks). Every extern "C" function validates its arguments, launches on the caller's stream and
// returns WF_OK / WF_EINVAL / WF_EHIP / WF_ENOTSUP; the message is kept in wf_last_error().
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "wf_bitnet.h"

namespace wf {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return WF_EHIP;
    }
    return WF_OK;
}

// Batch < 16 / untiled-cache decode attention (k_attn_sdpa, wf_attn.hip): splits per (sequence, kv
// head) and the model-owned buffers of its in-launch exchange (sizes in 8-byte granules).
constexpr int kSdpaNSMax = 48;         // splits per (sequence, kv head)
constexpr int kSdpaMaxT = 1024;        // keys per split: a split spans <= 3 512-key blocks
constexpr int kSdpaXG = 32;            // exchange granules per split: G heads x 3 blocks (G <= 8), padded
constexpr int kSdpaRec = 8 * 128 + 8;  // record granules per split: G x 128 o, then G l (G <= 8), padded
// ~240 blocks per launch at batch 1 (one per CU), at least 8 splits per (sequence, kv head)
inline int sdpa_splits(int B, int Hkv) {
    const int n = 240 / (B * Hkv > 0 ? B * Hkv : 1);
    return n < 8 ? 8 : (n > kSdpaNSMax ? kSdpaNSMax : n);
}
// codes of the model's host-visible error word (wf_model_check)
enum { WF_ATTN_ERR_SDPA = 1, WF_ATTN_ERR_SPLIT2 = 2 };
struct SdpaBufs {
    uint64_t* xg = nullptr;     // exchange granules [B][Hkv][ns][kSdpaXG]
    uint64_t* rec = nullptr;    // record granules [B][Hkv][ns][kSdpaRec]
    unsigned* epoch = nullptr;  // per-block launch counts [B][Hkv][ns]
    unsigned* err = nullptr;    // host-mapped error word (device address)
    int ns = 0;
    int stall = 0;              // test hook: polls expect a tag no block stores (the timeout path)
};

}  // namespace wf

#define WF_REQUIRE(cond, ...)                 \
    do {                                      \
        if (!(cond)) {                        \
            ::wf::set_error(__VA_ARGS__);     \
            return WF_EINVAL;                 \
        }                                     \
    } while (0)

#define WF_HIP(call)                                                          \
    do {                                                                      \
        hipError_t e_ = (call);                                               \
        if (e_ != hipSuccess) {                                               \
            ::wf::set_error("%s: %s", #call, hipGetErrorString(e_));          \
            return WF_EHIP;                                                   \
        }                                                                     \
    } while (0)
