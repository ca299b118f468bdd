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

// Decode attention's in-launch exchanges (k_attn_sdpa, k_attn_sdpa_mfma's split-2 sequences): codes of
// the model's host-visible error word (wf_model_check) and the model-owned hook the launches take.
enum { WF_ATTN_ERR_SDPA = 1, WF_ATTN_ERR_SPLIT2 = 2 };
struct SdpaBufs {
    unsigned* err = nullptr;  // host-mapped error word (device address)
    int stall = 0;            // test hook: k_attn_sdpa polls for a tag no block stores (the timeout path)
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
