"""ctypes binding of the C-ABI in include/wf_bitnet.h (lib/libwfbitnet.so, built by `make`).

The product path has exactly one implementation: the HIP kernels behind this library. If the
library is missing or cannot load, every op raises (ImportError at the first call, like
`sgl_kernel` missing in the reference, kernels/bitnet_patch.py:14-25); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[2]          # wrinklefree-inference-engine_amd/
LIB_PATH = Path(os.environ.get("WF_BITNET_LIB", PKG_ROOT / "lib" / "libwfbitnet.so"))

WF_OK, WF_EINVAL, WF_EHIP, WF_ENOTSUP = 0, 1, 2, 3
WF_F32, WF_BF16, WF_F16, WF_I8, WF_U8 = 0, 1, 2, 3, 4
WF_FMT_I2S, WF_FMT_TQ, WF_FMT_I2S_MFMA = 0, 1, 2
WF_KV_BF16, WF_KV_FP8, WF_KV_INT8 = 0, 1, 2  # wf_model_desc.kv_quant
WF_PREFILL_ROW_GROUP = 32  # include/wf_bitnet.h
(WF_OP_EMBED, WF_OP_QKV, WF_OP_ATTN, WF_OP_O, WF_OP_GATE_UP, WF_OP_DOWN, WF_OP_LM_HEAD) = range(7)

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_float

# name -> (restype, argtypes); must list every function declared in include/wf_bitnet.h
SIGNATURES = {
    "wf_last_error": (C.c_char_p, []),
    "wf_abi_version": (i32, []),
    "wf_check_kernel_available": (i32, []),
    "wf_bitnet_gemv": (i32, [vp, vp, f32, i32, i32, vp, vp]),
    "wf_bitnet_gemm": (i32, [vp, vp, f32, i32, i32, i32, vp, vp]),
    "wf_bitnet_gemm_ex": (i32, [i32, vp, vp, i64, f32, i32, i32, i32, vp, i64, vp]),
    "wf_bitnet_gemm_lsb": (i32, [vp, vp, f32, i32, i32, i32, vp, vp]),
    "wf_bitnet_linear_ws_bytes": (i64, [i32, i32]),
    "wf_bitnet_linear": (i32, [i32, vp, vp, i64, f32, i32, i32, i32, vp, i64, vp, vp]),
    "wf_bitnet_linear_fused": (i32, [i32, vp, i32, vp, vp, vp, i64, i32, i32, vp, vp, vp, vp]),
    "wf_bitnet_mlp_ws_bytes": (i64, [i32, i32, i32]),
    "wf_bitnet_mlp": (i32, [i32, vp, vp, f32, f32, f32, vp, f32, vp, i64, i32, i32, i32, vp, i64, vp, vp]),
    "wf_quantize_i8": (i32, [vp, i32, i64, vp, vp, vp]),
    "wf_quantize_i8_rows": (i32, [vp, i32, i32, i32, vp, vp, vp]),
    "wf_quantize_i8_trunc": (i32, [vp, i32, i64, vp, vp, vp]),
    "wf_pack_i2s": (i32, [vp, i32, i32, i32, vp, vp]),
    "wf_hf_to_i2s": (i32, [vp, i32, i32, vp, vp]),
    "wf_i2s_to_tq": (i32, [vp, i32, i32, vp, vp]),
    "wf_tq_to_i2s": (i32, [vp, i32, i32, vp, vp]),
    "wf_tq_row_bytes": (i64, [i32]),
    "wf_i2s_to_mfma": (i32, [vp, i32, i32, vp, vp]),
    "wf_mfma_to_i2s": (i32, [vp, i32, i32, vp, vp]),
    "wf_codes_to_tiles": (i32, [vp, i64, i32, i32, vp, vp]),
    "wf_bitnet_gemm_tiled": (i32, [vp, vp, f32, i32, i32, i32, vp, i64, vp]),
    "wf_kv_scatter": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp]),
    "wf_kv_gather": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp]),
    "wf_kv_scatter_tiles": (i32, [vp, vp, i32, i32, i32, vp, vp, vp, vp, i32, vp, vp]),
    "wf_kv_gather_tiles": (i32, [vp, vp, i32, i32, i32, vp, vp, vp, vp, i32, vp, vp]),
    "wf_kv_quant_i8": (i32, [vp, i32, i64, vp, vp, vp]),
    "wf_kv_dequant_i8": (i32, [vp, i64, vp, vp, i32, vp]),
    "wf_decode_attention_ws_bytes": (i64, [i32, i32, i32, i32]),
    "wf_decode_attention": (i32, [vp, i32, i64, i64, vp, vp, i32, i64, i64, i64, f32, f32, i32, i32, i32, i32, i32,
                                  vp, f32, vp, i32, i64, i64, vp, vp]),
    "wf_absmax": (i32, [vp, i32, i64, vp, vp]),
    "wf_msb_ternarize": (i32, [vp, i32, i32, i32, f32, vp, vp]),
    "wf_msb_dequant": (i32, [vp, i32, i32, f32, vp, i32, vp]),
    "wf_msb_linear": (i32, [vp, f32, vp, i32, i64, i32, i32, i32, vp, vp, i64, vp]),
    "wf_model_create": (i32, [vp, vp]),
    "wf_model_destroy": (i32, [vp]),
    "wf_model_step": (i32, [vp, vp]),
    "wf_model_graph_launch": (i32, [vp, vp]),
    "wf_model_launch_op": (i32, [vp, i32, i32, vp]),
    "wf_model_attn_view": (i32, [vp, vp]),
    "wf_model_check": (i32, [vp]),
    "wf_model_debug_stall_attention": (i32, [vp, i32]),
    "wf_model_fused_norm": (i32, [vp, vp]),
    "wf_model_prefill_reserve": (i32, [vp, i32]),
    "wf_model_prefill": (i32, [vp, vp, vp, vp, i32, vp]),
    "wf_model_prefill_view": (i32, [vp, vp, vp]),
}


class WFModelDesc(C.Structure):
    """Mirror of wf_model_desc (include/wf_bitnet.h)."""
    _fields_ = [(n, C.c_int) for n in ("hidden", "layers", "n_heads", "n_kv_heads", "head_dim", "inter", "vocab",
                                        "max_seq", "batch")] + \
               [("eps", C.c_float), ("wfmt", C.c_int)] + \
               [(n, C.c_void_p) for n in ("embed", "final_norm", "rope_cos", "rope_sin", "ln_in", "ln_post",
                                          "attn_sub", "ffn_sub", "w_qkv", "w_o", "w_gu", "w_d", "wscale",
                                          "tokens", "positions", "logits", "k_cache", "v_cache")] + \
               [("debug_flags", C.c_int), ("page_table", C.c_void_p), ("num_pages", C.c_int),
                ("kv_quant", C.c_int), ("kv_scale", C.c_void_p)]


class WFAttnView(C.Structure):
    """Mirror of wf_attn_records (include/wf_bitnet.h wf_model_attn_view)."""
    _fields_ = [("q", C.c_void_p), ("part_ml", C.c_void_p), ("part_o", C.c_void_p), ("records", C.c_int),
                ("attn_row", C.c_void_p)]


class KernelError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load():
    """Load lib/libwfbitnet.so (raises ImportError when it is missing: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise ImportError(f"HIP library {LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                                  "(or __graft_entry__.build())")
            lib = C.CDLL(str(LIB_PATH))
            study = LIB_PATH.name != "libwfbitnet.so"  # an A/B study build (WF_BITNET_LIB) may predate symbols
            for name, (res, args) in SIGNATURES.items():
                if study and not hasattr(lib, name):
                    continue
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    """Map C-ABI status codes to the reference's error behaviour (TORCH_CHECK -> RuntimeError,
    Python shape checks -> ValueError; SURVEY §8b Errors)."""
    if rc == WF_OK:
        return
    msg = load().wf_last_error().decode(errors="replace")
    if rc == WF_EINVAL:
        raise ValueError(f"{what}: {msg}" if what else msg)
    if rc == WF_ENOTSUP:
        raise NotImplementedError(msg)
    raise KernelError(f"{what}: {msg}" if what else msg)


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)


def kernel_available() -> bool:
    try:
        lib = load()
    except (ImportError, OSError):
        return False
    try:
        import torch
        if not torch.cuda.is_available():
            return False
    except Exception:
        return False
    return bool(lib.wf_check_kernel_available())
