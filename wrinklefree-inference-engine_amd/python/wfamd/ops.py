"""Tensor-level wrappers over the C-ABI (torch is plumbing here: device memory and streams).

Every function runs the gfx950 HIP kernel on the caller's current HIP stream. Inputs that live on
the host are staged to the current device and results are copied back (the reference's sgl-kernel
ops take host tensors; see DESIGN.md for the PCIe-inclusive cost). Errors follow the reference:
ValueError for shape/dtype problems (kernels/bitnet_patch.py:186, bitnet_quantization.py:98),
RuntimeError (KernelError) for HIP failures.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import WF_BF16, WF_F16, WF_F32, WF_FMT_I2S, WF_FMT_TQ, WF_I8, call

BITNET_BLOCK_SIZE = 128

_DT = {torch.float32: WF_F32, torch.bfloat16: WF_BF16, torch.float16: WF_F16, torch.int8: WF_I8}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dtcode(t: torch.Tensor, allowed=(WF_F32, WF_BF16, WF_F16)) -> int:
    code = _DT.get(t.dtype)
    if code is None or code not in allowed:
        raise ValueError(f"unsupported dtype {t.dtype}")
    return code


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the BitNet kernels run on gfx950 only")
    return torch.device("cuda", torch.cuda.current_device())


def _on_device(t: torch.Tensor) -> torch.Tensor:
    if t.is_cuda:
        return t.contiguous()
    return t.to(_device(), non_blocking=False).contiguous()


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_hip_rt = None


def device_copy(dst: int, src: int, nbytes: int) -> None:
    """Stream-ordered device-to-device copy between raw device pointers (hipMemcpyAsync on torch's
    current stream): reads library-owned buffers exposed by the C-ABI (wf_model_attn_view)."""
    global _hip_rt
    if _hip_rt is None:
        import ctypes as C
        _hip_rt = C.CDLL("libamdhip64.so")
        _hip_rt.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip_rt.hipMemcpyAsync.restype = C.c_int
    rc = _hip_rt.hipMemcpyAsync(dst, src, nbytes, 3, _stream())  # hipMemcpyDeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync failed ({rc})")


def check_kernel_available() -> bool:
    return _lib.kernel_available()


# ---------------------------------------------------------------------------------------------
# a1/a2: raw ternary GEMV/GEMM (sgl-kernel semantics: y = float(sum enc*a) * scale)
# ---------------------------------------------------------------------------------------------
def _check_packed(packed: torch.Tensor, k: int, fmt: int) -> None:
    if packed.dtype != torch.uint8 or packed.dim() != 2:
        raise ValueError(f"packed weights must be a 2-D uint8 tensor, got {packed.dtype} {tuple(packed.shape)}")
    if k % BITNET_BLOCK_SIZE != 0:
        raise ValueError(f"in_features ({k}) must be divisible by BITNET_BLOCK_SIZE={BITNET_BLOCK_SIZE}")
    want = k // 4 if fmt == WF_FMT_I2S else int(_lib.load().wf_tq_row_bytes(k))
    if packed.shape[1] != want:
        raise ValueError(f"packed weights have {packed.shape[1]} bytes per row, expected {want} for K={k}")


def bitnet_gemm_ex(packed: torch.Tensor, activations: torch.Tensor, scale: float, fmt: int = WF_FMT_I2S,
                   in_features: Optional[int] = None) -> torch.Tensor:
    if activations.dtype != torch.int8:
        raise ValueError(f"activations must be int8, got {activations.dtype}")
    a2 = activations.reshape(-1, activations.shape[-1]) if activations.dim() != 1 else activations.reshape(1, -1)
    k = a2.shape[1] if in_features is None else in_features
    _check_packed(packed, k, fmt)
    if a2.shape[1] != k:
        raise ValueError(f"activations have {a2.shape[1]} features, weights expect {k}")
    host = not (packed.is_cuda and activations.is_cuda)
    w = _on_device(packed)
    a = _on_device(a2)
    m, n = a.shape[0], w.shape[0]
    y = torch.empty((m, n), dtype=torch.float32, device=w.device)
    if m > 0 and n > 0:
        call("wf_bitnet_gemm_ex", fmt, w.data_ptr(), a.data_ptr(), a.stride(0), float(scale), m, n, k, y.data_ptr(),
             n, _stream())
    out = y.reshape(*activations.shape[:-1], n) if activations.dim() != 1 else y.reshape(n)
    return out.cpu() if host else out


def bitnet_gemv(packed_weights: torch.Tensor, activations: torch.Tensor, scale: float) -> torch.Tensor:
    """sgl_kernel.quantization.bitnet_gemv: packed [N, K/4] uint8 (blocked I2_S), act [K] int8 -> [N] f32."""
    if activations.dim() != 1:
        raise ValueError(f"bitnet_gemv expects 1-D activations, got shape {tuple(activations.shape)}")
    return bitnet_gemm_ex(packed_weights, activations, scale, WF_FMT_I2S)


def bitnet_gemm(packed_weights: torch.Tensor, activations: torch.Tensor, scale: float) -> torch.Tensor:
    """sgl_kernel.quantization.bitnet_gemm: act [M, K] int8 -> [M, N] f32 (one scale for the batch)."""
    if activations.dim() != 2:
        raise ValueError(f"bitnet_gemm expects 2-D activations, got shape {tuple(activations.shape)}")
    return bitnet_gemm_ex(packed_weights, activations, scale, WF_FMT_I2S)


def bitnet_gemm_lsb(packed: torch.Tensor, activations: torch.Tensor, scale: float) -> torch.Tensor:
    """kernels/native.py:27-93 semantics: signed dot on the LSB-interleaved layout."""
    if packed.dtype != torch.uint8 or packed.dim() != 2 or activations.dtype != torch.int8:
        raise ValueError("gemm_lsb expects uint8 [N, K/4] weights and int8 activations")
    a2 = activations.reshape(1, -1) if activations.dim() == 1 else activations
    k = packed.shape[1] * 4
    if a2.shape[1] != k:
        raise ValueError(f"activations have {a2.shape[1]} features, weights expect {k}")
    host = not (packed.is_cuda and activations.is_cuda)
    w, a = _on_device(packed), _on_device(a2)
    y = torch.empty((a.shape[0], w.shape[0]), dtype=torch.float32, device=w.device)
    call("wf_bitnet_gemm_lsb", w.data_ptr(), a.data_ptr(), float(scale), a.shape[0], w.shape[0], k, y.data_ptr(),
         _stream())
    out = y.reshape(w.shape[0]) if activations.dim() == 1 else y
    return out.cpu() if host else out


def bitnet_linear(x: torch.Tensor, packed: torch.Tensor, weight_scale: float, fmt: int = WF_FMT_I2S,
                  in_features: Optional[int] = None) -> torch.Tensor:
    """Fused BitNetLinear.forward (scripts/direct_inference_full.py:186-208): bf16 x [..., K] ->
    bf16 [..., N]; per-row int8 quantization, ternary GEMM and the reference's correction in one
    (M < 16) or two (M >= 16, int8 MFMA) launches."""
    if x.dtype != torch.bfloat16:
        raise ValueError(f"bitnet_linear expects bf16 activations, got {x.dtype}")
    k = x.shape[-1] if in_features is None else in_features
    _check_packed(packed, k, fmt)
    if x.shape[-1] != k:
        raise ValueError(f"activations have {x.shape[-1]} features, weights expect {k}")
    host = not (packed.is_cuda and x.is_cuda)
    w = _on_device(packed)
    x2 = _on_device(x.reshape(-1, k))
    if x2.stride(1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    m, n = x2.shape[0], w.shape[0]
    y = torch.empty((m, n), dtype=torch.bfloat16, device=w.device)
    if m > 0 and n > 0:
        nws = int(_lib.load().wf_bitnet_linear_ws_bytes(m, k))
        ws = torch.empty(nws, dtype=torch.uint8, device=w.device) if m >= 16 else None
        call("wf_bitnet_linear", fmt, w.data_ptr(), x2.data_ptr(), x2.stride(0), float(weight_scale), m, n, k,
             y.data_ptr(), n, _ptr(ws), _stream())
    out = y.reshape(*x.shape[:-1], n)
    return out.cpu() if host else out


def bitnet_linear_fused(x: torch.Tensor, packed: torch.Tensor, rows: Sequence[int], weight_scales: Sequence[float],
                        fmt: int = WF_FMT_I2S, in_features: Optional[int] = None) -> List[torch.Tensor]:
    """Several BitNetLinear layers on the same input with one shared activation quantization
    (include/wf_bitnet.h wf_bitnet_linear_fused; SURVEY §8f rank 1: fused q|k|v, gate|up).
    `packed` holds the layers' packed weights row-concatenated ([sum(rows), row bytes]); returns one
    bf16 tensor [..., rows[s]] per layer, each bit-identical to bitnet_linear on that layer."""
    if x.dtype != torch.bfloat16:
        raise ValueError(f"bitnet_linear_fused expects bf16 activations, got {x.dtype}")
    rows = [int(r) for r in rows]
    if not 1 <= len(rows) <= 3 or len(weight_scales) != len(rows) or min(rows) <= 0:
        raise ValueError("bitnet_linear_fused: 1..3 layers, one positive row count and one scale each")
    k = x.shape[-1] if in_features is None else in_features
    _check_packed(packed, k, fmt)
    if packed.shape[0] != sum(rows):
        raise ValueError(f"packed weights have {packed.shape[0]} rows, the layers {sum(rows)}")
    if x.shape[-1] != k:
        raise ValueError(f"activations have {x.shape[-1]} features, weights expect {k}")
    host = not (packed.is_cuda and x.is_cuda)
    w = _on_device(packed)
    x2 = _on_device(x.reshape(-1, k))
    if x2.stride(1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    m = x2.shape[0]
    ys = [torch.empty((m, r), dtype=torch.bfloat16, device=w.device) for r in rows]
    if m > 0:
        ns = len(rows)
        nws = int(_lib.load().wf_bitnet_linear_ws_bytes(m, k))
        ws = torch.empty(nws, dtype=torch.uint8, device=w.device) if m >= 16 else None
        c_n = (C.c_int * ns)(*rows)
        c_s = (C.c_float * ns)(*[float(v) for v in weight_scales])
        c_y = (C.c_void_p * ns)(*[y.data_ptr() for y in ys])
        c_l = (C.c_int64 * ns)(*rows)
        call("wf_bitnet_linear_fused", fmt, w.data_ptr(), ns, C.addressof(c_n), C.addressof(c_s), x2.data_ptr(),
             x2.stride(0), m, k, C.addressof(c_y), C.addressof(c_l), _ptr(ws), _stream())
    outs = [y.reshape(*x.shape[:-1], y.shape[1]) for y in ys]
    return [o.cpu() for o in outs] if host else outs


def bitnet_mlp(x: torch.Tensor, packed_gate_up: torch.Tensor, packed_down: torch.Tensor, ws_gate: float, ws_up: float,
               ws_down: float, ffn_sub_norm: torch.Tensor, eps: float = 1e-5, fmt: int = WF_FMT_I2S) -> torch.Tensor:
    """BitNet MLP in one call (include/wf_bitnet.h wf_bitnet_mlp; scripts/direct_inference_full.py:252-265):
    bf16 x [..., H] -> down(rms_norm(relu(gate(x))^2 * up(x), ffn_sub_norm)) bf16 [..., H]; gate|up
    row-concatenated with one shared activation quantization."""
    if x.dtype != torch.bfloat16 or ffn_sub_norm.dtype != torch.bfloat16:
        raise ValueError("bitnet_mlp expects bf16 activations and norm weight")
    h, i = x.shape[-1], ffn_sub_norm.shape[-1]
    _check_packed(packed_gate_up, h, fmt)
    _check_packed(packed_down, i, fmt)
    if packed_gate_up.shape[0] != 2 * i or packed_down.shape[0] != h:
        raise ValueError(f"gate|up must have {2 * i} rows and down {h} rows")
    if not (x.is_cuda and packed_gate_up.is_cuda and packed_down.is_cuda and ffn_sub_norm.is_cuda):
        raise ValueError("bitnet_mlp: device tensors only")
    x2 = x.reshape(-1, h)
    if x2.stride(1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    m = x2.shape[0]
    y = torch.empty((m, h), dtype=torch.bfloat16, device=x.device)
    if m > 0:
        nws = int(_lib.load().wf_bitnet_mlp_ws_bytes(m, h, i))
        ws = torch.empty(nws + 256, dtype=torch.uint8, device=x.device)
        base = (ws.data_ptr() + 255) // 256 * 256
        nw = ffn_sub_norm.contiguous()
        call("wf_bitnet_mlp", fmt, packed_gate_up.data_ptr(), packed_down.data_ptr(), float(ws_gate), float(ws_up),
             float(ws_down), nw.data_ptr(), float(eps), x2.data_ptr(), x2.stride(0), m, h, i, y.data_ptr(), h, base,
             _stream())
    return y.reshape(*x.shape[:-1], h)


# ---------------------------------------------------------------------------------------------
# a3: activation quantizers
# ---------------------------------------------------------------------------------------------
def quantize_activations_i8(activations: torch.Tensor) -> Tuple[torch.Tensor, float]:
    """bitnet_quantize_activations: per-tensor absmax int8, round-half-even (tests/test_bitnet_core.py:139-146).
    Returns (int8 tensor of the same shape, Python float scale = max|x| / 127)."""
    host = not activations.is_cuda
    x = _on_device(activations)
    code = _dtcode(x)
    n = x.numel()
    if n == 0:
        raise ValueError("cannot quantize an empty tensor")
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    mx = torch.empty(1, dtype=torch.float32, device=x.device)
    call("wf_quantize_i8", x.data_ptr(), code, n, q.data_ptr(), mx.data_ptr(), _stream())
    m = float(mx.item())
    if m < 1e-6:
        m = 1.0
    return (q.cpu() if host else q), m / 127.0


def quantize_activations_rows(activations: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-token variant: [M, K] -> (int8 [M, K], float64 scales [M]) computed on device."""
    x = _on_device(activations)
    code = _dtcode(x)
    m, k = x.reshape(-1, x.shape[-1]).shape
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    mx = torch.empty(m, dtype=torch.float32, device=x.device)
    call("wf_quantize_i8_rows", x.data_ptr(), code, m, k, q.data_ptr(), mx.data_ptr(), _stream())
    md = mx.double()
    md = torch.where(md < 1e-6, torch.ones_like(md), md)
    return q, md / 127.0


def quantize_activations_trunc(x: torch.Tensor) -> Tuple[torch.Tensor, float]:
    """kernels/native.py:244-256 (float32 scale, truncating cast)."""
    host = not x.is_cuda
    xd = _on_device(x)
    code = _dtcode(xd)
    q = torch.empty(xd.shape, dtype=torch.int8, device=xd.device)
    mx = torch.empty(1, dtype=torch.float32, device=xd.device)
    call("wf_quantize_i8_trunc", xd.data_ptr(), code, xd.numel(), q.data_ptr(), mx.data_ptr(), _stream())
    m = torch.tensor(mx.item(), dtype=torch.float32)
    s = float(m / 127.0) if float(m) > 1e-6 else 1.0
    return (q.cpu() if host else q), float(torch.tensor(s, dtype=torch.float32))


# ---------------------------------------------------------------------------------------------
# Load-time formats
# ---------------------------------------------------------------------------------------------
def pack_i2s(weight: torch.Tensor) -> torch.Tensor:
    """cache/bitnet_converter.py:26-77 on the device (K % 128 == 0)."""
    w = _on_device(weight)
    n, k = w.shape
    if k % 4 != 0:
        raise ValueError(f"in_features ({k}) must be divisible by 4")
    if k % BITNET_BLOCK_SIZE != 0:
        raise ValueError(f"in_features ({k}) must be divisible by {BITNET_BLOCK_SIZE}")
    if w.dtype not in _DT or w.dtype == torch.int8:
        w = w.float()
    out = torch.empty((n, k // 4), dtype=torch.uint8, device=w.device)
    call("wf_pack_i2s", w.data_ptr(), _dtcode(w), n, k, out.data_ptr(), _stream())
    return out


def hf_to_i2s(hf_packed: torch.Tensor) -> torch.Tensor:
    """HF [N/4, K] uint8 -> blocked I2_S [N, K/4] (tests/test_bitnet_core.py:21-106)."""
    p = _on_device(hf_packed)
    if p.dtype != torch.uint8 or p.dim() != 2:
        raise ValueError("HF packed weights must be 2-D uint8 [out/4, in]")
    np_, k = p.shape
    out = torch.empty((np_ * 4, k // 4), dtype=torch.uint8, device=p.device)
    call("wf_hf_to_i2s", p.data_ptr(), np_, k, out.data_ptr(), _stream())
    return out


def tq_row_bytes(k: int) -> int:
    return int(_lib.load().wf_tq_row_bytes(k))


def i2s_to_mfma(i2s: torch.Tensor) -> torch.Tensor:
    """I2_S [N, K/4] -> the matrix-core tile layout (include/wf_bitnet.h WF_FMT_I2S_MFMA), same shape."""
    w = _on_device(i2s).contiguous()
    n, k4 = w.shape
    out = torch.empty_like(w)
    call("wf_i2s_to_mfma", w.data_ptr(), n, 4 * k4, out.data_ptr(), _stream())
    return out


def codes_to_tiles(a: torch.Tensor) -> torch.Tensor:
    """int8 codes [M, K] -> matrix-core tile order (include/wf_bitnet.h wf_codes_to_tiles), flat
    int8 tensor of ceil(M/16)*16*K bytes."""
    a = _on_device(a).contiguous()
    m, k = a.shape
    out = torch.empty((m + 15) // 16 * 16 * k, dtype=torch.int8, device=a.device)
    call("wf_codes_to_tiles", a.data_ptr(), k, m, k, out.data_ptr(), _stream())
    return out


def bitnet_gemm_tiled(w_mfma: torch.Tensor, a_tiles: torch.Tensor, scale: float, m: int) -> torch.Tensor:
    """Prefill GEMM on tile layouts (wf_bitnet_gemm_tiled): float32 [m, N]."""
    n, k4 = w_mfma.shape
    y = torch.empty(m, n, dtype=torch.float32, device=w_mfma.device)
    call("wf_bitnet_gemm_tiled", w_mfma.data_ptr(), a_tiles.data_ptr(), float(scale), m, n, 4 * k4, y.data_ptr(), n,
         _stream())
    return y


def mfma_to_i2s(mf: torch.Tensor) -> torch.Tensor:
    w = _on_device(mf).contiguous()
    n, k4 = w.shape
    out = torch.empty_like(w)
    call("wf_mfma_to_i2s", w.data_ptr(), n, 4 * k4, out.data_ptr(), _stream())
    return out


def i2s_to_tq(i2s: torch.Tensor) -> torch.Tensor:
    p = _on_device(i2s)
    n, k = p.shape[0], p.shape[1] * 4
    out = torch.empty((n, tq_row_bytes(k)), dtype=torch.uint8, device=p.device)
    call("wf_i2s_to_tq", p.data_ptr(), n, k, out.data_ptr(), _stream())
    return out


def tq_to_i2s(tq: torch.Tensor, k: int) -> torch.Tensor:
    p = _on_device(tq)
    out = torch.empty((p.shape[0], k // 4), dtype=torch.uint8, device=p.device)
    call("wf_tq_to_i2s", p.data_ptr(), p.shape[0], k, out.data_ptr(), _stream())
    return out


# ---------------------------------------------------------------------------------------------
# KV cache helpers
# ---------------------------------------------------------------------------------------------
def kv_absmax(x: torch.Tensor) -> torch.Tensor:
    """max|x| on device (same reduction as the quantizer) -> float32 [1]."""
    mx = torch.empty(1, dtype=torch.float32, device=x.device)
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    call("wf_quantize_i8", x.data_ptr(), _dtcode(x), x.numel(), q.data_ptr(), mx.data_ptr(), _stream())
    return mx


def kv_quant_i8(x: torch.Tensor, absmax: torch.Tensor) -> torch.Tensor:
    q = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    call("wf_kv_quant_i8", x.data_ptr(), _dtcode(x), x.numel(), absmax.data_ptr(), q.data_ptr(), _stream())
    return q


def kv_dequant_i8(q: torch.Tensor, scale: torch.Tensor, out_dtype=torch.bfloat16) -> torch.Tensor:
    q = q.contiguous()
    out = torch.empty(q.shape, dtype=out_dtype, device=q.device)
    if q.numel():
        call("wf_kv_dequant_i8", q.data_ptr(), q.numel(), scale.data_ptr(), out.data_ptr(), _DT[out_dtype], _stream())
    return out


def decode_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *, kv_strides: Tuple[int, int, int],
                     B: int, Hq: int, Hkv: int, D: int, S: int, seq_lens: Optional[torch.Tensor] = None,
                     k_scale: float = 1.0, v_scale: float = 1.0, sm_scale: Optional[float] = None,
                     out_dtype=None) -> torch.Tensor:
    """Split-K decode attention. q: [B, Hq, D] (contiguous); k/v: base tensors addressed by
    kv_strides = (batch, head, position) element strides. Returns [B, Hq, D]."""
    q = q.contiguous()
    out_dtype = out_dtype or q.dtype
    out = torch.empty((B, Hq, D), dtype=out_dtype, device=q.device)
    ws = torch.empty(int(_lib.load().wf_decode_attention_ws_bytes(B, Hq, D, S)), dtype=torch.uint8, device=q.device)
    sm = float(sm_scale) if sm_scale is not None else 1.0 / math.sqrt(D)
    kvc = _dtcode(k, (WF_F32, WF_BF16, WF_F16, WF_I8))
    call("wf_decode_attention", q.data_ptr(), _dtcode(q), Hq * D, D, k.data_ptr(), v.data_ptr(), kvc,
         kv_strides[0], kv_strides[1], kv_strides[2], float(k_scale), float(v_scale), B, Hq, Hkv, D, S,
         _ptr(seq_lens), sm, out.data_ptr(), _DT[out_dtype], Hq * D, D, ws.data_ptr(), _stream())
    return out


# ---------------------------------------------------------------------------------------------
# torch.library schemas of the reference (docs/research/sglang_optimization_plan.md:61-74)
# ---------------------------------------------------------------------------------------------
_registered = False


def register_torch_ops() -> bool:
    """Define sgl_kernel::bitnet_{gemv,gemm,quantize_activations}_cpu with CUDA(HIP) and CPU(host
    buffers staged through the GPU) impls plus fake impls for torch.compile. Returns False if a
    real sgl_kernel already owns the namespace."""
    global _registered
    if _registered:
        return True
    try:
        lib = torch.library.Library("sgl_kernel", "DEF")
    except RuntimeError:
        try:
            lib = torch.library.Library("sgl_kernel", "FRAGMENT")
        except RuntimeError:
            return False
    try:
        lib.define("bitnet_gemv_cpu(Tensor packed_weights, Tensor activations, float scale) -> Tensor")
        lib.define("bitnet_gemm_cpu(Tensor packed_weights, Tensor activations, float scale) -> Tensor")
        lib.define("bitnet_quantize_activations_cpu(Tensor activations) -> (Tensor, Tensor)")
        # the fused ops the reference attempted (docs/research/sglang_optimization_plan.md:326-331;
        # their schemas are un-vendored, so these are this build's own): q|k|v on one shared
        # activation quantization, and the whole MLP block
        lib.define("bitnet_qkv_forward_cpu(Tensor x, Tensor packed_qkv, int q_rows, int k_rows, int v_rows, "
                   "float ws_q, float ws_k, float ws_v, int fmt=0) -> (Tensor, Tensor, Tensor)")
        lib.define("bitnet_mlp_forward_cpu(Tensor x, Tensor packed_gate_up, Tensor packed_down, float ws_gate, "
                   "float ws_up, float ws_down, Tensor ffn_sub_norm, float eps=1e-05, int fmt=0) -> Tensor")
    except RuntimeError:
        return False

    def _gemv(w, a, s):
        return bitnet_gemv(w, a, s)

    def _gemm(w, a, s):
        return bitnet_gemm(w, a, s)

    def _quant(x):
        q, s = quantize_activations_i8(x)
        return q, torch.tensor([s], dtype=torch.float32, device=q.device)

    def _qkv(x, w, qr, kr, vr, wq, wk, wv, fmt=0):  # torch drops arguments equal to the schema default
        return tuple(bitnet_linear_fused(x, w, [qr, kr, vr], [wq, wk, wv], fmt))

    def _mlp(x, wgu, wd, wg, wu, wdn, nw, eps=1e-5, fmt=0):
        return bitnet_mlp(x, wgu, wd, wg, wu, wdn, nw, eps, fmt)

    for key in ("CUDA", "CPU"):
        lib.impl("bitnet_gemv_cpu", _gemv, key)
        lib.impl("bitnet_gemm_cpu", _gemm, key)
        lib.impl("bitnet_quantize_activations_cpu", _quant, key)
        lib.impl("bitnet_qkv_forward_cpu", _qkv, key)  # host tensors are staged through the GPU
    lib.impl("bitnet_mlp_forward_cpu", _mlp, "CUDA")  # device tensors only (bitnet_mlp)

    @torch.library.register_fake("sgl_kernel::bitnet_qkv_forward_cpu", lib=lib)
    def _(x, packed_qkv, q_rows, k_rows, v_rows, ws_q, ws_k, ws_v, fmt=0):
        lead = x.shape[:-1]
        return tuple(x.new_empty((*lead, r), dtype=torch.bfloat16) for r in (q_rows, k_rows, v_rows))

    @torch.library.register_fake("sgl_kernel::bitnet_mlp_forward_cpu", lib=lib)
    def _(x, packed_gate_up, packed_down, ws_gate, ws_up, ws_down, ffn_sub_norm, eps=1e-5, fmt=0):
        return x.new_empty(x.shape, dtype=torch.bfloat16)

    @torch.library.register_fake("sgl_kernel::bitnet_gemv_cpu", lib=lib)
    def _(packed_weights, activations, scale):
        return torch.empty(packed_weights.shape[0], dtype=torch.float32, device=packed_weights.device)

    @torch.library.register_fake("sgl_kernel::bitnet_gemm_cpu", lib=lib)
    def _(packed_weights, activations, scale):
        return torch.empty(activations.shape[0], packed_weights.shape[0], dtype=torch.float32,
                           device=packed_weights.device)

    @torch.library.register_fake("sgl_kernel::bitnet_quantize_activations_cpu", lib=lib)
    def _(activations):
        return torch.empty_like(activations, dtype=torch.int8), torch.empty(1, dtype=torch.float32)

    globals()["_torch_lib"] = lib
    _registered = True
    return True


# ---------------------------------------------------------------------------------------------
# a12: the SGLang BitNet linear method on the MSB-interleaved layout
# (sglang_backend/bitnet_quantization.py:69-409)
# ---------------------------------------------------------------------------------------------
def absmax(x: torch.Tensor) -> float:
    """max|x| over the whole tensor (device reduction; `.item()` like the reference)."""
    xd = _on_device(x)
    out = torch.empty(1, dtype=torch.float32, device=xd.device)
    call("wf_absmax", xd.data_ptr(), _dtcode(xd), xd.numel(), out.data_ptr(), _stream())
    return float(out.item())


def msb_ternarize(weights: torch.Tensor, scale: float) -> torch.Tensor:
    """quantize_to_bitnet's ternarise + pack (bitnet_quantization.py:88-105) for a given scale."""
    n, k = weights.shape
    wd = _on_device(weights)
    out = torch.empty((n, k // 4), dtype=torch.uint8, device=wd.device)
    call("wf_msb_ternarize", wd.data_ptr(), _dtcode(wd), n, k, float(scale), out.data_ptr(), _stream())
    return out


def msb_dequant(packed: torch.Tensor, scale: float, out_features: int, in_features: int,
                dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """dequantize_bitnet (bitnet_quantization.py:211-252): (code - 1) * float(scale) -> dtype."""
    if packed.dtype != torch.uint8 or tuple(packed.shape) != (out_features, in_features // 4):
        raise ValueError(f"packed must be uint8 [{out_features}, {in_features // 4}], got {packed.dtype} "
                         f"{tuple(packed.shape)}")
    pd = _on_device(packed)
    out = torch.empty((out_features, in_features), dtype=dtype, device=pd.device)
    call("wf_msb_dequant", pd.data_ptr(), out_features, in_features, float(scale), out.data_ptr(), _dtcode(out),
         _stream())
    return out


def msb_linear(packed: torch.Tensor, scale: float, x: torch.Tensor, out_features: int, in_features: int,
               bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """x [..., K] (bf16/f16, the compute dtype) @ dequant(packed)^T (+ bias), read from the 2-bit
    bytes. Raises NotImplementedError for shapes the direct kernel does not take (K % 64 != 0 or
    K > 16384); the caller then uses the dequantised matrix."""
    if x.dtype not in (torch.bfloat16, torch.float16):
        raise ValueError(f"msb_linear computes in bf16/f16, got {x.dtype}")
    x2 = x.reshape(-1, in_features)
    if x2.stride(-1) != 1 or x2.stride(0) % 8 != 0 or x2.data_ptr() % 16 != 0:
        x2 = x2.contiguous()
    m = x2.shape[0]
    y = torch.empty((m, out_features), dtype=x.dtype, device=x2.device)
    b = None if bias is None else bias.to(device=x2.device, dtype=x.dtype).contiguous()
    call("wf_msb_linear", packed.data_ptr(), float(scale), x2.data_ptr(), _dtcode(x2), x2.stride(0), m, out_features,
         in_features, _ptr(b), y.data_ptr(), out_features, _stream())
    return y.reshape(*x.shape[:-1], out_features)
