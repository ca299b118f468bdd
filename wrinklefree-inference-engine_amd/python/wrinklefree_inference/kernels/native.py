"""HIP replacement of the reference's runtime-built pybind/OpenMP kernel
(src/wrinklefree_inference/kernels/native.py).

`build_kernel()` returns an object with the reference module's surface -- gemv, gemm, num_threads
(:105-109) -- whose gemv/gemm run the gfx950 LSB-layout kernel (wf_bitnet_gemm_lsb): signed
(bits-1) dot, float(sum) * scale (:27-93). numpy in, numpy out like the pybind module. The numpy
helpers pack_weights / unpack_weights / repack_hf_weights / quantize_activations keep the
reference's host-side semantics (:181-256), vectorised.
"""
from __future__ import annotations

import numpy as np
import torch

from wfamd import _lib
from wfamd import ops as _ops


class _HipNativeKernel:
    """Stands in for the `bitnet_native` pybind module."""

    @staticmethod
    def gemv(packed_weights: np.ndarray, activations: np.ndarray, scale: float) -> np.ndarray:
        w = torch.from_numpy(np.ascontiguousarray(packed_weights, dtype=np.uint8))
        a = torch.from_numpy(np.ascontiguousarray(activations, dtype=np.int8))
        return _ops.bitnet_gemm_lsb(w, a, float(np.float32(scale))).numpy()

    @staticmethod
    def gemm(packed_weights: np.ndarray, activations: np.ndarray, scale: float) -> np.ndarray:
        w = torch.from_numpy(np.ascontiguousarray(packed_weights, dtype=np.uint8))
        a = torch.from_numpy(np.ascontiguousarray(activations, dtype=np.int8))
        return _ops.bitnet_gemm_lsb(w, a, float(np.float32(scale))).numpy()

    @staticmethod
    def num_threads() -> int:
        """Compute units of the device (the OpenMP thread count's counterpart)."""
        if not torch.cuda.is_available():
            return 0
        return torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count


_kernel_module = None


def build_kernel(force: bool = False):
    """Load the prebuilt HIP library (built by `make`, never at runtime). RuntimeError if missing,
    matching the reference's failed-build behaviour (:164-165)."""
    global _kernel_module
    if _kernel_module is not None and not force:
        return _kernel_module
    try:
        _lib.load()
    except (ImportError, OSError) as e:
        raise RuntimeError(f"Kernel build failed: {e}") from e
    _kernel_module = _HipNativeKernel()
    return _kernel_module


def get_kernel():
    return build_kernel() if _kernel_module is None else _kernel_module


def pack_weights(weights: np.ndarray) -> np.ndarray:
    """byte[k] = w[4k] | w[4k+1]<<2 | w[4k+2]<<4 | w[4k+3]<<6, enc = clip(int(w)+1, 0, 2) (:181-198)."""
    out_f, in_f = weights.shape
    assert in_f % 4 == 0, f"in_features must be divisible by 4, got {in_f}"
    enc = (weights.astype(np.int32) + 1).clip(0, 2).astype(np.uint8)
    return (enc[:, 0::4] | (enc[:, 1::4] << 2) | (enc[:, 2::4] << 4) | (enc[:, 3::4] << 6)).astype(np.uint8)


def unpack_weights(packed: np.ndarray) -> np.ndarray:
    out_f, pk = packed.shape
    w = np.empty((out_f, pk * 4), dtype=np.float32)
    for j in range(4):
        w[:, j::4] = ((packed >> (2 * j)) & 0x03).astype(np.float32) - 1.0
    return w


def repack_hf_weights(packed_hf: np.ndarray) -> np.ndarray:
    """HF [out/4, in] with the interleaved (i::4) output convention of the reference (:218-241)."""
    out_packed, in_features = packed_hf.shape
    unpacked = np.zeros((out_packed * 4, in_features), dtype=np.float32)
    p = packed_hf.astype(np.int32)
    for i in range(4):
        unpacked[i::4, :] = ((p >> (i * 2)) & 0x03) - 1.0
    return pack_weights(unpacked)


def quantize_activations(x: np.ndarray):
    """float32 scale, truncating cast (:244-256)."""
    max_val = np.abs(x).max()
    scale = max_val / 127.0 if max_val > 1e-6 else 1.0
    quantized = np.clip(x / scale, -128, 127).astype(np.int8)
    return quantized, scale
