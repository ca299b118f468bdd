"""BitNet 1.58-bit linear method for SGLang on MI355X (drop-in for the reference's
sglang_backend/bitnet_quantization.py).

Weight format (bitnet_quantization.py:99-105): MSB-interleaved 2-bit codes, byte j of a row holds
w[4j] (bits 7-6) .. w[4j+3] (bits 1-0) as code = w + 1. The reference is a CPU method: dequantise
once (numba/LUT), cache the bf16 matrix and run `x @ W^T`. Here every piece runs on the GPU:

* `quantize_to_bitnet` / `dequantize_bitnet`: HIP kernels (wf_msb_ternarize / wf_msb_dequant).
* `BitNetLinearMethod.apply` for up to 4 rows reads the packed 2-bit bytes directly
  (wf_msb_linear: codes -> bf16/fp16 +-1/0 pairs in registers, v_dot2 accumulate; 8x fewer HBM bytes
  than the cached bf16 matrix the reference multiplies). Larger batches (or K the direct kernel
  does not take) multiply the cached dequantised matrix with the library GEMM (hipBLASLt), which
  is the reference's own algorithm on the device.

Numerics: the reference's bf16 weight is +-bf16(float(scale)); the direct kernel accumulates
sum (code-1) * x in fp32 and multiplies by that same bf16 scale, so results agree with the
reference up to fp32 summation order and the final bf16 rounding (the reference pins cosine
> 0.9999 vs fp32, tests/test_sglang_bitnet.py:243-283). Host tensors are staged to the GPU and
results returned on the host, like the other drop-in ops (PCIe-inclusive).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass
from enum import IntEnum
from typing import Any, Dict, List, Optional, Tuple

import torch

from wfamd import ops

from .activation_sparsity import ActivationSparsityConfig, apply_sparsity, get_default_config

logger = logging.getLogger(__name__)


class BitNetQuantType(IntEnum):
    """GGML BitNet quantisation types (bitnet_quantization.py:36-40)."""
    I2_S = 30
    TL1 = 31
    TL2 = 32


BITNET_QUANT_TYPES = {BitNetQuantType.I2_S, BitNetQuantType.TL1, BitNetQuantType.TL2}
BITNET_BLOCK_SIZE = 128

# rows up to which apply() reads the packed bytes directly (above: cached bf16 matrix + GEMM);
# measured crossover (tools/msb_bench.py): 4 rows 5.9-19 us vs GEMM 11-38 us, 16 rows 23-72 us vs 12-38 us
DIRECT_MAX_ROWS = 4


@dataclass
class BitNetWeightSpec:
    shape: Tuple[int, ...]
    quant_type: BitNetQuantType
    scale: float
    packed_shape: Tuple[int, ...]

    @property
    def bits_per_weight(self) -> float:
        return 1.58

    @property
    def compression_ratio(self) -> float:
        return 16.0 / self.bits_per_weight


def _to_host_if(t: torch.Tensor, host: bool) -> torch.Tensor:
    return t.cpu() if host else t


def quantize_to_bitnet(weights: torch.Tensor, block_size: int = BITNET_BLOCK_SIZE) -> Tuple[torch.Tensor, float]:
    """Ternarise (|w/scale| > 0.5 -> +-1) and pack (bitnet_quantization.py:69-109).
    Returns (uint8 [N, K/4] on the input's device, scale = max|w| or 1.0 below 1e-6)."""
    scale = ops.absmax(weights)
    if scale < 1e-6:
        scale = 1.0
    out_features, in_features = weights.shape
    assert in_features % block_size == 0, f"in_features must be divisible by {block_size}"
    packed = ops.msb_ternarize(weights, scale)
    return _to_host_if(packed, not weights.is_cuda), scale


def dequantize_bitnet(packed: torch.Tensor, scale: float, out_features: int, in_features: int,
                      use_numba: bool = True) -> torch.Tensor:
    """(code - 1) * scale as fp32 [N, K] (bitnet_quantization.py:211-252). `use_numba` is accepted
    for signature compatibility; the dequantisation is one HIP kernel either way."""
    out = ops.msb_dequant(packed, scale, out_features, in_features, torch.float32)
    return _to_host_if(out, not packed.is_cuda)


def dequantize_bitnet_reference(packed: torch.Tensor, scale: float, out_features: int,
                                in_features: int) -> torch.Tensor:
    """bitnet_quantization.py:115-137 -- same values as dequantize_bitnet."""
    return dequantize_bitnet(packed, scale, out_features, in_features)


def bitnet_matmul_reference(packed_weight: torch.Tensor, scale: float, x: torch.Tensor, out_features: int,
                            in_features: int) -> torch.Tensor:
    """bitnet_quantization.py:140-153: x @ dequant(W)^T in x's dtype."""
    w = dequantize_bitnet(packed_weight, scale, out_features, in_features).to(device=x.device, dtype=x.dtype)
    return torch.matmul(x, w.T)


class BitNetLinearMethod:
    """Linear method of the SGLang BitNet backend (bitnet_quantization.py:255-432) on the GPU.

    Same constructor and `apply` contract as the reference. `num_threads` only records the value
    (the reference sizes its CPU thread pool with it; the GPU path has none)."""

    def __init__(self, quant_type: BitNetQuantType = BitNetQuantType.I2_S,
                 compute_dtype: torch.dtype = torch.bfloat16, num_threads: Optional[int] = None,
                 pretranspose: bool = False, sparsity_config: Optional[ActivationSparsityConfig] = None):
        self.quant_type = quant_type
        self.compute_dtype = compute_dtype
        self.pretranspose = pretranspose
        self.sparsity_config = sparsity_config or get_default_config()
        self._weight_cache: Dict[tuple, torch.Tensor] = {}
        self._weight_cache_t: Dict[tuple, torch.Tensor] = {}
        self._packed_cache: Dict[int, torch.Tensor] = {}
        self._num_threads = num_threads or self._get_optimal_threads()
        self._last_sparsity: float = 0.0

    @staticmethod
    def _get_optimal_threads() -> int:
        return min(8, os.cpu_count() or 1)

    def _set_threads(self, n: int) -> None:
        self._num_threads = n

    @classmethod
    def get_optimal_dtype(cls) -> torch.dtype:
        return torch.bfloat16

    def _device_packed(self, packed_weight: torch.Tensor) -> torch.Tensor:
        if packed_weight.is_cuda:
            return packed_weight.contiguous()
        key = id(packed_weight)
        if key not in self._packed_cache:
            self._packed_cache[key] = ops._on_device(packed_weight)
        return self._packed_cache[key]

    def _get_cached_weight(self, packed_weight: torch.Tensor, scale: float, out_features: int,
                           in_features: int) -> torch.Tensor:
        key = (id(packed_weight), self.compute_dtype)
        if key not in self._weight_cache:
            self._weight_cache[key] = ops.msb_dequant(self._device_packed(packed_weight), scale, out_features,
                                                      in_features, self.compute_dtype)
        return self._weight_cache[key]

    def _get_cached_weight_t(self, packed_weight: torch.Tensor, scale: float, out_features: int,
                             in_features: int) -> torch.Tensor:
        key = (id(packed_weight), self.compute_dtype)
        if key not in self._weight_cache_t:
            w = self._get_cached_weight(packed_weight, scale, out_features, in_features)
            self._weight_cache_t[key] = w.T.contiguous()
        return self._weight_cache_t[key]

    def clear_cache(self) -> None:
        self._weight_cache.clear()
        self._weight_cache_t.clear()
        self._packed_cache.clear()

    def apply(self, packed_weight: torch.Tensor, scale: float, x: torch.Tensor, out_features: int,
              in_features: int, bias: Optional[torch.Tensor] = None,
              sparsity_config: Optional[ActivationSparsityConfig] = None) -> torch.Tensor:
        """y = x @ W^T (+ bias) in the compute dtype (bitnet_quantization.py:366-409)."""
        host = not x.is_cuda
        xc = ops._on_device(x)
        if xc.dtype != self.compute_dtype:
            xc = xc.to(self.compute_dtype)
        config = sparsity_config or self.sparsity_config
        if config.enabled:
            xc, self._last_sparsity = apply_sparsity(xc, config)
        rows = xc.numel() // max(in_features, 1)
        out = None
        if (self.compute_dtype in (torch.bfloat16, torch.float16) and rows <= DIRECT_MAX_ROWS
                and in_features % 64 == 0 and in_features <= 16384):
            out = ops.msb_linear(self._device_packed(packed_weight), scale, xc, out_features, in_features, bias)
        else:
            if self.pretranspose:
                out = torch.matmul(xc, self._get_cached_weight_t(packed_weight, scale, out_features, in_features))
            else:
                out = torch.matmul(xc, self._get_cached_weight(packed_weight, scale, out_features, in_features).T)
            if bias is not None:
                out = out + bias.to(device=out.device, dtype=self.compute_dtype)
        return _to_host_if(out, host)

    def get_last_sparsity(self) -> float:
        return self._last_sparsity

    def get_sparsity_stats(self) -> Dict[str, float]:
        if not self.sparsity_config.track_stats:
            return {"enabled": False}
        return {
            "enabled": True,
            "mode": self.sparsity_config.mode.value,
            "average_sparsity": self.sparsity_config.get_average_sparsity(),
            "last_sparsity": self._last_sparsity,
            "num_samples": len(self.sparsity_config._sparsity_history),
        }


class BitNetConfig:
    """Quantisation config registered with SGLang (bitnet_quantization.py:435-472)."""

    def __init__(self, quant_type: BitNetQuantType = BitNetQuantType.I2_S, block_size: int = BITNET_BLOCK_SIZE,
                 activation_bits: int = 8):
        self.quant_type = quant_type
        self.block_size = block_size
        self.activation_bits = activation_bits

    @classmethod
    def get_name(cls) -> str:
        return "bitnet"

    @classmethod
    def get_supported_act_dtypes(cls) -> List[torch.dtype]:
        return [torch.int8, torch.float16, torch.bfloat16, torch.float32]

    @classmethod
    def get_min_capability(cls) -> int:
        return 0

    def __repr__(self) -> str:
        return (f"BitNetConfig(quant_type={self.quant_type.name}, block_size={self.block_size}, "
                f"activation_bits={self.activation_bits})")


def validate_bitnet_model(model_path: str) -> Dict[str, Any]:
    """File-level checks of a BitNet GGUF path (bitnet_quantization.py:475-520)."""
    res: Dict[str, Any] = {"valid": False, "path": model_path, "exists": os.path.exists(model_path), "size_mb": 0,
                           "quant_type": None, "errors": []}
    if not res["exists"]:
        res["errors"].append(f"Model file not found: {model_path}")
        return res
    res["size_mb"] = os.path.getsize(model_path) / (1024 * 1024)
    if not model_path.endswith(".gguf"):
        res["errors"].append("Model file must have .gguf extension")
        return res
    low = model_path.lower()
    for tag, qt in (("i2_s", BitNetQuantType.I2_S), ("tl1", BitNetQuantType.TL1), ("tl2", BitNetQuantType.TL2)):
        if tag in low:
            res["quant_type"] = qt
            break
    else:
        res["errors"].append("Could not determine BitNet quant type from filename. "
                             "Expected 'i2_s', 'tl1', or 'tl2' in filename.")
        return res
    res["valid"] = not res["errors"]
    return res
