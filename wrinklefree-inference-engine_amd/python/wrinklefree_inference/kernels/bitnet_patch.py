"""Module-swap of BitNet linears onto the HIP ternary kernels.

API and behaviour of the reference's src/wrinklefree_inference/kernels/bitnet_patch.py:
  * NATIVE_KERNELS_AVAILABLE / BITNET_BLOCK_SIZE from sgl_kernel.quantization (:13-25);
  * BitNetLinearNative (:28-78): per-tensor int8 quantize, scale = weight_scale * act_scale,
    bitnet_gemv for one token, bitnet_gemm for a batch, + bias. Like the reference it applies no
    encoding correction and calls the blocked-layout kernel on whatever `packed_weight` holds;
  * pack_ternary_weights (:81-112): the LSB-interleaved layout byte |= enc(w[:, i::4]) << 2i;
  * extract_packed_weight_and_scale (:115-162), patch_model_with_native_kernels (:165-210),
    benchmark_kernels (:213-268).
"""
from __future__ import annotations

import logging
import time
from typing import Optional, Tuple

import torch
import torch.nn as nn

logger = logging.getLogger(__name__)

try:
    from sgl_kernel.quantization import (
        BITNET_BLOCK_SIZE,
        bitnet_check_kernel_available,
        bitnet_gemm,
        bitnet_gemv,
        bitnet_quantize_activations,
    )
    NATIVE_KERNELS_AVAILABLE = bitnet_check_kernel_available()
except ImportError:
    NATIVE_KERNELS_AVAILABLE = False
    BITNET_BLOCK_SIZE = 128


class BitNetLinearNative(nn.Module):
    """Linear layer on the HIP ternary kernels (reference kernels/bitnet_patch.py:28-78)."""

    def __init__(self, in_features: int, out_features: int, packed_weight: torch.Tensor,
                 weight_scale: torch.Tensor, bias: Optional[torch.Tensor] = None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.register_buffer("packed_weight", packed_weight)
        self.register_buffer("weight_scale", weight_scale)
        if bias is not None:
            self.register_buffer("bias", bias)
        else:
            self.bias = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        batch_shape = x.shape[:-1]
        x_flat = x.reshape(-1, self.in_features)
        x_int8, act_scale = bitnet_quantize_activations(x_flat)
        scale = self.weight_scale.item() * act_scale
        if x_flat.shape[0] == 1:
            output = bitnet_gemv(self.packed_weight, x_int8.squeeze(0), scale).unsqueeze(0)
        else:
            output = bitnet_gemm(self.packed_weight, x_int8, scale)
        if self.bias is not None:
            output = output + self.bias.to(output.device)
        return output.view(*batch_shape, self.out_features)


def pack_ternary_weights(weight: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """{-1,0,+1} -> LSB-interleaved uint8 [out, in/4] + scale (max|w|, 1.0 if < 1e-6)."""
    out_features, in_features = weight.shape
    if in_features % 4 != 0:
        raise ValueError(f"in_features ({in_features}) must be divisible by 4")
    enc = (torch.round(weight.float()).clamp(-1, 1).to(torch.int8) + 1).to(torch.uint8)
    packed = (enc[:, 0::4] | (enc[:, 1::4] << 2) | (enc[:, 2::4] << 4) | (enc[:, 3::4] << 6)).contiguous()
    scale = weight.abs().max().item()
    if scale < 1e-6:
        scale = 1.0
    return packed, torch.tensor(scale, dtype=torch.float32)


def extract_packed_weight_and_scale(linear: nn.Module, force_repack: bool = True):
    if not hasattr(linear, "weight"):
        return None, None, None
    weight = linear.weight.data
    if weight.dtype == torch.uint8:
        packed_weight = weight
        if hasattr(linear, "weight_scale"):
            weight_scale = linear.weight_scale.data
        elif hasattr(linear, "scale"):
            weight_scale = linear.scale.data
        else:
            weight_scale = torch.tensor(1.0)
    elif force_repack and weight.numel() > 0:
        uniq = torch.unique(torch.round(weight.float()))
        if len(uniq) <= 3 and uniq.abs().max() <= 1.0:
            try:
                packed_weight, weight_scale = pack_ternary_weights(weight)
            except Exception as e:  # mirrors the reference's warning path
                logger.warning(f"Failed to repack weights for {linear}: {e}")
                return None, None, None
        else:
            logger.warning(f"Non-ternary weights found (unique: {uniq.tolist()}), skipping {linear}")
            return None, None, None
    else:
        logger.warning(f"Non-packed weights found, skipping native kernel for {linear}")
        return None, None, None
    bias = linear.bias.data if getattr(linear, "bias", None) is not None else None
    return packed_weight, weight_scale, bias


def patch_model_with_native_kernels(model: nn.Module) -> int:
    if not NATIVE_KERNELS_AVAILABLE:
        logger.warning("Native BitNet kernels not available, skipping patch")
        return 0
    patched = 0
    for name, module in list(model.named_modules()):
        if isinstance(module, nn.Linear) or "Linear" in type(module).__name__:
            packed_weight, weight_scale, bias = extract_packed_weight_and_scale(module)
            if packed_weight is None:
                continue
            out_features, in_features = packed_weight.shape[0], packed_weight.shape[1] * 4
            if in_features % BITNET_BLOCK_SIZE != 0:
                continue
            dev = packed_weight.device if packed_weight.is_cuda else torch.device("cuda")
            native = BitNetLinearNative(in_features, out_features, packed_weight.to(dev), weight_scale,
                                        None if bias is None else bias.to(dev))
            parent_name, _, attr = name.rpartition(".")
            parent = model.get_submodule(parent_name) if parent_name else model
            setattr(parent, attr, native)
            patched += 1
    logger.info(f"Patched {patched} layers with native BitNet kernels")
    return patched


def benchmark_kernels(in_features: int = 2048, out_features: int = 2048, batch_size: int = 1,
                      num_iterations: int = 100) -> dict:
    if not NATIVE_KERNELS_AVAILABLE:
        return {"error": "Native kernels not available"}
    dev = torch.device("cuda")
    packed_weight = torch.randint(0, 256, (out_features, in_features // 4), dtype=torch.uint8, device=dev)
    weight_scale = torch.tensor(0.1)
    x = torch.randn(batch_size, in_features, device=dev)

    def run():
        x_int8, act_scale = bitnet_quantize_activations(x)
        if batch_size == 1:
            return bitnet_gemv(packed_weight, x_int8.squeeze(0), weight_scale.item() * act_scale)
        return bitnet_gemm(packed_weight, x_int8, weight_scale.item() * act_scale)

    for _ in range(10):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(num_iterations):
        run()
    torch.cuda.synchronize()
    native_time = (time.perf_counter() - t0) / num_iterations
    unpacked = torch.zeros(out_features, in_features, device=dev)
    packed = packed_weight.to(torch.int32)
    for i in range(4):
        unpacked[:, i::4] = ((packed >> (i * 2)) & 0x03).float() - 1.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(num_iterations):
        torch.matmul(x, unpacked.t())
    torch.cuda.synchronize()
    torch_time = (time.perf_counter() - t0) / num_iterations
    return {"native_ms": native_time * 1000, "torch_ms": torch_time * 1000, "speedup": torch_time / native_time,
            "in_features": in_features, "out_features": out_features, "batch_size": batch_size}
