"""sgl_kernel.quantization.bitnet drop-in (scripts/direct_inference_full.py:22,
scripts/profile_bitnet_ops.py:8, tests/test_vllm_cpu_stub.py:313, docs/research/notebook.md:92).

Semantics:
  bitnet_gemv(packed [N, K/4] uint8 blocked I2_S, act [K] int8, scale) -> float32 [N]
      y[n] = float(sum_k enc(W[n,k]) * act[k]) * scale,  enc = w + 1 in {0,1,2}  (raw, uncorrected)
  bitnet_gemm(packed, act [M, K] int8, scale) -> float32 [M, N]
  quantize_activations_i8(x) -> (int8 same shape, float s = max|x|/127), round-half-even
Device tensors run in place on the current HIP stream; host tensors are staged through the GPU.
"""
from wfamd import ops as _ops

BITNET_BLOCK_SIZE = _ops.BITNET_BLOCK_SIZE


def check_kernel_available() -> bool:
    return _ops.check_kernel_available()


bitnet_check_kernel_available = check_kernel_available


def bitnet_gemv(packed_weights, activations, scale):
    return _ops.bitnet_gemv(packed_weights, activations, scale)


def bitnet_gemm(packed_weights, activations, scale):
    return _ops.bitnet_gemm(packed_weights, activations, scale)


def quantize_activations_i8(activations):
    return _ops.quantize_activations_i8(activations)


bitnet_quantize_activations = quantize_activations_i8


def auto_tune_tiles(*args, **kwargs):
    """The reference stub (docs/research/notebook.md:92) returns nothing; the HIP kernels need no
    tile tuning at import time."""
    return None
