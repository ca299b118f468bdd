"""sgl_kernel.quantization drop-in (import sites: kernels/bitnet_patch.py:15-21,
scripts/benchmark_kernels.py:11-17, scripts/test_fallback.py:20)."""
from .bitnet import (  # noqa: F401
    BITNET_BLOCK_SIZE,
    auto_tune_tiles,
    bitnet_check_kernel_available,
    bitnet_gemm,
    bitnet_gemv,
    bitnet_quantize_activations,
    check_kernel_available,
    quantize_activations_i8,
)

__all__ = [
    "BITNET_BLOCK_SIZE",
    "bitnet_check_kernel_available",
    "bitnet_gemm",
    "bitnet_gemv",
    "bitnet_quantize_activations",
    "quantize_activations_i8",
]
