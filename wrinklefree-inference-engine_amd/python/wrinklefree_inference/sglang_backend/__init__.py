"""Drop-in for the reference's `wrinklefree_inference.sglang_backend` -- its BitNet linear method
(sglang_backend/__init__.py:3-8, bitnet_quantization.py), backed by the gfx950 kernels."""
from wrinklefree_inference.sglang_backend.bitnet_quantization import BITNET_QUANT_TYPES, BitNetConfig

__all__ = ["BitNetConfig", "BITNET_QUANT_TYPES"]
