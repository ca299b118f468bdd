# BitNet native kernels (reference: src/wrinklefree_inference/kernels/__init__.py)
from .bitnet_patch import (  # noqa: F401
    NATIVE_KERNELS_AVAILABLE,
    BitNetLinearNative,
    benchmark_kernels,
    patch_model_with_native_kernels,
)

__all__ = [
    "NATIVE_KERNELS_AVAILABLE",
    "BitNetLinearNative",
    "patch_model_with_native_kernels",
    "benchmark_kernels",
]
