"""Drop-in for the reference's `sgl_kernel` BitNet surface (extern/sglang-bitnet/sgl-kernel, un-vendored;
API recovered in SURVEY.md §8b), backed by the gfx950 HIP kernels of lib/libwfbitnet.so.

Importing registers torch.ops.sgl_kernel.bitnet_{gemv,gemm,quantize_activations}_cpu (schemas of
docs/research/sglang_optimization_plan.md:61-74) unless a real sgl_kernel already owns them.
"""
from wfamd import ops as _ops

_ops.register_torch_ops()

from . import quantization  # noqa: E402,F401
from . import kvcache  # noqa: E402,F401

__version__ = "0.1.0+mi355x"
