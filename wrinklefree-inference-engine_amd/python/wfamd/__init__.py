"""wfamd -- MI355X (gfx950) BitNet 1.58-bit hot path: host side of the C-ABI in include/wf_bitnet.h.

  wfamd._lib   ctypes binding of lib/libwfbitnet.so (fails loudly when missing)
  wfamd.ops    tensor-level ops (ternary GEMV/GEMM, int8 quantizer, formats, KV, attention)
  wfamd.model  fused decode step of bitnet-b1.58-2B-4T (graph-replayed)

The reference-facing drop-ins live next to this package: `sgl_kernel` and `wrinklefree_inference`.
"""
from ._lib import WF_FMT_I2S, WF_FMT_I2S_MFMA, WF_FMT_TQ, kernel_available  # noqa: F401

__version__ = "0.1.0"
