"""BitNetLinear on the fused HIP path.

The reference's decode runs this layer seven times per block (scripts/direct_inference_full.py:
186-208): per-row int8 activation quantization, ternary matmul on the packed weights, then the
encoding correction y = (raw - ws * sum(q)) * s, cast to bf16. `BitNetLinear.forward` is one C-ABI
call (wf_bitnet_linear): a single launch for fewer than 16 rows, else a quantize launch plus the
int8-MFMA GEMM.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from ._lib import WF_FMT_I2S, WF_FMT_TQ


class BitNetLinear(nn.Module):
    """bf16 [..., in_features] -> bf16 [..., out_features] with packed ternary weights.

    `packed` is the blocked I2_S layout [out, in/4] (cache/bitnet_converter.py:26-77) or, with
    fmt=WF_FMT_TQ, the ~1.6-bit layout; `weight_scale` is the layer's float scale.
    """

    def __init__(self, in_features: int, out_features: int, packed: torch.Tensor, weight_scale: float,
                 fmt: int = WF_FMT_I2S):
        super().__init__()
        if fmt not in (WF_FMT_I2S, WF_FMT_TQ):
            raise ValueError(f"unknown weight format {fmt}")
        if packed.shape[0] != out_features:
            raise ValueError(f"packed weights have {packed.shape[0]} rows, expected {out_features}")
        self.in_features = in_features
        self.out_features = out_features
        self.fmt = fmt
        self.weight_scale = float(weight_scale)
        self.register_buffer("packed_weight", packed)

    @classmethod
    def from_ternary(cls, weight: torch.Tensor, weight_scale: float, fmt: int = WF_FMT_I2S) -> "BitNetLinear":
        """Pack a {-1, 0, +1} weight [out, in] on the device."""
        w = weight.to("cuda") if not weight.is_cuda else weight
        packed = ops.pack_i2s(w)
        if fmt == WF_FMT_TQ:
            packed = ops.i2s_to_tq(packed)
        return cls(weight.shape[1], weight.shape[0], packed, weight_scale, fmt)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.bitnet_linear(x, self.packed_weight, self.weight_scale, self.fmt, self.in_features)

    def extra_repr(self) -> str:
        fmt = "i2s" if self.fmt == WF_FMT_I2S else "tq"
        return f"in_features={self.in_features}, out_features={self.out_features}, fmt={fmt}"


class BitNetFusedLinear(nn.Module):
    """Two or three BitNetLinear layers that read the same input (q|k|v, gate|up) as ONE op with one
    shared activation quantization (include/wf_bitnet.h wf_bitnet_linear_fused).
    forward returns a tuple with one bf16 tensor per layer, each bit-identical to that layer alone."""

    def __init__(self, layers: "list[BitNetLinear]"):
        super().__init__()
        if not 1 <= len(layers) <= 3:
            raise ValueError("BitNetFusedLinear takes 1..3 layers")
        k, fmt = layers[0].in_features, layers[0].fmt
        if any(l.in_features != k or l.fmt != fmt for l in layers):
            raise ValueError("fused layers must share in_features and the weight format")
        self.in_features = k
        self.fmt = fmt
        self.rows = [l.out_features for l in layers]
        self.weight_scales = [l.weight_scale for l in layers]
        self.register_buffer("packed_weight", torch.cat([l.packed_weight for l in layers], dim=0).contiguous())

    def forward(self, x: torch.Tensor):
        return tuple(ops.bitnet_linear_fused(x, self.packed_weight, self.rows, self.weight_scales, self.fmt,
                                             self.in_features))

    def extra_repr(self) -> str:
        return f"in_features={self.in_features}, rows={self.rows}, fmt={'i2s' if self.fmt == WF_FMT_I2S else 'tq'}"


class BitNetMLP(nn.Module):
    """The BitNet MLP block (scripts/direct_inference_full.py:252-265) as one op (wf_bitnet_mlp):
    down(rms_norm(relu(gate(x))^2 * up(x), ffn_sub_norm)), gate|up sharing one quantization."""

    def __init__(self, gate: BitNetLinear, up: BitNetLinear, down: BitNetLinear, ffn_sub_norm: torch.Tensor,
                 eps: float = 1e-5):
        super().__init__()
        if not (gate.in_features == up.in_features == down.out_features and gate.out_features == up.out_features
                == down.in_features and gate.fmt == up.fmt == down.fmt):
            raise ValueError("gate / up / down shapes or formats do not form an MLP")
        self.hidden, self.inter, self.fmt, self.eps = gate.in_features, gate.out_features, gate.fmt, float(eps)
        self.scales = (gate.weight_scale, up.weight_scale, down.weight_scale)
        self.register_buffer("packed_gate_up", torch.cat([gate.packed_weight, up.packed_weight], 0).contiguous())
        self.register_buffer("packed_down", down.packed_weight)
        self.register_buffer("ffn_sub_norm", ffn_sub_norm.to(torch.bfloat16).contiguous())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.bitnet_mlp(x, self.packed_gate_up, self.packed_down, *self.scales, self.ffn_sub_norm, self.eps,
                              self.fmt)

