"""Inference-time activation sparsity for the BitNet linear method (reference
sglang_backend/activation_sparsity.py:23-290: threshold, per-token top-k and variance-adaptive
top-k masks; default disabled). Evaluated with device tensor ops on the caller's stream; the
sparsity ratio is returned as a Python float like the reference (one host read per call)."""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Tuple

import torch


class SparsityMode(str, Enum):
    NONE = "none"
    THRESHOLD = "threshold"
    TOP_K = "top_k"
    ADAPTIVE = "adaptive"


@dataclass
class ActivationSparsityConfig:
    enabled: bool = False
    mode: SparsityMode = SparsityMode.NONE
    threshold: float = 0.01
    top_k_ratio: float = 0.4
    adaptive_min_ratio: float = 0.3
    adaptive_max_ratio: float = 0.7
    track_stats: bool = False
    _sparsity_history: list = field(default_factory=list, repr=False)

    def get_average_sparsity(self) -> float:
        h = self._sparsity_history
        return sum(h) / len(h) if h else 0.0

    def clear_stats(self) -> None:
        self._sparsity_history.clear()


def measure_sparsity(x: torch.Tensor, threshold: float = 1e-6) -> float:
    """Fraction of |x| < threshold (activation_sparsity.py:67-80)."""
    n = x.numel()
    return float((x.abs() < threshold).sum().item()) / n if n else 0.0


def apply_threshold_sparsity(x: torch.Tensor, threshold: float) -> Tuple[torch.Tensor, float]:
    """Keep |x| > threshold (activation_sparsity.py:83-99)."""
    keep = x.abs() > threshold
    return x * keep, 1.0 - float(keep.float().mean().item())


def _keep_topk(x: torch.Tensor, k: int) -> torch.Tensor:
    idx = torch.topk(x.abs(), k, dim=-1).indices
    return torch.zeros_like(x).scatter_(-1, idx, 1.0)


def apply_top_k_sparsity(x: torch.Tensor, ratio: float) -> Tuple[torch.Tensor, float]:
    """Keep the max(1, int(F * ratio)) largest |x| of every token (activation_sparsity.py:102-133)."""
    if ratio >= 1.0:
        return x, 0.0
    if ratio <= 0.0:
        return torch.zeros_like(x), 1.0
    k = max(1, int(x.shape[-1] * ratio))
    return x * _keep_topk(x, k), 1.0 - ratio


def apply_adaptive_sparsity(x: torch.Tensor, min_ratio: float = 0.3,
                            max_ratio: float = 0.7) -> Tuple[torch.Tensor, float]:
    """Per-token keep ratio interpolated by the token's normalised variance
    (activation_sparsity.py:136-195)."""
    var = x.var(dim=-1, keepdim=True)
    lo, hi = var.min(), var.max()
    if float(hi - lo) < 1e-8:
        return apply_top_k_sparsity(x, (min_ratio + max_ratio) / 2)
    keep_ratio = min_ratio + (max_ratio - min_ratio) * ((var - lo) / (hi - lo + 1e-8))
    feats = x.shape[-1]
    k_tok = (keep_ratio * feats).int().clamp(min=1, max=feats)
    kmax = int(k_tok.max().item())
    idx = torch.topk(x.abs(), kmax, dim=-1).indices
    rank = torch.arange(kmax, device=x.device).expand_as(idx)
    kept = rank < k_tok
    mask = torch.zeros_like(x, dtype=torch.float32).scatter_(-1, idx, kept.float())
    # the reference scatters a token's dropped ranks to feature 0 with value 0 after its kept ranks
    # (in-order scatter on the host): feature 0 ends dropped for every token with k < kmax
    mask[..., 0] = torch.where(k_tok[..., 0] < kmax, 0.0, mask[..., 0])
    return x * mask.to(x.dtype), 1.0 - float(keep_ratio.mean().item())


def apply_sparsity(x: torch.Tensor, config: ActivationSparsityConfig) -> Tuple[torch.Tensor, float]:
    if not config.enabled or config.mode == SparsityMode.NONE:
        return x, 0.0
    if config.mode == SparsityMode.THRESHOLD:
        out = apply_threshold_sparsity(x, config.threshold)
    elif config.mode == SparsityMode.TOP_K:
        out = apply_top_k_sparsity(x, config.top_k_ratio)
    elif config.mode == SparsityMode.ADAPTIVE:
        out = apply_adaptive_sparsity(x, config.adaptive_min_ratio, config.adaptive_max_ratio)
    else:
        raise ValueError(f"Unknown sparsity mode: {config.mode}")
    if config.track_stats:
        config._sparsity_history.append(out[1])
    return out


def get_default_config() -> ActivationSparsityConfig:
    return ActivationSparsityConfig(enabled=False)


def get_qsparse_config() -> ActivationSparsityConfig:
    return ActivationSparsityConfig(enabled=True, mode=SparsityMode.TOP_K, top_k_ratio=0.4, track_stats=True)


def get_conservative_config() -> ActivationSparsityConfig:
    return ActivationSparsityConfig(enabled=True, mode=SparsityMode.TOP_K, top_k_ratio=0.7, track_stats=True)


def get_adaptive_config() -> ActivationSparsityConfig:
    return ActivationSparsityConfig(enabled=True, mode=SparsityMode.ADAPTIVE, adaptive_min_ratio=0.3,
                                    adaptive_max_ratio=0.7, track_stats=True)
