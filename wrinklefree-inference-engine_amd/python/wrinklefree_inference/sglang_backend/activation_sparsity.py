"""Activation-sparsity configuration surface of the BitNet linear method -- API compatibility only.

The reference's inference-time activation sparsity (sglang_backend/activation_sparsity.py) is
SURVEY §2 row 4b: OUT of scope (disabled by default there; the reference measured a slowdown,
docs/research/notebook.md:802-813). `BitNetLinearMethod` (bitnet_quantization.py) keeps its
`sparsity_config` argument and stats accessors, so the config type and the disabled default exist
here; enabling a mode raises instead of silently computing something else.
"""
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
    track_stats: bool = False
    _sparsity_history: list = field(default_factory=list, repr=False)

    def get_average_sparsity(self) -> float:
        h = self._sparsity_history
        return sum(h) / len(h) if h else 0.0

    def clear_stats(self) -> None:
        self._sparsity_history.clear()


def apply_sparsity(x: torch.Tensor, config: ActivationSparsityConfig) -> Tuple[torch.Tensor, float]:
    """Identity for the disabled default (the reference's default path); any enabled mode raises."""
    if not config.enabled or config.mode == SparsityMode.NONE:
        return x, 0.0
    raise NotImplementedError(f"activation sparsity mode {config.mode.value!r} is out of scope "
                              "(SURVEY.md §2 row 4b); use the default (disabled) config")


def get_default_config() -> ActivationSparsityConfig:
    return ActivationSparsityConfig(enabled=False)
