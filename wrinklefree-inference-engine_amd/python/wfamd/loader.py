"""Checkpoint loader for the decode path: a bitnet-b1.58 checkpoint directory ->
BitNetConfig + the per-projection I2_S weight dict that `BitNetDecoder` takes.

Three on-disk forms of a ternary projection are recognised per tensor name (safetensors only --
nothing that unpickles):

* HF packed (microsoft/bitnet-b1.58-2B-4T; transformers integrations/bitnet.py:56-120, restated
  tests/test_bitnet_core.py:21-53): `<proj>.weight` uint8 [N/4, K] + `<proj>.weight_scale`.
  Repacked on the GPU by `wf_hf_to_i2s` exactly like scripts/direct_inference_full.py:110-114.
* The reference's converted cache (`cache_metadata.json` format_version "packed_bitnet_v1",
  cache/bitnet_converter.py:103-187): `<proj>.qweight` uint8 [N, K/4] already blocked I2_S +
  `<proj>.weight_scale`.
* Float ternary `<proj>.weight` [N, K] in {-1, 0, +1} (the converter's input,
  bitnet_converter.py:78-100): packed on the GPU by `wf_pack_i2s`; scale from `<proj>.weight_scale`
  when present, else 1.0.

The weight scale multiplies the integer sum like the reference's decode
(scripts/direct_inference_full.py:186-208; HF's BitLinear divides instead -- the reference's
convention is the one this path reproduces). The LM head is the tied embedding
(direct_inference_full.py:122-124). Norm weights and the embedding are loaded as bf16.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Tuple

import torch

from . import ops
from .model import BitNetConfig

PROJ = (("wq", "self_attn.q_proj"), ("wk", "self_attn.k_proj"), ("wv", "self_attn.v_proj"),
        ("wo", "self_attn.o_proj"), ("wg", "mlp.gate_proj"), ("wu", "mlp.up_proj"), ("wd", "mlp.down_proj"))
NORMS = (("ln_in", "input_layernorm"), ("ln_post", "post_attention_layernorm"),
         ("attn_sub", "self_attn.attn_sub_norm"), ("ffn_sub", "mlp.ffn_sub_norm"))


def config_from_hf(cfg: dict, max_seq: int = 4096) -> BitNetConfig:
    """HF config.json keys (as read by direct_inference_full.py:80-91)."""
    h, nh = int(cfg["hidden_size"]), int(cfg["num_attention_heads"])
    return BitNetConfig(hidden=h, layers=int(cfg["num_hidden_layers"]), n_heads=nh,
                        n_kv_heads=int(cfg.get("num_key_value_heads", nh)), head_dim=int(cfg.get("head_dim", h // nh)),
                        inter=int(cfg["intermediate_size"]), vocab=int(cfg["vocab_size"]), max_seq=int(max_seq),
                        eps=float(cfg.get("rms_norm_eps", 1e-5)), rope_theta=float(cfg.get("rope_theta", 500000.0)))


def checkpoint_format(path) -> str:
    """'packed_bitnet_v1' for the reference's converted cache, else 'hf'."""
    meta = Path(path) / "cache_metadata.json"
    if meta.exists():
        return str(json.loads(meta.read_text()).get("format_version", "hf"))
    return "hf"


class _Tensors:
    """Name -> tensor view over every *.safetensors file of a directory (lazy, memory-mapped)."""

    def __init__(self, path: Path):
        from safetensors import safe_open
        files = sorted(Path(path).glob("*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {path}")
        self._where: Dict[str, object] = {}
        self._handles = [safe_open(str(f), framework="pt", device="cpu") for f in files]
        for h in self._handles:
            for k in h.keys():
                self._where[k] = h

    def __contains__(self, name: str) -> bool:
        return name in self._where

    def get(self, name: str) -> torch.Tensor:
        if name not in self._where:
            raise KeyError(f"tensor {name!r} not in checkpoint")
        return self._where[name].get_tensor(name)

    def names(self):
        return list(self._where)


def _scale(t: _Tensors, base: str) -> float:
    name = f"{base}.weight_scale"
    return float(t.get(name).float().reshape(-1)[0].item()) if name in t else 1.0


def _projection(t: _Tensors, base: str, n: int, k: int, dev: torch.device) -> Tuple[torch.Tensor, float]:
    """One ternary projection -> (I2_S uint8 [n, k/4] on `dev`, weight scale)."""
    if f"{base}.qweight" in t:                                  # converted cache (blocked I2_S)
        q = t.get(f"{base}.qweight")
        if q.dtype != torch.uint8 or tuple(q.shape) != (n, k // 4):
            raise ValueError(f"{base}.qweight: expected uint8 [{n}, {k // 4}], got {q.dtype} {tuple(q.shape)}")
        return q.to(dev).contiguous(), _scale(t, base)
    w = t.get(f"{base}.weight")
    if w.dtype == torch.uint8:                                   # HF packed [n/4, k]
        if tuple(w.shape) != (n // 4, k):
            raise ValueError(f"{base}.weight: expected HF-packed uint8 [{n // 4}, {k}], got {tuple(w.shape)}")
        return ops.hf_to_i2s(w.to(dev)), _scale(t, base)
    if tuple(w.shape) != (n, k):                                 # float ternary [n, k]
        raise ValueError(f"{base}.weight: expected [{n}, {k}], got {tuple(w.shape)}")
    return ops.pack_i2s(w.to(dev)), _scale(t, base)


def load_checkpoint(path, device="cuda", max_seq: int = 4096) -> Tuple[BitNetConfig, Dict[str, torch.Tensor]]:
    """Load a checkpoint directory (config.json + *.safetensors) into the decoder's weight dict."""
    path = Path(path)
    cfg = config_from_hf(json.loads((path / "config.json").read_text()), max_seq=max_seq)
    if cfg.head_dim != 128:
        raise ValueError(f"head_dim {cfg.head_dim} unsupported (the decode kernels are built for 128)")
    dev = torch.device(device)
    t = _Tensors(path)
    h, i, kv, L = cfg.hidden, cfg.inter, cfg.kv_dim, cfg.layers
    shapes = {"wq": (h, h), "wk": (kv, h), "wv": (kv, h), "wo": (h, h), "wg": (i, h), "wu": (i, h), "wd": (h, i)}
    w: Dict[str, torch.Tensor] = {}
    wscale = torch.zeros(L, 7, dtype=torch.float32)
    for j, (key, sub) in enumerate(PROJ):
        per = []
        for l in range(L):
            p, s = _projection(t, f"model.layers.{l}.{sub}", *shapes[key], dev)
            per.append(p)
            wscale[l, j] = s
        w[key] = torch.stack(per)
    w["wscale"] = wscale
    for key, sub in NORMS:
        w[key] = torch.stack([t.get(f"model.layers.{l}.{sub}.weight").to(torch.bfloat16) for l in range(L)]).to(dev)
    w["embed"] = t.get("model.embed_tokens.weight").to(torch.bfloat16).to(dev).contiguous()
    w["final_norm"] = t.get("model.norm.weight").to(torch.bfloat16).to(dev)
    if tuple(w["embed"].shape) != (cfg.vocab, h):
        raise ValueError(f"embed_tokens {tuple(w['embed'].shape)} != ({cfg.vocab}, {h})")
    return cfg, w
