"""Inputs of the full-width reference golden (tests/golden/decode_full.npz): bitnet-b1.58-2B-4T
geometry (H 2560, I 6912, 20 / 5 heads x 128, vocab 128256; scripts/direct_inference_full.py:84-89)
with 2 layers, regenerated from torch CPU generator seeds wherever the fixture is checked (the
fixture stores outputs only, plus sha256 sums of these inputs so a generator mismatch fails loudly
instead of reading as a parity error).

* weights: wfamd.model.synthetic_weights(seed 21) on the CPU -- packed I2_S bytes (uniform ternary),
  embedding randn * 0.02, norm weights 1 + 0.1 randn, per-projection scales U[1.5, 2.0) -- with the
  q / k scales set to 0.05 so attention scores are O(1) as in a trained model (the random-init
  scales give |scores| ~ 30, a one-hot softmax);
* a random K/V history of CTX0 positions per layer (seed 22, N(0, 1) bf16), then POSITIONS decode
  steps from FIRST_TOKEN, teacher-forced by the reference's own greedy tokens.
"""
from __future__ import annotations

import hashlib

import torch

FULL = dict(hidden=2560, layers=2, n_heads=20, n_kv_heads=5, head_dim=128, inter=6912, vocab=128256, max_seq=4096)
WEIGHT_SEED, HIST_SEED = 21, 22
CTX0, POSITIONS, FIRST_TOKEN = 960, 64, 4242
TOPK = 64


def config():
    from wfamd.model import BitNetConfig
    return BitNetConfig(**FULL)


def weights(cfg):
    from wfamd.model import synthetic_weights
    w = synthetic_weights(cfg, seed=WEIGHT_SEED, device="cpu")
    w["wscale"][:, :2] = 0.05
    return w


def history(cfg):
    """K, V [layers, n_kv_heads, CTX0, head_dim] bf16."""
    g = torch.Generator().manual_seed(HIST_SEED)
    shape = (cfg.layers, cfg.n_kv_heads, CTX0, cfg.head_dim)
    k = torch.randn(shape, generator=g).to(torch.bfloat16)
    v = torch.randn(shape, generator=g).to(torch.bfloat16)
    return k, v


def input_digest(w, k, v) -> str:
    h = hashlib.sha256()
    for n in ("wq", "wk", "wv", "wo", "wg", "wu", "wd", "embed", "final_norm", "ln_in", "ln_post", "attn_sub",
              "ffn_sub", "wscale"):
        t = w[n].contiguous()
        h.update(t.view(torch.uint8).numpy().tobytes() if t.dtype != torch.float32 else t.numpy().tobytes())
    for t in (k, v):
        h.update(t.contiguous().view(torch.int16).numpy().tobytes())
    return h.hexdigest()
