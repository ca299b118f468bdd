#!/usr/bin/env python3
"""Diagnostic: the batched step at a batch that is not a multiple of 32 (test_gpu_configs (b) at
batch 40) -- per step and sampled row: position, logits / appended K/V vs the oracle.

    python tools/diag_ragged_batch.py [--batch 40] [--steps 3] [--eager]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_configs import bits, kv_bits, logical_kv, make_cfg, make_weights, oracle_arrays, rel_l2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=40)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--dense", action="store_true")
    args = ap.parse_args()
    from oracle import oracle as orc
    from wfamd.model import BitNetDecoder
    orc.build()
    cfg = make_cfg(2, 128256, 4128)
    w = make_weights(cfg, seed=2, trained_like=True)
    B, steps = args.batch, args.steps
    ctxs = np.random.default_rng(0).integers(1, 4096, size=B)
    pages = int(sum((c + steps + 1 + 31) // 32 for c in ctxs))
    dec = BitNetDecoder(cfg, w, batch=B, **({} if args.dense else dict(num_pages=pages, page_seed=0)))
    a = oracle_arrays(cfg, w)
    del w
    rows = sorted({int(np.argmin(ctxs)), int(np.argmax(ctxs))} | {r for r in (0, 1, 17, 22, 24, 33, 39) if r < B})
    print("rows", rows, "ctx", [int(ctxs[r]) for r in rows], flush=True)
    gen = torch.Generator(device="cuda").manual_seed(77)
    cmax = int(ctxs.max())
    models = {b: orc.DecodeModel(a) for b in rows}
    for l in range(cfg.layers):
        k = torch.randn(B, cfg.n_kv_heads, cmax, cfg.head_dim, generator=gen, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, cfg.n_kv_heads, cmax, cfg.head_dim, generator=gen, device="cuda").to(torch.bfloat16)
        dec.load_kv(l, k, v, lengths=ctxs)
        for b in rows:
            c = int(ctxs[b])
            kb, vb = logical_kv(dec, l, b, c)
            models[b].k_cache[l, :, :c] = kv_bits(dec, kb, l, 0)
            models[b].v_cache[l, :, :c] = kv_bits(dec, vb, l, 1)
    if dec.paged:
        for b in range(B):
            dec.reserve(b, int(ctxs[b]) + steps + 1)
    dec.set_state([(97 * b + 11) % cfg.vocab for b in range(B)], [int(c) for c in ctxs])
    for i in range(steps):
        toks = dec.tokens.cpu().numpy().copy()
        pos0 = dec.positions.cpu().numpy().copy()
        dec.step(graph=not args.eager)
        torch.cuda.synchronize()
        pos1 = dec.positions.cpu().numpy().copy()
        for b in rows:
            pos = int(ctxs[b]) + i
            ologits, onext = models[b].step(int(toks[b]), pos)
            err = rel_l2(orc.bf16_to_f32(bits(dec.logits[b])), orc.bf16_to_f32(ologits))
            kv = []
            for l in range(cfg.layers):
                kg, vg = logical_kv(dec, l, b, pos + 1)
                kv.append(rel_l2(orc.bf16_to_f32(kv_bits(dec, kg[:, pos], l, 0)), orc.bf16_to_f32(models[b].k_cache[l, :, pos])))
                kv.append(rel_l2(orc.bf16_to_f32(kv_bits(dec, vg[:, pos], l, 1)), orc.bf16_to_f32(models[b].v_cache[l, :, pos])))
            print(f"step {i} row {b:3d} pos {pos} (gpu pos {pos0[b]} -> {pos1[b]}) logits {err:.2e} kv {' '.join(f'{e:.1e}' for e in kv)}"
                  f" tok gpu {int(dec.tokens[b])} orc {onext}", flush=True)


if __name__ == "__main__":
    main()
