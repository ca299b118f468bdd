#!/usr/bin/env python3
"""Diagnostic: full-width prefill vs teacher-forced decode vs the oracle, per layer and position.

    python tools/diag_prefill.py [--n 64] [--seqs 1] [--trained]
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

from test_gpu_configs import bits, logical_kv, make_cfg, make_weights, oracle_arrays, rel_l2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--seqs", type=int, default=1)
    ap.add_argument("--trained", action="store_true")
    ap.add_argument("--inter", type=int, default=6912)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--batch", type=int, default=16, help="decode-side batch (1: the batch-1 VALU path)")
    ap.add_argument("--layers", type=int, default=2)
    args = ap.parse_args()
    from oracle import oracle as orc
    from wfamd.model import BitNetDecoder
    import dataclasses
    cfg = dataclasses.replace(make_cfg(args.layers, 128256, 2080), inter=args.inter)
    w = make_weights(cfg, seed=6, trained_like=args.trained)
    B, n = 16, args.n
    pf = BitNetDecoder(cfg, w, batch=B)
    dc = BitNetDecoder(cfg, w, batch=args.batch)
    a = oracle_arrays(cfg, w) if args.oracle else None
    rng = np.random.default_rng(12)
    prompts = [rng.integers(0, cfg.vocab, size=n + 1).tolist() for _ in range(args.seqs)]
    pf.prefill([(b, prompts[b][:n], 0) for b in range(args.seqs)], chunk_rows=16384)
    for t in range(n):
        dc.set_state([prompts[b][t] if b < args.seqs else 0 for b in range(args.batch)], [t] * args.batch)
        dc.step(graph=True)
    torch.cuda.synchronize()
    m = None
    if args.oracle:
        m = orc.DecodeModel(a)
        for t in range(n):
            m.step(prompts[0][t], t, logits=False)
    for l in range(cfg.layers):
        kp, vp = logical_kv(pf, l, 0, n)
        kd, vd = logical_kv(dc, l, 0, n)
        kp, vp, kd, vd = (orc.bf16_to_f32(bits(x)) for x in (kp, vp, kd, vd))
        ek = [rel_l2(kp[:, t], kd[:, t]) for t in range(n)]
        ev = [rel_l2(vp[:, t], vd[:, t]) for t in range(n)]
        print(f"layer {l} prefill vs decode: K max {max(ek):.2e} at {int(np.argmax(ek))}, V max {max(ev):.2e}")
        print("          prefill vs decode per position:", " ".join(f"{e:.1e}" for e in ek[:32]))
        if m is not None:
            kr, vr = orc.bf16_to_f32(m.k_cache[l, :, :n]), orc.bf16_to_f32(m.v_cache[l, :, :n])
            eo = [rel_l2(kd[:, t], kr[:, t]) for t in range(n)]
            ep = [rel_l2(kp[:, t], kr[:, t]) for t in range(n)]
            print(f"          decode vs oracle K max {max(eo):.2e}; prefill vs oracle K max {max(ep):.2e}")
            print(f"          positions > 1e-3: decode {sum(e > 1e-3 for e in eo)}/{n}, prefill {sum(e > 1e-3 for e in ep)}/{n}; "
                  f"layer rel-L2 decode {rel_l2(kd, kr):.2e} prefill {rel_l2(kp, kr):.2e}")
            print("          decode vs oracle per position:", " ".join(f"{e:.1e}" for e in eo[:32]))
            print("          prefill vs oracle per position:", " ".join(f"{e:.1e}" for e in ep[:32]))


if __name__ == "__main__":
    main()
