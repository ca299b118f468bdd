#!/usr/bin/env python3
"""End-to-end prefill of bitnet-b1.58-2B-4T (BASELINE configs[2]: 8 sequences x 2048 tokens =
16384 token rows) through wf_model_prefill on one MI355X: embed, 30 layers of row norm + fused
tile-layout int8-MFMA GEMMs (QKV + RoPE + K/V cache write, O + residual, gate|up + ReLU^2, down +
residual) and causal attention on the batched decoder's KV cache. Synthetic random-init weights.
Reports tokens/s and ms per prefill (HIP events around the whole call, inputs resident), and the
GEMM-only int8 TOPS share.

    python tools/prefill_bench.py [--seqs 8] [--seq-len 2048] [--iters 3] [--paged]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--paged", action="store_true")
    args = ap.parse_args()
    cfg = BITNET_2B
    B = max(16, args.seqs)  # the matrix-core decoder (batch >= 16) owns the KV slots
    n = args.seqs * args.seq_len
    pages = B * cfg.max_seq // 32 if args.paged else 0
    w = synthetic_weights(cfg, seed=0, device="cuda")
    dec = BitNetDecoder(cfg, w, batch=B, num_pages=pages, page_seed=0 if args.paged else None)
    del w
    torch.cuda.empty_cache()
    rng = np.random.default_rng(0)
    seqs = [(b, rng.integers(0, cfg.vocab, size=args.seq_len).tolist(), 0) for b in range(args.seqs)]
    dec.prefill(seqs, chunk_rows=args.chunk)  # warm (allocates the row workspace)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    times = []
    for _ in range(args.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dec.prefill(seqs, chunk_rows=args.chunk)
        e1.record(st)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times)[len(times) // 2]
    h, i, kv = cfg.hidden, cfg.inter, cfg.kv_dim
    gemm_ops = 2.0 * n * cfg.layers * ((h + 2 * kv) * h + h * h + 2 * i * h + h * i)
    print(json.dumps({"workload": f"prefill {args.seqs} x {args.seq_len} tokens (BASELINE configs[2])",
                      "rows": n, "ms": round(ms, 2), "tokens_per_s": round(n / (ms / 1000.0), 1),
                      "gemm_tops_if_all_time": round(gemm_ops / (ms / 1000.0) / 1e12, 1),
                      "kv": "paged" if args.paged else "dense", "chunk_rows": args.chunk}))


if __name__ == "__main__":
    main()
