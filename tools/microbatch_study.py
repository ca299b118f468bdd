"""Study: the batch-128 decode step as N concurrent micro-batches (N decoders of 128 / N sequences
sharing one weight set, each replaying its step graph on its own stream) against one decoder of 128.
The batched step is a chain of latency-bound launches (row norms, GEMMs) and one HBM-bound launch
(attention) per layer; independent micro-batch chains can fill each other's idle CUs.
Prints one JSON line per configuration. Usage: python tools/microbatch_study.py [--ctx-dist uniform]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402


def run(w, cfg, B: int, nmb: int, ctxs, steps: int, warmup: int, kv: str) -> dict:
    per = B // nmb
    total = steps + warmup
    decs, streams = [], []
    for i in range(nmb):
        c = ctxs[i * per:(i + 1) * per]
        paged = len(set(c.tolist())) > 1
        npages = int(sum((x + total + 1 + 31) // 32 for x in c)) if paged else 0
        d = BitNetDecoder(cfg, w, batch=per, num_pages=npages, page_seed=i if paged else None, kv_dtype=kv)
        if paged:
            for b in range(per):
                d.reserve(b, int(c[b]) + total + 1)
        d.fill_kv_random(int(c.max()), seed=1 + i)
        d.set_state([1] * per, [int(x) for x in c])
        decs.append(d)
        streams.append(torch.cuda.Stream())
    torch.cuda.synchronize()

    def step():
        for d, s in zip(decs, streams):
            with torch.cuda.stream(s):
                d.step(graph=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"batch": B, "micro_batches": nmb, "kv": kv, "ms_per_step": round(1000 * el / steps, 4),
           "tokens_per_s": round(B * steps / el, 1)}
    del decs
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx-dist", choices=["fixed", "uniform"], default="fixed")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--kv", choices=["bf16", "fp8"], default="bf16")
    ap.add_argument("--mb", default="1,2,4")
    a = ap.parse_args()
    cfg = BITNET_2B
    B = 128
    total = a.steps + a.warmup
    if a.ctx_dist == "uniform":
        ctxs = np.random.default_rng(0).integers(1, cfg.max_seq - total - 1, size=B)
    else:
        ctxs = np.full(B, 1024, dtype=np.int64)
    w = synthetic_weights(cfg, seed=0, device="cuda")
    for nmb in [int(x) for x in a.mb.split(",")]:
        r = run(w, cfg, B, nmb, ctxs, a.steps, a.warmup, a.kv)
        r["ctx_dist"] = a.ctx_dist
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
