#!/usr/bin/env python3
"""Node launcher of independent bitnet-b1.58-2B-4T replicas (BASELINE configs[4]; SURVEY §8d
config 5: "8 processes, HIP_VISIBLE_DEVICES=i, running configs 2 and 4 concurrently").

    python tools/replica_node.py [--replicas 8] [--workload mixed|b1|b128u] [--steps 100]
                                 [--same-gpu]

Process i sees GPU i only (HIP_VISIBLE_DEVICES=i), pins itself to a disjoint slice of the host
cores before its first GPU call (wfamd.replicas.pin_host_cores; the reference pins its server to 8
cores, scripts/launch_sglang_bitnet.sh:61-67) and runs its own decoder(s): no collective, no RCCL
communicator, nothing shared. Workloads per replica:
  b1    : decode batch 1 at context 1024 (configs[1] / SURVEY config 2),
  b128u : decode batch 128, contexts U[1, 4096 - steps) seed 0, paged KV (configs[3] / config 4),
  mixed : both at once on two HIP streams of the same GPU (a server with an interactive stream
          beside a full continuous batch) -- SURVEY config 5.
The parent prints one JSON line: node totals (sum over replicas) and the per-replica spread.
--same-gpu runs every replica on GPU 0 (a functional check on a one-GPU box; not a node number).
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

from wfamd.replicas import aggregate, launch, pin_host_cores  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--replica", type=int, default=-1, help="(internal) run as replica i")
    ap.add_argument("--workload", choices=["mixed", "b1", "b128u"], default="mixed")
    ap.add_argument("--steps", type=int, default=100, help="batch-128 steps (mixed: 4x as many batch-1 steps)")
    ap.add_argument("--same-gpu", action="store_true")
    ap.add_argument("--layers", type=int, default=30)
    return ap.parse_args()


def child(args):
    cores = pin_host_cores(args.replica, args.replicas)  # before any GPU call
    import numpy as np
    import torch
    from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights
    import dataclasses
    cfg = dataclasses.replace(BITNET_2B, layers=args.layers)
    torch.cuda.set_device(0)
    max_steps = 4 * args.steps + 8
    w = synthetic_weights(cfg, seed=args.replica)
    d1 = d128 = None
    if args.workload in ("b1", "mixed"):
        d1 = BitNetDecoder(cfg, w, batch=1)
        d1.fill_kv_random(1024, seed=1)
        d1.set_state([1], [1024])
    if args.workload in ("b128u", "mixed"):
        B = 128
        ctxs = np.random.default_rng(0).integers(1, cfg.max_seq - max_steps - 1, size=B)
        pages = int(sum((c + max_steps + 1 + 31) // 32 for c in ctxs))
        d128 = BitNetDecoder(cfg, w, batch=B, num_pages=pages, page_seed=0)
        for b in range(B):
            d128.reserve(b, int(ctxs[b]) + max_steps + 1)
        d128.fill_kv_random(int(ctxs.max()), seed=1)
        d128.set_state([1] * B, [int(c) for c in ctxs])
    del w
    torch.cuda.empty_cache()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):  # warm (graph capture)
        if d1:
            with torch.cuda.stream(s1):
                d1.step(graph=True)
        if d128:
            with torch.cuda.stream(s2):
                d128.step(graph=True)
    torch.cuda.synchronize()
    # batch-1 steps per batch-128 step so both streams stay busy for the whole window (a b128 step is
    # ~4x a b1 step); the host enqueues graph replays, the two streams run concurrently
    ratio = 4 if (d1 and d128) else 1
    steps = args.steps
    n1 = n128 = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        if d128:
            with torch.cuda.stream(s2):
                d128.step(graph=True)
            n128 += 1
        if d1:
            with torch.cuda.stream(s1):
                for _ in range(ratio):
                    d1.step(graph=True)
            n1 += ratio
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    r = {"replica": args.replica, "cores": len(cores), "core_range": [cores[0], cores[-1]],
         "seconds": round(el, 3), "b1_steps": n1, "b128_steps": n128,
         "b1_tokens_per_s": round(n1 / el, 2), "b128_tokens_per_s": round(128 * n128 / el, 2)}
    r["tokens_per_s"] = round(r["b1_tokens_per_s"] + r["b128_tokens_per_s"], 2)
    print(json.dumps(r), flush=True)


def main():
    args = parse()
    if args.replica >= 0:
        child(args)
        return
    argv = [str(Path(__file__).resolve()), "--workload", args.workload, "--steps", str(args.steps),
            "--layers", str(args.layers)]
    res = launch(args.replicas, argv, visible_devices=not args.same_gpu)
    line = {"workload": f"{args.replicas} independent replicas ({args.workload}; BASELINE configs[4])",
            "same_gpu": args.same_gpu, "node_tokens_per_s": aggregate(res),
            "b1": aggregate(res, "b1_tokens_per_s") if args.workload != "b128u" else None,
            "b128": aggregate(res, "b128_tokens_per_s") if args.workload != "b1" else None,
            "replicas": res}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
