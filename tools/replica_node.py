#!/usr/bin/env python3
"""Node launcher of independent bitnet-b1.58-2B-4T replicas (BASELINE configs[4]; SURVEY §8d
config 5: "8 processes, HIP_VISIBLE_DEVICES=i, running configs 2 and 4 concurrently").

    python tools/replica_node.py [--replicas 8] [--workload mixed|b1|b128u] [--steps 1000]
                                 [--same-gpu] [--layers 30] [--seed 0] [--verify]

Process i sees GPU i only (HIP_VISIBLE_DEVICES=i), pins itself to a disjoint slice of the host
cores before its first GPU call (wfamd.replicas.pin_host_cores; the reference pins its server to 8
cores, scripts/launch_sglang_bitnet.sh:61-67) and runs its own decoder(s): no collective, no RCCL
communicator, nothing shared. Workloads per replica:
  b1    : decode batch 1 at context 1024 (configs[1] / SURVEY config 2),
  b128u : decode batch 128, contexts U[1, 4096 - steps) seed 0, paged KV (configs[3] / config 4),
  mixed : both at once on two HIP streams of the same GPU (a server with an interactive stream
          beside a full continuous batch) -- SURVEY config 5.
The replicas start their timed windows together: a gloo barrier on the host (127.0.0.1 rendezvous
set up by wfamd.replicas.launch) brackets the window, so the windows overlap and the summed rate is a
concurrent node rate; each replica also reports its wall-clock window and the parent reports the
union of the windows and the node rate over it (total tokens / union).
The parent prints one JSON line: node totals (sum over replicas) and the per-replica spread.
--same-gpu runs every replica on GPU 0 (a functional check on a one-GPU box; not a node number).
--verify: each replica also records its greedy tokens of every step and a sha256 of its final
logits (replica i runs weights seed --seed + i, so a solo run with the same seed must agree).
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
    ap.add_argument("--steps", type=int, default=1000,
                    help="timed iterations: one batch-128 step (mixed: plus 4 batch-1 steps) each")
    ap.add_argument("--same-gpu", action="store_true")
    ap.add_argument("--layers", type=int, default=30)
    ap.add_argument("--seed", type=int, default=0, help="replica i uses synthetic weights seed --seed + i")
    ap.add_argument("--ctx", type=int, default=1024, help="batch-1 context")
    ap.add_argument("--verify", action="store_true", help="record greedy tokens and a logits hash")
    return ap.parse_args()


def child(args):
    cores = pin_host_cores(args.replica, args.replicas)  # before any GPU call
    import dataclasses
    import hashlib

    import numpy as np
    import torch
    import torch.distributed as dist
    from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights
    from wfamd.replicas import timed_window
    if args.replicas > 1:  # host-only rendezvous (gloo over 127.0.0.1): no RCCL communicator
        dist.init_process_group("gloo", rank=args.replica, world_size=args.replicas)
    cfg = dataclasses.replace(BITNET_2B, layers=args.layers)
    torch.cuda.set_device(0)
    ratio = 4 if args.workload == "mixed" else 1  # batch-1 steps per batch-128 step (a b128 step ~4x a b1 step)
    max_steps = ratio * (args.steps + 3) + 8
    w = synthetic_weights(cfg, seed=args.seed + args.replica)
    d1 = d128 = None
    if args.workload in ("b1", "mixed"):
        d1 = BitNetDecoder(cfg, w, batch=1)
        d1.fill_kv_random(args.ctx, seed=1)
        d1.set_state([1], [args.ctx])
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
    n_b1 = ratio if d1 else 0
    hist1 = torch.zeros(max(1, (args.steps + 3) * n_b1), dtype=torch.int32, device="cuda") if args.verify else None
    hist128 = torch.zeros(args.steps + 3, 128, dtype=torch.int32, device="cuda") if args.verify else None
    it = [0, 0]

    def one():
        # the host enqueues graph replays; the two streams run concurrently
        if d128:
            with torch.cuda.stream(s2):
                d128.step(graph=True)
                if hist128 is not None:
                    hist128[it[1]].copy_(d128.tokens)
            it[1] += 1
        if d1:
            with torch.cuda.stream(s1):
                for _ in range(n_b1):
                    d1.step(graph=True)
                    if hist1 is not None:
                        hist1[it[0]:it[0] + 1].copy_(d1.tokens)
                    it[0] += 1

    for _ in range(3):  # warm (graph capture)
        one()
    torch.cuda.synchronize()
    tw = timed_window(one, args.steps, torch.cuda.synchronize, dist if args.replicas > 1 else None)
    el = tw["local_s"]  # this replica's own clock: its rate; the node line keeps the max and the union
    n1, n128 = (n_b1 * args.steps if d1 else 0), (args.steps if d128 else 0)
    r = {"replica": args.replica, "cores": len(cores), "core_range": [cores[0], cores[-1]],
         "seed": args.seed + args.replica, "seconds": round(el, 4), "max_seconds": round(tw["max_s"], 4),
         "t_start": tw["t_start"], "t_end": tw["t_end"],
         "b1_steps": n1, "b128_steps": n128,
         "b1_tokens_per_s": round(n1 / el, 2), "b128_tokens_per_s": round(128 * n128 / el, 2)}
    r["tokens_per_s"] = round(r["b1_tokens_per_s"] + r["b128_tokens_per_s"], 2)
    r["tokens"] = n1 + 128 * n128
    if args.verify:
        torch.cuda.synchronize()
        h = hashlib.sha256()
        if d1:
            r["b1_tokens"] = hist1[:it[0]].cpu().tolist()
            h.update(d1.logits.view(torch.int16).cpu().numpy().tobytes())
        if d128:
            r["b128_tokens_sha256"] = hashlib.sha256(hist128[:it[1]].cpu().numpy().tobytes()).hexdigest()
            h.update(d128.logits.view(torch.int16).cpu().numpy().tobytes())
        r["logits_sha256"] = h.hexdigest()
    print(json.dumps(r), flush=True)
    if args.replicas > 1:
        dist.destroy_process_group()


def node_line(args, res) -> dict:
    """Node totals over the replicas' JSON lines. The headline is the whole-job clock of bench.py's
    contract: every token of every replica / the max over replicas of the timed window
    (`max_seconds`, all-reduced by the replicas). Beside it the conservative rate over the union of
    the wall-clock windows (last end - first start), and, as a diagnostic of the spread only, each
    replica's rate on its own clock (summing those would over-count replicas that share a GPU and
    finish at different times)."""
    union = max(r["t_end"] for r in res) - min(r["t_start"] for r in res)
    tokens = sum(r["tokens"] for r in res)
    job_s = max(r["max_seconds"] for r in res)
    return {"workload": f"{args.replicas} independent replicas ({args.workload}; BASELINE configs[4])",
            "same_gpu": args.same_gpu, "node_tokens_per_s": round(tokens / job_s, 2),
            "job_window_s": round(job_s, 4), "tokens": tokens,
            "union_window_s": round(union, 4),
            "node_tokens_per_s_over_union": round(tokens / union, 2),
            "per_replica_local_rates": aggregate(res),
            "b1": aggregate(res, "b1_tokens_per_s") if args.workload != "b128u" else None,
            "b128": aggregate(res, "b128_tokens_per_s") if args.workload != "b1" else None,
            "replicas": res}


def main():
    args = parse()
    if args.replica >= 0:
        child(args)
        return
    argv = [str(Path(__file__).resolve()), "--workload", args.workload, "--steps", str(args.steps),
            "--layers", str(args.layers), "--seed", str(args.seed), "--ctx", str(args.ctx)]
    if args.verify:
        argv.append("--verify")
    res = launch(args.replicas, argv, visible_devices=not args.same_gpu)
    print(json.dumps(node_line(args, res)))


if __name__ == "__main__":
    main()
