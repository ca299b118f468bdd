#!/usr/bin/env python3
"""Batch-1 decode ops with cold vs hot weights: each op's 30 launches captured in a HIP graph, once
over layers 0..29 (distinct weights: HBM-cold, the in-step case) and once as layer 0 thirty times
(the same 2.5-8.9 MB re-read: L2 / Infinity-Cache hot). The gap bounds what any cross-launch weight
prefetch could buy per op. Median of 5 replays, µs per launch.

    python tools/hot_cold_b1.py [--ctx 1024]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402

from wfamd import _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    args = ap.parse_args()
    cfg = BITNET_2B
    dec = BitNetDecoder(cfg, synthetic_weights(cfg, seed=0, device="cuda"), batch=1)
    dec.fill_kv_random(args.ctx, seed=1)
    dec.set_state([1], [args.ctx])
    for _ in range(5):
        dec.step(graph=True)
    ops = [(_lib.WF_OP_QKV, "qkv"), (_lib.WF_OP_ATTN, "attn"), (_lib.WF_OP_O, "o_proj"),
           (_lib.WF_OP_GATE_UP, "gate_up"), (_lib.WF_OP_DOWN, "down")]
    st = torch.cuda.current_stream()
    out = {}
    for op, name in ops:
        res = {}
        for kind, layers in (("cold", list(range(cfg.layers))), ("hot", [0] * cfg.layers)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for l in layers:
                    dec.launch_op(l, op)
            ts = []
            for _ in range(5):
                dec.step(graph=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                g.replay()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(1000.0 * e0.elapsed_time(e1) / len(layers))
            res[kind] = round(sorted(ts)[2], 3)
        out[name] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
