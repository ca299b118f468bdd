#!/usr/bin/env python3
"""Does the batched decode GEMM wait on its weight bytes? (the measured reason behind keeping I2_S,
not the ~1.6-bit TQ format, on the batch >= 16 path).

For each GEMM op of the batch-B decode step (B = 128 by default), the per-launch time of
  cold: one launch per layer, 30 distinct weight sets (the step's own cadence: weights from HBM), and
  hot : 30 launches of layer 0 (its 2.5-8.8 MB of weights stay in the XCD L2s / Infinity Cache),
each replayed from a HIP graph after a full decode step (bench.py op_timing). If hot ~= cold the
kernel is not bound by its weight stream, so a 20 % smaller weight format cannot make it faster
and TQ's base-3 digit extraction (about twice the I2_S decode VALU per code) can only cost.

    python tools/weight_bytes_study.py [--batch 128] [--ctx 1024]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402

from wfamd import _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402


def timed(dec, layers, op, reps=5):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for l in layers:
            dec.launch_op(l, op)
    st = torch.cuda.current_stream()
    out = []
    for _ in range(reps):
        dec.step(graph=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        out.append(1000.0 * e0.elapsed_time(e1) / len(layers))
    return sorted(out)[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=1024)
    args = ap.parse_args()
    w = synthetic_weights(BITNET_2B, seed=0)
    dec = BitNetDecoder(BITNET_2B, w, batch=args.batch)
    del w
    dec.fill_kv_random(args.ctx, seed=1)
    dec.set_state([1] * args.batch, [args.ctx] * args.batch)
    for _ in range(3):
        dec.step(graph=True)
    L = BITNET_2B.layers
    res = {}
    for op, name in ((_lib.WF_OP_QKV, "qkv"), (_lib.WF_OP_O, "o_proj"), (_lib.WF_OP_GATE_UP, "gate_up"),
                     (_lib.WF_OP_DOWN, "down")):
        cold = timed(dec, list(range(L)), op)
        hot = timed(dec, [0] * L, op)
        wb = {"qkv": dec.w_qkv, "o_proj": dec.w_o, "gate_up": dec.w_gu, "down": dec.w_d}[name][0].numel()
        res[name] = {"cold_us": round(cold, 3), "hot_us": round(hot, 3), "weight_bytes": wb,
                     "cold_weight_tbs": round(wb / cold / 1e6, 3), "hot_over_cold": round(hot / cold, 3)}
    print(json.dumps({"batch": args.batch, "ctx": args.ctx, "ops": res}))


if __name__ == "__main__":
    main()
