#!/usr/bin/env python3
"""Ablation timing of the decode ops on the full 2B model: production kernels vs builds without the
int8 activation staging (flag 1), without weight loads (flag 2), without the producer tail
(ticket + next-op norm, flag 4) or with the ticket but no norm (flag 8). Event-timed per op (30 layers
back to back after an Infinity-Cache flush), like bench.py. Results of flagged runs are garbage."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402

import bench  # noqa: E402
from wfamd import WF_FMT_I2S, WF_FMT_TQ  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402


def main():
    ctx = 1024
    w = synthetic_weights(BITNET_2B, seed=0)
    res = {}
    for fmt_name, fmt in (("tq", WF_FMT_TQ), ("i2s", WF_FMT_I2S)):
        for flags in (0, 1, 2, 4, 8, 5):
            if fmt == WF_FMT_I2S and flags:
                continue
            dec = BitNetDecoder(BITNET_2B, w, batch=1, wfmt=fmt, debug_flags=flags)
            dec.fill_kv_random(ctx)
            dec.set_state([1], [ctx])
            for _ in range(3):
                dec.step(graph=False)
            torch.cuda.synchronize()
            t = bench.op_timing(dec, ctx)
            res[f"{fmt_name}_flags{flags}"] = {k: v["us"] for k, v in t.items()}
            print(fmt_name, flags, json.dumps(res[f"{fmt_name}_flags{flags}"]), flush=True)
            del dec
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
