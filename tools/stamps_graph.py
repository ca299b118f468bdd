#!/usr/bin/env python3
"""In-graph latency timeline of one batch-1 decode layer (diagnostic build lib/libwfbitnet_stamps.so,
`make -C wrinklefree-inference-engine_amd stamps`). The whole decode step is replayed as its HIP graph
(warm clocks, warm code, the real inter-kernel gaps); every GEMV op stamps into its own region
(WF_STAMP_BASE), so after a replay the buffers hold the LAST layer's QKV / O / GU / DN, the attention
(its own translation unit) and the LM head. Prints, per op, the first / median block entry and the
median / last block exit on one 100 MHz clock (relative to the QKV's first entry), the gaps between
ops, per-stamp medians relative to each block's entry, and the shader clock (s_memtime / s_memrealtime).

    python tools/stamps_graph.py [--ctx 1024] [--reps 20] [--batch 128]

At batch > 1 the ops are the row norms (k_rownorm: ln_in and ln_post share a region, so the
ln_post one is shown; k_rownorm_attn), the k_dec_gemm_t GEMMs and k_attn_mfma.
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "wrinklefree-inference-engine_amd"
os.environ["WF_BITNET_LIB"] = os.environ.get("WF_STAMPS_LIB", str(PKG / "lib" / "libwfbitnet_stamps.so"))
sys.path.insert(0, str(PKG / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wfamd import _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402

SLOTS, NBLK = 80, 16384
GEMV_NAMES = {0: "entry", 1: "image", 2: "dot", 3: "out", 7: "qkv_out", 8: "p_ss", 9: "p_r", 10: "p_y", 11: "p_sf",
              12: "p_q", 13: "w_landed"}
ATTN_NAMES = {0: "entry", 1: "qk_done", 2: "exchanged", 3: "records", 4: "merged"}
LM_NAMES = {0: "entry", 1: "staged", 2: "dot", 3: "ticket", 4: "argmax"}
GEMM_NAMES = {0: "entry", 14: "norm_published", 15: "rows_ready", 1: "issued", 2: "first_mma", 3: "mma_done",
              4: "combined", 5: "epilogue"}
RN_NAMES = {0: "entry", 1: "normed", 2: "done"}


def read(lib, fn):
    buf = np.zeros(NBLK * SLOTS, dtype=np.uint64)
    assert getattr(lib, fn)(C.c_void_p(buf.ctypes.data), C.c_int(buf.size), C.c_int(0)) == 0
    return buf.reshape(NBLK, SLOTS).astype(np.int64)


def op_summary(rows, names, last_slot, t0):
    live = rows[rows[:, 0] > 0]
    ent = (live[:, 0] - t0) * 0.01
    ex = (live[:, last_slot] - t0) * 0.01
    out = {"blocks": int(len(live)), "entry_first": round(float(ent.min()), 2),
           "entry_med": round(float(np.median(ent)), 2), "exit_med": round(float(np.median(ex)), 2),
           "exit_last": round(float(ex.max()), 2)}
    per, foreign = {}, {}
    for sl, nm in names.items():
        # a stamp counts only inside its own block's window [entry, exit + 20 us]: a slot another launch
        # wrote (an earlier layer's op of the same region, a kernel that skips the stamp) is
        # reported as foreign, not folded into the medians
        ok = (live[:, sl] > 0) & (live[:, sl] >= live[:, 0]) & (live[:, sl] <= live[:, last_slot] + 2000)
        bad = int(((live[:, sl] > 0) & ~ok).sum())
        if sl and ok.any():
            per[nm] = round(float(np.median((live[ok, sl] - live[ok, 0]) * 0.01)), 2)
        if sl and bad:
            foreign[nm] = bad
    out["per_block_med"] = per
    if foreign:
        out["foreign_stamps"] = foreign
    ok = (live[:, 64] > 0) & (live[:, 64 + last_slot] > 0)
    if ok.any():
        dt = (live[ok, last_slot] - live[ok, 0]).astype(np.float64)
        dc = (live[ok, 64 + last_slot] - live[ok, 64]).astype(np.float64)
        good = dt > 0
        if good.any():
            out["clock_mhz"] = round(float(np.median(dc[good] / dt[good] * 100.0)), 0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1)
    args = ap.parse_args()
    lib = _lib.load()
    for fn in ("wf_debug_stamps_decode", "wf_debug_stamps_attn"):
        getattr(lib, fn).restype = C.c_int
        getattr(lib, fn).argtypes = [C.c_void_p, C.c_int, C.c_int]
    w = synthetic_weights(BITNET_2B, seed=0)
    B = args.batch
    dec = BitNetDecoder(BITNET_2B, w, batch=B)
    del w
    dec.fill_kv_random(args.ctx)
    dec.set_state([1 + b for b in range(B)], [args.ctx] * B)
    for _ in range(args.reps):
        dec.step(graph=True)
    torch.cuda.synchronize()
    for fn in ("wf_debug_stamps_decode", "wf_debug_stamps_attn"):
        assert getattr(lib, fn)(None, 0, 1) == 0
    torch.cuda.synchronize()
    for _ in range(3):
        dec.step(graph=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    dec.step(graph=True)
    e1.record()
    torch.cuda.synchronize()
    dc, at = read(lib, "wf_debug_stamps_decode"), read(lib, "wf_debug_stamps_attn")
    if B == 1:
        order = ("qkv", "attn", "o_proj", "gate_up", "down", "lm_head")
        ops = {"qkv": (dc[0:512], GEMV_NAMES, 7), "attn": (at[0:2048], ATTN_NAMES, 4),
               "o_proj": (dc[512:1024], GEMV_NAMES, 3), "gate_up": (dc[1024:1536], GEMV_NAMES, 3),
               "down": (dc[1536:2048], GEMV_NAMES, 3), "lm_head": (dc[4096:4096 + 8016], LM_NAMES, 3)}
    else:
        order = ("qkv", "attn", "rn_attn", "o_proj", "rn_post", "gate_up", "rn_ffn", "down")
        ops = {"qkv": (dc[0:512], GEMM_NAMES, 5), "attn": (at[0:16384], ATTN_NAMES, 2),
               "rn_attn": (dc[2560:2560 + B], RN_NAMES, 2), "o_proj": (dc[512:1024], GEMM_NAMES, 5),
               "rn_post": (dc[2048:2048 + B], RN_NAMES, 2), "gate_up": (dc[1024:1536], GEMM_NAMES, 5),
               "rn_ffn": (dc[2304:2304 + B], RN_NAMES, 2), "down": (dc[1536:2048], GEMM_NAMES, 5)}
    t0 = dc[0:512][dc[0:512, 0] > 0, 0].min()
    res = {name: op_summary(r, nm, ls, t0) for name, (r, nm, ls) in ops.items() if (r[:, 0] > 0).any()}
    order = [n for n in order if n in res]  # batch > 1 with the norm fused into the GEMMs: no k_rownorm
    prev = None
    for name in order:
        if prev:
            res[name]["gap_from_prev_last_exit"] = round(res[name]["entry_first"] - res[prev]["exit_last"], 2)
        prev = name
    res["step_ms"] = round(e0.elapsed_time(e1), 4)
    # per-block timeline of the attention (block index, then each named stamp in us from t0)
    ar = ops["attn"][0]
    live = np.nonzero(ar[:, 0] > 0)[0]
    raw = [[int(i)] + [round(float((ar[i, sl] - t0) * 0.01), 2) if ar[i, sl] > 0 else None for sl in ATTN_NAMES]
           for i in live]
    for k, v in res.items():
        print(k, json.dumps(v), flush=True)
    out = ROOT / "gpurun_out" / f"stamps_graph_b{B}.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))
    (out.parent / f"stamps_graph_b{B}_attn_raw.json").write_text(json.dumps(raw))
    if B == 1:  # per-block LM head stamps (entry, staged, dot, ticket, argmax), us from t0
        lr = ops["lm_head"][0]
        lraw = [[int(i)] + [round(float((lr[i, sl] - t0) * 0.01), 2) if lr[i, sl] > 0 else None for sl in LM_NAMES]
                for i in np.nonzero(lr[:, 0] > 0)[0]]
        (out.parent / f"stamps_graph_b{B}_lm_raw.json").write_text(json.dumps(lraw))


if __name__ == "__main__":
    main()
