#!/usr/bin/env python3
"""In-kernel latency breakdown of the decode ops (diagnostic build lib/libwfbitnet_stamps.so, made
with `make -C wrinklefree-inference-engine_amd stamps`). Thread 0 of every block records the
100 MHz wall clock at named points (WF_STAMP in csrc/); this tool launches one op of one layer after
an Infinity-Cache flush and prints, per stamp slot, min / median / max over blocks relative to the
first block's entry, plus the timeline of one block that reached the launch's last stage.

    python tools/stamps.py [--ctx 1024] [--wfmt tq|i2s] [--flags 0] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "wrinklefree-inference-engine_amd"
os.environ["WF_BITNET_LIB"] = str(PKG / "lib" / "libwfbitnet_stamps.so")
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(PKG / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wfamd import WF_FMT_I2S, WF_FMT_TQ, _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402

SLOTS, NBLK = 80, 16384  # wave 0 uses columns 0..15 (wf_norm.h)
NAMES = {  # slot names per kernel kind (WF_STAMP(i) in csrc/)
    "gemv": ["entry", "image", "dot", "out", "-", "-", "-", "qkv_out", "p_ss", "p_r", "p_y", "p_sf", "p_q", "w_landed",
             "-", "-"],
    "attn": ["entry", "kv_done", "out", "-", "-", "-", "-", "-"] + ["-"] * 8,
    "lm": ["entry", "staged", "dot", "ticket", "argmax", "-", "-", "-"] + ["-"] * 8,
    "dgemm": ["entry", "issued", "first_mma", "loop_done", "reduced", "epi_issued", "epi_drained"] + ["-"] * 9,
}


def read(lib, fn, nblocks):
    buf = np.zeros(nblocks * SLOTS, dtype=np.uint64)
    rc = getattr(lib, fn)(C.c_void_p(buf.ctypes.data), C.c_int(buf.size), C.c_int(0))
    assert rc == 0, rc
    return buf.reshape(nblocks, SLOTS)


def reset(lib):
    for fn in ("wf_debug_stamps_decode", "wf_debug_stamps_attn"):
        assert getattr(lib, fn)(None, 0, 1) == 0


def summarize(st, kind, tail_slot):
    """st: [NBLK, SLOTS]; block (x, y, z) of a launch sits in row x + 2048 y + 8192 z (wf_norm.h)."""
    live = st[:, 0] > 0
    st = st[live].astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 0.01  # 100 MHz -> us
    out = {"blocks": int(live.sum())}
    for s, name in enumerate(NAMES[kind][:16]):
        if name == "-":
            continue
        col = rel[st[:, s] > 0, s]
        if col.size:
            out[name] = [round(float(col.min()), 2), round(float(np.median(col)), 2), round(float(col.max()), 2),
                         int(col.size)]
    # per-block durations: median over blocks of (slot - own entry)
    for sl, name in enumerate(NAMES[kind][:16]):
        if name == "-" or sl == 0:
            continue
        ok = st[:, sl] > 0
        if ok.any():
            out.setdefault("block_dur", {})[name] = round(float(np.median((st[ok, sl] - st[ok, 0]) * 0.01)), 2)
    tails = np.nonzero(st[:, tail_slot] > 0)[0]
    if tails.size:
        i = tails[0]
        out["tail_block"] = {NAMES[kind][s]: round(float(rel[i, s]), 2) for s in range(16)
                             if st[i, s] > 0 and NAMES[kind][s] != "-"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--wfmt", choices=["tq", "i2s"], default="tq")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--layer", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--warm", action="store_true",
                    help="launch the same op of layer-1 right before (code and inputs warm, weights cold)")
    ap.add_argument("--hot", action="store_true",
                    help="launch the same op of the SAME layer right before (weights in L2 / Infinity Cache)")
    args = ap.parse_args()
    lib = _lib.load()
    for fn in ("wf_debug_stamps_decode", "wf_debug_stamps_attn"):
        getattr(lib, fn).restype = C.c_int
        getattr(lib, fn).argtypes = [C.c_void_p, C.c_int, C.c_int]
    w = synthetic_weights(BITNET_2B, seed=0)
    B = args.batch
    dec = BitNetDecoder(BITNET_2B, w, batch=B, wfmt=WF_FMT_TQ if args.wfmt == "tq" else WF_FMT_I2S,
                        debug_flags=args.flags)
    del w
    dec.fill_kv_random(args.ctx)
    dec.set_state([1] * B, [args.ctx] * B)
    for _ in range(3):
        dec.step(graph=False)
    torch.cuda.synchronize()
    flush = torch.empty(384 << 20, dtype=torch.uint8, device="cuda")
    ops = [(_lib.WF_OP_QKV, "qkv", "gemv", "decode", 7), (_lib.WF_OP_ATTN, "attn", "attn", "attn", 2),
           (_lib.WF_OP_O, "o_proj", "gemv", "decode", 3), (_lib.WF_OP_GATE_UP, "gate_up", "gemv", "decode", 3),
           (_lib.WF_OP_DOWN, "down", "gemv", "decode", 3), (_lib.WF_OP_LM_HEAD, "lm_head", "lm", "decode", 4)]
    if B >= 16:  # batched matrix-core path: GEMM stamps (slots 0-6), attention as before
        ops = [(_lib.WF_OP_QKV, "qkv", "dgemm", "decode", 6), (_lib.WF_OP_ATTN, "attn", "attn", "attn", 2),
               (_lib.WF_OP_O, "o_proj", "dgemm", "decode", 6), (_lib.WF_OP_GATE_UP, "gate_up", "dgemm", "decode", 6),
               (_lib.WF_OP_DOWN, "down", "dgemm", "decode", 6)]
    res = {}
    for op, name, kind, tu, tail in ops:
        for rep in range(args.reps):
            flush.fill_(rep + 1)
            torch.cuda.synchronize()
            reset(lib)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if args.warm:
                dec.launch_op(args.layer - 1, op)
            if args.hot:
                dec.launch_op(args.layer, op)
            e0.record()
            dec.launch_op(args.layer, op)
            e1.record()
            torch.cuda.synchronize()
            st = read(lib, f"wf_debug_stamps_{tu}", NBLK)
            s = summarize(st, kind, tail)
            s["event_us"] = round(1000 * e0.elapsed_time(e1), 2)
            res.setdefault(name, []).append(s)
        print(name, json.dumps(res[name][-1]), flush=True)
    out = ROOT / "gpurun_out" / "stamps.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
