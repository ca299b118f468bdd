#!/usr/bin/env python3
"""In-kernel timeline of the batch-1 fused QKV + attention launch (k_qkv_attn; diagnostic build
lib/libwfbitnet_stamps.so from `make -C wrinklefree-inference-engine_amd stamps`). Runs whole decode
steps (graph replay) so the launch sees its in-step cache state, then one more step with stamps
reset and reads the last layer's QKV launch: per stamp, min / median / max over blocks in µs
relative to the launch's first block entry.

    python tools/stamps_qkv_attn.py [--ctx 1024]
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "wrinklefree-inference-engine_amd"
os.environ["WF_BITNET_LIB"] = str(PKG / "lib" / os.environ.get("WF_STAMPS_LIB", "libwfbitnet_stamps.so"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(PKG / "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wfamd import _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402

SLOTS, NBLK = 80, 16384
QKV = {0: "entry", 1: "image", 2: "dot", 14: "published"}
ATT = {0: "entry", 8: "kv_issued", 9: "poll_passed", 10: "q_landed", 11: "keys_done", 15: "wave_merged",
       13: "merge_barrier", 12: "records"}
WAVE_SLOTS = (0, 8, 10, 11, 15, 13)  # also shown for waves 1..3 (stamp columns 16 w + slot)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    cfg = BITNET_2B
    dec = BitNetDecoder(cfg, synthetic_weights(cfg, seed=0, device="cuda"), batch=1)
    dec.fill_kv_random(args.ctx, seed=1)
    dec.set_state([1], [args.ctx])
    lib = _lib.load()
    nq = (cfg.n_heads + 2 * cfg.n_kv_heads) * cfg.head_dim // 16
    na = cfg.n_heads * 8
    for rep in range(args.reps):
        for _ in range(3):
            dec.step(graph=True)
        torch.cuda.synchronize()
        assert lib.wf_debug_stamps_decode(None, 0, 1) == 0
        dec.step(graph=False)  # eager: the last layer's launch leaves its stamps (rows 0 .. nq + na)
        torch.cuda.synchronize()
        buf = np.zeros(NBLK * SLOTS, dtype=np.uint64)
        assert lib.wf_debug_stamps_decode(C.c_void_p(buf.ctypes.data), C.c_int(buf.size), C.c_int(0)) == 0
        st = buf.reshape(NBLK, SLOTS)[: nq + na].astype(np.int64)
        t0 = st[:, 0].min()
        print(f"rep {rep}: qkv blocks {nq}, attention blocks {na}")
        for rows, names, tag in ((st[:nq], QKV, "qkv "), (st[nq:], ATT, "attn")):
            for slot, name in names.items():
                v = rows[:, slot]
                v = (v[v > 0] - t0) * 0.01
                if v.size:
                    print(f"  {tag} {name:12s} min {v.min():6.2f}  med {np.median(v):6.2f}  max {v.max():6.2f}  (n {v.size})")
                if tag == "attn" and slot in WAVE_SLOTS:
                    for w in (1, 2, 3):
                        vw = rows[:, 16 * w + slot]
                        vw = (vw[vw > 0] - t0) * 0.01
                        if vw.size:
                            print(f"       wave {w} {name:12s} med {np.median(vw):6.2f}  max {vw.max():6.2f}")


if __name__ == "__main__":
    main()
