#!/usr/bin/env python3
"""Per-wave view of the stamp build (tools/stamps.py layout: 80 words per block = 4 waves x 16
realtime slots + 16 shader-clock slots of wave 0). Launches one op of one layer after the same op
of the previous layer (code warm, weights cold) and prints, for a few blocks, each wave's slot
times (us from the block's first entry) and the shader clock of wave 0 between two slots."""
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

from wfamd import WF_FMT_TQ, _lib  # noqa: E402
from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights  # noqa: E402

W = 80
NAMES = ["entry", "image", "dot", "out", "4", "5", "6", "qkv_out", "p_ss", "p_r", "p_y", "p_sf", "p_q", "w_landed",
         "14", "15"]


def main():
    lib = _lib.load()
    fn = lib.wf_debug_stamps_decode
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int, C.c_int]
    w = synthetic_weights(BITNET_2B, seed=0)
    dec = BitNetDecoder(BITNET_2B, w, batch=1, wfmt=WF_FMT_TQ)
    del w
    dec.fill_kv_random(1024)
    dec.set_state([1], [1024])
    for _ in range(3):
        dec.step(graph=False)
    torch.cuda.synchronize()
    flush = torch.empty(384 << 20, dtype=torch.uint8, device="cuda")
    out = {}
    for op, name in ((_lib.WF_OP_O, "o_proj"), (_lib.WF_OP_DOWN, "down")):
        flush.fill_(3)
        torch.cuda.synchronize()
        assert fn(None, 0, 1) == 0
        torch.cuda.synchronize()
        dec.launch_op(4, op)
        dec.launch_op(5, op)
        torch.cuda.synchronize()
        buf = np.zeros(16384 * W, dtype=np.uint64)
        assert fn(C.c_void_p(buf.ctypes.data), buf.size, 0) == 0
        st = buf.reshape(16384, W).astype(np.int64)
        live = np.nonzero(st[:, 0])[0]
        res = []
        for b in live[:: max(1, len(live) // 4)][:4]:
            t0 = min(st[b, 16 * wv] for wv in range(4) if st[b, 16 * wv])
            waves = {}
            for wv in range(4):
                row = {NAMES[i]: round((st[b, 16 * wv + i] - t0) * 0.01, 2) for i in range(16) if st[b, 16 * wv + i]}
                waves[f"w{wv}"] = row
            clk = {}
            i0, i1 = 0, 3  # entry -> out on wave 0
            if st[b, 64 + i0] and st[b, 64 + i1] and st[b, i1] > st[b, i0]:
                clk["mhz"] = round((st[b, 64 + i1] - st[b, 64 + i0]) / ((st[b, i1] - st[b, i0]) * 0.01), 1)
            res.append({"block": int(b), **waves, **clk})
        out[name] = res
        for r in res:
            print(name, json.dumps(r), flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "stamps_waves.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
