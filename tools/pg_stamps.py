#!/usr/bin/env python3
"""In-kernel timeline of the prefill GEMM main loop (diagnostic stamps build): per block, stamps at
stages 8 and 9 of pgemm_tile (before the DMA wait, after it, after the barrier, after the DMA issue +
fragment reads, after the MFMA issue) and at kernel entry / main-loop end. Prints medians over
blocks of each interval (us), per wave 0..3.

    python tools/pg_stamps.py [--n 13824] [--k 2560] [--m 16384]
"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "wrinklefree-inference-engine_amd"
os.environ["WF_BITNET_LIB"] = str(PKG / "lib" / os.environ.get("WF_STAMPS_LIB", "libwfbitnet_stamps.so"))
sys.path.insert(0, str(PKG / "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from wfamd import _lib, ops  # noqa: E402

SLOTS, NBLK = 80, 16384


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=13824)
    ap.add_argument("--k", type=int, default=2560)
    args = ap.parse_args()
    lib = _lib.load()
    fn = lib.wf_debug_stamps_mfma
    fn.restype, fn.argtypes = C.c_int, [C.c_void_p, C.c_int, C.c_int]
    M, N, K = args.m, args.n, args.k
    g = torch.Generator(device="cuda").manual_seed(0)
    w = torch.randint(0, 255, (N, K // 4), dtype=torch.uint8, device="cuda", generator=g)
    wt = ops.i2s_to_mfma(w) if hasattr(ops, "i2s_to_mfma") else w
    a = ops.codes_to_tiles(torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda", generator=g))
    for rep in range(3):
        assert fn(None, 0, 1) == 0
        torch.cuda.synchronize()
        y = ops.bitnet_gemm_tiled(wt, a, 1.0, M)
        torch.cuda.synchronize()
    buf = np.zeros(NBLK * SLOTS, dtype=np.uint64)
    assert fn(C.c_void_p(buf.ctypes.data), buf.size, 0) == 0
    st = buf.reshape(NBLK, SLOTS).astype(np.int64)
    live = st[:, 0] > 0
    st = st[live]
    print("blocks", int(live.sum()))
    t0 = st[:, 0].min()
    for w in range(4):  # waves 0..3, or 0, 2, 4, 6 with the WF_STAMPS_EVEN build
        col = lambda i: st[:, 16 * w + i]
        names = ["wait", "barrier", "issue+read", "mma-issue", "->next"]
        out = []
        for c in range(2):
            base = 1 + 5 * c
            for i in range(4):
                d = (col(base + i + 1) - col(base + i)) * 0.01
                out.append(f"{names[i]}{c}={np.median(d):.3f}")
            if c == 0:
                out.append(f"->next={np.median((col(6) - col(5)) * 0.01):.3f}")
        life = (st[:, 11] - st[:, 0]) * 0.01 if w == 0 else None
        print(f"wave {w}:", " ".join(out), "" if life is None else f"life={np.median(life):.2f}us")
    print("kernel span us", (st[:, 11].max() - t0) * 0.01)
    # shader clock over the block's life (wave 0 records s_memtime in column 64 + slot)
    ok = (st[:, 64] > 0) & (st[:, 64 + 11] > 0)
    clk = (st[ok, 64 + 11] - st[ok, 64]) / np.maximum(st[ok, 11] - st[ok, 0], 1) * 100.0  # MHz
    print("shader clock MHz median", float(np.median(clk)), "p10", float(np.percentile(clk, 10)), "p90", float(np.percentile(clk, 90)))


if __name__ == "__main__":
    main()
