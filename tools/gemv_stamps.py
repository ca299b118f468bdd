#!/usr/bin/env python3
"""Kernel-only duration of the standalone GEMV (sgl_kernel bitnet_gemv, wf_bitnet_gemv) from in-kernel
wall-clock stamps (diagnostic build lib/libwfbitnet_stamps.so, `make stamps`): for each of the
reference's benchmark shapes (scripts/benchmark_kernels.py:132-138, plus k/v) the graph of bench.py's
gemv_bench (cold weights rotating through >= 1.2 GB) is replayed, and the LAST launch's first block
entry -> last block exit (s_memrealtime, 100 MHz) is its duration: no launch gap, no profiler in the
way (rocprofv3's per-dispatch durations of these ~1-3 us kernels read 1-2 us high, see
profiles/README.md). GB/s = (N K / 4 + K + 4 N) / duration.

    python tools/gemv_stamps.py [--reps 7]
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
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import GEMV_SHAPES  # noqa: E402
from wfamd import _lib  # noqa: E402

SLOTS, NBLK = 80, 16384


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    lib = _lib.load()
    rd = lib.wf_debug_stamps_gemv
    rd.restype, rd.argtypes = C.c_int, [C.c_void_p, C.c_int, C.c_int]
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {}
    for name, N, K in GEMV_SHAPES:
        wb = N * K // 4
        nbuf = max(8, int(1.2e9 // wb) + 1)
        w = torch.randint(0, 255, (nbuf, N, K // 4), dtype=torch.uint8, device="cuda", generator=g)
        w &= 0xAA
        a = torch.randint(-128, 128, (K,), dtype=torch.int8, device="cuda", generator=g)
        y = torch.empty(N, dtype=torch.float32, device="cuda")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cs = torch.cuda.current_stream().cuda_stream
            for i in range(nbuf):
                _lib.check(lib.wf_bitnet_gemv(w[i].data_ptr(), a.data_ptr(), 0.01, N, K, y.data_ptr(), cs), "gemv")
        graph.replay()
        spans = []
        nblk = (N + 3) // 4  # an upper bound of the launch's blocks (4-16 rows per block)
        for _ in range(args.reps):
            assert rd(None, 0, 1) == 0
            torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            buf = np.zeros(NBLK * SLOTS, dtype=np.uint64)
            assert rd(C.c_void_p(buf.ctypes.data), buf.size, 0) == 0
            s = buf.reshape(NBLK, SLOTS).astype(np.int64)[:nblk]
            ent = s[:, 0][s[:, 0] > 0]
            ex = np.concatenate([s[:, 16 * wv + 1][s[:, 16 * wv + 1] > 0] for wv in range(4)])
            spans.append((ex.max() - ent.min()) * 0.01)
        us = float(np.median(spans))
        nbytes = wb + K + 4 * N
        out[name] = {"N": N, "K": K, "kernel_us": round(us, 3), "gbs": round(nbytes / us / 1e3, 1),
                     "spans_us": [round(x, 2) for x in spans]}
        print(name, json.dumps(out[name]), flush=True)
        del w, graph
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
