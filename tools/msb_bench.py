#!/usr/bin/env python3
"""Micro-benchmark of the SGLang BitNet linear method on the GPU: the direct 2-bit
kernel (wf_msb_linear) vs the reference's algorithm on the device (cached dequantised bf16 matrix +
library GEMM). Cycles through enough distinct weight buffers (>= 1 GB) that the weights come from
HBM, not the 256 MB Infinity Cache (SURVEY §8d cache hygiene). Prints one JSON line per shape."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402

from wfamd import ops  # noqa: E402


def timed(fn, iters):
    """Average device time per call: `iters` calls captured into one HIP graph (no host launch gaps),
    replayed after a warm-up replay."""
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    torch.cuda.set_device(0)
    for (n, k) in ((2560, 2560), (6912, 2560), (2560, 6912), (4096, 4096), (11008, 4096), (4096, 11008)):
        nbuf = max(2, int(1.2e9 // (n * k // 4)))
        ws = [torch.randint(0, 256, (n, k // 4), dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
        for m in (1, 4, 16):
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            us = timed(lambda i: ops.msb_linear(ws[i % nbuf], 1.0, x, n, k), 100)
            byts = n * k // 4 + m * k * 2 + m * n * 2
            wd = ops.msb_dequant(ws[0], 1.0, n, k, torch.bfloat16)
            nb2 = max(2, int(1.2e9 // (n * k * 2)))
            wds = [wd.clone() for _ in range(nb2)]
            us_ref = timed(lambda i: torch.matmul(x, wds[i % nb2].T), 50)
            del wds
            print(json.dumps({"n": n, "k": k, "m": m, "direct_us": round(us, 2), "direct_gbs": round(byts / us / 1e3, 1),
                              "frac_8tbs": round(byts / us / 1e3 / 8000, 3), "bf16_gemm_us": round(us_ref, 2)}),
                  flush=True)
        del ws


if __name__ == "__main__":
    main()
