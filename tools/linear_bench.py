#!/usr/bin/env python3
"""BitNetLinear (wf_bitnet_linear: row quantizer + ternary GEMM + correction, bf16 out) at decode-batch
row counts on the 2B shapes, captured in a HIP graph (20 calls per replay), us per call.

    python tools/linear_bench.py
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402
from wfamd import ops  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {}
    for (n, k) in ((2560, 2560), (6912, 2560), (2560, 6912)):
        w = torch.randint(0, 255, (n, k // 4), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
        w = w & 0xAA  # codes 0 / 2 only in the high bit of each field: valid I2_S
        for m in (16, 32, 64, 128, 256):
            x = torch.randn(m, k, generator=g, device="cuda").to(torch.bfloat16)
            for _ in range(3):
                ops.bitnet_linear(x, w, 1.0)
            torch.cuda.synchronize()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                ops.bitnet_linear(x, w, 1.0)
                with torch.cuda.graph(graph, stream=s):
                    for _ in range(20):
                        ops.bitnet_linear(x, w, 1.0)
            torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            out[f"{n}x{k} M{m}"] = round(e0.elapsed_time(e1) * 1000.0 / 100, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
