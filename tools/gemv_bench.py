#!/usr/bin/env python3
"""Standalone sgl_kernel bitnet_gemv on the reference's benchmark shapes (scripts/benchmark_kernels.py:
40-66, 132-138, plus k/v), through the C-ABI wf_bitnet_gemv, weights rotating through >= 1.2 GB
(bench.py gemv_bench). Run under `rocprofv3 --kernel-trace --stats` for kernel-only durations:
each k_gemv_rows launch is one GEMV; GB/s = (N K / 4 + K + 4 N) / duration.

    python tools/gemv_bench.py [--reps 5]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    print(json.dumps(bench.gemv_bench(reps=args.reps)))


if __name__ == "__main__":
    main()
