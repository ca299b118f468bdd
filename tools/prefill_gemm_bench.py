#!/usr/bin/env python3
"""Prefill-shaped ternary GEMMs on the int8 matrix cores (BASELINE configs[2]: seq 2048 x batch 8
-> M = 16384 token rows), 2B-4T layer shapes: the tile-layout GEMM wf_bitnet_gemm_tiled (the
prefill path's operands: WF_FMT_I2S_MFMA weights, tile-ordered codes) and, for comparison, the
row-major C-ABI wf_bitnet_gemm_ex. Reports per shape: us, TOPS (2*M*N*K), fraction of the int8
dense peak, and the fp32 output write rate (the raw sgl-kernel contract returns fp32).

    python tools/prefill_gemm_bench.py [--m 16384] [--iters 20]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

import torch  # noqa: E402

from wfamd import WF_FMT_I2S, _lib, ops  # noqa: E402

INT8_DENSE_PEAK_TOPS = 5000.0  # MI355X int8 dense: 2x the ~2.5 PF bf16 dense rate (MI355X_MICROARCH.md Matrix cores)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    M = args.m
    lib = _lib.load()
    shapes = [("qkv", 3840, 2560), ("o_proj", 2560, 2560), ("gate_up", 13824, 2560), ("down", 2560, 6912)]
    g = torch.Generator(device="cuda").manual_seed(0)
    st = torch.cuda.current_stream()
    res = {}
    for name, N, K in shapes:
        w = torch.randint(0, 256, (N, K // 4), dtype=torch.uint8, device="cuda", generator=g)
        a = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda", generator=g)
        y = torch.empty(M, N, dtype=torch.float32, device="cuda")

        wt = ops.i2s_to_mfma(w)
        at = ops.codes_to_tiles(a)

        def run_rowmajor():
            _lib.check(lib.wf_bitnet_gemm_ex(WF_FMT_I2S, w.data_ptr(), a.data_ptr(), K, 1.0, M, N, K, y.data_ptr(),
                                             N, st.cuda_stream), "gemm")

        def run_tiled():
            _lib.check(lib.wf_bitnet_gemm_tiled(wt.data_ptr(), at.data_ptr(), 1.0, M, N, K, y.data_ptr(), N,
                                                st.cuda_stream), "gemm_tiled")

        def timed(run):
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.iters):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            return 1000.0 * e0.elapsed_time(e1) / args.iters

        us_rm = timed(run_rowmajor)
        us = timed(run_tiled)
        tops = 2.0 * M * N * K / us / 1e6
        res[name] = {"M": M, "N": N, "K": K, "us": round(us, 1), "tops": round(tops, 1),
                     "frac_int8_peak": round(tops / INT8_DENSE_PEAK_TOPS, 3),
                     "out_gbs": round(4.0 * M * N / us / 1e3, 1), "rowmajor_us": round(us_rm, 1)}
        print(name, json.dumps(res[name]), flush=True)
        del w, a, y, wt, at
    layer_us = sum(v["us"] for v in res.values())
    print(json.dumps({"prefill_gemm_us_per_layer": round(layer_us, 1),
                      "prefill_gemm_ms_30_layers": round(30 * layer_us / 1000, 2),
                      "gemm_tokens_per_s": round(M / (30 * layer_us / 1e6), 1)}))


if __name__ == "__main__":
    main()
