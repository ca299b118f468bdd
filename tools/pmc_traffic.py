#!/usr/bin/env python3
"""Per-launch HBM traffic of the decode-step kernels from two rocprofv3 PMC passes (run separately,
`--pmc FETCH_SIZE --kernel-trace --output-format csv` and `--pmc WRITE_SIZE ...`, MI355X_MICROARCH.md
HBM/rocprofv3 section). FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE
reports half the bytes of 16-byte-per-lane coalesced streaming reads (every weight / KV load of
these kernels), so the read side is doubled. Writes profiles/pmc_traffic.json keyed by bench.py's
op names, plus a copy named per round.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write r01 [pmc_traffic]

The last argument names the unsuffixed copy bench.py reads (pmc_traffic.json for batch 1,
pmc_traffic_b128.json for the batched step).
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
MODES = {"0": "qkv", "1": "o_proj", "2": "gate_up", "3": "down"}


def op_name(kernel: str):
    m = re.search(r"k_gemv<wf::Fmt(\w+), (\d)", kernel)
    if m:
        return MODES[m.group(2)], m.group(1)
    m = re.search(r"k_dec_gemm(?:_t)?<\d+, \d+, \d+, (\d)[,>]", kernel)
    if m:  # batched matrix-core GEMMs (last template argument = mode)
        return MODES[m.group(1)], "I2S_MFMA" if "k_dec_gemm_t" in kernel else "I2S"
    if "k_attn_sdpa" in kernel or "k_attn_part" in kernel or "k_attn_mfma" in kernel:  # r05 / earlier rounds
        return "attn", None
    if "k_seq_order" in kernel:
        return "seq_order", None
    if "k_lm_head" in kernel:
        return "lm_head", None
    if "k_rownorm_attn" in kernel:
        return "rownorm_attn", None
    if "k_rownorm" in kernel:
        return "rownorm", None
    if "k_embed" in kernel:
        return "embed", None
    return None, None


def read(d: Path, counter: str):
    f = next(d.glob("*counter_collection.csv"))
    acc = defaultdict(list)
    fmts = {}
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            op, fmt = op_name(r["Kernel_Name"])
            if op:
                acc[op].append(float(r["Counter_Value"]) * 1024.0)
                if fmt:
                    fmts[op] = fmt
    return acc, fmts


def main():
    fetch_dir, write_dir = Path(sys.argv[1]), Path(sys.argv[2])
    tag = sys.argv[3] if len(sys.argv) > 3 else "r01"
    stem = sys.argv[4] if len(sys.argv) > 4 else "pmc_traffic"
    fetch, fmts = read(fetch_dir, "FETCH_SIZE")
    write, _ = read(write_dir, "WRITE_SIZE")
    out = {"_note": "bytes per launch; read side = 2 x FETCH_SIZE (gfx950 wide-read correction), "
                    "write side = WRITE_SIZE; averages over every dispatch of the profiled bench run",
           "_weight_format": sorted(set(fmts.values()))}
    for op in sorted(set(fetch) | set(write)):
        f = fetch.get(op, [0.0])
        w = write.get(op, [0.0])
        fb = 2.0 * sum(f) / len(f)
        wb = sum(w) / len(w)
        out[op] = {"calls": len(f), "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                   "hbm_bytes_per_launch": round(fb + wb)}
    (ROOT / "profiles").mkdir(exist_ok=True)
    txt = json.dumps(out, indent=1)
    (ROOT / "profiles" / f"{stem}.json").write_text(txt + "\n")
    (ROOT / "profiles" / f"{stem}_{tag}.json").write_text(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
