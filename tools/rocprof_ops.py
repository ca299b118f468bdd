#!/usr/bin/env python3
"""Per-op rocprofv3 kernel time of a profiled bench run, keyed by bench.py's op names, and the
dominant op by TOTAL rocprof time (what bench.py's `roofline` reports, so the choice does not flip
between near-equal ops on run-to-run noise of the live timing).

    python tools/rocprof_ops.py profiles/rocprof_r04_bench_kernel_stats.txt r04 [rocprof_ops]

Input: a tools/prof_summary.py table (calls total_us avg_us med_us min_us max_us pct kernel).
Writes profiles/<stem>.json (read by bench.py) and profiles/<stem>_<tag>.json.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from pmc_traffic import op_name  # noqa: E402


def parse(path: Path) -> dict:
    ops = {}
    for line in path.read_text().splitlines():
        parts = line.split(None, 7)
        if len(parts) < 8 or not parts[0].isdigit():
            continue
        op, _ = op_name(parts[7])
        if not op:
            continue
        calls, total = int(parts[0]), float(parts[1])
        o = ops.setdefault(op, {"calls": 0, "total_us": 0.0, "kernels": []})
        o["calls"] += calls
        o["total_us"] = round(o["total_us"] + total, 1)
        o["kernels"].append(parts[7][:120])
    for o in ops.values():
        o["avg_us"] = round(o["total_us"] / o["calls"], 3)
    return ops


def main():
    src = Path(sys.argv[1])
    tag = sys.argv[2] if len(sys.argv) > 2 else "r04"
    stem = sys.argv[3] if len(sys.argv) > 3 else "rocprof_ops"
    ops = parse(src)
    dom = max(ops, key=lambda k: ops[k]["total_us"])
    out = {"_note": "per-op rocprofv3 kernel time of a profiled bench run; _dominant = largest total time",
           "_source": src.name, "_dominant": dom, **ops}
    txt = json.dumps(out, indent=1)
    (ROOT / "profiles" / f"{stem}.json").write_text(txt + "\n")
    (ROOT / "profiles" / f"{stem}_{tag}.json").write_text(txt + "\n")
    print(f"dominant: {dom}")


if __name__ == "__main__":
    main()
