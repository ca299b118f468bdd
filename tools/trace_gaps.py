#!/usr/bin/env python3
"""Per-kernel durations and dispatch-to-dispatch gaps from a rocprofv3 kernel trace
(`rocprofv3 --kernel-trace --output-format csv`). For each kernel name: the trace's own duration
(End - Start) and the gap from the previous dispatch's End on the same queue to this Start, so
duration + gap = the per-call time a back-to-back replay (graph or stream) sees. Reconciles the
three GEMV clocks of DESIGN.md (rocprof duration, graph-replay µs per call, in-kernel stamps).

    python tools/trace_gaps.py gpurun_out/gtrace [filter-substring] > profiles/gemv_trace_r04.txt
"""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")[:90]


def main():
    d = Path(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    f = next(d.rglob("*kernel_trace.csv"))
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Queue_Id"]) if r.get("Queue_Id") else 0, int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort(key=lambda t: (t[0], t[1]))
    dur = defaultdict(list)
    gap = defaultdict(list)
    prev_end = {}
    for q, s, e, name in rows:
        k = short(name)
        if filt and filt not in name:
            prev_end[q] = e
            continue
        dur[k].append((e - s) / 1000.0)
        if q in prev_end and 0 <= s - prev_end[q] < 50_000:  # same replay (gaps under 50 us)
            gap[k].append((s - prev_end[q]) / 1000.0)
        prev_end[q] = e
    print(f"# {f.name}: {len(rows)} dispatches; us; gap = this Start - previous End on the same queue")
    print(f"{'kernel':90s} {'calls':>6s} {'dur_med':>8s} {'dur_mean':>8s} {'gap_med':>8s} {'dur+gap':>8s}")
    for k in sorted(dur, key=lambda x: -sum(dur[x])):
        dm = statistics.median(dur[k])
        gm = statistics.median(gap[k]) if gap[k] else float("nan")
        print(f"{k:90s} {len(dur[k]):6d} {dm:8.3f} {statistics.fmean(dur[k]):8.3f} {gm:8.3f} {dm + gm:8.3f}")


if __name__ == "__main__":
    main()
