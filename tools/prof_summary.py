#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace output (rocpd SQLite .db or kernel_trace.csv) per kernel:
calls, total/avg/median/min/max duration in microseconds, sorted by total time."""
import csv
import glob
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
    name_col = "display_name" if "display_name" in cols else ("kernel_name" if "kernel_name" in cols else "name")
    q = f"select s.{name_col}, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id"
    return [(n, (e - s) / 1000.0) for n, s, e in cur.execute(q)]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0))
    return out


def summarize(rows):
    agg = defaultdict(list)
    for n, us in rows:
        agg[n].append(us)
    tot = sum(sum(v) for v in agg.values())
    lines = []
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        lines.append((n, len(v), sum(v), sum(v) / len(v), v[len(v) // 2], min(v), max(v), 100.0 * sum(v) / tot))
    return lines


def main():
    path = sys.argv[1]
    if path.endswith(".db"):
        rows = from_db(path)
    elif path.endswith(".csv"):
        rows = from_csv(path)
    else:
        cands = glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True) or glob.glob(f"{path}/**/*.db", recursive=True)
        rows = from_csv(cands[0]) if cands[0].endswith(".csv") else from_db(cands[0])
    print(f"{'calls':>7} {'total_us':>12} {'avg_us':>10} {'med_us':>9} {'min_us':>9} {'max_us':>9} {'pct':>6}  kernel")
    for n, c, t, a, md, mn, mx, p in summarize(rows):
        short = n if len(n) < 110 else n[:107] + "..."
        print(f"{c:7d} {t:12.1f} {a:10.3f} {md:9.3f} {mn:9.3f} {mx:9.3f} {p:6.2f}  {short}")


if __name__ == "__main__":
    main()
