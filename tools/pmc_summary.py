#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel from a `--pmc ... --kernel-trace --output-format csv`
output directory: python tools/pmc_summary.py <dir> [kernel-regex]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "")
                if pat and not pat.search(k):
                    continue
                acc[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
