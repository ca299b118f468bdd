#!/usr/bin/env python3
"""Per-phase summary of the batch-1 attention's in-graph stamps (gpurun_out/stamps_graph_b1_attn_raw.json,
written by tools/stamps_graph.py): per stamp the min / median / max over blocks (µs on the QKV clock) and
the per-block phase durations."""
import json
import sys

import numpy as np
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from stamps_graph import ATTN_NAMES  # noqa: E402

raw = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps_graph_b1_attn_raw.json"))
a = np.array([[np.nan if v is None else v for v in r] for r in raw], dtype=float)
names = list(ATTN_NAMES.values())
print("blocks", a.shape[0])
for j, n in enumerate(names):
    c = a[:, 1 + j]
    if np.isnan(c).all():
        continue
    print(f"{n:>10}: min {np.nanmin(c):6.2f} med {np.nanmedian(c):6.2f} max {np.nanmax(c):6.2f}")
for j in range(1, len(names)):
    d = a[:, 1 + j] - a[:, j]
    if np.isnan(d).all():
        continue
    print(f"{names[j]:>10} - {names[j - 1]:<10}: min {np.nanmin(d):5.2f} med {np.nanmedian(d):5.2f} max {np.nanmax(d):5.2f}")
