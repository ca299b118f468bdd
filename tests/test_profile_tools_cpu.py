"""Host-side profile tooling on synthetic inputs (no GPU): the kernel-trace gap reconciliation
(tools/trace_gaps.py), the per-op rocprof table (tools/rocprof_ops.py) and the PMC traffic summary
(tools/pmc_traffic.py) that bench.py's `roofline` reads."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))


def _trace(path: Path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Queue_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for q, name, s, e in rows:
            w.writerow(["KERNEL_DISPATCH", q, name, s, e])


def test_trace_gaps_duration_plus_gap(tmp_path):
    # three back-to-back dispatches of one kernel: 2 us each, 1 us apart; another queue interleaved
    rows = [(1, "void wf::k_gemv_rows<wf::FmtI2S, 4, 1>(args)", 1000 + 3000 * i, 3000 + 3000 * i) for i in range(3)]
    rows += [(2, "other(args)", 500, 700)]
    _trace(tmp_path / "run_kernel_trace.csv", rows)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "trace_gaps.py"), str(tmp_path), "k_gemv_rows"],
                         check=True, capture_output=True, text=True).stdout
    line = next(ln for ln in out.splitlines() if ln.startswith("wf::k_gemv_rows"))
    calls, dur_med, dur_mean, gap_med, tot = line.split()[-5:]
    assert int(calls) == 3
    assert float(dur_med) == 2.0 and float(dur_mean) == 2.0
    assert float(gap_med) == 1.0 and float(tot) == 3.0


def test_rocprof_ops_dominant_by_total(tmp_path):
    import rocprof_ops
    table = tmp_path / "stats.txt"
    table.write_text(
        "  calls     total_us     avg_us    med_us    min_us    max_us    pct  kernel\n"
        "   4350      26036.2      5.985     5.520     4.800     9.641  17.94  void wf::k_attn_part<1, 8>(unsigned short const*, long)\n"
        "   4350      25512.4      5.865     5.520     4.440     9.120  17.58  void wf::k_gemv<wf::FmtI2S, 2, 8, 1, 1>(wf::GemvArgs)\n"
        "    145      14727.9    101.572   101.280    98.320   107.840  10.15  void wf::k_lm_head_p<1, 1>(unsigned short const*)\n")
    ops = rocprof_ops.parse(table)
    assert set(ops) >= {"attn", "gate_up", "lm_head"}
    assert max(ops, key=lambda k: ops[k]["total_us"]) == "attn"
    assert abs(ops["gate_up"]["avg_us"] - 5.865) < 1e-9


def test_pmc_traffic_doubles_fetch(tmp_path):
    import pmc_traffic
    for sub, counter, val in (("f", "FETCH_SIZE", 1000.0), ("w", "WRITE_SIZE", 5.0)):
        d = tmp_path / sub
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writerow(["void wf::k_gemv<wf::FmtI2S, 1, 32, 1, 1>(wf::GemvArgs)", counter, val])
    fetch, fmts = pmc_traffic.read(tmp_path / "f", "FETCH_SIZE")
    write, _ = pmc_traffic.read(tmp_path / "w", "WRITE_SIZE")
    assert fetch["o_proj"] == [1000.0 * 1024] and fmts["o_proj"] == "I2S"
    assert write["o_proj"] == [5.0 * 1024]
    assert json.dumps(pmc_traffic.op_name("void wf::k_lm_head_p<1, 1>(x)")) == '["lm_head", null]'
