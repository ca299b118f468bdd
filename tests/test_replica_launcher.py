"""Node-level replica plumbing on CPU (BASELINE configs[4]; wfamd/replicas.py, tools/replica_node.py):
disjoint host-core slices, the launcher starting N processes and aggregating their JSON lines, and
the AVX512-VNNI CPU-baseline build of the oracle agreeing bit for bit with the checker build."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))


def test_core_slices_partition_the_mask():
    from wfamd.replicas import core_slice
    cores = list(range(3, 3 + 37))
    for world in (1, 2, 3, 8, 37):
        sl = [core_slice(r, world, cores) for r in range(world)]
        flat = [c for s in sl for c in s]
        assert sorted(flat) == cores and len(set(flat)) == len(flat)  # disjoint, complete
        assert max(map(len, sl)) - min(map(len, sl)) <= 1               # balanced
        assert all(s == sorted(s) and s[-1] - s[0] == len(s) - 1 for s in sl)  # contiguous
    assert core_slice(5, 8, [0, 1, 2]) == [2]  # more replicas than cores: shared, never empty
    with pytest.raises(ValueError):
        core_slice(2, 2, cores)


def test_aggregate_sum_and_spread():
    from wfamd.replicas import aggregate
    a = aggregate([{"tokens_per_s": 100.0}, {"tokens_per_s": 110.0}, {"tokens_per_s": 90.0}])
    assert a["sum"] == 300.0 and a["replicas"] == 3 and a["min"] == 90.0 and a["max"] == 110.0
    assert a["spread"] == pytest.approx(0.2)
    with pytest.raises(ValueError):
        aggregate([])


_FAKE = r"""
import json, os, sys, time
sys.path.insert(0, os.environ["WF_PY"])
from wfamd.replicas import pin_host_cores
i = int(sys.argv[sys.argv.index("--replica") + 1]); n = int(sys.argv[sys.argv.index("--replicas") + 1])
cores = pin_host_cores(i, n)
assert sorted(os.sched_getaffinity(0)) == cores
t0 = time.perf_counter(); s = 0
while time.perf_counter() - t0 < 0.2: s += 1
print(json.dumps({"replica": i, "cores": cores, "tokens_per_s": 10.0 * (i + 1), "omp": os.environ["OMP_NUM_THREADS"],
                  "hip": os.environ.get("HIP_VISIBLE_DEVICES")}))
"""


def test_launcher_runs_replicas_on_disjoint_cores():
    from wfamd.replicas import aggregate, launch
    n = 3
    res = launch(n, ["-c", _FAKE], timeout_s=120, env_extra={"WF_PY": str(ROOT / "wrinklefree-inference-engine_amd"
                                                                          / "python")})
    assert [r["replica"] for r in res] == list(range(n))
    assert [r["hip"] for r in res] == ["0", "1", "2"]  # process i sees GPU i only
    sets = [set(r["cores"]) for r in res]
    assert all(not (sets[a] & sets[b]) for a in range(n) for b in range(a + 1, n))
    assert all(r["omp"] == str(len(r["cores"])) for r in res)
    agg = aggregate(res)
    assert agg["sum"] == 60.0 and agg["per_replica"] == [10.0, 20.0, 30.0]


def test_launcher_reports_a_failed_replica():
    from wfamd.replicas import launch
    with pytest.raises(RuntimeError, match="replica 1"):
        launch(2, ["-c", "import sys; i = sys.argv[sys.argv.index('--replica') + 1]; "
                         "sys.exit(3) if i == '1' else print('{\"tokens_per_s\": 1}')"], timeout_s=60,
               visible_devices=False)


def _has_vnni() -> bool:
    try:
        return "avx512_vnni" in Path("/proc/cpuinfo").read_text()
    except OSError:
        return False


@pytest.mark.skipif(not _has_vnni(), reason="host without AVX512-VNNI")
def test_vnni_baseline_build_equals_checker():
    """The CPU baseline's AVX512-VNNI enc-sums (oracle/wf_oracle.c -DORC_VNNI) are the checker's
    integer sums bit for bit: raw GEMV and the corrected BitNet linear at the 2B-4T shapes and a
    shape the vector loop does not cover (odd block count: scalar path)."""
    from oracle import oracle as orc
    orc.build()
    orc.build(march="native", name="liborc_vnni.so", defines=("ORC_VNNI",))
    fast = orc.lib("liborc_vnni.so")
    assert fast.orc_vnni_build() == 1 and orc.lib().orc_vnni_build() == 0
    rng = np.random.default_rng(0)
    for n, k in ((2560, 2560), (640, 2560), (2560, 6912), (96, 384)):
        c = rng.integers(0, 3, size=(n, k // 4, 4)).astype(np.uint8)
        p = np.ascontiguousarray((c[..., 0] << 6) | (c[..., 1] << 4) | (c[..., 2] << 2) | c[..., 3])
        a = rng.integers(-128, 128, size=k).astype(np.int8)
        y0, y1 = np.zeros(n, np.float32), np.zeros(n, np.float32)
        assert orc.lib().orc_gemv_i2s(p.ctypes.data, a.ctypes.data, 0.37, n, k, y0.ctypes.data) == 0
        assert fast.orc_gemv_i2s(p.ctypes.data, a.ctypes.data, 0.37, n, k, y1.ctypes.data) == 0
        assert np.array_equal(y0.view(np.uint32), y1.view(np.uint32)), (n, k)
        x = orc.f32_to_bf16(rng.standard_normal(k).astype(np.float32))
        l0, l1 = np.zeros(n, np.uint16), np.zeros(n, np.uint16)
        assert orc.lib().orc_bitnet_linear_bf16(x.ctypes.data, p.ctypes.data, 1.5, n, k, l0.ctypes.data) == 0
        assert fast.orc_bitnet_linear_bf16(x.ctypes.data, p.ctypes.data, 1.5, n, k, l1.ctypes.data) == 0
        assert np.array_equal(l0, l1), (n, k)


def test_host_cores_respect_the_cgroup_quota(monkeypatch):
    """A GPU box may show every CPU of the machine in the affinity mask while its cgroup quota is a
    slice of them: the replicas' core slices come from the mask capped at the quota."""
    import os
    from wfamd import replicas
    mask = sorted(os.sched_getaffinity(0))
    monkeypatch.setattr(replicas.os, "sched_getaffinity", lambda pid: set(range(128)))
    monkeypatch.setattr(replicas, "cgroup_cpu_quota", lambda: 16.0)
    assert replicas.host_cores() == list(range(16))
    sl = [replicas.core_slice(r, 8) for r in range(8)]
    assert sl == [[2 * r, 2 * r + 1] for r in range(8)]  # 8 replicas x 2 cores, all within the quota
    monkeypatch.setattr(replicas, "cgroup_cpu_quota", lambda: None)
    assert replicas.host_cores() == list(range(128))
    assert mask  # (the real mask is untouched)


def test_timed_window_single_rank():
    from wfamd.replicas import timed_steps, timed_window
    calls = []
    tw = timed_window(lambda: calls.append(1), 5, lambda: None)
    assert len(calls) == 5 and tw["max_s"] == tw["local_s"] >= 0 and tw["t_end"] >= tw["t_start"]
    assert timed_steps(lambda: None, 3, lambda: None) >= 0


def test_node_line_uses_the_whole_job_clock():
    """tools/replica_node.py's node headline is every replica's tokens over the max-over-replicas
    window (bench.py's whole-job clock), not the sum of per-replica rates on their own clocks."""
    import argparse
    import importlib.util
    spec = importlib.util.spec_from_file_location("replica_node", ROOT / "tools" / "replica_node.py")
    rn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rn)
    args = argparse.Namespace(replicas=2, workload="mixed", same_gpu=True)
    res = [{"tokens": 1000, "max_seconds": 2.0, "seconds": 1.0, "t_start": 10.0, "t_end": 11.0, "tokens_per_s": 1000.0,
            "b1_tokens_per_s": 0.0, "b128_tokens_per_s": 1000.0},
           {"tokens": 1000, "max_seconds": 2.0, "seconds": 2.0, "t_start": 10.0, "t_end": 12.5, "tokens_per_s": 500.0,
            "b1_tokens_per_s": 0.0, "b128_tokens_per_s": 500.0}]
    line = rn.node_line(args, res)
    assert line["node_tokens_per_s"] == 1000.0            # 2000 tokens / 2.0 s
    assert line["node_tokens_per_s_over_union"] == 800.0  # 2000 tokens / 2.5 s
    assert line["per_replica_local_rates"]["sum"] == 1500.0  # diagnostic only
