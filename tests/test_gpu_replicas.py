"""BASELINE configs[4] ("8 independent replicas (one bitnet-b1.58-2B-4T server per MI355X), aggregate
node tokens/sec") exercised on the GPU box: replica processes started by the node launcher
(wfamd.replicas.launch, tools/replica_node.py) on the one GPU, each with its own weights seed, host
core slice and gloo start barrier (no RCCL), running the mixed workload (batch-1 decode beside a
batch-128 continuous batch at config-4 contexts, paged KV) over the full 30-layer model. Each replica
records its greedy tokens of every step and a hash of its final logits; a replica's results must be
bit-identical to a solo run of the same seed in a fresh process (independence: nothing shared,
nothing order-dependent between replicas). Two replicas, then the configs[4] process count (eight,
two host cores each within the box's quota). Reference: scripts/launch_sglang_bitnet.sh:60-61.

This module runs FIRST in the session (tests/conftest.py orders it) so the children start before
the pytest process has touched the GPU; the parent itself never makes a GPU call."""
import json
import os
import sys
import threading
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

pytestmark = pytest.mark.gpu

NODE = str(ROOT / "tools" / "replica_node.py")
_SOLO = {}  # seed -> solo result, shared by the two tests


def _argv(seed: int, steps: int = 6):
    return [NODE, "--workload", "mixed", "--steps", str(steps), "--layers", "30", "--seed", str(seed), "--verify"]


class _Heartbeat:
    """The children's output is collected at their end: a line a minute under gpurun_out/ (when the
    directory exists) shows a long launch is alive."""

    def __init__(self, name: str):
        self.path = ROOT / "gpurun_out" / f"heartbeat_{name}.txt"
        self.stop = threading.Event()

    def __enter__(self):
        if self.path.parent.is_dir():
            threading.Thread(target=self._run, daemon=True).start()
        return self

    def _run(self):
        t0 = time.time()
        while not self.stop.wait(30.0):
            with open(self.path, "a") as f:
                f.write(f"{time.time() - t0:.0f} s\n")

    def __exit__(self, *exc):
        self.stop.set()


def _solo(seed: int):
    from wfamd.replicas import launch
    if seed not in _SOLO:
        _SOLO[seed] = launch(1, _argv(seed), timeout_s=400, visible_devices=False)[0]
    return _SOLO[seed]


def _same(got, solo):
    assert got["seed"] == solo["seed"]
    assert got["b1_tokens"] == solo["b1_tokens"] and len(got["b1_tokens"]) == 4 * 9
    assert got["b128_tokens_sha256"] == solo["b128_tokens_sha256"]
    assert got["logits_sha256"] == solo["logits_sha256"]


def test_replicas_on_one_gpu_match_solo_runs():
    import torch
    from wfamd.replicas import aggregate, launch
    assert not torch.cuda.is_initialized(), "the replica children must start before this process uses the GPU"
    with _Heartbeat("replicas2"):
        res = launch(2, _argv(100), timeout_s=400, visible_devices=False)
        assert [r["replica"] for r in res] == [0, 1] and [r["seed"] for r in res] == [100, 101]
        # the barrier aligns the timed windows: they overlap
        assert max(r["t_start"] for r in res) < min(r["t_end"] for r in res)
        _same(res[1], _solo(101))
    # different weights seeds give different outputs: the comparison above is not vacuous
    assert res[0]["logits_sha256"] != res[1]["logits_sha256"]
    print(json.dumps({"node": aggregate(res), "solo_seed101": {k: _SOLO[101][k] for k in ("tokens_per_s", "seconds")}}))


def test_eight_replicas_on_one_gpu():
    """The configs[4] process count: eight 30-layer replicas at once on the one GPU, two host cores
    each (the box's 16-CPU quota split by wfamd.replicas.core_slice). Every replica completes inside
    the shared barrier-aligned window, the core slices are disjoint, and replica 1 (seed 101) is
    bit-identical to the solo run of seed 101 although seven other processes share the GPU."""
    import torch
    from wfamd.replicas import host_cores, launch
    assert not torch.cuda.is_initialized(), "the replica children must start before this process uses the GPU"
    with _Heartbeat("replicas8"):
        res = launch(8, _argv(100), timeout_s=900, visible_devices=False)
        assert [r["replica"] for r in res] == list(range(8)) and [r["seed"] for r in res] == list(range(100, 108))
        assert max(r["t_start"] for r in res) < min(r["t_end"] for r in res)
        ncores = len(host_cores())
        ranges = sorted(tuple(r["core_range"]) for r in res)
        if ncores >= 8:
            assert all(a[1] < b[0] for a, b in zip(ranges, ranges[1:])), ranges  # disjoint slices
        assert all(r["cores"] == max(1, ncores // 8) or r["cores"] == ncores // 8 + 1 for r in res), res
        _same(res[1], _solo(101))
    assert len({r["logits_sha256"] for r in res}) == 8
    tokens = sum(r["tokens"] for r in res)
    job = max(r["max_seconds"] for r in res)
    print(json.dumps({"replicas": 8, "node_tokens_per_s": round(tokens / job, 1), "job_s": round(job, 3),
                      "cores": [r["cores"] for r in res]}))
