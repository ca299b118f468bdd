"""BASELINE configs[4] ("8 independent replicas (one bitnet-b1.58-2B-4T server per MI355X), aggregate
node tokens/sec") exercised on the GPU box: replica processes started by the node launcher
(wfamd.replicas.launch, tools/replica_node.py) on the one GPU, each with its own weights seed, host
core slice and gloo start barrier (no RCCL), running the mixed workload (batch-1 decode beside a
batch-128 continuous batch at config-4 contexts, paged KV) over the full 30-layer model. Each replica
records its greedy tokens of every step and a hash of its final logits; a replica's results must be
bit-identical to a solo run of the same seed in a fresh process (independence: nothing shared,
nothing order-dependent between replicas). Reference: scripts/launch_sglang_bitnet.sh:60-61.

This module runs FIRST in the session (tests/conftest.py orders it) so the children start before
the pytest process has touched the GPU; the parent itself never makes a GPU call."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

pytestmark = pytest.mark.gpu

NODE = str(ROOT / "tools" / "replica_node.py")


def _argv(seed: int, steps: int = 6):
    return [NODE, "--workload", "mixed", "--steps", str(steps), "--layers", "30", "--seed", str(seed), "--verify"]


def test_replicas_on_one_gpu_match_solo_runs():
    import torch
    from wfamd.replicas import aggregate, launch
    assert not torch.cuda.is_initialized(), "the replica children must start before this process uses the GPU"
    res = launch(2, _argv(100), timeout_s=400, visible_devices=False)
    assert [r["replica"] for r in res] == [0, 1] and [r["seed"] for r in res] == [100, 101]
    # the barrier aligns the timed windows: they overlap
    assert max(r["t_start"] for r in res) < min(r["t_end"] for r in res)
    solo = launch(1, _argv(101), timeout_s=400, visible_devices=False)[0]
    assert solo["seed"] == 101
    got = res[1]
    assert got["b1_tokens"] == solo["b1_tokens"] and len(got["b1_tokens"]) == 4 * 9
    assert got["b128_tokens_sha256"] == solo["b128_tokens_sha256"]
    assert got["logits_sha256"] == solo["logits_sha256"]
    # different weights seeds give different outputs: the comparison above is not vacuous
    assert res[0]["logits_sha256"] != got["logits_sha256"]
    print(json.dumps({"node": aggregate(res), "solo_seed101": {k: solo[k] for k in ("tokens_per_s", "seconds")}}))
