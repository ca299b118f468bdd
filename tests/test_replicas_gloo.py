"""The N>1 bench path (replicas, no data-path collective) on CPU: two gloo ranks, barrier +
max-over-ranks timing and the whole-job rate (wfamd/replicas.py, used by bench.py)."""
import os
import socket
import sys
import time
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "wrinklefree-inference-engine_amd" / "python"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    from wfamd.replicas import replica_rate, timed_steps
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []
        per_step = 0.02 * (rank + 1)  # rank 1 is the slow replica

        def step():
            calls.append(1)
            time.sleep(per_step)
        el = timed_steps(step, 5, lambda: None, dist)
        out[rank] = (el, len(calls), replica_rate(128, 5, world, el))
    finally:
        dist.destroy_process_group()


def test_two_replicas_max_over_ranks():
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    (el0, n0, r0), (el1, n1, r1) = res[0], res[1]
    assert n0 == n1 == 5
    assert el0 == el1  # every rank reports the same (max) time
    assert el0 >= 5 * 0.04  # at least the slow replica's work
    assert r0 == pytest.approx(128 * 5 * 2 / el0)


def test_single_process_rate():
    from wfamd.replicas import replica_rate, timed_steps
    el = timed_steps(lambda: None, 3, lambda: None, None)
    assert el >= 0
    assert replica_rate(1, 10, 1, 0.5) == 20.0
    with pytest.raises(ValueError):
        replica_rate(1, 1, 1, 0.0)
