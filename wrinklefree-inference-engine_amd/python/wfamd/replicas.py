"""Replica timing for the multi-GPU bench (the decode path does not shard -- one
independent wf_model per GPU, no data-path collective).

`timed_steps` brackets K steps with barrier + device sync on both sides and returns the MAX
elapsed time over ranks (one all_reduce of a scalar, outside the timed region); `replica_rate`
turns that into the whole-job rate. Backend-agnostic: nccl (RCCL) on the GPU node, gloo in the
CPU tests.
"""
from __future__ import annotations

import time
from typing import Callable, Optional


def timed_steps(step: Callable[[], None], steps: int, sync: Callable[[], None], dist=None,
                device: Optional[str] = None) -> float:
    """Run `step` `steps` times between synchronised barriers; return max-over-ranks seconds."""
    import torch
    on = dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    sync()
    if on:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if on:
        dist.barrier()
    el = time.perf_counter() - t0
    if on:
        t = torch.tensor([el], dtype=torch.float64, device=device or "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def replica_rate(units_per_step_per_rank: int, steps: int, world: int, elapsed_s: float) -> float:
    """Whole-job throughput: every rank processed units_per_step_per_rank * steps units."""
    if elapsed_s <= 0:
        raise ValueError("elapsed time must be positive")
    return units_per_step_per_rank * steps * world / elapsed_s
