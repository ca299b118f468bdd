"""Independent replicas: the node-level deployment of the decode path (BASELINE
configs[4]: "8 independent replicas (one bitnet-b1.58-2B-4T server per MI355X), aggregate node
tokens/sec"). The path does not shard -- one wf_model per GPU, no data-path collective and no
RCCL communicator: the only cross-process traffic is a gloo barrier and a scalar max around the
timed region, on the host.

* `core_slice` / `pin_host_cores`: each replica process gets a disjoint slice of the host cores
  (the reference pins its CPU server to 8 cores, scripts/launch_sglang_bitnet.sh:61-67); set
  before the process touches the GPU.
* `timed_steps` brackets K steps with barrier + device sync on both sides and returns the MAX
  elapsed time over ranks (`timed_window` also returns each rank's own time and window);
  `replica_rate` turns that into the whole-job rate.
* `aggregate` sums per-replica results and reports the spread (BASELINE configs[4]).
* `launch` starts N replica processes, process i with HIP_VISIBLE_DEVICES=i, and collects the one
  JSON line each prints (tools/replica_node.py); it hands them a host rendezvous (MASTER_ADDR
  127.0.0.1 and a free MASTER_PORT) so they can bracket their timed windows with a gloo barrier.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time
from typing import Callable, Dict, List, Optional, Sequence


def cgroup_cpu_quota() -> Optional[float]:
    """CPUs the cgroup allows (v2 cpu.max, or v1 cfs quota / period); None when unlimited. A GPU box
    may show every CPU of the machine in the affinity mask while its quota is a slice of them."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def host_cores() -> List[int]:
    """The host cores this process may really use: its affinity mask, sorted, capped at the cgroup
    CPU quota (the first floor(quota) CPUs of the mask)."""
    mask = sorted(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    if quota is not None and int(quota) < len(mask):
        return mask[:max(1, int(quota))]
    return mask


def core_slice(rank: int, world: int, cores: Optional[Sequence[int]] = None) -> List[int]:
    """Disjoint, contiguous, near-equal slices of `cores` (default: host_cores(), the affinity mask
    within the cgroup quota); slice `rank` of `world`. Every core belongs to exactly one slice when
    world <= cores."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} out of range for world {world}")
    cs = sorted(cores if cores is not None else host_cores())
    if not cs:
        raise ValueError("no host cores")
    if world > len(cs):  # more replicas than cores: share round-robin (never an empty slice)
        return [cs[rank % len(cs)]]
    base, extra = divmod(len(cs), world)
    start = rank * base + min(rank, extra)
    return cs[start:start + base + (1 if rank < extra else 0)]


def pin_host_cores(rank: int, world: int, cores: Optional[Sequence[int]] = None) -> List[int]:
    """Pin this process (all its threads created afterwards, OpenMP included) to its core slice and
    size the intra-op thread pools to it. Call before the first GPU / torch call of the process."""
    sl = core_slice(rank, world, cores)
    os.sched_setaffinity(0, sl)
    os.environ["OMP_NUM_THREADS"] = str(len(sl))
    try:
        import torch
        torch.set_num_threads(len(sl))
    except Exception:
        pass
    return sl


def timed_window(step: Callable[[], None], steps: int, sync: Callable[[], None], dist=None,
                 device: Optional[str] = None) -> Dict[str, float]:
    """Run `step` `steps` times between synchronised barriers. Returns this rank's own elapsed time
    (`local_s`, measured from after the start barrier to the device sync after its last step), the
    max of that over ranks (`max_s`) and this rank's wall-clock window (`t_start`, `t_end`, stamped
    inside the barriers, so the window holds no barrier wait). `dist` is torch.distributed
    initialised with a host backend (gloo): the barriers and the max-reduce of one scalar run on the
    host, outside the timed device work."""
    import torch
    on = dist is not None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    sync()
    if on:
        dist.barrier()
    sync()
    w0, t0 = time.time(), time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    local, w1 = time.perf_counter() - t0, time.time()
    el = local
    if on:
        dist.barrier()
        t = torch.tensor([local], dtype=torch.float64, device=device or "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return {"max_s": el, "local_s": local, "t_start": w0, "t_end": w1}


def timed_steps(step: Callable[[], None], steps: int, sync: Callable[[], None], dist=None,
                device: Optional[str] = None) -> float:
    """timed_window's max-over-ranks seconds (the whole-job clock of bench.py's contract)."""
    return timed_window(step, steps, sync, dist, device)["max_s"]


def replica_rate(units_per_step_per_rank: int, steps: int, world: int, elapsed_s: float) -> float:
    """Whole-job throughput: every rank processed units_per_step_per_rank * steps units."""
    if elapsed_s <= 0:
        raise ValueError("elapsed time must be positive")
    return units_per_step_per_rank * steps * world / elapsed_s


def aggregate(results: List[Dict], key: str = "tokens_per_s") -> Dict:
    """Node total and per-replica spread of `key` over the replicas' result dicts."""
    if not results:
        raise ValueError("no replica results")
    vals = [float(r[key]) for r in results]
    mean = sum(vals) / len(vals)
    return {"replicas": len(vals), "sum": round(sum(vals), 2), "mean": round(mean, 2),
            "min": round(min(vals), 2), "max": round(max(vals), 2),
            "spread": round((max(vals) - min(vals)) / mean, 4) if mean > 0 else 0.0,
            "per_replica": [round(v, 2) for v in vals]}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv: List[str], timeout_s: float = 900.0, env_extra: Optional[Dict[str, str]] = None,
           visible_devices: bool = True) -> List[Dict]:
    """Start n replica processes `python argv... --replica i --replicas n` (process i sees GPU i only
    when visible_devices), wait for all, and return the last JSON line each printed. Raises if a
    replica fails (its stderr tail in the message). The parent never touches the GPU. Every child
    gets MASTER_ADDR=127.0.0.1 / MASTER_PORT (one free port per launch), RANK and WORLD_SIZE for
    an optional gloo rendezvous."""
    procs = []
    port = str(free_port())
    for i in range(n):
        env = dict(os.environ, **(env_extra or {}))
        env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK=str(i), WORLD_SIZE=str(n))
        if visible_devices:
            env["HIP_VISIBLE_DEVICES"] = str(i)
        cmd = [sys.executable] + list(argv) + ["--replica", str(i), "--replicas", str(n)]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    out, errs = [], []
    t_end = time.time() + timeout_s
    for i, p in enumerate(procs):
        try:
            so, se = p.communicate(timeout=max(1.0, t_end - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise RuntimeError(f"replica {i} timed out")
        lines = [ln for ln in so.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not lines:
            errs.append(f"replica {i} rc={p.returncode}: {se[-1500:]}")
            continue
        out.append(json.loads(lines[-1]))
    if errs:
        raise RuntimeError("\n".join(errs))
    return out
