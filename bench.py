#!/usr/bin/env python3
"""Decode benchmark of the MI355X BitNet b1.58 hot path (BASELINE.json metric: decode tokens/sec +
GEMV HBM GB/s, bitnet-b1.58-2B-4T).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--ctx C] [--wfmt tq|i2s]

One "step" = one decode token for every sequence of the batch through all 30 layers and the bf16
LM head (greedy), replayed as one HIP graph; inputs (weights, KV context, token) resident in HBM.
Default workload = BASELINE configs[1]: batch 1 on one MI355X, synthetic random-init weights of the
2B-4T architecture (no checkpoint offline), KV context pre-filled to --ctx positions.
N > 1 (torch.distributed.run, one rank per GPU): independent replicas, each pinned to its own slice
of the host cores, no data-path collective and no RCCL communicator (a gloo barrier on the host;
SURVEY §8e); value = all ranks' tokens / max-over-ranks time.

Also measured live: per-op kernel durations with HIP events (graph replays of each op's 30
launches, each after a full decode step so caches are in their in-step state), the dominant
kernel's achieved HBM GB/s vs the 8 TB/s peak (PMC traffic from profiles/pmc_traffic.json), and the
CPU baseline (oracle/cpu_baseline.py: AVX512-VNNI build of the oracle's decode step) on this host's
cores, all cores and pinned to 8 (rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--wfmt", choices=["tq", "i2s"], default="i2s")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-op-timing", action="store_true")
    ap.add_argument("--max-seq", type=int, default=0, help="KV rows per (sequence, kv head); 0 = model default")
    ap.add_argument("--ctx-dist", choices=["fixed", "uniform"], default="fixed",
                    help="uniform: per-sequence contexts drawn from U[1, max_seq - steps) with seed 0 (SURVEY §8d "
                         "config 4), on paged KV")
    ap.add_argument("--paged", action="store_true", help="paged KV (32-token pages; batch >= 16)")
    ap.add_argument("--no-gemv", action="store_true", help="skip the standalone GEMV / GEMM-sweep benchmarks")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the sub-records (batch 128 at ctx 1024 and at config-4 contexts, prefill 8 x 2048) "
                         "that the default N = 1 batch-1 run appends")
    ap.add_argument("--sub-steps", type=int, default=10, help="timed steps of each batch-128 sub-record")
    ap.add_argument("--kv", choices=["bf16", "fp8", "int8"], default="bf16",
                    help="K/V cache element type (batch >= 16): fp8 = OCP e4m3fn, scale 1.0; int8 = the "
                         "reference's INT8 KVCacheDtype, scale 4/127 (unit-variance synthetic K/V)")
    return ap.parse_args()


def op_timing(dec, ctx, reps: int = 5):
    """Per-op average kernel duration measured with HIP events on the launch stream. Each op's
    launches for all 30 layers (its in-step cadence: one launch per layer, distinct weights each
    time; the LM head is one launch) are captured into a HIP graph like the decode step itself, and
    every timed replay follows one full decode step, so the caches hold what they hold inside the
    step (weights streamed from HBM, the previous token's KV partly in the Infinity Cache). Graph
    replay keeps host launch gaps out of the per-launch average; the numbers agree with rocprofv3's
    in-step kernel durations (profiles/). Median of `reps`. Also returns algorithmic bytes."""
    import torch
    from wfamd import _lib
    L = dec.cfg.layers
    ops = [(_lib.WF_OP_QKV, "qkv"), (_lib.WF_OP_ATTN, "attn"), (_lib.WF_OP_O, "o_proj"),
           (_lib.WF_OP_GATE_UP, "gate_up"), (_lib.WF_OP_DOWN, "down"), (_lib.WF_OP_LM_HEAD, "lm_head")]
    graphs = {}
    for op, name in ops:
        layers = [0] if op == _lib.WF_OP_LM_HEAD else list(range(L))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for l in layers:
                dec.launch_op(l, op)
        graphs[name] = (g, len(layers))
    rec = []
    st = torch.cuda.current_stream()
    for rep in range(reps):
        for op, name in ops:
            g, n = graphs[name]
            dec.step(graph=True)  # the cache state the op sees inside the decode step
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            g.replay()
            e1.record(st)
            rec.append((name, op, n, e0, e1))
    torch.cuda.synchronize()
    out = {}
    for name, op, n, e0, e1 in rec:
        out.setdefault(name, {"op": op, "us": []})["us"].append(1000.0 * e0.elapsed_time(e1) / n)
    res = {}
    for name, v in out.items():
        us = sorted(v["us"])[len(v["us"]) // 2]
        nbytes = dec.op_bytes(v["op"], ctx)
        per_tok = 1 if v["op"] == _lib.WF_OP_LM_HEAD else L
        res[name] = {"us": round(us, 3), "bytes": nbytes, "gbs": round(nbytes / us / 1e3, 1),
                     "launches_per_step": per_tok, "us_per_step": round(us * per_tok, 2)}
    return res


GEMV_SHAPES = [("q_proj/o_proj", 2560, 2560), ("k_proj/v_proj", 640, 2560), ("gate/up", 6912, 2560),
               ("down", 2560, 6912)]  # (N, K): scripts/benchmark_kernels.py:132-138 plus k/v


def gemv_bench(rotate_bytes: float = 1.2e9, reps: int = 3):
    """The reference's kernel benchmark (scripts/benchmark_kernels.py:40-66) on the GPU: one
    sgl_kernel bitnet_gemv call (C-ABI wf_bitnet_gemv, raw enc-sum GEMV + scale, output
    preallocated) per launch, random ternary I2_S weights, int8 activations. The launches of one
    timed replay rotate through >= 1.2 GB of distinct weight buffers (SURVEY §8d cache hygiene: the
    256 MB Infinity Cache cannot serve them), captured in a HIP graph (no host gaps); per-call µs =
    replay time / calls, GB/s = (W_bytes + K + 4N) / µs as benchmark_kernels.py:61-66."""
    import torch
    from wfamd import _lib
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    st = torch.cuda.current_stream()
    out = {}
    for name, N, K in GEMV_SHAPES:
        wb = N * K // 4
        nbuf = max(8, int(rotate_bytes // wb) + 1)
        w = torch.randint(0, 255, (nbuf, N, K // 4), dtype=torch.uint8, device="cuda", generator=g)
        w &= 0xAA  # every 2-bit field in {0, 2}: valid enc codes (w = -1 / +1)
        a = torch.randint(-128, 128, (K,), dtype=torch.int8, device="cuda", generator=g)
        y = torch.empty(N, dtype=torch.float32, device="cuda")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cs = torch.cuda.current_stream().cuda_stream
            for i in range(nbuf):
                _lib.check(lib.wf_bitnet_gemv(w[i].data_ptr(), a.data_ptr(), 0.01, N, K, y.data_ptr(), cs), "gemv")
        graph.replay()
        times = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            graph.replay()
            e1.record(st)
            torch.cuda.synchronize()
            times.append(1000.0 * e0.elapsed_time(e1) / nbuf)
        us = sorted(times)[len(times) // 2]
        nbytes = wb + K + 4 * N
        out[name] = {"N": N, "K": K, "us": round(us, 3), "bytes": nbytes, "gbs": round(nbytes / us / 1e3, 1),
                     "calls_per_replay": nbuf}
        del w, graph
        torch.cuda.empty_cache()
    return out


GEMM_SWEEP = (6912, 2560, (1, 4, 8, 16, 32))  # (K, N, M): scripts/benchmark_kernels.py:140,162-170 (down proj)


def gemm_sweep(rotate_bytes: float = 1.2e9, reps: int = 3):
    """The reference's GEMM batch sweep (scripts/benchmark_kernels.py:75-106, :162-170): sgl_kernel
    bitnet_gemm (C-ABI wf_bitnet_gemm: Y = float(sum enc(W) A) * scale, fp32 out) on the down
    projection 6912 -> 2560 at M in {1, 4, 8, 16, 32}, the launches of one graph replay rotating
    through >= 1.2 GB of distinct I2_S weight buffers. Per M: µs per call, GOPS = 2 M K N / t and
    GB/s = (W + M K + 4 M N) / t, as benchmark_kernels.py:98-106 computes them."""
    import torch
    from wfamd import _lib
    lib = _lib.load()
    K, N, Ms = GEMM_SWEEP
    g = torch.Generator(device="cuda").manual_seed(1)
    st = torch.cuda.current_stream()
    wb = N * K // 4
    nbuf = max(8, int(rotate_bytes // wb) + 1)
    w = torch.randint(0, 255, (nbuf, N, K // 4), dtype=torch.uint8, device="cuda", generator=g)
    w &= 0xAA
    out = {}
    for M in Ms:
        a = torch.randint(-128, 128, (M, K), dtype=torch.int8, device="cuda", generator=g)
        y = torch.empty(M, N, dtype=torch.float32, device="cuda")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            cs = torch.cuda.current_stream().cuda_stream
            for i in range(nbuf):
                _lib.check(lib.wf_bitnet_gemm(w[i].data_ptr(), a.data_ptr(), 0.01, M, N, K, y.data_ptr(), cs), "gemm")
        graph.replay()
        times = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            graph.replay()
            e1.record(st)
            torch.cuda.synchronize()
            times.append(1000.0 * e0.elapsed_time(e1) / nbuf)
        us = sorted(times)[len(times) // 2]
        nbytes = wb + M * K + 4 * M * N
        out[str(M)] = {"M": M, "us": round(us, 3), "gops": round(2.0 * M * K * N / us / 1e3, 1),
                       "gbs": round(nbytes / us / 1e3, 1), "bytes": nbytes,
                       "hbm_frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4)}
        del graph
    del w
    torch.cuda.empty_cache()
    return {"layer": f"down proj {K} -> {N}", "calls_per_replay": nbuf, "by_M": out}


INT8_DENSE_PEAK_TOPS = 5000.0  # MI355X dense int8 MFMA (MI355X_MICROARCH.md; no 2:1 sparsity)


def sub_records(cfg, steps: int, warmup: int = 3) -> dict:
    """BASELINE's other single-GPU configurations under the same clock, each
    with its own roofline:
      b1_tq     -- decode batch 1 at ctx 1024 on the ~1.6-bit TQ weights (configs[1], the other format);
      b128      -- decode batch 128, every sequence at ctx 1024 (configs[3] at a fixed context);
      b128_cfg4 -- decode batch 128 on paged KV, contexts U[1, max_seq - steps) seed 0 (configs[3]);
      prefill   -- 8 sequences x 2048 tokens through wf_model_prefill (configs[2]).
    Decode records: tokens/s over `steps` graph-replayed steps (barrier + sync both sides), the
    per-op HIP-event timing and the dominant op's HBM fraction as in the headline line; prefill: the
    median of 3 HIP-event-timed calls, int8 GEMM tera-ops (2 M N K summed over the 4 GEMMs x 30
    layers, as scripts/benchmark_kernels.py:99) per second against the dense int8 peak."""
    import numpy as np
    import torch
    from wfamd.model import BitNetDecoder, synthetic_weights
    from wfamd import WF_FMT_TQ
    out = {}
    st = torch.cuda.current_stream()
    w = synthetic_weights(cfg, seed=0, device="cuda")
    # batch 1 on the ~1.6-bit TQ weights (north_star: "packs weights at ~1.6 bit"; the reference's
    # 1.58 bits / weight, sglang_backend/bitnet_quantization.py:58-61), the headline's workload
    dec = BitNetDecoder(cfg, w, batch=1, wfmt=WF_FMT_TQ)
    dec.fill_kv_random(1024, seed=1)
    dec.set_state([1], [1024])
    n_tq = max(steps, 100)
    for _ in range(warmup):
        dec.step(graph=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_tq):
        dec.step(graph=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    wb = cfg.weight_bytes_per_token(WF_FMT_TQ)
    out["b1_tq"] = {"workload": "decode batch 1, ctx 1024, TQ weights (5 trits / byte, ~1.6 bit; BASELINE configs[1])",
                    "tokens_per_s": round(n_tq / el, 1), "ms_per_step": round(1000.0 * el / n_tq, 4), "steps": n_tq,
                    "weight_bytes_per_token": wb, "weight_gbs": round(wb / (el / n_tq) / 1e9, 1)}
    del dec
    torch.cuda.empty_cache()
    for name, dist_ in (("b128", "fixed"), ("b128_cfg4", "uniform")):
        B, total = 128, warmup + steps
        if dist_ == "uniform":
            ctxs = np.random.default_rng(0).integers(1, cfg.max_seq - total - 1, size=B)
        else:
            ctxs = np.full(B, 1024, dtype=np.int64)
        paged = dist_ == "uniform"
        pages = int(sum((c + total + 1 + 31) // 32 for c in ctxs)) if paged else 0
        dec = BitNetDecoder(cfg, w, batch=B, num_pages=pages, page_seed=0 if paged else None)
        if paged:
            for b in range(B):
                dec.reserve(b, int(ctxs[b]) + total + 1)
        dec.fill_kv_random(int(ctxs.max()), seed=1)
        dec.set_state([1] * B, [int(c) for c in ctxs])
        for _ in range(warmup):
            dec.step(graph=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            dec.step(graph=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ctx = int(round(float(ctxs.mean()))) + total // 2
        kern = op_timing(dec, ctx, reps=3)
        att = kern["attn"]
        out[name] = {"workload": f"decode batch 128, ctx {'1024' if dist_ == 'fixed' else 'U[1, max_seq)'}, "
                                 f"kv bf16{', paged' if paged else ''} (BASELINE configs[3])",
                     "tokens_per_s": round(B * steps / el, 1), "ms_per_step": round(1000.0 * el / steps, 4),
                     "steps": steps, "ctx_mean": int(round(float(ctxs.mean()))),
                     "roofline": {"bound": "hbm", "kernel": "attn", "achieved": att["gbs"], "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(att["gbs"] / HBM_PEAK_GBS, 4),
                                  "bytes_per_launch": att["bytes"], "us_per_launch": att["us"],
                                  "ops": {k: {"us": v["us"], "gbs": v["gbs"], "frac": round(v["gbs"] / HBM_PEAK_GBS, 4)}
                                          for k, v in kern.items()}}}
        del dec
        torch.cuda.empty_cache()
    # prefill 8 x 2048 (the batched decoder owns the KV slots)
    seqs_n, seq_len = 8, 2048
    dec = BitNetDecoder(cfg, w, batch=16)
    rng = np.random.default_rng(0)
    seqs = [(b, rng.integers(0, cfg.vocab, size=seq_len).tolist(), 0) for b in range(seqs_n)]
    n_rows = seqs_n * seq_len  # one 16384-row chunk (tools/prefill_bench.py's default)
    dec.prefill(seqs, chunk_rows=n_rows)
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dec.prefill(seqs, chunk_rows=n_rows)
        e1.record(st)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times)[1]
    n = seqs_n * seq_len
    h, i, kv = cfg.hidden, cfg.inter, cfg.kv_dim
    gemm_ops = 2.0 * n * cfg.layers * ((h + 2 * kv) * h + h * h + 2 * i * h + h * i)
    tops = gemm_ops / (ms / 1000.0) / 1e12
    out["prefill"] = {"workload": f"prefill {seqs_n} x {seq_len} tokens (BASELINE configs[2])", "ms": round(ms, 2),
                      "tokens_per_s": round(n / (ms / 1000.0), 1), "gemm_tera_ops": round(gemm_ops / 1e12, 2),
                      "roofline": {"bound": "mfma", "kernel": "whole prefill (GEMM ops over the end-to-end time)",
                                   "achieved": round(tops, 1), "peak": INT8_DENSE_PEAK_TOPS, "unit": "TOPS",
                                   "frac": round(tops / INT8_DENSE_PEAK_TOPS, 4)}}
    del dec, w
    torch.cuda.empty_cache()
    return out


def cpu_baseline(ctx: int, seconds: float, pin_cores: int = 8):
    """The CPU baseline on this host (oracle/cpu_baseline.py, run as a child process so its core
    affinity and OpenMP pool are its own): the oracle's full decode step of the 2B model shape and the
    standalone GEMV shapes, AVX512-VNNI build where the host has it, timed (1) on the process's whole
    CPU share (every physical core of its affinity mask, capped by the cgroup CPU quota) and (2)
    pinned to `pin_cores` physical cores (the reference's server pin,
    scripts/launch_sglang_bitnet.sh:61); one OpenMP thread per core, OMP_PROC_BIND=close,
    OMP_PLACES=cores. Bounded samples of `seconds` each; random weights (timing only)."""
    import subprocess
    runs = {}
    for name, cores in (("all", 0), (f"pin{pin_cores}", pin_cores)):
        env = dict(os.environ)
        cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--ctx", str(ctx), "--seconds", str(seconds),
               "--gemv-seconds", "1.0", "--cores", str(cores)]
        r = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=600)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            raise RuntimeError(f"cpu baseline ({name}) failed: {r.stderr[-1500:]}")
        runs[name] = json.loads(lines[-1])
    a, p = runs["all"], runs[f"pin{pin_cores}"]
    return {"value": a["decode"]["tokens_per_s"], "unit": "tokens/s", "cores": a["threads"], "kind": "port",
            "sample": f"oracle/wf_oracle.c orc_decode_step ({a['build']}), full 30-layer bitnet-b1.58-2B-4T shape, "
                      f"batch 1, ctx {ctx}, {a['decode']['tokens']} tokens in {a['decode']['seconds']}s (random weights)",
            "ms_per_token": a["decode"]["ms_per_token"], "cpu_model": a["cpu_model"], "isa": a["isa"],
            "omp_threads": a["threads"], "affinity_cpus": a["affinity_cpus"],
            "logical_cpus_total": a["logical_cpus_total"], "core_choice": a["core_choice"],
            "omp_proc_bind": a["omp_proc_bind"], "omp_places": a["omp_places"],
            f"pinned_{pin_cores}_cores": {"value": p["decode"]["tokens_per_s"], "omp_threads": p["threads"],
                                          "ms_per_token": p["decode"]["ms_per_token"], "gemv": p["gemv"]},
            "gemv": a["gemv"]}


def _profile_json(name: str):
    f = ROOT / "profiles" / name
    try:
        return json.loads(f.read_text()) if f.exists() else None
    except Exception:
        return None


def roofline(kern: dict, B: int, args, step_gbs: float) -> dict:
    """The `roofline` object. The dominant kernel is fixed by the committed rocprofv3 profile of this
    workload (profiles/rocprof_ops*.json, `_dominant` = the op with the largest TOTAL kernel time,
    tools/rocprof_ops.py), so the choice does not flip between near-equal ops on the live timing's
    noise; its achieved GB/s is measured live (HIP events over graph replays of its launches).
    `traffic` = PMC HBM bytes per launch (profiles/pmc_traffic*.json, FETCH_SIZE x 2 + WRITE_SIZE).
    `ops` carries every op's live fraction and its PMC traffic / algorithmic-bytes ratio; `step_frac`
    is the whole step's (weights + KV) bytes per step over the step time, against the same peak."""
    fixed_ctx = args.ctx_dist == "fixed" and args.kv == "bf16"  # the profiled workload
    suffix = "" if B < 16 else f"_b{B}"
    prof = _profile_json(f"rocprof_ops{suffix}.json") if fixed_ctx else None
    pmc = (_profile_json(f"pmc_traffic{suffix}.json") or {}) if fixed_ctx else {}
    if prof and prof.get("_dominant") in kern:
        dom_name, how = prof["_dominant"], f"largest total rocprofv3 time in profiles/{prof.get('_source')}"
    else:
        dom_name, how = max(kern, key=lambda k: kern[k]["us_per_step"]), "largest live us per step (no profile)"
    ops = {}
    for name, k in kern.items():
        t = pmc.get(name, {}).get("hbm_bytes_per_launch")
        ops[name] = {"us": k["us"], "gbs": k["gbs"], "frac": round(k["gbs"] / HBM_PEAK_GBS, 4),
                     "traffic": t, "traffic_ratio": round(t / k["bytes"], 3) if t else None,
                     "rocprof_avg_us": (prof or {}).get(name, {}).get("avg_us")}
    dom = kern[dom_name]
    return {"bound": "hbm", "achieved": dom["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(dom["gbs"] / HBM_PEAK_GBS, 4), "traffic": ops[dom_name]["traffic"],
            "kernel": dom_name, "dominant_by": how, "bytes_per_launch": dom["bytes"], "us_per_launch": dom["us"],
            "step_gbs": round(step_gbs, 1), "step_frac": round(step_gbs / HBM_PEAK_GBS, 4), "ops": ops}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from wfamd import WF_FMT_I2S, WF_FMT_TQ, _lib
    from wfamd.model import BITNET_2B, BitNetDecoder, synthetic_weights
    from wfamd.replicas import pin_host_cores, replica_rate, timed_steps

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # the CPU baseline runs in child processes BEFORE this process touches the GPU (no fork of a
    # GPU-initialised process; the host is idle while it runs)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(max(1, min(args.ctx, 4096 - args.warmup - args.steps - 2)), args.cpu_seconds)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1:
        # independent replicas: a disjoint host-core slice per rank, set before the
        # first GPU call; a host (gloo) barrier only -- no RCCL communicator exists
        pin_host_cores(local, local_world)
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    if not _lib.kernel_available():
        raise SystemExit("gfx950 HIP kernels unavailable: build with __graft_entry__.build()")

    cfg = BITNET_2B
    if args.max_seq:
        import dataclasses
        cfg = dataclasses.replace(cfg, max_seq=args.max_seq)
    B = args.batch
    wfmt = WF_FMT_TQ if args.wfmt == "tq" else WF_FMT_I2S
    total = args.warmup + args.steps
    ctx = max(1, min(args.ctx, cfg.max_seq - total - 1))
    import numpy as np
    paged = args.paged or args.ctx_dist == "uniform"
    if args.ctx_dist == "uniform":
        ctxs = np.random.default_rng(0).integers(1, cfg.max_seq - total - 1, size=B)
    else:
        ctxs = np.full(B, ctx, dtype=np.int64)
    num_pages = int(sum((c + total + 1 + 31) // 32 for c in ctxs)) if paged else 0
    w = synthetic_weights(cfg, seed=0, device="cuda")
    dec = BitNetDecoder(cfg, w, batch=B, wfmt=wfmt, num_pages=num_pages, page_seed=0 if paged else None,
                        kv_dtype=args.kv, kv_scale=(4.0 / 127, 4.0 / 127) if args.kv == "int8" else None)
    del w
    torch.cuda.empty_cache()
    if paged:
        for b in range(B):
            dec.reserve(b, int(ctxs[b]) + total + 1)
    dec.fill_kv_random(ctx, seed=1)
    dec.set_state([1] * B, [int(c) for c in ctxs])
    ctx = int(round(float(ctxs.mean())))

    for _ in range(args.warmup):
        dec.step(graph=True)
    el = timed_steps(lambda: dec.step(graph=True), args.steps, torch.cuda.synchronize,
                     dist if world > 1 else None)
    tok_s = replica_rate(B, args.steps, world, el)
    ms_step = 1000.0 * el / args.steps

    kern = {} if args.no_op_timing else op_timing(dec, ctx + total // 2)
    kv_esz = 1 if args.kv in ("fp8", "int8") else 2
    step_bytes = cfg.weight_bytes_per_token(wfmt) + B * cfg.kv_bytes_per_token(ctx + total // 2) * kv_esz // 2
    step_gbs = step_bytes / (ms_step / 1000.0) / 1e9
    roof = roofline(kern, B, args, step_gbs) if kern else None
    gemv = None if (args.no_gemv or B != 1) else gemv_bench()
    gsweep = None if (args.no_gemv or B != 1) else gemm_sweep()
    sub = None
    if rank == 0 and world == 1 and B == 1 and not args.no_sub and args.ctx_dist == "fixed":
        del dec
        torch.cuda.empty_cache()
        sub = sub_records(cfg, args.sub_steps)
        if wfmt == WF_FMT_I2S:  # the TQ batch-1 rate against this run's I2_S headline
            sub["b1_tq"]["vs_i2s"] = round(sub["b1_tq"]["tokens_per_s"] / tok_s, 4)
    if cpu:
        cpu_gemv = cpu.pop("gemv")
        if gemv:
            for k, v in cpu_gemv.items():
                gemv[k]["cpu_us"], gemv[k]["cpu_gbs"] = v["us"], v["gbs"]

    if rank == 0:
        line = {
            "metric": "decode tokens/sec + GEMV HBM GB/s, bitnet-b1.58-2B-4T, batch 1/128",
            "value": round(tok_s, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int8", "data": "synthetic",
            "config": {"workload": f"decode batch={B} (BASELINE configs[1])" if B == 1 else
                       f"decode batch={B}" + (" (BASELINE configs[3]: contexts U[1, max_seq), continuous decode)"
                                              if args.ctx_dist == "uniform" else ""),
                       "model": "bitnet-b1.58-2B-4T (random init)", "global_batch": B * world, "seq_len": ctx,
                       "parallelism": f"replicas{world}", "weights": "ternary " + ("TQ ~1.6-bit" if wfmt else "I2_S 2-bit"),
                       "activations": "int8 per-token", "lm_head": "bf16",
                       "kv": args.kv + (", paged (32-token pages)" if paged else ""),
                       **({"ctx_mean": ctx, "ctx_min": int(ctxs.min()), "ctx_max": int(ctxs.max())}
                          if args.ctx_dist == "uniform" else {})},
            "step_hbm_gbs": round(step_gbs, 1),
            "gemv_hbm_gbs": kern.get("gate_up", {}).get("gbs") if kern else None,
            "gemv": gemv, "gemm_sweep": gsweep,
            "roofline": roof, "cpu_baseline": cpu, "kernels": kern, "sub_records": sub,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
