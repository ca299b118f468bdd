"""CPU baseline of the hot path on the host cores -- BASELINE INFRASTRUCTURE ONLY (bench.py's
cpu_baseline leg runs this module in a child process, once on every core of its affinity mask and
once pinned to 8 cores like the reference's server, scripts/launch_sglang_bitnet.sh:61-67).

It times the oracle's C code (oracle/wf_oracle.c), built for the host: with -DORC_VNNI on an
AVX512-VNNI host the ternary enc-sums run on vpdpbusd and the LM head on vdpbf16ps (the
reference's own CPU ISA: legacy/src/native/bitnet_kernel.cpp:104-249; SURVEY §8d "CPU baseline":
the build's own AVX512-VNNI restatement of a1-a3), else the autovectorised scalar build
(-march=native). Random weights of the full bitnet-b1.58-2B-4T shape, bounded samples.

    python -m oracle.cpu_baseline --ctx 1024 --seconds 6 [--cores 8]   -> one JSON line

Threads and placement: --cores N pins to N distinct physical cores of the affinity mask (one
logical CPU per core, SMT siblings skipped); --cores 0 uses the process's whole CPU share: the
affinity mask capped by the cgroup CPU quota (a GPU box may show every CPU of the machine in its
mask while its quota allows a slice of them). One OpenMP thread per chosen core with
OMP_PROC_BIND=close and OMP_PLACES=cores, set before the OpenMP runtime loads.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from pathlib import Path

import numpy as np

from oracle import oracle as orc

GEMV_SHAPES = [("q_proj/o_proj", 2560, 2560), ("k_proj/v_proj", 640, 2560), ("gate/up", 6912, 2560),
               ("down", 2560, 6912)]  # scripts/benchmark_kernels.py:132-138 plus k/v


def host_info() -> dict:
    model, flags = "unknown", set()
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name") and model == "unknown":
                model = line.split(":", 1)[1].strip()
            elif line.startswith("flags") and not flags:
                flags = set(line.split(":", 1)[1].split())
    except OSError:
        pass
    isa = sorted(f for f in flags if f.startswith(("avx512", "amx")) or f in ("avx2", "avx_vnni", "fma"))
    return {"cpu_model": model, "isa": isa, "logical_cpus_total": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "_flags": flags}


def cgroup_cpu_quota() -> float | None:
    """CPUs allowed by the cgroup (v2 cpu.max, or v1 cfs quota / period); None when unlimited."""
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        p = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def physical_cores(cpus) -> list[int]:
    """One logical CPU per physical core (first sibling), in CPU order."""
    seen, out = set(), []
    for c in sorted(cpus):
        base = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
        try:
            key = (base.joinpath("physical_package_id").read_text().strip(), base.joinpath("core_id").read_text().strip())
        except OSError:
            key = ("cpu", str(c))
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def choose_cores(n: int) -> tuple[list[int], str]:
    """(cores to run on, how their count was chosen)."""
    mask = sorted(os.sched_getaffinity(0))
    phys = physical_cores(mask) or mask
    if n > 0:
        return phys[:n], f"pinned to {min(n, len(phys))} physical cores"
    quota = cgroup_cpu_quota()
    if quota is not None and int(quota) < len(phys):
        k = max(1, int(quota))
        return phys[:k], f"cgroup CPU quota {quota:g} of {len(mask)} CPUs in the affinity mask"
    return phys, f"every physical core of the {len(mask)}-CPU affinity mask"


def build_lib(flags, extra=()) -> tuple[str, str]:
    """(library name, build kind) for this host; `extra` = study defines (tools/ab_cpu_team.sh)."""
    if "avx512_vnni" in flags and "avx512bw" in flags:
        name = "liborc_vnni" + "".join("_" + d.lower() for d in extra) + ".so"
        try:
            orc.build(march="native", name=name, defines=("ORC_VNNI",) + tuple(extra))
            return name, "avx512-vnni (vpdpbusd enc-sums" + (", vdpbf16ps LM head)" if "avx512_bf16" in flags
                                                             else ", scalar-fp32 LM head)")
        except Exception:
            pass
    name = "liborc_native.so"
    try:
        orc.build(march="native", name=name)
        return name, "scalar C, -march=native autovectorised"
    except Exception:
        orc.build()
        return "liborc.so", "scalar C, x86-64-v3"


def model_arrays(ctx_room: int, rng) -> dict:
    import torch  # rope tables only (no GPU use)
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "wrinklefree-inference-engine_amd" / "python"))
    from wfamd.model import BITNET_2B as cfg, rope_tables
    H, L, HQ, HKV, D, I, V = cfg.hidden, cfg.layers, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.inter, cfg.vocab
    S = ctx_room
    lut = np.array([((v // 27) % 3) << 6 | ((v // 9) % 3) << 4 | ((v // 3) % 3) << 2 | (v % 3) for v in range(81)],
                   dtype=np.uint8)

    def tern(*shape):
        return lut[rng.integers(0, 81, size=shape, dtype=np.uint8)]

    def bf16_small(*shape):  # random bf16 bit patterns of magnitude ~0.01 (timing only)
        sign = rng.integers(0, 2, size=shape, dtype=np.uint16) << 15
        return (0x3C00 + rng.integers(0, 0x100, size=shape, dtype=np.uint16)) | sign

    def bf16_one(*shape):
        return np.full(shape, 0x3F80, dtype=np.uint16)

    cos, sin = rope_tables(D, S, cfg.rope_theta)
    return {
        "cfg": np.array([H, L, HQ, HKV, D, I, V, S], dtype=np.int64), "eps": np.float32(cfg.eps),
        "embed": bf16_small(V, H), "final_norm": bf16_one(H),
        "rope_cos": cos.view(torch.int16).numpy().view(np.uint16),
        "rope_sin": sin.view(torch.int16).numpy().view(np.uint16),
        "ln_in": bf16_one(L, H), "ln_post": bf16_one(L, H), "attn_sub": bf16_one(L, H), "ffn_sub": bf16_one(L, I),
        "wq": tern(L, H, H // 4), "wk": tern(L, HKV * D, H // 4), "wv": tern(L, HKV * D, H // 4),
        "wo": tern(L, H, H // 4), "wg": tern(L, I, H // 4), "wu": tern(L, I, H // 4), "wd": tern(L, H, I // 4),
        "wscale": np.full((L, 7), 1.75, dtype=np.float32), "_bf16_small": bf16_small,
    }


def decode_rate(libname: str, ctx: int, seconds: float) -> dict:
    rng = np.random.default_rng(0)
    a = model_arrays(ctx + 2048, rng)
    small = a.pop("_bf16_small")
    m = orc.DecodeModel(a, libname)
    L, HKV, D = m.k_cache.shape[0], m.k_cache.shape[1], m.k_cache.shape[3]
    m.k_cache[:, :, :ctx] = small(L, HKV, ctx, D)
    m.v_cache[:, :, :ctx] = small(L, HKV, ctx, D)
    m.step(1, ctx)  # warm (page in weights)
    n, t0, tok = 0, time.perf_counter(), 1
    while True:
        _, tok = m.step(tok, ctx + 1 + n)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or ctx + 2 + n >= ctx + 2048:
            break
    return {"tokens_per_s": round(n / el, 3), "ms_per_token": round(1000 * el / n, 2), "tokens": n,
            "seconds": round(el, 2)}


def gemv_rates(libname: str, seconds_per_shape: float) -> dict:
    rng = np.random.default_rng(0)
    L = orc.lib(libname)
    out = {}
    for name, N, K in GEMV_SHAPES:
        p = (rng.integers(0, 256, size=(N, K // 4), dtype=np.uint8) & 0xAA).astype(np.uint8)
        act = rng.integers(-128, 128, size=K, dtype=np.int8)
        y = np.zeros(N, np.float32)
        args = (p.ctypes.data, act.ctypes.data, 0.01, N, K, y.ctypes.data)
        L.orc_gemv_i2s(*args)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds_per_shape:
            L.orc_gemv_i2s(*args)
            n += 1
        us = 1e6 * (time.perf_counter() - t0) / n
        nbytes = N * K // 4 + K + 4 * N
        out[name] = {"us": round(us, 1), "gbs": round(nbytes / us / 1e3, 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--gemv-seconds", type=float, default=1.0)
    ap.add_argument("--cores", type=int, default=0,
                    help="pin to N physical cores of the affinity mask; 0 = the process's whole CPU share")
    ap.add_argument("--define", action="append", default=[], help="study define for the VNNI build (A/B only)")
    args = ap.parse_args()
    info = host_info()  # the mask as given, before pinning
    cores, how = choose_cores(args.cores)
    os.sched_setaffinity(0, cores)
    # one OpenMP thread per chosen core, bound (read when the OpenMP runtime loads with the library)
    os.environ.update(OMP_NUM_THREADS=str(len(cores)), OMP_PROC_BIND="close", OMP_PLACES="cores")
    info.update(cores_used=len(cores), core_choice=how, omp_proc_bind="close", omp_places="cores")
    flags = info.pop("_flags")
    libname, kind = build_lib(flags, args.define)
    threads = orc.num_threads(libname)
    res = {**info, "threads": threads, "build": kind, "vnni": bool(orc.lib(libname).orc_vnni_build()),
           "decode": decode_rate(libname, args.ctx, args.seconds),
           "gemv": gemv_rates(libname, args.gemv_seconds) if args.gemv_seconds > 0 else None}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
