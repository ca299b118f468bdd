"""CPU sanitizers (SURVEY.md §5 "race detection / sanitizers"): the oracle (oracle/wf_oracle.c, with
oracle/asan_driver.c as its command-line front end) and the fast-arithmetic check
(tools/check_fast_arith.c) built with -fsanitize=address,undefined (no recovery: the first finding
fails the run) and run on the golden fixtures' inputs; every sanitized output must equal the
regular oracle build's output bit for bit. GPU code has no sanitizer on this pool; the host side of
the HIP library is plain C++ argument checking covered by tests/test_cabi_cpu.py."""
import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

ROOT = Path(__file__).resolve().parents[1]
SAN = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"]
pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="no host C compiler")


def _env():
    e = dict(os.environ)
    # the runtime's own link-order check is off: this process may start with other preloaded objects
    e["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:abort_on_error=0:halt_on_error=1"
    e["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    e["OMP_NUM_THREADS"] = "2"
    return e


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("asan")
    exe = d / "asan_driver"
    subprocess.run(["gcc", *SAN, "-fopenmp", "-std=c11", "-ffp-contract=off", "-march=x86-64-v3", "-I", str(ROOT / "oracle"),
                    str(ROOT / "oracle" / "wf_oracle.c"), str(ROOT / "oracle" / "asan_driver.c"), "-o", str(exe), "-lm"],
                   check=True)
    return exe, d


def run(driver, *args):
    exe, _ = driver
    r = subprocess.run([str(exe), *map(str, args)], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, (args[0], r.returncode, r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]


def test_oracle_kernels_under_asan_ubsan(driver, orc):
    """Quantizers, the raw ternary GEMM, the packers and the corrected linear on the reference's
    golden inputs (tests/golden/quant, gemv, linear .npz): sanitized == golden == regular build."""
    _, d = driver
    qg = load_golden("quant")
    for i in range(3):
        x = np.ascontiguousarray(qg[f"x{i}"], np.float32)
        x.tofile(d / "x.f32")
        run(driver, "quant", x.size, d / "x.f32", d / "q.i8", d / "s.f64")
        assert np.array_equal(np.fromfile(d / "q.i8", np.int8), qg[f"q{i}"]) and np.fromfile(d / "s.f64")[0] == qg[f"s{i}"]
    rng = np.random.default_rng(1)
    xr = (rng.standard_normal((5, 640)) * rng.uniform(0.01, 3, (5, 1))).astype(np.float32)
    xr.tofile(d / "xr.f32")
    run(driver, "qrows", 5, 640, d / "xr.f32", d / "qr.i8", d / "sr.f64")
    qr, sr = orc.quantize_i8_rows(xr)
    assert np.array_equal(np.fromfile(d / "qr.i8", np.int8).reshape(5, 640), qr)
    assert np.array_equal(np.fromfile(d / "sr.f64"), sr)
    gg = load_golden("gemv")
    for i in range(3):
        w, a = np.ascontiguousarray(gg[f"p{i}"]), np.ascontiguousarray(gg[f"a{i}"])
        n, k = w.shape[0], w.shape[1] * 4
        w.tofile(d / "w.u8")
        a.tofile(d / "a.i8")
        run(driver, "gemm", a.shape[0], n, k, float(np.float32(gg[f"scale{i}"])), d / "w.u8", d / "a.i8", d / "y.f32")
        assert np.array_equal(np.fromfile(d / "y.f32", np.float32).reshape(gg[f"y{i}"].shape), gg[f"y{i}"]), i
    wt = rng.integers(-1, 2, size=(48, 384)).astype(np.float32)
    wt.tofile(d / "wt.f32")
    run(driver, "packs", 48, 384, d / "wt.f32", d / "i2s.u8", d / "tq.u8", d / "back.u8")
    p = orc.pack_i2s(wt)
    assert np.array_equal(np.fromfile(d / "i2s.u8", np.uint8).reshape(p.shape), p)
    assert np.array_equal(np.fromfile(d / "tq.u8", np.uint8).reshape(48, -1), orc.pack_tq(p))
    assert np.array_equal(np.fromfile(d / "back.u8", np.uint8).reshape(p.shape), p)
    lg = load_golden("linear")
    for i in range(3):
        x, w = np.ascontiguousarray(lg[f"x{i}"]), np.ascontiguousarray(lg[f"p{i}"])
        x.tofile(d / "xb.u16")
        w.tofile(d / "wl.u8")
        run(driver, "linear", w.shape[0], x.size, repr(float(lg[f"ws{i}"])), d / "xb.u16", d / "wl.u8", d / "yl.u16")
        assert np.array_equal(np.fromfile(d / "yl.u16", np.uint16), lg[f"y{i}"]), i


@pytest.mark.parametrize("mode,S", [(0, 300), (1, 300), (1, 1025)])
def test_oracle_attention_under_asan_ubsan(driver, orc, mode, S):
    _, d = driver
    rng = np.random.default_rng(S + mode)
    hq, hkv, D, smax = 8, 2, 128, 1040
    bf = lambda *sh: orc.f32_to_bf16(rng.standard_normal(sh).astype(np.float32))
    q, k, v = bf(hq, D), bf(hkv, smax, D), bf(hkv, smax, D)
    for n, a in (("q", q), ("k", k), ("v", v)):
        a.tofile(d / f"{n}.u16")
    run(driver, "attn", hq, hkv, D, smax, S, mode, d / "q.u16", d / "k.u16", d / "v.u16", d / "o.u16")
    ref = orc.attention_sdpa_cpu_bf16(q, k, v, S) if mode else orc.attention_gqa_bf16(q, k, v, S)
    assert np.array_equal(np.fromfile(d / "o.u16", np.uint16).reshape(hq, D), ref)


@pytest.mark.parametrize("attn_mode", [0, 1])
def test_oracle_decode_step_under_asan_ubsan(driver, orc, attn_mode):
    """Six steps of the whole decode step on the golden small model (tests/golden/decode.npz)."""
    _, d = driver
    g = load_golden("decode")
    md = d / f"model{attn_mode}"
    md.mkdir(exist_ok=True)
    cfg = [int(v) for v in g["cfg"]]
    (md / "cfg.txt").write_text(" ".join(map(str, cfg)) + f" {float(g.get('eps', np.float32(1e-5))):.9g}\n")
    for n in ("embed", "final_norm", "rope_cos", "rope_sin", "ln_in", "ln_post", "attn_sub", "ffn_sub",
              "wq", "wk", "wv", "wo", "wg", "wu", "wd"):
        np.ascontiguousarray(g[n]).tofile(md / f"{n}.bin")
    np.ascontiguousarray(g["wscale"], np.float32).tofile(md / "wscale.bin")
    toks = np.ascontiguousarray(g["tokens"], np.int32)
    toks.tofile(md / "tokens.i32")
    run(driver, "decode", md, len(toks), attn_mode)
    got = np.fromfile(md / "logits.u16", np.uint16).reshape(len(toks), -1)
    m = orc.DecodeModel(g, attn_mode=attn_mode)
    for i, t in enumerate(toks):
        ref, _ = m.step(int(t), i)
        assert np.array_equal(got[i], ref), i


def test_fast_arith_under_asan_ubsan(tmp_path):
    exe = tmp_path / "check_fast_arith"
    subprocess.run(["gcc", *SAN, "-mfma", "-o", str(exe), str(ROOT / "tools" / "check_fast_arith.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "0.002"], capture_output=True, text=True, env=_env(), timeout=600)
    print(r.stdout)
    assert r.returncode == 0 and "runtime error" not in r.stderr, (r.stdout, r.stderr[-3000:])
    assert "every bf16 x: 0 mismatches" in r.stdout
