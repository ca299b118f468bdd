"""Pin the CPU oracle (oracle/wf_oracle.c) to the reference: every oracle function is checked
against golden vectors that tests/golden/make_golden.py produced by running the reference's own
Python, plus the reference's known-answer cases. CPU only."""
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, load_golden


def test_manifest_hashes():
    man = json.loads((GOLDEN / "manifest.json").read_text())
    for name, digest in man.items():
        if name.startswith("_"):
            continue
        assert hashlib.sha256((GOLDEN / name).read_bytes()).hexdigest() == digest, name


class TestPacking:
    """a5/a6/a7: cache/bitnet_converter.py:26-77, tests/test_bitnet_core.py:21-136, kernels/native.py:181-241."""

    def test_pack_i2s_matches_reference(self, orc):
        g = load_golden("packing")
        for i in range(6):
            w, p = g[f"w{i}"], g[f"p{i}"]
            assert np.array_equal(orc.pack_i2s(w.astype(np.float32)), p), i
            k = w.shape[1]
            assert np.array_equal(orc.unpack_i2s(p, k).astype(np.int8), g[f"un{i}"]), i

    def test_pack_rounding_and_known_answers(self, orc):
        g = load_golden("packing")
        assert np.array_equal(orc.pack_i2s(g["wf"]), g["pf"])
        ka = orc.pack_i2s(g["ka_w"].astype(np.float32))
        assert np.array_equal(ka, g["ka_p"])
        assert (ka[0, 0], ka[0, 1], ka[0, 31]) == (149, 69, 86)
        ones = orc.pack_i2s(np.ones((2, 256), np.float32))
        assert np.array_equal(ones, g["ones_p"]) and np.all(ones == 170)

    def test_hf_unpack(self, orc):
        g = load_golden("packing")
        assert np.array_equal(orc.unpack_hf(g["hf_p"]).astype(np.int8), g["hf_un"])

    def test_lsb_layout(self, orc):
        g = load_golden("packing")
        assert np.array_equal(orc.pack_lsb(g["lsb_w"].astype(np.float32)), g["lsb_p"])
        assert np.array_equal(orc.unpack_lsb(g["lsb_p"]).astype(np.int8), g["lsb_w"])

    def test_tq_bijection(self, orc):
        """The ~1.6-bit device format is a bijection of I2_S (all 243 byte codes, pad handling)."""
        rng = np.random.default_rng(0)
        for n, k in [(3, 128), (5, 2560), (2, 6912), (4, 640)]:
            w = rng.integers(-1, 2, size=(n, k)).astype(np.float32)
            p = orc.pack_i2s(w)
            tq = orc.pack_tq(p)
            assert tq.shape == (n, ((k + 79) // 80) * 16)
            assert np.array_equal(orc.unpack_tq(tq, k), p)
        assert orc.tq_row_bytes(2560) == 512 and orc.tq_row_bytes(6912) == 1392
        # every base-3 code decodes back (q = ceil(v*256/243) trick)
        for v in range(243):
            q = (v * 256 + 242) // 243
            digits = []
            for _ in range(5):
                digits.append((q * 3) >> 8)
                q = (q * 3) & 0xFF
            assert sum(d * 3 ** (4 - i) for i, d in enumerate(digits)) == v


class TestQuant:
    """a3: tests/test_bitnet_core.py:139-146 and kernels/native.py:244-256."""

    def test_quantize_rne(self, orc):
        g = load_golden("quant")
        for i in range(8):
            q, s = orc.quantize_i8(g[f"x{i}"])
            assert np.array_equal(q, g[f"q{i}"]), i
            assert s == float(g[f"s{i}"]), i

    def test_quantize_trunc(self, orc):
        g = load_golden("quant")
        for i in range(8):
            q, s = orc.quantize_i8_trunc(g[f"x{i}"])
            assert np.array_equal(q, g[f"qt{i}"]), i
            assert np.float32(s) == g[f"st{i}"], i

    def test_rows_equal_per_row_calls(self, orc):
        x = np.random.default_rng(1).standard_normal((5, 640)).astype(np.float32)
        q, s = orc.quantize_i8_rows(x)
        for r in range(5):
            qr, sr = orc.quantize_i8(x[r])
            assert np.array_equal(q[r], qr) and s[r] == sr


class TestGemv:
    """a1/a2: tests/test_bitnet_core.py:149-167; known answer tests/test_bitnet_weight_loading.py:141-169."""

    def test_raw_gemv_gemm_bitexact(self, orc):
        g = load_golden("gemv")
        for i in range(7):
            y = orc.gemm_i2s(g[f"p{i}"], g[f"a{i}"], float(g[f"scale{i}"]))
            assert np.array_equal(y.view(np.uint32), g[f"y{i}"].view(np.uint32)), i

    def test_known_answer(self, orc):
        g = load_golden("gemv")
        p = orc.pack_i2s(np.ones((4, 256), np.float32))
        q, s = orc.quantize_i8(np.ones(256, np.float32))
        raw = orc.gemv_i2s(p, q, 2.0)
        assert np.array_equal(raw, g["ka_raw"]) and np.all(raw == 130048.0)
        assert s == float(g["ka_s"])
        corr = ((raw - np.float32(2.0 * q.astype(np.float32).sum())) * np.float32(s)).astype(np.float32)
        assert np.allclose(corr, g["ka_corr"]) and np.allclose(corr, 512.0)

    def test_lsb_signed(self, orc):
        g = load_golden("gemv")
        y = orc.gemv_lsb_signed(g["lsb_p"], g["lsb_a"], float(g["lsb_scale"]))
        np.testing.assert_allclose(y, g["lsb_y"], rtol=1e-6, atol=1e-6)


class TestLinearAndAttention:
    def test_corrected_linear_bitexact(self, orc):
        """a4: scripts/direct_inference_full.py:186-208 float sequence reproduced exactly."""
        g = load_golden("linear")
        for i in range(3):
            y = orc.bitnet_linear_bf16(g[f"x{i}"], g[f"p{i}"], float(g[f"ws{i}"]))
            assert np.array_equal(y, g[f"y{i}"]), i

    def test_gqa_attention(self, orc):
        """a10: F.scaled_dot_product_attention(..., enable_gqa=True) in bf16; oracle in double.
        Tolerance: relative L2 error <= 5e-3 (torch's bf16 CPU SDPA rounds P to bf16 internally)."""
        g = load_golden("attention")
        for i in range(4):
            s = int(g[f"s{i}"])
            k = g[f"k{i}"].transpose(1, 0, 2)  # [S, Hkv, D] -> [Hkv, S, D]
            v = g[f"v{i}"].transpose(1, 0, 2)
            o = orc.attention_gqa_bf16(g[f"q{i}"], k, v, s).reshape(-1)
            ref = orc.bf16_to_f32(g[f"o{i}"])
            got = orc.bf16_to_f32(o)
            rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
            assert rel < 5e-3, (i, rel)


def test_decode_step_matches_reference(orc):
    """Whole decode step (scripts/direct_inference_full.py:267-302) on the small golden model.
    Tolerance: relative L2 error of bf16 logits <= 1e-3 (torch CPU reduction order and
    bf16 SDPA internals differ from the oracle's double accumulation; quantization boundaries can
    flip single int8 codes), and the greedy token must agree."""
    g = load_golden("decode")
    m = orc.DecodeModel(g)
    for pos, tok in enumerate(g["tokens"]):
        logits, nxt = m.step(int(tok), pos)
        ref = orc.bf16_to_f32(g["logits"][pos])
        got = orc.bf16_to_f32(logits)
        rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
        assert rel < 1e-3, (pos, rel)
        top2 = np.sort(ref)[-2:]
        if top2[1] - top2[0] > 0.05 * abs(top2[1]):
            assert nxt == int(np.argmax(ref)), pos


def _bits_to_f32(bits: np.ndarray, half: bool) -> np.ndarray:
    if half:
        return bits.view(np.float16).astype(np.float32)
    return (bits.astype(np.uint32) << 16).view(np.float32)


def _round_dt(x: np.ndarray, dt: str) -> np.ndarray:
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    return t.to(getattr(torch, dt)).float().numpy()


class TestMsbLinearMethod:
    """a12: sglang_backend/bitnet_quantization.py:69-153, :211-252, :366-409."""

    def test_ternarize_matches_reference(self, orc):
        g = load_golden("msb")
        for name in ("w32", "wb", "wh", "wz", "wt"):
            dt = ["float32", "bfloat16", "float16"][int(g[f"{name}_dtype"])]
            got = orc.msb_ternarize(g[f"{name}_in"], float(g[f"{name}_scale"]), dt)
            assert np.array_equal(got, g[f"{name}_packed"]), name
        assert float(g["wz_scale"]) == 1.0 and np.all(g["wz_packed"] == 0x55)
        # the exact +-0.5 ties of row 0 (w / max|w| with max = 2): 0.5 -> 0, -0.5 -> 0, 0.4995 -> 0
        assert g["wt_packed"][0, 0] == (2 << 6 | 1 << 4 | 1 << 2 | 1)

    def test_dequant_matches_reference(self, orc):
        g = load_golden("msb")
        for name in ("w32", "wb", "wh", "wz", "wt"):
            assert np.array_equal(orc.msb_dequant(g[f"{name}_packed"], float(g[f"{name}_scale"])), g[f"{name}_deq"])

    @pytest.mark.parametrize("tag,dt", [("bf", "bfloat16"), ("h", "float16")])
    def test_linear_matches_reference(self, orc, tag, dt):
        """The reference multiplies rnd(+-scale) weights in its GEMM order; the oracle sums in double and
        applies rnd(scale) once: equal up to one rounding of the output (1 ulp of the compute dtype)."""
        g = load_golden("msb")
        ws = float(_round_dt(np.array([g["lin_scale"]], np.float32), dt)[0])
        bias = _round_dt(g["lin_bias"], dt)
        ulp = 2.0 ** -7 if tag == "bf" else 2.0 ** -10
        for m in (1, 3, 32):
            x = _round_dt(g[f"lin_x{m}"], dt)
            for key, b in ((f"lin_y{m}_{tag}", None), (f"lin_yb{m}_{tag}", bias)):
                ref = _bits_to_f32(g[key], tag == "h")
                got = orc.msb_linear(g["lin_packed"], ws, x, b, dt)
                err = np.abs(got - ref)
                assert np.all(err <= ulp * np.abs(ref) + 1e-3 * ws), (key, float(err.max()))
                assert np.mean(got == ref) > 0.9, key


class TestActivationSparsity:
    """Our device-op restatement of sglang_backend/activation_sparsity.py (host logic, runs on CPU
    tensors too) against the reference's outputs (threshold :83-99, top-k :102-133, adaptive
    :136-195; disabled by default :240-242)."""

    def test_masks_match_reference(self):
        import torch
        from wrinklefree_inference.sglang_backend import activation_sparsity as sp
        g = load_golden("msb")
        x = torch.from_numpy(g["sp_x"])
        y, r = sp.apply_top_k_sparsity(x, 0.4)
        assert np.array_equal(y.numpy(), g["sp_topk"]) and r == pytest.approx(float(g["sp_topk_r"]))
        y, r = sp.apply_threshold_sparsity(x, 0.5)
        assert np.array_equal(y.numpy(), g["sp_thr"]) and r == pytest.approx(float(g["sp_thr_r"]))
        y, r = sp.apply_adaptive_sparsity(x, 0.3, 0.7)
        assert np.array_equal(y.numpy(), g["sp_adapt"]) and r == pytest.approx(float(g["sp_adapt_r"]))
        cfg = sp.get_qsparse_config()
        y, r = sp.apply_sparsity(x, cfg)
        assert np.array_equal(y.numpy(), g["sp_topk"]) and cfg.get_average_sparsity() == pytest.approx(0.6)
        y, r = sp.apply_sparsity(x, sp.get_default_config())
        assert y is x and r == 0.0


def test_sdpa_cpu_bf16_restatement_vs_torch(orc):
    """The reference's attention call (scripts/direct_inference_full.py:241) as it runs: torch
    2.10's CPU flash SDPA on bf16 (a third-party dependency; tests/golden/sdpa_probe.py). The
    oracle's restatement (orc_attention_sdpa_cpu_bf16: 512-key blocks, running max, fexp_u20,
    bf16 probabilities, unrounded sums) against torch's own outputs over block edges (1, 15-17,
    511-513, 527 keys), the decode_full geometry (961 keys, 20 / 5 heads), 1024-4096 keys and
    peaky / flat scores: <= 0.1 % of the bf16 elements differ, each head within 2e-3 rel-L2 (the
    QK / P.V GEMM summation order of oneDNN is unpublished; those elements are fp32-order ties).
    The exact softmax rounded once differs in > 20 % of them, so the fixture discriminates."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    import sdpa_probe as sp
    z = load_golden("sdpa_cpu_bf16")
    assert str(z["input_sha256"]) == sp.digest(), "regenerated SDPA inputs differ from the fixture's"
    assert int(z["backend"]) == 1  # torch._fused_sdp_choice: FLASH_ATTENTION
    mis = tot = mis_exact = 0
    for c in sp.CASES:
        q, k, v = sp.inputs(*c)
        qb, kb, vb = sp.bits(q[0, :, 0]), sp.bits(k[0]), sp.bits(v[0])
        o = orc.attention_sdpa_cpu_bf16(qb, kb, vb, c[1])
        ref = z[f"out_{c[0]}"]
        of, rf = orc.bf16_to_f32(o), orc.bf16_to_f32(ref)
        for h in range(c[2]):
            err = np.linalg.norm(of[h] - rf[h]) / np.linalg.norm(rf[h])
            assert err <= 2e-3, (c, h, err)
        mis += int((o != ref).sum())
        tot += o.size
        mis_exact += int((orc.attention_gqa_bf16(qb, kb, vb, c[1]) != ref).sum())
    print(f"SDPA restatement: {mis} / {tot} bf16 elements differ from torch; exact softmax: {mis_exact}")
    assert mis <= 1e-3 * tot, (mis, tot)
    assert mis_exact >= 0.2 * tot, (mis_exact, tot)
    # fexp_u20 is a ~1e-4-accurate exponential: fexp_u20(0) = 0.9999466 (the row maximum's own term
    # of the sum; its bf16 P rounds to 1.0), flushed to 0 below ln(FLT_MIN)
    x = np.array([0.0, -1.0, -2.5, -10.0, -87.0, -88.0, -200.0], np.float32)
    e = orc.fexp_u20(x)
    assert e[0] == np.float32(0.9999466) and e[-1] == 0.0 and e[-2] == 0.0
    assert np.allclose(e[:5], np.exp(x[:5].astype(np.float64)), rtol=1.5e-4, atol=0)
