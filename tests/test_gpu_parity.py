"""GPU parity: every HIP kernel, called through the C-ABI, against the reference's golden vectors
and the CPU oracle on the same seeded inputs. Integer/byte/index work is bit-exact; bf16 outputs
use relative-L2 tolerances stated per test."""
import math

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from wfamd import _lib
    assert _lib.kernel_available(), "gfx950 kernels must load on the GPU box (no fallback)"
    torch.cuda.set_device(0)


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def bits(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


# ------------------------------------------------------------------------------------------------
# a1/a2 raw GEMV/GEMM
# ------------------------------------------------------------------------------------------------
def test_gemv_gemm_golden_bitexact():
    from wfamd import ops
    g = load_golden("gemv")
    for i in range(7):
        m, n, k = (int(v) for v in g[f"shape{i}"])
        if k % 128:
            with pytest.raises(ValueError):
                ops.bitnet_gemm(cu(g[f"p{i}"]), cu(g[f"a{i}"]), float(g[f"scale{i}"]))
            continue
        y = ops.bitnet_gemm(cu(g[f"p{i}"]), cu(g[f"a{i}"]), float(g[f"scale{i}"])).cpu().numpy()
        assert np.array_equal(y.view(np.uint32), g[f"y{i}"].view(np.uint32)), i
        if m == 1:
            y1 = ops.bitnet_gemv(cu(g[f"p{i}"]), cu(g[f"a{i}"][0]), float(g[f"scale{i}"])).cpu().numpy()
            assert np.array_equal(y1, g[f"y{i}"][0]), i


@pytest.mark.parametrize("n,k", [(2560, 2560), (640, 2560), (6912, 2560), (2560, 6912), (13824, 2560), (3840, 2560)])
def test_gemv_model_shapes_vs_oracle(orc, n, k):
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    rng = np.random.default_rng(n * 7 + k)
    p = rng.integers(0, 81, size=(n, k // 4))
    lut = np.array([((v // 27) % 3) << 6 | ((v // 9) % 3) << 4 | ((v // 3) % 3) << 2 | (v % 3) for v in range(81)],
                   dtype=np.uint8)
    p = lut[p]
    a = rng.integers(-128, 128, size=k).astype(np.int8)
    ref = orc.gemv_i2s(p, a, 0.01)
    y = ops.bitnet_gemv(cu(p), cu(a), 0.01).cpu().numpy()
    assert np.array_equal(y, ref)
    # the ~1.6-bit TQ format gives the identical raw result
    tq = ops.i2s_to_tq(cu(p))
    assert np.array_equal(tq.cpu().numpy(), orc.pack_tq(p))
    y2 = ops.bitnet_gemm_ex(tq, cu(a), 0.01, WF_FMT_TQ, in_features=k).cpu().numpy()
    assert np.array_equal(y2, ref)
    assert np.array_equal(ops.tq_to_i2s(tq, k).cpu().numpy(), p)


@pytest.mark.parametrize("n,k", [(1, 128), (5, 1280), (63, 8192), (640, 6912), (1001, 2560), (17, 7936)])
def test_gemv_rows_ragged_vs_oracle(orc, n, k):
    """The wave-per-row GEMV (k_gemv_rows: a row split over 1, 2 or 4 waves, ragged last block, 1-2
    chunks per lane) bit-exact with the oracle, I2_S and TQ, including row counts that leave part of
    the last block idle and K at the 8192-element limit of the LDS image."""
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    rng = np.random.default_rng(n + k)
    c = rng.integers(0, 3, size=(n, k // 4, 4)).astype(np.uint8)
    p = np.ascontiguousarray((c[..., 0] << 6) | (c[..., 1] << 4) | (c[..., 2] << 2) | c[..., 3])
    a = rng.integers(-128, 128, size=k).astype(np.int8)
    ref = orc.gemv_i2s(p, a, 0.37)
    assert np.array_equal(ops.bitnet_gemv(cu(p), cu(a), 0.37).cpu().numpy(), ref)
    tq = ops.i2s_to_tq(cu(p))
    assert np.array_equal(ops.bitnet_gemm_ex(tq, cu(a), 0.37, WF_FMT_TQ, in_features=k).cpu().numpy(), ref)


@pytest.mark.parametrize("m", [2, 3, 5, 8, 16, 33, 128, 600])
def test_gemm_batches_vs_oracle(orc, m):
    """VALU path (M < 16) and int8-MFMA path (M >= 16, wf_mfma.hip): bit-exact vs the oracle."""
    from wfamd import ops
    rng = np.random.default_rng(m)
    w = rng.integers(-1, 2, size=(320, 1280)).astype(np.float32)
    p = orc.pack_i2s(w)
    a = rng.integers(-128, 128, size=(m, 1280)).astype(np.int8)
    y = ops.bitnet_gemm(cu(p), cu(a), 1.7).cpu().numpy()
    assert np.array_equal(y, orc.gemm_i2s(p, a, 1.7))
    # GEMV == GEMM row consistency (tests/test_bitnet_weight_loading.py:270-302)
    y0 = ops.bitnet_gemv(cu(p), cu(a[0]), 1.7).cpu().numpy()
    assert np.array_equal(y0, y[0])


def test_known_answer_and_errors():
    """tests/test_bitnet_weight_loading.py:141-169: W=1, x=1, ws=2 -> raw 130048, corrected 2*K."""
    from wfamd import ops
    g = load_golden("gemv")
    p = ops.pack_i2s(torch.ones(4, 256, device="cuda"))
    q, s = ops.quantize_activations_i8(torch.ones(256, device="cuda"))
    raw = ops.bitnet_gemv(p, q, 2.0).cpu().numpy()
    assert np.array_equal(raw, g["ka_raw"]) and s == float(g["ka_s"])
    corr = (torch.from_numpy(raw) - 2.0 * q.float().sum().item()) * s
    assert np.allclose(corr.numpy(), g["ka_corr"])
    with pytest.raises(ValueError):
        ops.bitnet_gemv(torch.zeros(4, 40, dtype=torch.uint8, device="cuda"), torch.zeros(160, dtype=torch.int8,
                                                                                          device="cuda"), 1.0)
    with pytest.raises(ValueError):
        ops.bitnet_gemv(torch.zeros(4, 64, dtype=torch.uint8, device="cuda"), torch.zeros(256, dtype=torch.float32,
                                                                                          device="cuda"), 1.0)


def test_host_tensors_roundtrip_through_gpu():
    """Reference callers pass host tensors to the sgl-kernel ops: same values, returned on the host."""
    from sgl_kernel.quantization import bitnet_gemv, bitnet_quantize_activations
    g = load_golden("gemv")
    y = bitnet_gemv(torch.from_numpy(g["p1"]), torch.from_numpy(g["a1"][0]), float(g["scale1"]))
    assert not y.is_cuda and np.array_equal(y.numpy(), g["y1"][0])
    q, s = bitnet_quantize_activations(torch.from_numpy(load_golden("quant")["x0"]))
    assert not q.is_cuda
    y2 = torch.ops.sgl_kernel.bitnet_gemv_cpu(torch.from_numpy(g["p1"]).cuda(), torch.from_numpy(g["a1"][0]).cuda(),
                                              float(g["scale1"]))
    assert np.array_equal(y2.cpu().numpy(), g["y1"][0])


# ------------------------------------------------------------------------------------------------
# a3 quantizers
# ------------------------------------------------------------------------------------------------
def test_quantize_golden_bitexact():
    from wfamd import ops
    g = load_golden("quant")
    for i in range(8):
        x = cu(g[f"x{i}"])
        q, s = ops.quantize_activations_i8(x)
        assert np.array_equal(q.cpu().numpy(), g[f"q{i}"]), i
        assert s == float(g[f"s{i}"]), i
        qt, st = ops.quantize_activations_trunc(x)
        assert np.array_equal(qt.cpu().numpy(), g[f"qt{i}"]), i
        assert np.float32(st) == g[f"st{i}"], i
        # bf16 input path
        xb = x.to(torch.bfloat16)
        qb, sb = ops.quantize_activations_i8(xb)
        from oracle import oracle as orc
        qo, so = orc.quantize_i8(xb.float().cpu().numpy())
        assert np.array_equal(qb.cpu().numpy(), qo) and sb == so


def test_quantize_half_integer_boundaries(orc):
    """The fast quantizer (quant8: x * (1/s) with an exact-divide fallback near x.5, used by every
    decode-step GEMV prologue) against the oracle's IEEE divide on inputs packed around the
    rounding boundaries x/s = k + 0.5 (tests/test_bitnet_core.py:139-146 semantics), bit-exact."""
    from wfamd import ops
    m = np.float32(3.7)
    sf = np.float32(np.float64(m) / 127.0)
    k = np.arange(-127, 127, dtype=np.float64) + 0.5
    vals = [np.float32(m), -np.float32(m)]
    for rel in (-3, -2, -1, 0, 1, 2, 3):
        base = (k * np.float64(sf)).astype(np.float32)
        vals.append(np.nextafter(base, np.float32(np.inf) * np.sign(rel)) if rel else base)
        for _ in range(abs(rel) - 1):
            vals[-1] = np.nextafter(vals[-1], np.float32(np.inf) * np.sign(rel))
    x = np.concatenate([np.atleast_1d(v) for v in vals]).astype(np.float32)
    x = x[np.abs(x) <= m]
    pad = (-x.size) % 8
    x = np.concatenate([x, np.zeros(pad + 8, np.float32)])  # 8-wide body + scalar tail both run
    x = np.concatenate([x, np.float32([0.25, -0.5, 1.0])])
    q, s = ops.quantize_activations_i8(cu(x))
    qo, so = orc.quantize_i8(x)
    assert s == so
    assert np.array_equal(q.cpu().numpy(), qo)


def test_quantize_rows_vs_oracle(orc):
    from wfamd import ops
    x = np.random.default_rng(3).standard_normal((7, 2560)).astype(np.float32) * 5
    q, s = ops.quantize_activations_rows(cu(x))
    qo, so = orc.quantize_i8_rows(x)
    assert np.array_equal(q.cpu().numpy(), qo)
    assert np.array_equal(s.cpu().numpy(), so)


# ------------------------------------------------------------------------------------------------
# formats
# ------------------------------------------------------------------------------------------------
def test_pack_formats_golden():
    from wfamd import ops
    g = load_golden("packing")
    for i in range(4):  # K % 128 == 0 cases
        p = ops.pack_i2s(cu(g[f"w{i}"].astype(np.float32))).cpu().numpy()
        assert np.array_equal(p, g[f"p{i}"]), i
    # HF [N/4, K] -> I2_S through the reference's unpack+pack (incl. invalid code 3)
    rng = np.random.default_rng(5)
    hf = rng.integers(0, 256, size=(32, 256)).astype(np.uint8)
    from oracle import oracle as orc
    ref = orc.pack_i2s(orc.unpack_hf(hf))
    assert np.array_equal(ops.hf_to_i2s(cu(hf)).cpu().numpy(), ref)


def test_lsb_native_kernel_golden():
    from wrinklefree_inference.kernels.native import build_kernel
    g = load_golden("gemv")
    k = build_kernel()
    y = k.gemv(g["lsb_p"], g["lsb_a"], float(g["lsb_scale"]))
    np.testing.assert_allclose(y, g["lsb_y"], rtol=1e-6, atol=1e-6)
    assert k.num_threads() > 0


# ------------------------------------------------------------------------------------------------
# KV cache (a8/a9/a11)
# ------------------------------------------------------------------------------------------------
def test_kvcache_golden_all_dtypes():
    from wrinklefree_inference.kv_cache import KVCache, KVCacheConfig, KVCacheDtype
    g = load_golden("kv")
    for name in ["BF16", "FP16", "FP32", "INT8", "FP8_E4M3"]:
        cfg = KVCacheConfig(max_seq_len=32, num_layers=2, num_heads=4, head_dim=16, dtype=KVCacheDtype[name])
        c = KVCache(cfg)
        c.update(1, torch.from_numpy(g[f"{name}_k1"]), torch.from_numpy(g[f"{name}_v1"]), 0)
        c.update(1, torch.from_numpy(g[f"{name}_k2"]), torch.from_numpy(g[f"{name}_v2"]), 5)
        kg, vg = c.get(1)
        assert np.array_equal(kg.float().cpu().numpy(), g[f"{name}_kget"]), name
        assert np.array_equal(vg.float().cpu().numpy(), g[f"{name}_vget"]), name
        st = c.cache[1, :, :8]
        st = st.float() if name in ("BF16", "FP16", "FP32") else st.view(torch.int8)
        assert np.array_equal(st.cpu().numpy(), g[f"{name}_storage"]), name
        assert np.array_equal(c.k_scales.cpu().numpy(), g[f"{name}_kscale"]), name
        assert np.array_equal(c.v_scales.cpu().numpy(), g[f"{name}_vscale"]), name


def test_attention_with_kv_cache_golden():
    """kv_cache.py:316-369 with a float32 query; tolerance rel-L2 1e-5 (fp32 summation order)."""
    from wrinklefree_inference.kv_cache import KVCache, KVCacheConfig, KVCacheDtype, attention_with_kv_cache
    g = load_golden("kv")
    c = KVCache(KVCacheConfig(max_seq_len=64, num_layers=1, num_heads=4, head_dim=32, dtype=KVCacheDtype.BF16))
    for pos in range(6):
        o = attention_with_kv_cache(torch.from_numpy(g["att_q"][pos]), c, 0, torch.from_numpy(g["att_k"][pos]),
                                    torch.from_numpy(g["att_v"][pos]), pos)
        assert o.shape == (1, 4, 1, 32)
        assert rel_l2(o.numpy(), g["att_o"][pos]) < 1e-5, pos


def test_kv_manager_scatter_gather():
    from sgl_kernel.kvcache import KVCacheManager
    g = load_golden("kv")
    m = KVCacheManager(num_layers=3, num_heads=2, head_dim=8, page_size=16, max_pages=10)
    a = m.allocate_pages(4)
    m.free_pages(a[1:3])
    b = m.allocate_pages(3)
    m.scatter_kv(torch.from_numpy(g["pg_k"]).reshape(3, -1), torch.from_numpy(g["pg_v"]).reshape(3, -1), b,
                 torch.zeros(3, dtype=torch.int32), 2)
    ko, vo = torch.zeros(3, 16), torch.zeros(3, 16)
    m.gather_kv(ko, vo, b, torch.zeros(3, dtype=torch.int32), 2)
    assert np.array_equal(ko.reshape(3, 2, 8).numpy(), g["pg_ko"])
    assert np.array_equal(vo.reshape(3, 2, 8).numpy(), g["pg_vo"])
    # reference shape: BitNet 20 heads x 128, 32 layers, all layers independent (tests/test_kv_cache_cpp.py:347-373)
    m = KVCacheManager(num_layers=32, num_heads=20, head_dim=128, page_size=256, max_pages=100)
    pages = m.allocate_pages(8)
    ks = [torch.randn(8, 2560, device="cuda") for _ in range(32)]
    vs = [torch.randn(8, 2560, device="cuda") for _ in range(32)]
    for l in range(32):
        m.scatter_kv(ks[l], vs[l], pages, None, l)
    for l in range(32):
        ko = torch.zeros(8, 2560, device="cuda")
        vo = torch.zeros(8, 2560, device="cuda")
        m.gather_kv(ko, vo, pages, None, l)
        assert torch.equal(ko, ks[l]) and torch.equal(vo, vs[l])
    bad = torch.tensor([0, 999], dtype=torch.int32)
    m.scatter_kv(ks[0][:2], vs[0][:2], bad, None, 0)
    assert m.invalid_page_count() == 1


# ------------------------------------------------------------------------------------------------
# decode attention (a10)
# ------------------------------------------------------------------------------------------------
def test_gqa_attention_golden():
    """F.scaled_dot_product_attention(enable_gqa) in bf16 (golden) vs the HIP kernel: rel-L2 <= 5e-3."""
    from wfamd import ops
    g = load_golden("attention")
    for i in range(4):
        s = int(g[f"s{i}"])
        q = cu(g[f"q{i}"].astype(np.int16)).view(torch.bfloat16).reshape(1, 20, 128)
        k = cu(g[f"k{i}"].astype(np.int16)).view(torch.bfloat16)  # [S, Hkv, D]
        v = cu(g[f"v{i}"].astype(np.int16)).view(torch.bfloat16)
        o = ops.decode_attention(q, k, v, kv_strides=(0, 128, 5 * 128), B=1, Hq=20, Hkv=5, D=128, S=s)
        got = o.float().cpu().numpy().reshape(-1)
        ref = (g[f"o{i}"].astype(np.uint32) << 16).view(np.float32)
        assert rel_l2(got, ref) < 5e-3, (i, rel_l2(got, ref))


@pytest.mark.parametrize("S,B", [(4096, 1), (1000, 3), (64, 128)])
def test_decode_attention_vs_oracle(orc, S, B):
    """Long contexts / batches with ragged lengths vs the double-precision oracle: rel-L2 <= 4e-3 (bf16 out)."""
    from wfamd import ops
    rng = np.random.default_rng(S + B)
    Hq, Hkv, D = 20, 5, 128
    k = torch.randn(B, Hkv, S, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device="cuda").to(torch.bfloat16)
    q = torch.randn(B, Hq, D, device="cuda").to(torch.bfloat16)
    lens = torch.from_numpy(rng.integers(1, S + 1, size=B).astype(np.int32))
    lens[0] = S
    o = ops.decode_attention(q, k, v, kv_strides=(Hkv * S * D, S * D, D), B=B, Hq=Hq, Hkv=Hkv, D=D, S=S,
                             seq_lens=lens.cuda())
    for b in range(min(B, 4)):
        ref = orc.attention_gqa_bf16(bits(q[b]), bits(k[b]), bits(v[b]), int(lens[b]))
        assert rel_l2(orc.bf16_to_f32(bits(o[b])), orc.bf16_to_f32(ref)) < 4e-3, b


# ------------------------------------------------------------------------------------------------
# whole decode step (§8f rank 4)
# ------------------------------------------------------------------------------------------------
def _small_decoder(wfmt, batch=1):
    from wfamd.model import BitNetConfig, BitNetDecoder, weights_from_arrays
    g = load_golden("decode")
    H, L, HQ, HKV, D, I, V, S = (int(v) for v in g["cfg"])
    cfg = BitNetConfig(hidden=H, layers=L, n_heads=HQ, n_kv_heads=HKV, head_dim=D, inter=I, vocab=V, max_seq=S)
    return g, BitNetDecoder(cfg, weights_from_arrays(g), batch=batch, wfmt=wfmt)


@pytest.mark.parametrize("wfmt", [0, 1])
def test_decode_steps_match_reference(orc, wfmt):
    """Six decode tokens through the fused, graph-replayed step vs the reference golden logits
    (scripts/direct_inference_full.py:267-302 run on the reference's functions) and vs the oracle.
    Tolerance: rel-L2 of bf16 logits <= 1e-3; greedy token identical when the top-2 gap is clear."""
    g, dec = _small_decoder(wfmt)
    m = orc.DecodeModel(g, attn_mode=1)  # batch 1: the reference's SDPA (k_attn_sdpa)
    for pos, tok in enumerate(g["tokens"]):
        dec.set_state([int(tok)], [pos])
        dec.step(graph=True)
        torch.cuda.synchronize()
        got = orc.bf16_to_f32(bits(dec.logits[0]))
        ref = orc.bf16_to_f32(g["logits"][pos])
        assert rel_l2(got, ref) < 1e-3, (pos, rel_l2(got, ref))
        ologits, onext = m.step(int(tok), pos)
        assert rel_l2(got, orc.bf16_to_f32(ologits)) < 1e-3
        top2 = np.sort(ref)[-2:]
        if top2[1] - top2[0] > 0.05 * abs(top2[1]):
            assert int(dec.tokens[0].item()) == int(np.argmax(ref))
        assert int(dec.positions[0].item()) == pos + 1
    # the cache holds exactly what the reference wrote: compare K/V of layer 0 at the last position
    kref = m.k_cache[0, :, len(g["tokens"]) - 1]
    kgot = bits(dec.k_cache[0, 0, :, len(g["tokens"]) - 1])
    assert rel_l2(orc.bf16_to_f32(kgot), orc.bf16_to_f32(kref)) < 1e-2


def test_decode_graph_equals_eager_and_batch_rows_independent():
    g, dec1 = _small_decoder(1, batch=1)
    _, dec2 = _small_decoder(1, batch=1)
    _, decb = _small_decoder(1, batch=4)
    toks = [int(t) for t in g["tokens"]]
    dec1.set_state([toks[0]], [0])
    dec2.set_state([toks[0]], [0])
    decb.set_state([toks[0]] * 4, [0] * 4)
    for _ in range(4):
        dec1.step(graph=True)
        dec2.step(graph=False)
        decb.step(graph=True)
    torch.cuda.synchronize()
    assert torch.equal(dec1.logits, dec2.logits)
    assert torch.equal(dec1.tokens, dec2.tokens)
    for b in range(4):
        assert torch.equal(decb.logits[b], dec1.logits[0])
        assert int(decb.tokens[b]) == int(dec1.tokens[0])


@pytest.mark.parametrize("B,wfmt", [(5, 1), (6, 0)])
def test_decode_small_batch_distinct_rows_match_single(B, wfmt):
    """Batch 2..15 runs the batch-1 kernels per row (GEMV blocks per row, one attention block per
    (split, head, sequence) with the per-(sequence, head) merge ticket, the LM head stream with 1 or 2
    rows per block): every row, each with its own start token, must equal a batch-1 run of that
    token bit for bit over 4 greedy steps (distinct rows catch a ticket or row index mixed across
    sequences, which identical rows would hide)."""
    g, decb = _small_decoder(wfmt, batch=B)
    toks = [int(t) for t in g["tokens"]]
    starts = [toks[(3 * b + 1) % len(toks)] for b in range(B)]
    assert len(set(starts)) > 1
    decb.set_state(starts, [0] * B)
    singles = {}
    for t in sorted(set(starts)):
        _, d1 = _small_decoder(wfmt, batch=1)
        d1.set_state([t], [0])
        singles[t] = d1
    for _ in range(4):
        decb.step(graph=True)
        for d1 in singles.values():
            d1.step(graph=True)
        torch.cuda.synchronize()
        for b in range(B):
            d1 = singles[starts[b]]
            assert torch.equal(decb.logits[b], d1.logits[0]), b
            assert int(decb.tokens[b]) == int(d1.tokens[0]), b


def test_decode_batched_mfma_rows_match_single():
    """Batch >= 16 runs the int8-MFMA GEMMs, the bf16-MFMA LM head and the row argmax; every row
    (its own start token, positions 0..3) must match a batch-1 run of the same sequence: logits
    within 1e-4 rel-L2 (the LM head sums in a different fp32 order), same greedy tokens when the
    top-2 gap is clear."""
    g, decb = _small_decoder(0, batch=24)
    toks = [int(t) for t in g["tokens"]]
    starts = [toks[b % len(toks)] for b in range(24)]
    decb.set_state(starts, [0] * 24)
    singles = {}
    for t in sorted(set(starts)):
        _, d1 = _small_decoder(0, batch=1)
        d1.set_state([t], [0])
        singles[t] = d1
    for step in range(4):
        decb.step(graph=True)
        for d1 in singles.values():
            d1.step(graph=True)
        torch.cuda.synchronize()
        for b in range(24):
            ref = singles[starts[b]]
            got = decb.logits[b].float().cpu().numpy()
            exp = ref.logits[0].float().cpu().numpy()
            assert rel_l2(got, exp) < 1e-4, (step, b, rel_l2(got, exp))
            top2 = np.sort(exp)[-2:]
            if top2[1] - top2[0] > 1e-2 * abs(top2[1]):
                assert int(decb.tokens[b]) == int(ref.tokens[0]), (step, b)
            assert int(decb.positions[b]) == step + 1


@pytest.mark.parametrize("m", [3, 40, 300])
def test_bitnet_linear_native_patch(m):
    """kernels/bitnet_patch.py BitNetLinearNative on the HIP kernels equals the reference formula
    (per-tensor quantize, scale = ws * act_scale, raw blocked-layout kernel, no correction): the
    reference's batched linear (kernels/bitnet_patch.py:55-78) pinned at M > 1, on the batched GEMV
    (M < 16) and the int8 matrix-core GEMM (M >= 16) -- one activation scale for the whole tensor."""
    from oracle import oracle as orc
    from wrinklefree_inference.kernels.bitnet_patch import BitNetLinearNative
    rng = np.random.default_rng(9)
    w = rng.integers(-1, 2, size=(256, 512)).astype(np.float32)
    p = orc.pack_i2s(w)
    lin = BitNetLinearNative(512, 256, cu(p), torch.tensor(1.5))
    x = rng.standard_normal((m, 512)).astype(np.float32)
    x[m // 2, 7] = 9.0  # one outlier row sets the shared scale
    y = lin(cu(x)).cpu().numpy()
    q, s = orc.quantize_i8(x)
    ref = orc.gemm_i2s(p, q, np.float32(1.5 * s))
    assert np.array_equal(y, ref)
    y1 = lin(cu(x[:1])).cpu().numpy()
    q1, s1 = orc.quantize_i8(x[:1])
    assert np.array_equal(y1, orc.gemm_i2s(p, q1, np.float32(1.5 * s1)))


# ------------------------------------------------------------------------------------------------
# f1: fused BitNetLinear (scripts/direct_inference_full.py:186-208)
# ------------------------------------------------------------------------------------------------
def test_bitnet_linear_golden_bitexact():
    """One row: quantize + ternary GEMV + correction in one launch, bf16 bit-exact with the vectors
    the reference's own functions produced (tests/golden/make_golden.py gen_linear)."""
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    g = load_golden("linear")
    for i in range(3):
        p, x, ws, y = g[f"p{i}"], g[f"x{i}"], float(g[f"ws{i}"]), g[f"y{i}"]
        xt = cu(x.view(np.int16)).view(torch.bfloat16)
        out = ops.bitnet_linear(xt, cu(p), ws)
        assert np.array_equal(bits(out), y), i
        tq = ops.i2s_to_tq(cu(p))
        out_tq = ops.bitnet_linear(xt, tq, ws, WF_FMT_TQ, in_features=x.shape[0])
        assert np.array_equal(bits(out_tq), y), i


@pytest.mark.parametrize("m,n,k", [(1, 2560, 2560), (3, 100, 640), (7, 640, 2560), (16, 2560, 2560),
                                   (40, 136, 6912), (129, 3840, 2560), (300, 13824, 2560)])
def test_bitnet_linear_rows_vs_oracle(orc, m, n, k):
    """Every row bf16 bit-exact with the oracle's per-row linear (M < 16: GEMV prologue path;
    M >= 16: row quantizer + int8 MFMA GEMM), ragged N, strided input rows."""
    from wfamd import ops
    rng = np.random.default_rng(m * 131 + n + k)
    w = rng.integers(-1, 2, size=(n, k)).astype(np.float32)
    p = orc.pack_i2s(w)
    x = (rng.standard_normal((m, k + 64)) * rng.uniform(0.05, 3.0, size=(m, 1))).astype(np.float32)
    x[0, 5] = 40.0  # an outlier sets a row's scale
    xb = orc.f32_to_bf16(x)
    xt = cu(xb.view(np.int16)).view(torch.bfloat16)[:, :k]  # row stride k + 64
    out = bits(ops.bitnet_linear(xt, cu(p), 1.25))
    for r in range(m):
        ref = orc.bitnet_linear_bf16(np.ascontiguousarray(xb[r, :k]), p, 1.25)
        assert np.array_equal(out[r], ref), r


@pytest.mark.parametrize("m,k,rows,fmt", [(1, 2560, (2560, 640, 640), 0), (5, 2560, (6912, 6912), 0),
                                           (1, 2560, (2560, 640, 640), 1), (3, 6912, (2560,), 1),
                                           (16, 2560, (2560, 640, 640), 0), (130, 2560, (6912, 6912), 0),
                                           (40, 640, (136, 40, 8), 0)])
def test_bitnet_linear_fused_vs_oracle(orc, m, k, rows, fmt):
    """wf_bitnet_linear_fused (q|k|v, gate|up: one shared activation quantization):
    every segment bf16 bit-exact with the oracle's per-row linear on that segment's weights and
    scale, and with ops.bitnet_linear on the segment alone; M < 16 (one GEMV launch, I2_S and TQ),
    M >= 16 (one row quantizer + one int8-MFMA GEMM over all segments), ragged segments, strided rows."""
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    from wfamd.linear import BitNetFusedLinear, BitNetLinear
    rng = np.random.default_rng(m * 7 + k + sum(rows))
    ws = [1.25 + 0.25 * i for i in range(len(rows))]
    ps = [orc.pack_i2s(rng.integers(-1, 2, size=(n, k)).astype(np.float32)) for n in rows]
    x = (rng.standard_normal((m, k + 32)) * rng.uniform(0.05, 3.0, size=(m, 1))).astype(np.float32)
    xb = orc.f32_to_bf16(x)
    xt = cu(xb.view(np.int16)).view(torch.bfloat16)[:, :k]  # row stride k + 32
    packed = torch.cat([cu(p) for p in ps], dim=0)
    if fmt == WF_FMT_TQ:
        packed = torch.cat([ops.i2s_to_tq(cu(p)) for p in ps], dim=0)
    outs = ops.bitnet_linear_fused(xt, packed, rows, ws, fmt, in_features=k)
    layers = [BitNetLinear(k, n, ops.i2s_to_tq(cu(p)) if fmt == WF_FMT_TQ else cu(p), w, fmt)
              for n, p, w in zip(rows, ps, ws)]
    mod = BitNetFusedLinear(layers)(xt)
    for s, (n, p, w) in enumerate(zip(rows, ps, ws)):
        got = bits(outs[s])
        assert got.shape == (m, n)
        assert np.array_equal(got, bits(mod[s])), s
        assert np.array_equal(got, bits(layers[s](xt))), s
        for r in ([0, m - 1] if m > 16 else range(m)):
            ref = orc.bitnet_linear_bf16(np.ascontiguousarray(xb[r, :k]), p, w)
            assert np.array_equal(got[r], ref), (s, r)
    if len(rows) == 3:  # the torch.ops schema (sgl_kernel::bitnet_qkv_forward_cpu) runs the same launch
        assert ops.register_torch_ops()
        top = torch.ops.sgl_kernel.bitnet_qkv_forward_cpu(xt[:, :k].contiguous(), packed, *rows, *ws, fmt)
        for s in range(3):
            assert np.array_equal(bits(top[s]), bits(outs[s])), s
    with pytest.raises(ValueError):
        ops.bitnet_linear_fused(xt, packed, [rows[0] + 16] + list(rows[1:]), ws, fmt, in_features=k)


@pytest.mark.parametrize("m,h,i,fmt", [(1, 2560, 6912, 0), (3, 512, 1536, 1), (20, 512, 1536, 0), (1, 2560, 6912, 1)])
def test_bitnet_mlp_vs_oracle(orc, m, h, i, fmt):
    """wf_bitnet_mlp (BitNetMLP) against the reference's mlp() (scripts/direct_inference_full.py:252-265)
    composed from the oracle: per row gate / up = BitNetLinear (bit-exact pieces), act =
    bf16(bf16(relu(gate)^2) * up), rms_norm(ffn_sub_norm) (oracle orc_rmsnorm_bf16, double sum), down.
    The GPU's fp32 norm sum can move one activation across a bf16 / int8 rounding boundary, so the bar
    is rel-L2 <= 2e-3 per row (the decode step's 1e-3 at the logits), most rows bit-exact."""
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    from wfamd.linear import BitNetLinear, BitNetMLP
    rng = np.random.default_rng(m + h + i + fmt)
    ws = (1.6, 1.8, 1.7)
    pg, pu = (orc.pack_i2s(rng.integers(-1, 2, size=(i, h)).astype(np.float32)) for _ in range(2))
    pd = orc.pack_i2s(rng.integers(-1, 2, size=(h, i)).astype(np.float32))
    fw = orc.f32_to_bf16(rng.uniform(0.5, 1.5, size=i).astype(np.float32))
    xb = orc.f32_to_bf16(rng.standard_normal((m, h)).astype(np.float32))
    dev = lambda p: ops.i2s_to_tq(cu(p)) if fmt == WF_FMT_TQ else cu(p)  # noqa: E731
    layers = [BitNetLinear(h, i, dev(pg), ws[0], fmt), BitNetLinear(h, i, dev(pu), ws[1], fmt),
              BitNetLinear(i, h, dev(pd), ws[2], fmt)]
    mlp = BitNetMLP(*layers, cu(fw.view(np.int16)).view(torch.bfloat16), eps=1e-5)
    xt = cu(xb.view(np.int16)).view(torch.bfloat16)
    got = bits(mlp(xt))
    assert ops.register_torch_ops()  # sgl_kernel::bitnet_mlp_forward_cpu: the same launch
    top = torch.ops.sgl_kernel.bitnet_mlp_forward_cpu(xt, mlp.packed_gate_up, mlp.packed_down, *ws, mlp.ffn_sub_norm,
                                                      1e-5, fmt)
    assert np.array_equal(bits(top), got)
    exact = 0
    for r in range(m):
        g = orc.bf16_to_f32(orc.bitnet_linear_bf16(xb[r], pg, ws[0]))
        u = orc.bf16_to_f32(orc.bitnet_linear_bf16(xb[r], pu, ws[1]))
        sq = orc.bf16_to_f32(orc.f32_to_bf16(np.maximum(g, 0) * np.maximum(g, 0)))
        act = orc.f32_to_bf16(sq * u)
        ref = orc.bitnet_linear_bf16(orc.rms_norm_bf16(act, fw, 1e-5), pd, ws[2])
        a, b = orc.bf16_to_f32(got[r]), orc.bf16_to_f32(ref)
        e = float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
        assert e <= 2e-3, (r, e)
        exact += int(np.array_equal(got[r], ref))
    assert exact >= (m + 1) // 2, (exact, m)


def test_bitnet_linear_module_and_errors():
    from wfamd import ops
    from wfamd._lib import WF_FMT_TQ
    from wfamd.linear import BitNetLinear
    from oracle import oracle as orc
    rng = np.random.default_rng(21)
    w = rng.integers(-1, 2, size=(256, 512)).astype(np.float32)
    x = torch.randn(2, 3, 512, device="cuda").to(torch.bfloat16)
    lin = BitNetLinear.from_ternary(torch.from_numpy(w), 0.75)
    lin_tq = BitNetLinear.from_ternary(torch.from_numpy(w), 0.75, fmt=WF_FMT_TQ)
    y, y_tq = lin(x), lin_tq(x)
    assert y.shape == (2, 3, 256) and y.dtype == torch.bfloat16
    assert torch.equal(y, y_tq)
    p = orc.pack_i2s(w)
    xb = bits(x.reshape(6, 512))
    for r in range(6):
        assert np.array_equal(bits(y.reshape(6, 256))[r], orc.bitnet_linear_bf16(xb[r], p, 0.75))
    with pytest.raises(ValueError):
        ops.bitnet_linear(x.float(), lin.packed_weight, 0.75)
    with pytest.raises(ValueError):
        ops.bitnet_linear(x[..., :384], lin.packed_weight, 0.75)


def test_decode_batched_long_ragged_context_matches_single():
    """Batched (matrix-core attention on the transposed V cache) vs batch-1 (VALU attention on the
    row-major cache) over ragged contexts of 0..1900 cached keys: same logical K/V, per-row logits
    within 1e-4 rel-L2 (attention sums in a different fp32 order; P enters as bf16 hi + lo)."""
    from wfamd.model import BitNetConfig, BitNetDecoder, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=2048)
    w = synthetic_weights(cfg, seed=3)
    B = 20
    decb = BitNetDecoder(cfg, w, batch=B)
    assert decb.kv_tiled
    gen = torch.Generator(device="cuda").manual_seed(11)
    ctx = 1900
    kv = [(torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16),
           torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16)) for _ in range(2)]
    for l in range(2):
        decb.load_kv(l, *kv[l])
    pos = [0, 1, 5, 31, 32, 33, 127, 128, 129, 255, 256, 300, 511, 777, 1000, 1023, 1024, 1500, 1899, 1700]
    toks = [(37 * b + 5) % cfg.vocab for b in range(B)]
    decb.set_state(toks, pos)
    decb.step(graph=True)
    torch.cuda.synchronize()
    for b in (0, 1, 3, 4, 7, 8, 10, 13, 15, 16, 18):
        d1 = BitNetDecoder(cfg, w, batch=1)
        assert not d1.kv_tiled
        for l in range(2):
            d1.load_kv(l, kv[l][0][b:b + 1], kv[l][1][b:b + 1])
        d1.set_state([toks[b]], [pos[b]])
        d1.step(graph=False)
        torch.cuda.synchronize()
        got = decb.logits[b].float().cpu().numpy()
        exp = d1.logits[0].float().cpu().numpy()
        assert rel_l2(got, exp) < 1e-4, (b, pos[b], rel_l2(got, exp))
        del d1


def test_decode_paged_kv_equals_dense():
    """Paged KV (32-token pages from a shuffled pool, page table per sequence) vs
    the dense tile-layout planes: the same arithmetic on the same keys, so logits, next tokens and
    the K/V rows the steps append are bit-identical, over ragged contexts (0..1900, page edges),
    several graph-replayed steps that cross page boundaries, and a sequence released and
    re-admitted onto recycled pages."""
    from wfamd.model import BitNetConfig, BitNetDecoder, from_kv_tiles, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=2048)
    w = synthetic_weights(cfg, seed=5)
    B = 20
    dense = BitNetDecoder(cfg, w, batch=B)
    paged = BitNetDecoder(cfg, w, batch=B, num_pages=B * cfg.max_seq // 32 // 2, page_seed=7)
    assert dense.kv_tiled and paged.paged
    gen = torch.Generator(device="cuda").manual_seed(13)
    ctx = 1900
    pos = [0, 1, 5, 31, 32, 33, 127, 128, 129, 255, 256, 300, 511, 777, 1000, 1023, 1024, 1500, 1899, 1700]
    for l in range(2):
        k = torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16)
        for b in range(B):  # keys past a sequence's position are never read: keep them out of the pool
            k[b, :, pos[b]:] = 0
            v[b, :, pos[b]:] = 0
        dense.load_kv(l, k, v)
        paged.load_kv(l, k[:, :, :max(pos)], v[:, :, :max(pos)], lengths=pos)
    steps = 6
    for b in range(B):
        paged.reserve(b, pos[b] + steps + 3)
    assert paged.pool.num_free_pages() < paged.pool.num_pages
    toks = [(37 * b + 5) % cfg.vocab for b in range(B)]
    for dec in (dense, paged):
        dec.set_state(toks, pos)
    for i in range(steps):
        dense.step(graph=True)
        paged.step(graph=True)
        torch.cuda.synchronize()
        assert torch.equal(dense.logits.view(torch.int16), paged.logits.view(torch.int16)), i
        assert torch.equal(dense.tokens, paged.tokens) and torch.equal(dense.positions, paged.positions)
    # the appended rows sit in the right pages: compare every sequence's K/V through the page table
    for l in range(2):
        kd, vd = from_kv_tiles(dense.k_cache[l], dense.v_cache[l])
        for b in (0, 3, 4, 5, 8, 17, 18):
            n = pos[b] + steps
            nblk = (n + 31) // 32
            ids = torch.from_numpy(paged.seq_pages[b][:nblk].astype(np.int64)).cuda()
            kt = paged.k_cache[l].index_select(0, ids).transpose(0, 1).reshape(1, nblk * 32, 128)
            vt = paged.v_cache[l].index_select(0, ids).transpose(0, 1).reshape(1, nblk * 32, 128)
            kp, vp = from_kv_tiles(kt, vt)
            assert torch.equal(kp[:, :n], kd[b, :, :n]) and torch.equal(vp[:, :n], vd[b, :, :n]), (l, b)
    # release + re-admit sequence 3 at position 0 on recycled pages: it decodes like a fresh dense row
    free0 = paged.pool.num_free_pages()
    paged.release(3)
    assert paged.pool.num_free_pages() > free0
    paged.reserve(3, 40)
    t3 = int(dense.tokens[3])
    for dec in (dense, paged):
        p = dec.positions.clone()
        p[3] = 0
        dec.positions.copy_(p)
    for i in range(3):
        dense.step(graph=True)
        paged.step(graph=True)
    torch.cuda.synchronize()
    assert torch.equal(dense.logits[3].view(torch.int16), paged.logits[3].view(torch.int16)), t3


def test_kv_manager_backed_by_decoder_pool():
    """One paged pool behind both APIs (tests/test_kv_cache_cpp.py:283-373): the
    reference's KVCacheManager, backed by a paged decoder, allocates the decoder's own 32-token pages,
    scatters token rows [T, H*D] into them (slots = position within a page, the tile layouts the
    batched attention reads), and the decoder -- its sequences mapped onto those pages -- decodes
    bit-identically to the dense decoder holding the same history; gather_kv returns the rows, the
    K/V rows the steps append included; freeing through the manager refills the decoder's pool."""
    from sgl_kernel.kvcache import KVCacheManager
    from wfamd.model import BitNetConfig, BitNetDecoder, from_kv_tiles, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=2048)
    w = synthetic_weights(cfg, seed=5)
    B, steps = 16, 5
    dense = BitNetDecoder(cfg, w, batch=B)
    paged = BitNetDecoder(cfg, w, batch=B, num_pages=B * cfg.max_seq // 32 // 2, page_seed=3)
    mgr = KVCacheManager.from_decoder(paged)
    free0 = mgr.num_free_pages()
    assert free0 == paged.pool.num_free_pages() == paged.pool.num_pages
    pos = [0, 1, 31, 32, 33, 100, 255, 256, 257, 511, 700, 1000, 1023, 1024, 1300, 1800]
    gen = torch.Generator(device="cuda").manual_seed(21)
    pages = []
    for b in range(B):  # every sequence's pages for its history and the steps ahead, via the reference API
        pg = mgr.allocate_pages((pos[b] + steps + 32) // 32)
        assert len(pg) == (pos[b] + steps + 32) // 32
        paged.map_pages(b, pg.numpy())
        pages.append(pg)
    assert mgr.num_free_pages() == paged.pool.num_free_pages() < free0
    rows = {}
    for l in range(cfg.layers):
        k = torch.randn(B, 1, max(pos), 128, generator=gen, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, 1, max(pos), 128, generator=gen, device="cuda").to(torch.bfloat16)
        for b in range(B):
            k[b, :, pos[b]:] = 0
            v[b, :, pos[b]:] = 0
        dense.load_kv(l, k, v)
        for b in range(B):
            n = pos[b]
            if n == 0:
                continue
            t = torch.arange(n)
            pg, sl = pages[b][t // 32], (t % 32).to(torch.int32)
            kr, vr = k[b, 0, :n].contiguous(), v[b, 0, :n].contiguous()  # [T, H*D], H = 1
            mgr.scatter_kv(kr, vr, pg, sl, l)
            rows[(l, b)] = (kr, vr, pg, sl)
    for l, b in ((0, 5), (1, 14)):  # the reference's round trip, from the engine's tile layout
        kr, vr, pg, sl = rows[(l, b)]
        ko, vo = torch.zeros_like(kr), torch.zeros_like(vr)
        mgr.gather_kv(ko, vo, pg, sl, l)
        assert torch.equal(ko, kr) and torch.equal(vo, vr), (l, b)
    toks = [(41 * b + 7) % cfg.vocab for b in range(B)]
    for dec in (dense, paged):
        dec.set_state(toks, pos)
    for i in range(steps):
        dense.step(graph=True)
        paged.step(graph=True)
        torch.cuda.synchronize()
        assert torch.equal(dense.logits.view(torch.int16), paged.logits.view(torch.int16)), i
        assert torch.equal(dense.tokens, paged.tokens)
    assert mgr.invalid_page_count() == 0
    for l in range(cfg.layers):  # the rows the steps appended, read back through the manager
        kd, vd = from_kv_tiles(dense.k_cache[l], dense.v_cache[l])
        for b in (0, 3, 9, 15):
            n = pos[b] + steps
            t = torch.arange(n)
            ko = torch.zeros(n, 128, dtype=torch.bfloat16, device="cuda")
            vo = torch.zeros_like(ko)
            mgr.gather_kv(ko, vo, pages[b][t // 32], (t % 32).to(torch.int32), l)
            assert torch.equal(ko, kd[b, 0, :n]) and torch.equal(vo, vd[b, 0, :n]), (l, b)
    for b in range(B):
        mgr.free_pages(pages[b])
    assert mgr.num_free_pages() == paged.pool.num_free_pages() == free0


@pytest.mark.parametrize("m,n,k", [(16, 16, 128), (130, 272, 384), (300, 3840, 2560), (513, 2560, 6912),
                                   (1024, 13824, 2560)])
def test_prefill_gemm_tiled_vs_oracle(orc, m, n, k):
    """wf_bitnet_gemm_tiled (tile-layout prefill GEMM, XCD-grouped 128 x 256 tiles) is bit-exact with
    the oracle's raw enc-sum GEMM and with wf_bitnet_gemm on the same operands, over ragged M / N
    tails (partial row and column blocks) and the 2B-4T layer shapes."""
    from wfamd import ops
    rng = np.random.default_rng(m + n + k)
    c = rng.integers(0, 3, size=(n, k // 4, 4)).astype(np.uint8)  # enc codes in {0, 1, 2}
    p = (c[..., 0] << 6) | (c[..., 1] << 4) | (c[..., 2] << 2) | c[..., 3]
    a = rng.integers(-128, 128, size=(m, k)).astype(np.int8)
    at = ops.codes_to_tiles(cu(a))
    y = ops.bitnet_gemm_tiled(ops.i2s_to_mfma(cu(p)), at, 0.37, m).cpu().numpy()
    rows = slice(None) if m * n * k < 2e9 else slice(0, 64)
    assert np.array_equal(y[rows], orc.gemm_i2s(p, a[rows], 0.37))
    assert np.array_equal(y, ops.bitnet_gemm(cu(p), cu(a), 0.37).cpu().numpy())


def test_prefill_matches_teacher_forced_decode():
    """wf_model_prefill (tile GEMMs with the decode epilogues, one-pass causal attention) vs the
    batched decode step run token by token over the same prompts (teacher forcing): the K/V rows
    written for every prompt position and the next step's logits agree within 5e-3 rel-L2 (the
    attention sums in a different fp32 order: one pass vs 8 merged splits), the greedy tokens
    match; prefill on paged KV is bit-identical to prefill on the dense planes."""
    from wfamd.model import BitNetConfig, BitNetDecoder, from_kv_tiles, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=512)
    w = synthetic_weights(cfg, seed=9)
    B = 16
    rng = np.random.default_rng(4)
    lens = [2, 3, 5, 33, 64, 65, 100, 130, 7, 31, 32, 200, 4, 17, 96, 150]
    prompts = [rng.integers(0, cfg.vocab, size=n).tolist() for n in lens]
    ref = BitNetDecoder(cfg, w, batch=B)
    for t in range(max(lens) - 1):
        ref.set_state([p[min(t, len(p) - 2)] for p in prompts], [min(t, len(p) - 2) for p in prompts])
        ref.step(graph=False)
    pf = BitNetDecoder(cfg, w, batch=B)
    pf.prefill([(b, p[:-1], 0) for b, p in enumerate(prompts)], chunk_rows=256)  # several chunks
    pg = BitNetDecoder(cfg, w, batch=B, num_pages=B * cfg.max_seq // 32, page_seed=1)
    pg.prefill([(b, p[:-1], 0) for b, p in enumerate(prompts)])
    torch.cuda.synchronize()
    for l in range(cfg.layers):
        kr, vr = from_kv_tiles(ref.k_cache[l], ref.v_cache[l])
        kp, vp = from_kv_tiles(pf.k_cache[l], pf.v_cache[l])
        for b, n in enumerate(lens):
            for a_, b_ in ((kr, kp), (vr, vp)):
                x, y = a_[b, :, :n - 1].float().cpu().numpy(), b_[b, :, :n - 1].float().cpu().numpy()
                assert rel_l2(y, x) < 5e-3, (l, b, rel_l2(y, x))
    for dec in (ref, pf, pg):
        for b, p in enumerate(prompts):
            dec.tokens[b] = p[-1]
            dec.positions[b] = len(p) - 1
        dec.step(graph=True)
    torch.cuda.synchronize()
    assert torch.equal(pf.logits.view(torch.int16), pg.logits.view(torch.int16))
    for b in range(B):
        got, exp = pf.logits[b].float().cpu().numpy(), ref.logits[b].float().cpu().numpy()
        assert rel_l2(got, exp) < 5e-3, (b, rel_l2(got, exp))
    assert (pf.tokens == ref.tokens).float().mean().item() >= 0.9


def test_prefill_in_pieces_equals_one_shot():
    """Chunked prefill (a prompt split over calls, later pieces at start > 0 attending to the K/V
    the earlier calls wrote; rows of several slots interleaved per call) is bit-identical to one
    prefill call of the whole prompts, on paged KV."""
    from wfamd.model import BitNetConfig, BitNetDecoder, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=512)
    w = synthetic_weights(cfg, seed=21)
    B = 16
    rng = np.random.default_rng(8)
    prompts = {b: rng.integers(0, cfg.vocab, size=int(n)).tolist() for b, n in zip(range(0, B, 3), (70, 33, 129, 5, 64, 200))}
    one = BitNetDecoder(cfg, w, batch=B, num_pages=B * 16, page_seed=2)
    one.prefill([(b, p, 0) for b, p in prompts.items()])
    parts = BitNetDecoder(cfg, w, batch=B, num_pages=B * 16, page_seed=3)
    cuts = {b: sorted(rng.integers(1, len(p), size=2).tolist()) if len(p) > 2 else [1, 1] for b, p in prompts.items()}
    for k in range(3):
        batch = []
        for b, p in prompts.items():
            e = [0] + cuts[b] + [len(p)]
            batch.append((b, p[e[k]:e[k + 1]], e[k]))
        parts.prefill(batch, chunk_rows=64)
    for dec in (one, parts):
        for b, p in prompts.items():
            dec.tokens[b] = p[-1]
            dec.positions[b] = len(p)
            if dec.paged:
                dec.reserve(b, len(p) + 1)
        dec.step(graph=False)
    torch.cuda.synchronize()
    for b in prompts:
        assert torch.equal(one.logits[b].view(torch.int16), parts.logits[b].view(torch.int16)), b


def _cos_rows(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return torch.nn.functional.cosine_similarity(a.float(), b.float(), dim=-1)


@pytest.mark.parametrize("kvd", ["fp8", "int8", "int8-absmax"])
def test_fp8_kv_codes_and_decode_quality(kvd):
    """One-byte K/V for the batched decode step (FP8 e4m3fn; int8 = the reference's INT8
    KVCacheDtype): (1) the K/V codes a step writes equal torch's e4m3fn / int8 rounding
    (wfamd.model.to_fp8_codes / to_int8_codes) of the bf16 values a bf16-KV decoder writes, divided
    by the per-layer scale (bit-exact, layer 0 where both see the same input); (2) decoding over ragged contexts
    with FP8 K/V keeps the logits close to bf16 K/V. The reference's quantized-KV bar is cosine >=
    0.998 on one attention output (docs/research/notebook.md:690-700); here it is the logits after
    two layers of a random-init model and the LM head, measured at mean ~0.997 (e4m3 keeps 3
    mantissa bits), so the bar is mean >= 0.995, floor 0.99, and >= 80 % equal greedy tokens;
    (3) paged FP8 == dense FP8 bit for bit. int8-absmax: int8 codes at non-power-of-two scales of the
    reference's absmax / 127 form (kv_cache/kv_cache.py:159-185), where rne(y / s) and rne(y * (1 / s))
    differ near ties: the device divides, as the header, the oracle and to_int8_codes do."""
    from wfamd.model import KV_CODES, BitNetConfig, BitNetDecoder, from_kv_tiles, synthetic_weights
    absmax = kvd == "int8-absmax"
    kvd = "int8" if absmax else kvd
    enc = KV_CODES[kvd][0]
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=2048)
    w = synthetic_weights(cfg, seed=31)
    # q/k/v projection scales such that attention scores are O(1), as in a trained model (the
    # random-init scales give |scores| ~ 30: one-hot softmax where any rounding flips the winner)
    w["wscale"][:, :3] = 0.05
    B = 20
    scale = [(0.5, 0.25), (1.0, 0.5)] if kvd == "fp8" else [(1 / 16, 1 / 32), (1 / 8, 1 / 16)]
    if absmax:
        scale = [(4.37 / 127, 3.91 / 127), (5.03 / 127, 4.66 / 127)]
    bf = BitNetDecoder(cfg, w, batch=B)
    f8 = BitNetDecoder(cfg, w, batch=B, kv_dtype=kvd, kv_scale=scale)
    f8p = BitNetDecoder(cfg, w, batch=B, kv_dtype=kvd, kv_scale=scale, num_pages=B * 64, page_seed=4)
    gen = torch.Generator(device="cuda").manual_seed(5)
    ctx = 1500
    pos = [0, 1, 5, 31, 32, 33, 127, 128, 129, 255, 256, 300, 511, 777, 1000, 1023, 1024, 1300, 1499, 1400]
    for l in range(cfg.layers):
        k = torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, 1, ctx, 128, generator=gen, device="cuda").to(torch.bfloat16)
        for dec in (bf, f8):
            dec.load_kv(l, k, v)
        f8p.load_kv(l, k, v, lengths=pos)
    for b in range(B):
        f8p.reserve(b, pos[b] + 1)
    toks = [(53 * b + 7) % cfg.vocab for b in range(B)]
    for dec in (bf, f8, f8p):
        dec.set_state(toks, pos)
        dec.step(graph=True)
    torch.cuda.synchronize()
    kb, vb = from_kv_tiles(bf.k_cache[0], bf.v_cache[0])
    k8, v8 = from_kv_tiles(f8.k_cache[0], f8.v_cache[0])
    for b in range(B):
        p = pos[b]
        assert torch.equal(k8[b, :, p], enc(kb[b, :, p], scale[0][0])), b
        assert torch.equal(v8[b, :, p], enc(vb[b, :, p], scale[0][1])), b
    assert torch.equal(f8.logits.view(torch.int16), f8p.logits.view(torch.int16))
    cos = _cos_rows(f8.logits, bf.logits)
    assert cos.mean().item() >= 0.995 and cos.min().item() >= 0.99, cos
    assert (f8.tokens == bf.tokens).float().mean().item() >= 0.8


@pytest.mark.parametrize("kvd", ["fp8", "int8"])
def test_fp8_kv_prefill(kvd):
    """Prefill into one-byte K/V (FP8 / int8): paged == dense bit-exact, and the next step's logits stay within the
    FP8 bar of test_fp8_kv_codes_and_decode_quality (mean cosine >= 0.995, floor 0.99) of the same
    prefill + step on bf16 K/V."""
    from wfamd.model import BitNetConfig, BitNetDecoder, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=2, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=512)
    w = synthetic_weights(cfg, seed=41)
    w["wscale"][:, :3] = 0.05  # O(1) attention scores (see test_fp8_kv_codes_and_decode_quality)
    B = 16
    rng = np.random.default_rng(6)
    prompts = {b: rng.integers(0, cfg.vocab, size=int(n)).tolist() for b, n in zip(range(0, B, 2), (40, 3, 150, 64, 97, 200, 17, 33))}
    sc = (0.5, 0.5) if kvd == "fp8" else (1 / 16, 1 / 16)
    decs = [BitNetDecoder(cfg, w, batch=B), BitNetDecoder(cfg, w, batch=B, kv_dtype=kvd, kv_scale=sc),
            BitNetDecoder(cfg, w, batch=B, kv_dtype=kvd, kv_scale=sc, num_pages=B * 16, page_seed=9)]
    for dec in decs:
        for b, p in prompts.items():
            dec.admit(b, p)
        dec.step(graph=False)
    torch.cuda.synchronize()
    assert torch.equal(decs[1].logits.view(torch.int16), decs[2].logits.view(torch.int16))
    rows = list(prompts)
    cos = _cos_rows(decs[1].logits[rows], decs[0].logits[rows])
    assert cos.mean().item() >= 0.995 and cos.min().item() >= 0.99, cos


def test_prefill_fp8_paged_argument_errors():
    """The new entry points fail loudly on contract violations (ValueError for WF_EINVAL, as the
    reference's shape checks; nothing silently ignored): prefill on a batch-1 decoder, rows not in whole groups, FP8 / paged K/V on a
    decoder without the matrix-core path, bad FP8 scales, tiled GEMM shape checks."""
    import ctypes as C
    from wfamd import _lib, ops
    from wfamd.model import BitNetConfig, BitNetDecoder, synthetic_weights
    cfg = BitNetConfig(hidden=512, layers=1, n_heads=4, n_kv_heads=1, head_dim=128, inter=768, vocab=1024,
                       max_seq=256)
    w = synthetic_weights(cfg, seed=1)
    d1 = BitNetDecoder(cfg, w, batch=1)
    with pytest.raises(ValueError):  # C-ABI WF_EINVAL -> ValueError (wfamd._lib.check)
        d1.prefill([(0, [1, 2, 3], 0)])
    with pytest.raises(ValueError):
        BitNetDecoder(cfg, w, batch=4, kv_dtype="fp8")
    with pytest.raises(ValueError):
        BitNetDecoder(cfg, w, batch=4, kv_dtype="int8")
    with pytest.raises(ValueError):
        BitNetDecoder(cfg, w, batch=16, kv_dtype="int4")
    with pytest.raises(ValueError):
        BitNetDecoder(cfg, w, batch=4, num_pages=64)
    with pytest.raises(ValueError):
        BitNetDecoder(cfg, w, batch=16, kv_dtype="fp8", kv_scale=(0.0, 1.0))
    d16 = BitNetDecoder(cfg, w, batch=16)
    with pytest.raises(ValueError):
        d16.prefill([(0, list(range(300)), 0)])  # beyond max_seq
    _lib.call("wf_model_prefill_reserve", d16._h, 32)
    t = torch.zeros(20, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    with pytest.raises(ValueError):
        _lib.call("wf_model_prefill", d16._h, t.data_ptr(), t.data_ptr(), t.data_ptr(), 20, st)  # not whole groups
    with pytest.raises(ValueError):
        _lib.call("wf_model_prefill", d16._h, t.data_ptr(), t.data_ptr(), t.data_ptr(), 64, st)  # > reserved rows
    wq = torch.zeros(24, 32, dtype=torch.uint8, device="cuda")  # N = 24: not a multiple of 16
    a = ops.codes_to_tiles(torch.zeros(16, 128, dtype=torch.int8, device="cuda"))
    with pytest.raises(ValueError):
        ops.bitnet_gemm_tiled(wq, a, 1.0, 16)


def test_mfma_tile_format_roundtrip_and_gemv(orc):
    """WF_FMT_I2S_MFMA is a bijection of I2_S (device repack both ways; include/wf_bitnet.h layout)."""
    from wfamd import ops
    rng = np.random.default_rng(17)
    for n, k in ((64, 512), (3840, 2560), (2560, 6912)):
        p = rng.integers(0, 256, size=(n, k // 4)).astype(np.uint8)
        mf = ops.i2s_to_mfma(cu(p))
        mfn = mf.cpu().numpy().reshape(-1).view(np.uint32)
        # spot-check the documented dword order
        nkb = k // 128
        for t in rng.integers(0, mfn.size, size=64):
            h, lane, blk = t & 1, (t >> 1) & 63, t >> 7
            kb, ct = blk % nkb, blk // nkb
            row = ct * 16 + (lane & 15)
            off = 32 * kb + 16 * h + 4 * (lane >> 4)
            assert mfn[t] == p[row, off:off + 4].view(np.uint32)[0]
        assert np.array_equal(ops.mfma_to_i2s(mf).cpu().numpy(), p)
