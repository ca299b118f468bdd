#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE's own Python.

Run ONLY in the build container (the reference tree does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Every expected output below is produced by a reference function (cited file:line) or by the
reference's call pattern composed from those functions; inputs are seeded. The resulting
``*.npz`` files hold only numeric arrays (load with ``numpy.load(..., allow_pickle=False)``), and
``manifest.json`` records their sha256 sums. No reference source text is stored.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import math
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent

sys.dont_write_bytecode = True
sys.path.insert(0, str(REF / "src"))
sys.path.insert(0, str(REF / "tests"))

import test_bitnet_core as tbc  # noqa: E402  (reference tests/test_bitnet_core.py)
import test_kv_cache_cpp as tkv  # noqa: E402  (reference tests/test_kv_cache_cpp.py)
from wrinklefree_inference.kernels import bitnet_patch  # noqa: E402
from wrinklefree_inference.kernels import native as rnative  # noqa: E402
from wrinklefree_inference.kv_cache import kv_cache as rkv  # noqa: E402


def _load_by_path(name: str, path: Path):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# cache/__init__.py pulls google.cloud; load the converter module by file path.
conv = _load_by_path("ref_bitnet_converter", REF / "src/wrinklefree_inference/cache/bitnet_converter.py")


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16).copy()


def save(name: str, **arrays):
    path = OUT / f"{name}.npz"
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    return path


def gen_packing():
    g = torch.Generator().manual_seed(0)
    out = {}
    # (N, K): standard blocks, multiple blocks, degenerate K<128 block (converter.py:58-61), K%128 tail
    shapes = [(16, 128), (8, 512), (4, 2560), (2, 6912), (6, 64), (5, 160)]
    for i, (n, k) in enumerate(shapes):
        w = torch.randint(-1, 2, (n, k), generator=g).float()
        p1, s1 = conv._pack_ternary_weights(w)          # cache/bitnet_converter.py:26-77
        p2, s2 = tbc._pack_ternary_weights(w)           # tests/test_bitnet_core.py:56-106
        assert torch.equal(p1, p2) and torch.equal(s1, s2)
        un = tbc._unpack_i2_to_ternary(p1, n, k)        # tests/test_bitnet_core.py:109-136
        out[f"w{i}"] = w.to(torch.int8).numpy()
        out[f"p{i}"] = p1.numpy()
        out[f"un{i}"] = un.to(torch.int8).numpy()
        out[f"scale{i}"] = s1.numpy()
    # non-integer weights: round-half-even then clamp (converter.py:47)
    w = torch.tensor([[0.5, -0.5, 1.5, -2.7, 0.49, -0.51, 2.0, -1.0] * 16])
    out["wf"] = w.numpy().astype(np.float32)
    out["pf"] = conv._pack_ternary_weights(w)[0].numpy()
    # known answers: w0=+1, w33=-1, w127=+1 else 0 -> bytes[0,1,31] = 149, 69, 86 ; all +1 -> 170
    w = torch.zeros(1, 128)
    w[0, 0], w[0, 33], w[0, 127] = 1, -1, 1
    out["ka_w"] = w.to(torch.int8).numpy()
    out["ka_p"] = conv._pack_ternary_weights(w)[0].numpy()
    out["ones_p"] = conv._pack_ternary_weights(torch.ones(2, 256))[0].numpy()
    # HF [N/4, K] unpack (tests/test_bitnet_core.py:21-53), random bytes incl. the invalid code 3
    hf = torch.randint(0, 256, (16, 96), generator=g, dtype=torch.uint8)
    out["hf_p"] = hf.numpy()
    out["hf_un"] = tbc._unpack_ternary_weights(hf).to(torch.int8).numpy()
    # LSB layout: kernels/bitnet_patch.py:81-112 and kernels/native.py:181-215
    w = torch.randint(-1, 2, (12, 256), generator=g).float()
    pl, sl = bitnet_patch.pack_ternary_weights(w)
    pn = rnative.pack_weights(w.numpy())
    assert np.array_equal(pl.numpy(), pn)
    out["lsb_w"] = w.to(torch.int8).numpy()
    out["lsb_p"] = pn
    # HF -> LSB kernel repack (kernels/native.py:218-241, interleaved i::4 convention)
    hfw = torch.randint(0, 81, (8, 128), generator=g)
    hfb = torch.zeros(8, 128, dtype=torch.int32)
    for i in range(4):
        hfb |= ((hfw // (3 ** i)) % 3) << (2 * i)
    out["hf2lsb_in"] = hfb.to(torch.uint8).numpy()
    out["hf2lsb_out"] = rnative.repack_hf_weights(hfb.to(torch.uint8).numpy())
    return save("packing", **out)


def gen_quant():
    g = torch.Generator().manual_seed(1)
    out = {}
    xs = [
        torch.randn(2560, generator=g),
        torch.randn(6912, generator=g) * 37.0,
        torch.randn(128, generator=g) * 1e-3,
        torch.full((64,), 3e-7),                       # |x| < 1e-6 -> scale 1.0 branch
        torch.zeros(16),
        torch.tensor([127.0, 0.5, 1.5, 2.5, -0.5, -1.5, -2.5, 126.5, -127.0, 3.49999]),  # RNE ties
        torch.randn(4, 2560, generator=g),             # 2-D: one per-tensor scale
        torch.randn(2560, generator=g).to(torch.bfloat16).float(),  # bf16-origin activations
    ]
    for i, x in enumerate(xs):
        q, s = tbc.quantize_activations_i8(x)           # tests/test_bitnet_core.py:139-146
        out[f"x{i}"] = x.numpy().astype(np.float32)
        out[f"q{i}"] = q.numpy()
        out[f"s{i}"] = np.float64(s)
        qn, sn = rnative.quantize_activations(x.numpy().astype(np.float32))  # kernels/native.py:244-256
        out[f"qt{i}"] = qn
        out[f"st{i}"] = np.float32(sn)
    return save("quant", **out)


def gen_gemv():
    g = torch.Generator().manual_seed(2)
    out = {}
    # (N, K, M): reference formula tests/test_bitnet_core.py:149-167, batched row by row (GEMM a2)
    cases = [(64, 128, 1), (40, 2560, 1), (24, 6912, 1), (33, 512, 3), (16, 2560, 4), (7, 160, 2), (9, 64, 1)]
    for i, (n, k, m) in enumerate(cases):
        w = torch.randint(-1, 2, (n, k), generator=g).float()
        p, _ = tbc._pack_ternary_weights(w)
        x = torch.randn(m, k, generator=g)
        q, s = tbc.quantize_activations_i8(x)
        scale = [0.01, 1.7, 0.3333, 2.0, 1e-3, 1.0, 0.7][i]
        y = torch.stack([tbc.bitnet_gemv_reference(p, q[r], scale) for r in range(m)])
        out[f"p{i}"] = p.numpy()
        out[f"a{i}"] = q.numpy()
        out[f"scale{i}"] = np.float64(scale)
        out[f"y{i}"] = y.numpy().astype(np.float32)
        out[f"shape{i}"] = np.array([m, n, k], dtype=np.int64)
    # known answer (tests/test_bitnet_weight_loading.py:141-169): W=1, x=1, ws=2 -> 2*K corrected
    k = 256
    p, _ = tbc._pack_ternary_weights(torch.ones(4, k))
    q, s = tbc.quantize_activations_i8(torch.ones(k))
    raw = tbc.bitnet_gemv_reference(p, q, 2.0)
    corr = (raw - 2.0 * q.float().sum()) * s
    out["ka_raw"] = raw.numpy()
    out["ka_corr"] = corr.numpy()
    out["ka_s"] = np.float64(s)
    # LSB signed GEMV, kernels/native.py:27-65 (checked by the reference as np.dot(W, a) * scale,
    # tests/test_bitnet_model.py:57)
    w = np.random.default_rng(3).choice([-1, 0, 1], size=(48, 512)).astype(np.float32)
    pl = rnative.pack_weights(w)
    act = np.random.default_rng(4).standard_normal(512).astype(np.float32)
    ai, sc = rnative.quantize_activations(act)
    out["lsb_p"] = pl
    out["lsb_a"] = ai
    out["lsb_scale"] = np.float32(sc)
    out["lsb_y"] = (np.dot(w, ai.astype(np.float32)) * sc).astype(np.float32)
    return save("gemv", **out)


def ref_linear(x_bf16: torch.Tensor, packed: torch.Tensor, ws: float) -> torch.Tensor:
    """scripts/direct_inference_full.py:186-208 composed from the reference's own functions."""
    q, s = tbc.quantize_activations_i8(x_bf16.float())
    raw = tbc.bitnet_gemv_reference(packed, q, ws)
    act_sum = q.float().sum().item()
    return ((raw - ws * act_sum) * s).to(torch.bfloat16)


def gen_linear():
    g = torch.Generator().manual_seed(5)
    out = {}
    for i, (n, k, ws) in enumerate([(256, 512, 1.796875), (96, 2560, 1.5), (64, 6912, 2.0)]):
        w = torch.randint(-1, 2, (n, k), generator=g).float()
        p, _ = tbc._pack_ternary_weights(w)
        x = (torch.randn(k, generator=g) * 0.7).to(torch.bfloat16)
        y = ref_linear(x, p, ws)
        out[f"p{i}"] = p.numpy()
        out[f"x{i}"] = bf16_bits(x)
        out[f"ws{i}"] = np.float32(ws)
        out[f"y{i}"] = bf16_bits(y)
    return save("linear", **out)


def gen_kv():
    g = torch.Generator().manual_seed(6)
    out = {}
    # KVCache (kv_cache/kv_cache.py:96-313) update/get per dtype, incl. the per-layer scale overwrite
    for name in ["BF16", "FP16", "FP32", "INT8", "FP8_E4M3"]:
        cfg = rkv.KVCacheConfig(max_seq_len=32, num_layers=2, num_heads=4, head_dim=16, dtype=rkv.KVCacheDtype[name])
        c = rkv.KVCache(cfg)
        k1 = torch.randn(1, 5, 4, 16, generator=g)
        v1 = torch.randn(1, 5, 4, 16, generator=g)
        k2 = torch.randn(1, 3, 4, 16, generator=g) * 3
        v2 = torch.randn(1, 3, 4, 16, generator=g) * 0.2
        c.update(1, k1, v1, 0)
        c.update(1, k2, v2, 5)
        kg, vg = c.get(1)
        out[f"{name}_k1"], out[f"{name}_v1"] = k1.numpy(), v1.numpy()
        out[f"{name}_k2"], out[f"{name}_v2"] = k2.numpy(), v2.numpy()
        out[f"{name}_kget"] = kg.float().numpy()
        out[f"{name}_vget"] = vg.float().numpy()
        out[f"{name}_storage"] = c.cache[1, :, :8].float().numpy() if name in ("BF16", "FP16", "FP32") \
            else c.cache[1, :, :8].view(torch.int8).numpy()
        out[f"{name}_kscale"] = c.k_scales.numpy()
        out[f"{name}_vscale"] = c.v_scales.numpy()
    # attention_with_kv_cache (kv_cache/kv_cache.py:316-369), BF16 cache, float32 query
    cfg = rkv.KVCacheConfig(max_seq_len=64, num_layers=1, num_heads=4, head_dim=32, dtype=rkv.KVCacheDtype.BF16)
    c = rkv.KVCache(cfg)
    outs = []
    qs, ks, vs = [], [], []
    for pos in range(6):
        q = torch.randn(1, 4, 1, 32, generator=g)
        k = torch.randn(1, 1, 4, 32, generator=g)
        v = torch.randn(1, 1, 4, 32, generator=g)
        o = rkv.attention_with_kv_cache(q, c, 0, k, v, pos)
        qs.append(q.numpy()); ks.append(k.numpy()); vs.append(v.numpy()); outs.append(o.numpy())
    out["att_q"], out["att_k"], out["att_v"], out["att_o"] = map(np.stack, (qs, ks, vs, outs))
    mem = rkv.compute_kv_cache_memory({"num_layers": 30, "num_heads": 5, "head_dim": 128}, 4096, rkv.KVCacheDtype.BF16)
    out["mem_total_mb"] = np.float64(mem["total_mb"])
    out["mem_per_token_kb"] = np.float64(mem["per_token_kb"])
    # Paged KVCacheManager twin (tests/test_kv_cache_cpp.py:20-127): allocation order + roundtrip
    ref = tkv.PythonKVCacheReference(num_layers=3, num_heads=2, head_dim=8, page_size=16, max_pages=10)
    a = ref.allocate_pages(4)
    ref.free_pages_batch(a[1:3])
    b = ref.allocate_pages(3)
    single = ref.allocate_page()
    too_many = ref.allocate_pages(100)
    out["pg_a"], out["pg_b"], out["pg_single"] = a.numpy(), b.numpy(), np.int64(single)
    out["pg_too_many"] = np.int64(too_many.numel())
    out["pg_free_after"] = np.int64(ref.num_free_pages())
    k_in = torch.randn(3, 2, 8, generator=g)
    v_in = torch.randn(3, 2, 8, generator=g)
    ref.scatter_kv(k_in, v_in, b, torch.zeros(3, dtype=torch.int32), 2)
    ko, vo = ref.gather_kv(b, torch.zeros(3, dtype=torch.int32), 2)
    out["pg_k"], out["pg_v"], out["pg_ko"], out["pg_vo"] = k_in.numpy(), v_in.numpy(), ko.numpy(), vo.numpy()
    return save("kv", **out)


def sdpa_gqa(q_bf16: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, s: int) -> torch.Tensor:
    """scripts/direct_inference_full.py:229-244: q [Hq, D] bf16; kc/vc [S_max, Hkv, D]."""
    qa = q_bf16.unsqueeze(0).unsqueeze(2)
    ka = kc[:s].transpose(0, 1).unsqueeze(0)
    va = vc[:s].transpose(0, 1).unsqueeze(0)
    return F.scaled_dot_product_attention(qa, ka, va, enable_gqa=True).squeeze(0).squeeze(1).flatten()


def gen_attention():
    g = torch.Generator().manual_seed(7)
    out = {}
    hq, hkv, d = 20, 5, 128
    for i, s in enumerate([1, 7, 50, 300]):
        q = torch.randn(hq, d, generator=g).to(torch.bfloat16)
        kc = torch.randn(s, hkv, d, generator=g).to(torch.bfloat16)
        vc = torch.randn(s, hkv, d, generator=g).to(torch.bfloat16)
        o = sdpa_gqa(q, kc, vc, s)
        out[f"q{i}"], out[f"k{i}"], out[f"v{i}"] = bf16_bits(q), bf16_bits(kc), bf16_bits(vc)
        out[f"o{i}"] = bf16_bits(o)
        out[f"s{i}"] = np.int64(s)
    return save("attention", **out)


def rms_norm(x, w, eps):
    """scripts/direct_inference_full.py:181-184."""
    var = x.float().pow(2).mean(-1, keepdim=True)
    return (x * torch.rsqrt(var + eps).to(x.dtype)) * w


def rope_tables(head_dim, max_seq, base):
    """scripts/direct_inference_full.py:31-44."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float32) / head_dim))
    fr = torch.outer(torch.arange(max_seq, dtype=torch.float32), inv)
    return torch.cos(fr).to(torch.bfloat16), torch.sin(fr).to(torch.bfloat16)


def rotate(x, cos, sin):
    """scripts/direct_inference_full.py:58-70."""
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    return torch.cat([x1 * cos - x2 * sin, x1 * sin + x2 * cos], dim=-1)


def gen_decode():
    """A small BitNet model stepped through the decode loop of scripts/direct_inference_full.py:267-302."""
    g = torch.Generator().manual_seed(8)
    H, L, HQ, HKV, D, I, V, S = 512, 2, 4, 2, 128, 768, 1024, 64
    eps, theta = 1e-5, 500000.0
    bf = torch.bfloat16
    out = dict(cfg=np.array([H, L, HQ, HKV, D, I, V, S], dtype=np.int64), eps=np.float32(eps))
    embed = (torch.randn(V, H, generator=g) * 0.02).to(bf)
    fnorm = (1.0 + 0.1 * torch.randn(H, generator=g)).to(bf)
    cos, sin = rope_tables(D, S, theta)
    out["embed"], out["final_norm"], out["rope_cos"], out["rope_sin"] = map(bf16_bits, (embed, fnorm, cos, sin))
    names = ["wq", "wk", "wv", "wo", "wg", "wu", "wd"]
    shapes = [(H, H), (HKV * D, H), (HKV * D, H), (H, H), (I, H), (I, H), (H, I)]
    layers = []
    for li in range(L):
        lay = {}
        for nm, (n, k) in zip(names, shapes):
            lay[nm] = tbc._pack_ternary_weights(torch.randint(-1, 2, (n, k), generator=g).float())[0]
        lay["ws"] = [float(torch.empty(1).uniform_(1.5, 2.0, generator=g).item()) for _ in range(7)]
        lay["ws"] = [float(np.float32(w)) for w in lay["ws"]]
        for nm, n in [("ln_in", H), ("ln_post", H), ("attn_sub", H), ("ffn_sub", I)]:
            lay[nm] = (1.0 + 0.1 * torch.randn(n, generator=g)).to(bf)
        layers.append(lay)
    for nm in names:
        out[nm] = np.stack([layers[i][nm].numpy() for i in range(L)])
    for nm in ["ln_in", "ln_post", "attn_sub", "ffn_sub"]:
        out[nm] = np.stack([bf16_bits(layers[i][nm]) for i in range(L)])
    out["wscale"] = np.array([layers[i]["ws"] for i in range(L)], dtype=np.float32)

    kc = torch.zeros(L, S, HKV, D, dtype=bf)
    vc = torch.zeros(L, S, HKV, D, dtype=bf)
    tokens = [3, 17, 999, 256, 42, 7]
    logits_all, hidden_all = [], []
    for pos, tok in enumerate(tokens):
        hid = embed[tok]
        for li, lay in enumerate(layers):
            ws = lay["ws"]
            x = rms_norm(hid, lay["ln_in"], eps)
            q = ref_linear(x, lay["wq"], ws[0]).view(HQ, D)
            k = ref_linear(x, lay["wk"], ws[1]).view(HKV, D)
            v = ref_linear(x, lay["wv"], ws[2]).view(HKV, D)
            q, k = rotate(q, cos[pos], sin[pos]), rotate(k, cos[pos], sin[pos])
            kc[li, pos], vc[li, pos] = k, v
            a = sdpa_gqa(q, kc[li], vc[li], pos + 1)
            a = rms_norm(a, lay["attn_sub"], eps)
            hid = hid + ref_linear(a, lay["wo"], ws[3])
            x = rms_norm(hid, lay["ln_post"], eps)
            gt = ref_linear(x, lay["wg"], ws[4])
            up = ref_linear(x, lay["wu"], ws[5])
            act = torch.relu(gt.to(bf)).square() * up.to(bf)
            act = rms_norm(act, lay["ffn_sub"], eps)
            hid = hid + ref_linear(act, lay["wd"], ws[6])
        hn = rms_norm(hid, fnorm, eps)
        logits = F.linear(hn, embed)
        logits_all.append(bf16_bits(logits))
        hidden_all.append(bf16_bits(hid))
    out["tokens"] = np.array(tokens, dtype=np.int64)
    out["logits"] = np.stack(logits_all)
    out["hidden"] = np.stack(hidden_all)
    return save("decode", **out)


def reference_decoder():
    """(DirectBitNetInference instance with the full_inputs weights and history, cfg, weights, K, V,
    the full_inputs module); see gen_decode_full."""
    import types
    sys.path.insert(0, str(OUT))
    import full_inputs as fi
    sys.path.insert(0, str(OUT.parents[1] / "wrinklefree-inference-engine_amd" / "python"))
    cache = {}
    orig_unpack = tbc._unpack_i2_to_ternary

    def unpack_memo(p, n, k):
        key = (p.data_ptr(), n, k)
        if key not in cache:
            cache[key] = orig_unpack(p, n, k)
        return cache[key]

    tbc._unpack_i2_to_ternary = unpack_memo
    mods = {"sglang": types.ModuleType("sglang"), "sglang.srt": types.ModuleType("sglang.srt"),
            "sglang.srt.models": types.ModuleType("sglang.srt.models"),
            "sglang.srt.models.bitnet": types.ModuleType("sglang.srt.models.bitnet"),
            "sgl_kernel": types.ModuleType("sgl_kernel"), "sgl_kernel.quantization": types.ModuleType("sgl_kernel.quantization"),
            "sgl_kernel.quantization.bitnet": types.ModuleType("sgl_kernel.quantization.bitnet")}
    mods["sglang.srt.models.bitnet"]._unpack_ternary_weights = tbc._unpack_ternary_weights
    mods["sglang.srt.models.bitnet"]._pack_ternary_weights = tbc._pack_ternary_weights
    mods["sgl_kernel.quantization.bitnet"].bitnet_gemv = tbc.bitnet_gemv_reference
    mods["sgl_kernel.quantization.bitnet"].quantize_activations_i8 = tbc.quantize_activations_i8
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        dif = _load_by_path("ref_direct_inference_full", REF / "scripts/direct_inference_full.py")
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
        tbc._unpack_i2_to_ternary = orig_unpack
    sys.modules["ref_direct_inference_full"] = dif
    tbc._unpack_i2_to_ternary = unpack_memo
    cfg = fi.config()
    w = fi.weights(cfg)
    kh, vh = fi.history(cfg)
    L, H, HKV, D = cfg.layers, cfg.hidden, cfg.n_kv_heads, cfg.head_dim
    bf = torch.bfloat16
    m = object.__new__(dif.DirectBitNetInference)
    m.device, m.dtype = "cpu", bf
    m.hidden_dim, m.n_layers, m.n_heads, m.n_kv_heads = H, L, cfg.n_heads, HKV
    m.head_dim, m.mlp_hidden, m.vocab_size, m.rms_eps, m.rope_theta = D, cfg.inter, cfg.vocab, cfg.eps, cfg.rope_theta
    m.rope = dif.RotaryEmbedding(D, max_seq_len=cfg.max_seq, base=cfg.rope_theta)
    m.embed_tokens = w["embed"]
    m.lm_head = m.embed_tokens
    m.final_norm = w["final_norm"]
    ws = w["wscale"].numpy()
    names = [("q_proj", "wq"), ("k_proj", "wk"), ("v_proj", "wv"), ("o_proj", "wo"), ("gate_proj", "wg"),
             ("up_proj", "wu"), ("down_proj", "wd")]
    m.layers = []
    for li in range(L):
        lay = {"input_layernorm": w["ln_in"][li], "post_attention_layernorm": w["ln_post"][li],
               "attn_sub_norm": w["attn_sub"][li], "ffn_sub_norm": w["ffn_sub"][li]}
        for j, (rn, wn) in enumerate(names):
            lay[rn] = w[wn][li].contiguous()
            lay[rn.replace("_proj", "_scale")] = float(ws[li, j])
        m.layers.append(lay)
    m.max_seq_len = cfg.max_seq
    m.k_cache = torch.zeros(L, cfg.max_seq, HKV, D, dtype=bf)
    m.v_cache = torch.zeros(L, cfg.max_seq, HKV, D, dtype=bf)
    m.k_cache[:, :fi.CTX0] = kh.transpose(1, 2)
    m.v_cache[:, :fi.CTX0] = vh.transpose(1, 2)
    return m, cfg, w, kh, vh, fi, unpack_memo, orig_unpack


def gen_decode_full(sdpa_fp32: bool = False):
    """The reference's OWN decode loop at the 2B-4T geometry (2 layers, full width and vocabulary):
    scripts/direct_inference_full.py's DirectBitNetInference.forward_layer / rms_norm / attention /
    mlp / bitnet_linear and its RotaryEmbedding, run on an instance whose weights are set directly
    (its __init__ reads a checkpoint from disk, :74-112). The script imports two un-vendored modules
    (sglang.srt.models.bitnet, sgl_kernel.quantization.bitnet, :21-22); they are provided here by the
    reference's own restatements of the same functions in tests/test_bitnet_core.py (the
    _unpack/_pack_ternary_weights copies :21-106, quantize_activations_i8 :139-146 and
    bitnet_gemv_reference :149-167, which `ref_linear` above uses too), with the unpacked weights
    memoised per tensor (same values, fewer host loops). Inputs: tests/golden/full_inputs.py.
    Stored: per position the hidden state after each layer, the K / V rows each layer appends, the
    top-64 logits (indices + bf16 values) and the greedy token; sha256 of the regenerated inputs.

    sdpa_fp32 (decode_full_f32attn.npz): the same loop with the one call whose CPU bf16 arithmetic
    is not reproducible elsewhere -- torch's CPU flash SDPA on bf16 tensors, which rounds the
    softmax probabilities to bf16 before P.V (measured: ~20-40 % of a 961-key output's elements
    differ from the exactly rounded result by >= 1 bf16 ulp) -- evaluated on the same bf16 q / K /
    V upcast to fp32 and rounded to bf16 once (the script's F.scaled_dot_product_attention call
    :241 routed through an upcasting wrapper); every other op is the reference's own."""
    m, cfg, w, kh, vh, fi, unpack_memo, orig_unpack = reference_decoder()
    dif = sys.modules["ref_direct_inference_full"]
    if sdpa_fp32:
        class _F:  # the script's `F` module with the SDPA call upcast
            def __getattr__(self, name):
                return getattr(F, name)

            @staticmethod
            def scaled_dot_product_attention(q, k, v, **kw):
                return F.scaled_dot_product_attention(q.float(), k.float(), v.float(), **kw).to(q.dtype)
        dif.F = _F()
    L = cfg.layers
    tbc._unpack_i2_to_ternary = unpack_memo
    tokens, nexts, hidden, krows, vrows, tidx, tval = [], [], [], [], [], [], []
    tok = fi.FIRST_TOKEN
    with torch.no_grad():
        for i in range(fi.POSITIONS):
            pos = fi.CTX0 + i
            hid = m.embed_tokens[tok]  # DirectBitNetInference.forward (:285-300), one layer at a time
            hs = []
            for li in range(L):
                hid = m.forward_layer(hid, li, pos)
                hs.append(bf16_bits(hid))
            logits = F.linear(m.rms_norm(hid, m.final_norm), m.lm_head)
            nxt = int(logits.argmax().item())  # sample(temperature=0) (:304-306)
            top = torch.topk(logits.float(), fi.TOPK)
            tokens.append(tok)
            nexts.append(nxt)
            hidden.append(np.stack(hs))
            krows.append(np.stack([bf16_bits(m.k_cache[li, pos].flatten()) for li in range(L)]))
            vrows.append(np.stack([bf16_bits(m.v_cache[li, pos].flatten()) for li in range(L)]))
            tidx.append(top.indices.numpy().astype(np.int32))
            tval.append(bf16_bits(logits[top.indices]))
            tok = nxt
    tbc._unpack_i2_to_ternary = orig_unpack
    dif.F = F
    return save("decode_full_f32attn" if sdpa_fp32 else "decode_full", tokens=np.array(tokens, np.int64), next=np.array(nexts, np.int64),
                hidden=np.stack(hidden), k_rows=np.stack(krows), v_rows=np.stack(vrows),
                top_idx=np.stack(tidx), top_val=np.stack(tval), ctx0=np.int64(fi.CTX0),
                input_sha256=np.array(fi.input_digest(w, kh, vh)))


def gen_msb():
    """SGLang BitNet linear method: quantize_to_bitnet (bitnet_quantization.py:69-109),
    dequantize_bitnet (:211-252, LUT path: numba is absent), BitNetLinearMethod.apply (:366-409) in
    bf16 and fp16 with and without bias, and the activation-sparsity masks (activation_sparsity.py)."""
    from wrinklefree_inference.sglang_backend import activation_sparsity as rsp
    from wrinklefree_inference.sglang_backend import bitnet_quantization as rbq
    g = torch.Generator().manual_seed(12)
    out = {}
    # ternarisation: fp32 / bf16 / fp16 weights, an all-zero matrix (scale -> 1.0) and exact +-0.5 ties
    w32 = torch.randn(96, 256, generator=g)
    wb = (torch.randn(64, 384, generator=g) * 0.3).to(torch.bfloat16)
    wh = (torch.randn(32, 128, generator=g) * 3.0).to(torch.float16)
    wz = torch.zeros(8, 128)
    wt = torch.zeros(4, 128)
    wt[0, :8] = torch.tensor([2.0, 1.0, -1.0, 0.999, -1.001, 1.001, -2.0, 0.0])
    wt[1:, :] = torch.randn(3, 128, generator=g)
    for name, w in (("w32", w32), ("wb", wb), ("wh", wh), ("wz", wz), ("wt", wt)):
        packed, scale = rbq.quantize_to_bitnet(w)
        out[f"{name}_in"] = w.float().numpy()
        out[f"{name}_dtype"] = np.array({torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[w.dtype])
        out[f"{name}_packed"] = packed.numpy()
        out[f"{name}_scale"] = np.array(scale, dtype=np.float64)
        out[f"{name}_deq"] = rbq.dequantize_bitnet(packed, scale, w.shape[0], w.shape[1]).numpy()
    # linear: N=192, K=1024 packed from random weights
    wl = torch.randn(192, 1024, generator=g)
    pl, sl = rbq.quantize_to_bitnet(wl)
    out["lin_packed"], out["lin_scale"] = pl.numpy(), np.array(sl, dtype=np.float64)
    bias = torch.randn(192, generator=g)
    out["lin_bias"] = bias.numpy()
    for m in (1, 3, 32):
        x = torch.randn(m, 1024, generator=g)
        out[f"lin_x{m}"] = x.numpy()
        for dt, tag in ((torch.bfloat16, "bf"), (torch.float16, "h")):
            meth = rbq.BitNetLinearMethod(compute_dtype=dt)
            y = meth.apply(pl, sl, x, 192, 1024)
            yb = meth.apply(pl, sl, x, 192, 1024, bias=bias)
            out[f"lin_y{m}_{tag}"] = y.view(torch.int16).numpy().view(np.uint16)
            out[f"lin_yb{m}_{tag}"] = yb.view(torch.int16).numpy().view(np.uint16)
    # activation sparsity (float32 activations, 4 tokens; checked in tests/test_oracle_golden.py)
    xs = torch.randn(4, 256, generator=g) * torch.linspace(0.2, 3.0, 4).unsqueeze(1)
    out["sp_x"] = xs.numpy()
    out["sp_topk"], out["sp_topk_r"] = rsp.apply_top_k_sparsity(xs, 0.4)[0].numpy(), np.array(0.6)
    thr, r = rsp.apply_threshold_sparsity(xs, 0.5)
    out["sp_thr"], out["sp_thr_r"] = thr.numpy(), np.array(r)
    ad, r = rsp.apply_adaptive_sparsity(xs, 0.3, 0.7)
    out["sp_adapt"], out["sp_adapt_r"] = ad.numpy(), np.array(r)
    return save("msb", **out)


GENERATORS = {"packing": lambda: gen_packing(), "quant": lambda: gen_quant(), "gemv": lambda: gen_gemv(),
              "linear": lambda: gen_linear(), "kv": lambda: gen_kv(), "attention": lambda: gen_attention(),
              "decode": lambda: gen_decode(), "msb": lambda: gen_msb(), "decode_full": lambda: gen_decode_full(),
              "decode_full_f32attn": lambda: gen_decode_full(sdpa_fp32=True)}


def main():
    torch.set_num_threads(8)
    names = sys.argv[1:] or list(GENERATORS)
    paths = [GENERATORS[n]() for n in names]
    mpath = OUT / "manifest.json"
    manifest = json.loads(mpath.read_text()) if mpath.exists() else {}
    manifest.update({p.name: hashlib.sha256(p.read_bytes()).hexdigest() for p in paths})
    manifest["_generator"] = "tests/golden/make_golden.py (reference @ /root/reference, torch " + torch.__version__ + ")"
    mpath.write_text(json.dumps(manifest, indent=2, sort_keys=True) + "\n")
    for p in paths:
        print(f"{p.name}: {p.stat().st_size} bytes")


if __name__ == "__main__":
    main()
