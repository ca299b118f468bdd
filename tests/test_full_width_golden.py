"""The oracle against the reference's OWN decode loop at the 2B-4T geometry (tests/golden/
decode_full.npz, made by tests/golden/make_golden.py gen_decode_full from
scripts/direct_inference_full.py's DirectBitNetInference methods): 2 full-width layers, vocab
128256, a 960-position random K/V history, 64 teacher-forced decode positions.

This pins the oracle where every batched / prefill / full-width GPU test uses it as the checker,
and MEASURES the oracle-vs-reference flip rate those tests' allowances are derived from: a
position "flips" when one bf16 element of an attention output lands on the other side of a
rounding boundary between two implementations (the reference's bf16 SDPA vs the oracle's double
attention) and the int8 requantisation of the next GEMV input turns it into whole code steps."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(GOLDEN))
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))

FLIP = 1e-3  # north_star's bf16 tolerance; a position above it in any compared quantity is a flip


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def load_fixture(name: str = "decode_full"):
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def regenerate(name: str = "decode_full"):
    """(cfg, weights, K history, V history) on the CPU, checked against the fixture's input sha256."""
    import full_inputs as fi
    g = load_fixture(name)
    cfg = fi.config()
    w = fi.weights(cfg)
    kh, vh = fi.history(cfg)
    assert fi.input_digest(w, kh, vh) == str(g["input_sha256"]), "regenerated inputs differ from the fixture's"
    return cfg, w, kh, vh, g


def compare_position(g, i, krows, vrows, top_vals, layers):
    """Per-layer K / V row rel-L2 and the top-64 logits' rel-L2 of position i (bf16 bits in)."""
    from oracle.oracle import bf16_to_f32
    ek = [rel_l2(bf16_to_f32(krows[l]), bf16_to_f32(g["k_rows"][i, l])) for l in range(layers)]
    ev = [rel_l2(bf16_to_f32(vrows[l]), bf16_to_f32(g["v_rows"][i, l])) for l in range(layers)]
    el = rel_l2(bf16_to_f32(top_vals), bf16_to_f32(g["top_val"][i]))
    return ek, ev, el


@pytest.mark.parametrize("fixture,attn_mode", [("decode_full", 1), ("decode_full_f32attn", 0)])
def test_oracle_full_width_vs_reference_decode_loop(orc, fixture, attn_mode):
    """K / V rows of both layers and the top-64 logits of all 64 positions vs the reference, teacher
    forced (the token AND, for decode_full, the reference's K / V rows: each position then starts
    from the reference's own state, so one position's flip does not follow every later position
    through its cache row); layer 0's rows (computed from the token embedding alone) bit-exact;
    greedy token equal wherever the reference's top-2 gap is clear.
    decode_full (the reference exactly as it runs, CPU bf16 SDPA) against the oracle's restatement
    of that SDPA (attn_mode 1): <= 3 flipped positions of 64 (measured 3: positions 0, 25, 63 --
    summation-order ties of the SDPA's GEMMs, tests/golden/sdpa_probe.py).
    decode_full_f32attn (the reference's loop with its SDPA evaluated in fp32) against the exact
    softmax (attn_mode 0): bit-exact everywhere, cache not forced."""
    cfg, w, kh, vh, g = regenerate(fixture)
    import torch
    from wfamd.model import rope_tables
    cos, sin = rope_tables(cfg.head_dim, cfg.max_seq, cfg.rope_theta)
    bits = lambda t: t.contiguous().view(torch.int16).numpy().view(np.uint16)
    a = {"cfg": np.array([cfg.hidden, cfg.layers, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.inter, cfg.vocab,
                          cfg.max_seq], dtype=np.int64),
         "eps": np.float32(cfg.eps), "rope_cos": bits(cos), "rope_sin": bits(sin),
         "wscale": w["wscale"].numpy().astype(np.float32)}
    for n in ("wq", "wk", "wv", "wo", "wg", "wu", "wd"):
        a[n] = w[n].numpy()
    for n in ("embed", "final_norm", "ln_in", "ln_post", "attn_sub", "ffn_sub"):
        a[n] = bits(w[n])
    m = orc.DecodeModel(a, attn_mode=attn_mode)
    ctx0 = int(g["ctx0"])
    m.k_cache[:, :, :ctx0] = bits(kh)
    m.v_cache[:, :, :ctx0] = bits(vh)
    flips, worst = [], 0.0
    P = len(g["tokens"])
    for i in range(P):
        pos = ctx0 + i
        logits, nxt = m.step(int(g["tokens"][i]), pos)
        kr = m.k_cache[:, :, pos].reshape(cfg.layers, -1)
        vr = m.v_cache[:, :, pos].reshape(cfg.layers, -1)
        ek, ev, el = compare_position(g, i, kr, vr, logits[g["top_idx"][i]], cfg.layers)
        assert ek[0] == 0.0 and ev[0] == 0.0, (i, ek, ev)  # layer 0: bit-exact
        if max(ek + ev + [el]) >= FLIP:
            flips.append((i, [round(e, 4) for e in ek + ev], round(el, 4)))
        if attn_mode == 1:
            L, HKV, D = cfg.layers, cfg.n_kv_heads, cfg.head_dim
            m.k_cache[:, :, pos] = g["k_rows"][i].reshape(L, HKV, D)
            m.v_cache[:, :, pos] = g["v_rows"][i].reshape(L, HKV, D)
        if flips and flips[-1][0] == i:
            continue
        worst = max(worst, el)
        ref = orc.bf16_to_f32(g["top_val"][i])
        if ref[0] - ref[1] > 1e-2 * abs(ref[0]):
            assert nxt == int(g["next"][i]), i
    print(f"oracle (attn_mode {attn_mode}) vs reference ({fixture}), {P} positions: worst clean top-64 logits rel-L2 {worst:.2e}; "
          f"flips {len(flips)}: {flips}")
    if fixture == "decode_full_f32attn":
        # the reference's loop with its SDPA evaluated in fp32 and rounded once: the oracle IS that
        # computation -- every K / V row and every top-64 logit bit-identical, every greedy token equal
        assert not flips and worst == 0.0, flips
    else:
        # a flip is one bf16 attention element on the other side of a rounding boundary (an fp32
        # summation-order tie) turned into an int8 code step by attn_sub_norm's quantization
        assert len(flips) <= 3 and all(e < 3e-2 for _, es, el in flips for e in es + [el]), flips
