"""The GPU decode path against the REFERENCE's own decode loop at the 2B-4T geometry
(tests/golden/decode_full*.npz; tests/test_full_width_golden.py pins the oracle to the same
fixtures): 2 full-width layers, vocab 128256, a 960-position K/V history, 64 teacher-forced
positions.

* decode_full_f32attn -- the reference's loop (scripts/direct_inference_full.py) with its SDPA
  evaluated in fp32: the oracle reproduces it bit for bit, so this is north_star's 1e-3 bar against
  the reference itself. Compared per position: the K / V rows both layers append, the top-64 logits
  (the reference's indices), the greedy token where the top-2 gap is clear. A "flip" = a position
  above 1e-3 in any of them (see test_full_width_golden.py for why one bf16 boundary case becomes a
  ~1e-2 change two ops later); the allowed count is derived from the measurement recorded in
  DESIGN.md §5, and a flip must stay below 2e-2.
* decode_full (the reference exactly as it runs, CPU bf16 SDPA): the paths whose attention follows
  that SDPA's arithmetic (k_attn_sdpa: 512-key blocks, running max, fexp_u20 probabilities rounded
  to bf16; oracle/wf_oracle.c orc_attention_sdpa_cpu_bf16) are held to north_star's bar against it,
  teacher-forced per position (the token and the reference's K / V rows of the position, so one
  position's flip does not follow every later position through its cache row): <= 3 flips of 64,
  each < 3e-2 -- the oracle's own restatement measures 3 (tests/test_full_width_golden.py).

Paths: batch 1 (graph-replayed step), the batched matrix-core step at batch 128 (the golden sequence
in row 0 of a paged batch, other rows at random contexts) and the prefill (the 64 tokens as one
prompt chunk on top of the history: every K / V row it writes; the compared rows of layers 0 and 1
depend only on the position's own layer-0 output, so a flip stays in its position without forcing)."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
from test_full_width_golden import regenerate, rel_l2  # noqa: E402

pytestmark = pytest.mark.gpu

FLIP = 1e-3
FLIP_MAX = 2e-2


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from wfamd import _lib
    assert _lib.kernel_available(), "gfx950 kernels must load on the GPU box (no fallback)"
    torch.cuda.set_device(0)


def bits(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().view(torch.int16).cpu().numpy().view(np.uint16)


def f32(b) -> np.ndarray:
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def to_dev(w):
    return {k: (v if k == "wscale" else v.cuda()) for k, v in w.items()}


def check(fixture, g, i, krows, vrows, logits, token, flips, stats):
    """Compare position i; returns nothing, appends to flips / stats."""
    L = g["k_rows"].shape[1]
    ek = [rel_l2(f32(krows[l]), f32(g["k_rows"][i, l])) for l in range(L)]
    ev = [rel_l2(f32(vrows[l]), f32(g["v_rows"][i, l])) for l in range(L)]
    el = rel_l2(f32(logits[g["top_idx"][i]]), f32(g["top_val"][i])) if logits is not None else 0.0
    assert ek[0] < FLIP and ev[0] < FLIP, (fixture, i, ek, ev)  # layer 0: no attention upstream
    worst = max(ek + ev + [el])
    stats.append(worst)
    if worst >= FLIP:
        flips.append((i, [round(e, 4) for e in ek + ev], round(el, 4)))
        return
    if token is not None:
        top = f32(g["top_val"][i])
        if top[0] - top[1] > 1e-2 * abs(top[0]):
            assert token == int(g["next"][i]), (fixture, i)


def verdict(fixture, path, flips, stats, P):
    print(f"{path} vs reference {fixture}: {P} positions, median worst rel-L2 {np.median(stats):.2e}, "
          f"flips {len(flips)}: {flips}")
    # decode_full_f32attn (measured): 0-2 flips per 64 positions; decode_full: the
    # oracle's restatement of the reference's SDPA flips 3 (summation-order ties); allowance 3
    assert len(flips) <= 3, flips
    bound = FLIP_MAX if fixture == "decode_full_f32attn" else 3e-2
    assert all(e < bound for _, es, el in flips for e in es + [el]), flips


@pytest.mark.parametrize("fixture", ["decode_full"])
def test_batch1_vs_reference_decode_loop(fixture):
    from wfamd.model import BitNetDecoder
    cfg, w, kh, vh, g = regenerate(fixture)
    dec = BitNetDecoder(cfg, to_dev(w), batch=1)
    del w
    for l in range(cfg.layers):
        dec.load_kv(l, kh[l][None].cuda(), vh[l][None].cuda())
    ctx0, P = int(g["ctx0"]), len(g["tokens"])
    flips, stats = [], []
    for i in range(P):
        pos = ctx0 + i
        dec.set_state([int(g["tokens"][i])], [pos])
        dec.step(graph=True)
        torch.cuda.synchronize()
        kr = [bits(dec.k_cache[l, 0, :, pos].flatten()) for l in range(cfg.layers)]
        vr = [bits(dec.v_cache[l, 0, :, pos].flatten()) for l in range(cfg.layers)]
        check(fixture, g, i, kr, vr, bits(dec.logits[0]), int(dec.tokens[0]), flips, stats)
        for l in range(cfg.layers):  # teacher-forced cache: the reference's rows of this position
            dec.k_cache[l, 0, :, pos] = torch.from_numpy(g["k_rows"][i, l].view(np.int16)).view(torch.bfloat16).view(
                cfg.n_kv_heads, cfg.head_dim).cuda()
            dec.v_cache[l, 0, :, pos] = torch.from_numpy(g["v_rows"][i, l].view(np.int16)).view(torch.bfloat16).view(
                cfg.n_kv_heads, cfg.head_dim).cuda()
    verdict(fixture, "batch 1", flips, stats, P)


def force_paged_row(dec, l, b, pos, krow, vrow):
    """Write the reference's K / V row (bf16 bits [Hkv * D]) at position pos of sequence b into its
    page (tile layouts): the teacher-forced cache of the batched path."""
    from wfamd.model import from_kv_tiles, to_kv_tiles
    H, D = dec.cfg.n_kv_heads, dec.cfg.head_dim
    page = int(dec.seq_pages[b][pos // 32])
    kt = dec.k_cache[l][page].reshape(H, 32, D)
    vt = dec.v_cache[l][page].reshape(H, 32, D)
    k, v = from_kv_tiles(kt, vt)
    k[:, pos % 32] = torch.from_numpy(krow.view(np.int16)).view(torch.bfloat16).view(H, D).cuda()
    v[:, pos % 32] = torch.from_numpy(vrow.view(np.int16)).view(torch.bfloat16).view(H, D).cuda()
    k2, v2 = to_kv_tiles(k, v)
    dec.k_cache[l][page].copy_(k2.reshape(dec.k_cache[l][page].shape))
    dec.v_cache[l][page].copy_(v2.reshape(dec.v_cache[l][page].shape))


@pytest.mark.parametrize("fixture", ["decode_full"])
def test_batch128_paged_vs_reference_decode_loop(fixture):
    from test_gpu_configs import logical_kv
    from wfamd.model import BitNetDecoder
    cfg, w, kh, vh, g = regenerate(fixture)
    B = 128
    ctx0, P = int(g["ctx0"]), len(g["tokens"])
    ctxs = np.random.default_rng(3).integers(1, 2048, size=B)
    ctxs[0] = ctx0
    pages = int(sum((c + P + 1 + 31) // 32 for c in ctxs))
    dec = BitNetDecoder(cfg, to_dev(w), batch=B, num_pages=pages, page_seed=1)
    del w
    gen = torch.Generator(device="cuda").manual_seed(9)
    cmax = int(ctxs.max())
    for l in range(cfg.layers):
        k = torch.randn(B, cfg.n_kv_heads, cmax, cfg.head_dim, generator=gen, device="cuda").to(torch.bfloat16)
        v = torch.randn(B, cfg.n_kv_heads, cmax, cfg.head_dim, generator=gen, device="cuda").to(torch.bfloat16)
        k[0, :, :ctx0] = kh[l].cuda()
        v[0, :, :ctx0] = vh[l].cuda()
        dec.load_kv(l, k, v, lengths=ctxs)
        del k, v
    for b in range(B):
        dec.reserve(b, int(ctxs[b]) + P + 1)
    dec.set_state([(31 * b + 5) % cfg.vocab for b in range(B)], [int(c) for c in ctxs])
    flips, stats = [], []
    for i in range(P):
        pos = ctx0 + i
        dec.tokens[0] = int(g["tokens"][i])  # teacher-forced row 0; the other rows run greedy
        dec.step(graph=True)
        torch.cuda.synchronize()
        kr, vr = [], []
        for l in range(cfg.layers):
            kg, vg = logical_kv(dec, l, 0, pos + 1)
            kr.append(bits(kg[:, pos].flatten()))
            vr.append(bits(vg[:, pos].flatten()))
        check(fixture, g, i, kr, vr, bits(dec.logits[0]), int(dec.tokens[0]), flips, stats)
        for l in range(cfg.layers):  # teacher-forced cache: the reference's rows of this position
            force_paged_row(dec, l, 0, pos, g["k_rows"][i, l], g["v_rows"][i, l])
    verdict(fixture, "batch 128 (row 0, paged)", flips, stats, P)


@pytest.mark.parametrize("fixture", ["decode_full"])
def test_prefill_vs_reference_decode_loop(fixture):
    """The 64 golden tokens as one prompt chunk at positions 960..1023 of a slot holding the
    history (batch-16 paged decoder): every K / V row the prefill writes vs the reference's rows."""
    from test_gpu_configs import logical_kv
    from wfamd.model import BitNetDecoder
    cfg, w, kh, vh, g = regenerate(fixture)
    B = 16
    ctx0, P = int(g["ctx0"]), len(g["tokens"])
    dec = BitNetDecoder(cfg, to_dev(w), batch=B, num_pages=B * ((ctx0 + P + 32) // 32 + 1), page_seed=2)
    del w
    ln = np.zeros(B, dtype=np.int64)
    ln[3] = ctx0
    for l in range(cfg.layers):
        k = torch.zeros(B, cfg.n_kv_heads, ctx0, cfg.head_dim, dtype=torch.bfloat16, device="cuda")
        v = torch.zeros_like(k)
        k[3], v[3] = kh[l].cuda(), vh[l].cuda()
        dec.load_kv(l, k, v, lengths=ln)
    dec.prefill([(3, [int(t) for t in g["tokens"]], ctx0)])
    torch.cuda.synchronize()
    flips, stats = [], []
    kl = [logical_kv(dec, l, 3, ctx0 + P) for l in range(cfg.layers)]
    for i in range(P):
        pos = ctx0 + i
        kr = [bits(kl[l][0][:, pos].flatten()) for l in range(cfg.layers)]
        vr = [bits(kl[l][1][:, pos].flatten()) for l in range(cfg.layers)]
        check(fixture, g, i, kr, vr, None, None, flips, stats)
    verdict(fixture, "prefill (64-token chunk)", flips, stats, P)
