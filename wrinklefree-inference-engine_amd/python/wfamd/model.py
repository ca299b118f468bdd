"""BitNet b1.58 decode runner on the fused HIP decode step (wf_model_* in include/wf_bitnet.h).

Semantics follow scripts/direct_inference_full.py:181-302 (RMSNorm, BitNet linear with the
encoding correction, half-split RoPE θ=5e5, GQA SDPA, attn_sub_norm, ReLU² MLP with ffn_sub_norm,
tied bf16 LM head, greedy argmax). Per-token activation scales: sequence b of a batch computes
exactly what a batch-1 decode of that sequence computes.

Weights enter in the reference's canonical per-projection blocked I2_S layout
([layers, out, in/4]); `build_device_layout` fuses them into the kernel layout:
  * q|k|v rows concatenated; inside each 128-row head, row tile t holds dims 8t..8t+7 and
    64+8t..64+8t+7 (so the RoPE pairs land in one block);
  * gate/up interleaved in 8-row tiles [gate 8t..8t+7 | up 8t..8t+7];
  * optionally repacked to the ~1.6-bit TQ format (lossless, wf_i2s_to_tq).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib, ops
from ._lib import WF_FMT_I2S, WF_FMT_I2S_MFMA, WF_FMT_TQ, WFModelDesc, call


@dataclass
class BitNetConfig:
    hidden: int = 2560
    layers: int = 30
    n_heads: int = 20
    n_kv_heads: int = 5
    head_dim: int = 128
    inter: int = 6912
    vocab: int = 128256
    max_seq: int = 4096
    eps: float = 1e-5
    rope_theta: float = 500000.0

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    def ternary_weights(self) -> int:
        h, i, kv = self.hidden, self.inter, self.kv_dim
        return self.layers * (2 * h * h + 2 * kv * h + 3 * i * h)

    def weight_bytes_per_token(self, wfmt: int) -> int:
        """Algorithmic HBM bytes of one batch-1 decode step's weight stream (ternary + bf16 LM head)."""
        h, i, kv = self.hidden, self.inter, self.kv_dim
        rb = ops.tq_row_bytes if wfmt == WF_FMT_TQ else (lambda k: k // 4)
        tern = self.layers * ((h + 2 * kv) * rb(h) + h * rb(h) + 2 * i * rb(h) + h * rb(i))
        return tern + self.vocab * h * 2

    def kv_bytes_per_token(self, ctx: int) -> int:
        return self.layers * 2 * self.kv_dim * 2 * ctx


BITNET_2B = BitNetConfig()


def rope_tables(head_dim: int, max_seq: int, base: float):
    """scripts/direct_inference_full.py:31-44 (fp32 freqs, cos/sin cast to bf16)."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float32) / head_dim))
    fr = torch.outer(torch.arange(max_seq, dtype=torch.float32), inv)
    return torch.cos(fr).to(torch.bfloat16), torch.sin(fr).to(torch.bfloat16)


def _as_bf16(x, device) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        if x.dtype == np.uint16:
            return torch.from_numpy(x.astype(np.int16)).view(torch.bfloat16).to(device)
        return torch.from_numpy(x).to(device=device, dtype=torch.bfloat16)
    return x.to(device=device, dtype=torch.bfloat16)


def _as_u8(x, device) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x)).to(device)
    return x.to(device)


def qkv_row_permutation(n_heads_total: int, head_dim: int = 128) -> torch.Tensor:
    half = head_dim // 2
    per = []
    for t in range(half // 8):
        per.extend(range(8 * t, 8 * t + 8))
        per.extend(range(half + 8 * t, half + 8 * t + 8))
    per = torch.tensor(per, dtype=torch.long)
    return torch.cat([h * head_dim + per for h in range(n_heads_total)])


def gate_up_interleave(inter: int) -> torch.Tensor:
    idx = []
    for t in range(inter // 8):
        idx.extend(range(8 * t, 8 * t + 8))
        idx.extend(range(inter + 8 * t, inter + 8 * t + 8))
    return torch.tensor(idx, dtype=torch.long)


_LUT81 = None


def random_i2s(shape, generator: torch.Generator) -> torch.Tensor:
    """Uniform ternary weights (randint(-1, 2), scripts/benchmark_kernels.py:35) packed as I2_S bytes:
    every byte holds 4 independent enc codes in {0,1,2}. Generated on the generator's device."""
    global _LUT81
    dev = generator.device
    if _LUT81 is None or _LUT81.device != dev:
        lut = torch.zeros(81, dtype=torch.uint8)
        for v in range(81):
            d = [(v // 3 ** i) % 3 for i in range(4)]
            lut[v] = (d[0] << 6) | (d[1] << 4) | (d[2] << 2) | d[3]
        _LUT81 = lut.to(dev)
    idx = torch.randint(0, 81, shape, generator=generator, device=dev, dtype=torch.int64)
    return _LUT81[idx]


def synthetic_weights(cfg: BitNetConfig, seed: int = 0, device="cuda") -> Dict[str, torch.Tensor]:
    """Random-init weights of the bitnet-b1.58-2B-4T architecture (no checkpoint offline)."""
    device = torch.device(device)
    g = torch.Generator(device=device).manual_seed(seed)
    h, i, kv, L = cfg.hidden, cfg.inter, cfg.kv_dim, cfg.layers
    w = {}
    shapes = {"wq": (h, h // 4), "wk": (kv, h // 4), "wv": (kv, h // 4), "wo": (h, h // 4),
              "wg": (i, h // 4), "wu": (i, h // 4), "wd": (h, i // 4)}
    for name, shp in shapes.items():
        w[name] = torch.stack([random_i2s(shp, g) for _ in range(L)])
    w["embed"] = (torch.randn(cfg.vocab, h, generator=g, device=device) * 0.02).to(torch.bfloat16)
    w["final_norm"] = (1.0 + 0.1 * torch.randn(h, generator=g, device=device)).to(torch.bfloat16)
    for name, n in (("ln_in", h), ("ln_post", h), ("attn_sub", h), ("ffn_sub", i)):
        w[name] = (1.0 + 0.1 * torch.randn(L, n, generator=g, device=device)).to(torch.bfloat16)
    w["wscale"] = (torch.rand(L, 7, generator=g, device=device) * 0.5 + 1.5).to(torch.float32).cpu()
    return w


def weights_from_arrays(a: dict, device="cuda") -> Dict[str, torch.Tensor]:
    """Host arrays in the tests/golden/decode.npz layout -> device tensors."""
    w = {n: _as_u8(a[n], device) for n in ("wq", "wk", "wv", "wo", "wg", "wu", "wd")}
    for n in ("embed", "final_norm", "ln_in", "ln_post", "attn_sub", "ffn_sub"):
        w[n] = _as_bf16(a[n], device)
    w["wscale"] = torch.from_numpy(np.asarray(a["wscale"], dtype=np.float32))
    return w


def build_device_layout(cfg: BitNetConfig, w: Dict[str, torch.Tensor], wfmt: int = WF_FMT_I2S):
    """Fuse per-projection I2_S weights into the kernel layout (and repack to TQ if asked)."""
    dev = w["wq"].device
    hq_tot = cfg.n_heads + 2 * cfg.n_kv_heads
    perm = qkv_row_permutation(hq_tot, cfg.head_dim).to(dev)
    gu = gate_up_interleave(cfg.inter).to(dev)
    out = {"w_qkv": [], "w_o": [], "w_gu": [], "w_d": []}
    for l in range(cfg.layers):
        qkv = torch.cat([w["wq"][l], w["wk"][l], w["wv"][l]], dim=0).index_select(0, perm)
        gate_up = torch.cat([w["wg"][l], w["wu"][l]], dim=0).index_select(0, gu)
        parts = {"w_qkv": qkv, "w_o": w["wo"][l], "w_gu": gate_up, "w_d": w["wd"][l]}
        for name, t in parts.items():
            t = t.contiguous()
            if wfmt == WF_FMT_TQ:
                t = ops.i2s_to_tq(t)
            elif wfmt == WF_FMT_I2S_MFMA:
                t = ops.i2s_to_mfma(t)
            out[name].append(t)
    return {k: torch.stack(v).contiguous() for k, v in out.items()}


def to_kv_tiles(k: torch.Tensor, v: torch.Tensor):
    """Logical K/V [..., S, 128] -> the tile layouts of the batched decode (include/wf_bitnet.h;
    csrc/wf_norm.h k_tile_off / v_tile_off), same shapes. Key t = 32 blk + 8 a + 4 tau + r."""
    *lead, S, D = k.shape
    assert D == 128 and S % 32 == 0
    kt = k.reshape(*lead, S // 32, 4, 2, 4, 16, 8)            # blk, a, tau, r, dg, e
    nl = len(lead)
    kt = kt.permute(*range(nl), nl, nl + 2, nl + 4, nl + 1, nl + 3, nl + 5)  # blk, tau, dg, a, r, e
    vt = v.reshape(*lead, S // 32, 4, 8, 8, 16)                # blk, q, e, n, l
    vt = vt.permute(*range(nl), nl, nl + 3, nl + 1, nl + 4, nl + 2)          # blk, n, q, l, e
    return kt.reshape(*lead, S, D).contiguous(), vt.reshape(*lead, S, D).contiguous()


def from_kv_tiles(kt: torch.Tensor, vt: torch.Tensor):
    """Inverse of to_kv_tiles."""
    *lead, S, D = kt.shape
    nl = len(lead)
    k = kt.reshape(*lead, S // 32, 2, 16, 4, 4, 8)            # blk, tau, dg, a, r, e
    k = k.permute(*range(nl), nl, nl + 3, nl + 1, nl + 4, nl + 2, nl + 5)   # blk, a, tau, r, dg, e
    v = vt.reshape(*lead, S // 32, 8, 4, 16, 8)                # blk, n, q, l, e
    v = v.permute(*range(nl), nl, nl + 2, nl + 4, nl + 1, nl + 3)           # blk, q, e, n, l
    return k.reshape(*lead, S, D).contiguous(), v.reshape(*lead, S, D).contiguous()


def to_fp8_codes(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """bf16/fp32 values -> OCP e4m3fn codes (uint8) of clamp(x / scale, +-448), round to nearest even:
    what the decode step's cache epilogue stores for an FP8 K/V cache."""
    y = (x.float() / scale).clamp(-448.0, 448.0)
    return y.to(torch.float8_e4m3fn).view(torch.uint8)


def from_fp8_codes(c: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    return c.view(torch.float8_e4m3fn).float() * scale


def to_int8_codes(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """bf16/fp32 values -> int8 codes clamp(rne(x / scale), -127, 127) (stored as uint8 bytes): what
    the decode step's cache epilogue stores for an int8 K/V cache (the reference's KVCacheDtype.INT8,
    kv_cache/kv_cache.py:159-185, with a static scale)."""
    y = torch.round(x.float() / scale).clamp(-127.0, 127.0)
    return y.to(torch.int8).view(torch.uint8)


def from_int8_codes(c: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    return c.view(torch.int8).float() * scale


KV_CODES = {"fp8": (to_fp8_codes, from_fp8_codes), "int8": (to_int8_codes, from_int8_codes)}


def pack_prefill_rows(seqs, group: int = _lib.WF_PREFILL_ROW_GROUP):
    """(slot, tokens, start) triples -> the row arrays of wf_model_prefill (tokens, slots,
    positions): each slot's tokens at positions start, start + 1, ..., padded to a multiple of
    `group` rows by repeating its last (token, position) -- a repeat recomputes the same K/V row, so
    the pad is harmless -- so that every aligned group of `group` rows belongs to one slot."""
    tok, slot, pos = [], [], []
    for b, toks, start in seqs:
        n = len(toks)
        if n == 0:
            continue
        pad = (-n) % group
        tok += list(toks) + [toks[-1]] * pad
        pos += list(range(start, start + n)) + [start + n - 1] * pad
        slot += [b] * (n + pad)
    return tok, slot, pos


class PagePool:
    """Host-side free list of KV pages, with the semantics of sgl_kernel.kvcache.KVCacheManager's
    allocator (tests/test_kv_cache_cpp.py:283-373: allocate_pages(n) -> int32 ids, empty when the
    pool is short; free_pages(ids); num_free_pages()). Pages here hold 32 tokens of every kv head
    of every layer (the tile block of the batched attention); ids index the pool dimension of the
    decoder's k_cache / v_cache."""

    def __init__(self, num_pages: int, seed: Optional[int] = None):
        self.num_pages = int(num_pages)
        order = np.arange(self.num_pages, dtype=np.int32)
        if seed is not None:  # scattered placement (a long-running server's pool), not id order
            np.random.default_rng(seed).shuffle(order)
        self._free = list(order[::-1])

    def num_free_pages(self) -> int:
        return len(self._free)

    def allocate_pages(self, n: int) -> np.ndarray:
        if n > len(self._free):
            return np.zeros(0, dtype=np.int32)
        out = [self._free.pop() for _ in range(n)]
        return np.asarray(out, dtype=np.int32)

    def free_pages(self, ids) -> None:
        for i in np.asarray(ids, dtype=np.int64).reshape(-1):
            if 0 <= i < self.num_pages:  # out-of-range ids are ignored, as the reference twin's free_page (:66-69)
                self._free.append(int(i))


class BitNetDecoder:
    """Owns the device layout, the caller-side state tensors and the wf_model handle.

    num_pages > 0 (batch >= 16, I2_S): paged KV. k_cache / v_cache become a pool of 32-token pages
    [layers, num_pages, n_kv_heads, 32 * head_dim] and `page_table` [batch, max_seq / 32] maps each
    sequence's 32-token blocks to pages (include/wf_bitnet.h wf_model_desc.page_table); `reserve`
    / `release` grow and free a sequence's pages from `pool` between steps."""

    def __init__(self, cfg: BitNetConfig, weights: Dict[str, torch.Tensor], batch: int = 1,
                 wfmt: int = WF_FMT_I2S, device="cuda", debug_flags: int = 0, num_pages: int = 0,
                 page_seed: Optional[int] = None, kv_dtype: str = "bf16", kv_scale=None):
        self.cfg, self.batch, self.wfmt = cfg, batch, wfmt
        self.dev = torch.device(device)
        # batch >= 16 on I2_S runs the matrix-core GEMMs on their tile layout (same bytes, re-tiled)
        if wfmt == WF_FMT_I2S and batch >= 16 and cfg.hidden % 16 == 0 and cfg.inter % 16 == 0:
            wfmt = WF_FMT_I2S_MFMA
        self.wfmt_device = wfmt
        lay = build_device_layout(cfg, weights, wfmt)
        self.w_qkv, self.w_o, self.w_gu, self.w_d = lay["w_qkv"], lay["w_o"], lay["w_gu"], lay["w_d"]
        self.embed = weights["embed"].contiguous()
        self.final_norm = weights["final_norm"].contiguous()
        self.norms = {n: weights[n].contiguous() for n in ("ln_in", "ln_post", "attn_sub", "ffn_sub")}
        cos, sin = rope_tables(cfg.head_dim, cfg.max_seq, cfg.rope_theta)
        self.rope_cos, self.rope_sin = cos.to(self.dev).contiguous(), sin.to(self.dev).contiguous()
        self.wscale = weights["wscale"].detach().cpu().to(torch.float32).contiguous()
        L, B = cfg.layers, batch
        self.tokens = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.positions = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.logits = torch.zeros(B, cfg.vocab, dtype=torch.bfloat16, device=self.dev)
        # batch >= 16 on I2_S (the matrix-core decode path) keeps K and V in the tile layouts of
        # include/wf_bitnet.h (wf_model_desc.k_cache); to_kv_tiles / from_kv_tiles convert
        self.kv_tiled = batch >= 16 and wfmt in (WF_FMT_I2S, WF_FMT_I2S_MFMA) and cfg.max_seq % 32 == 0
        self.paged = num_pages > 0
        if self.paged:
            if not (self.kv_tiled and cfg.head_dim == 128):
                raise ValueError("paged KV needs batch >= 16, I2_S weights, head_dim 128 and max_seq % 32 == 0")
            kv_shape = (L, num_pages, cfg.n_kv_heads, 32 * cfg.head_dim)
            self.pool = PagePool(num_pages, page_seed)
            self.seq_pages = [np.zeros(0, dtype=np.int32) for _ in range(B)]
            self._pt_host = np.zeros((B, cfg.max_seq // 32), dtype=np.int32)
            self.page_table = torch.zeros((B, cfg.max_seq // 32), dtype=torch.int32, device=self.dev)
        else:
            kv_shape = (L, B, cfg.n_kv_heads, cfg.max_seq, cfg.head_dim)
        if kv_dtype not in ("bf16", "fp8", "int8"):
            raise ValueError(f"kv_dtype must be 'bf16', 'fp8' or 'int8', got {kv_dtype!r}")
        self.kv_dtype = kv_dtype
        self.kv_quant = {"bf16": _lib.WF_KV_BF16, "fp8": _lib.WF_KV_FP8, "int8": _lib.WF_KV_INT8}[kv_dtype]
        self.kv_fp8 = self.kv_quant != _lib.WF_KV_BF16  # one-byte codes (e4m3 or int8)
        if self.kv_fp8 and not self.kv_tiled:
            raise ValueError("FP8 / int8 K/V need the batched matrix-core decoder (batch >= 16, I2_S, max_seq % 32 == 0)")
        # one-byte codes as uint8 storage, per-layer (K, V) scales (include/wf_bitnet.h kv_quant)
        sc = np.ones((L, 2), dtype=np.float32) if kv_scale is None else np.broadcast_to(
            np.asarray(kv_scale, dtype=np.float32), (L, 2)).copy()
        self.kv_scale = torch.from_numpy(np.ascontiguousarray(sc))
        kv_dt = torch.uint8 if self.kv_fp8 else torch.bfloat16
        self.k_cache = torch.zeros(kv_shape, dtype=kv_dt, device=self.dev)
        self.v_cache = torch.zeros(kv_shape, dtype=kv_dt, device=self.dev)
        d = WFModelDesc()
        d.hidden, d.layers, d.n_heads, d.n_kv_heads = cfg.hidden, L, cfg.n_heads, cfg.n_kv_heads
        d.head_dim, d.inter, d.vocab, d.max_seq, d.batch = cfg.head_dim, cfg.inter, cfg.vocab, cfg.max_seq, B
        d.eps, d.wfmt = cfg.eps, wfmt
        d.embed, d.final_norm = self.embed.data_ptr(), self.final_norm.data_ptr()
        d.rope_cos, d.rope_sin = self.rope_cos.data_ptr(), self.rope_sin.data_ptr()
        d.ln_in, d.ln_post = self.norms["ln_in"].data_ptr(), self.norms["ln_post"].data_ptr()
        d.attn_sub, d.ffn_sub = self.norms["attn_sub"].data_ptr(), self.norms["ffn_sub"].data_ptr()
        d.w_qkv, d.w_o, d.w_gu, d.w_d = (t.data_ptr() for t in (self.w_qkv, self.w_o, self.w_gu, self.w_d))
        d.wscale = self.wscale.data_ptr()
        d.tokens, d.positions, d.logits = self.tokens.data_ptr(), self.positions.data_ptr(), self.logits.data_ptr()
        d.k_cache, d.v_cache = self.k_cache.data_ptr(), self.v_cache.data_ptr()
        d.debug_flags = int(debug_flags)
        if self.paged:
            d.page_table, d.num_pages = self.page_table.data_ptr(), int(num_pages)
        if self.kv_fp8:
            d.kv_quant, d.kv_scale = self.kv_quant, self.kv_scale.data_ptr()
        self._desc = d
        h = C.c_void_p()
        call("wf_model_create", C.addressof(d), C.addressof(h))
        self._h = h

    def __del__(self):
        try:
            if getattr(self, "_h", None) and self._h.value:
                _lib.load().wf_model_destroy(self._h)
                self._h = C.c_void_p()
        except Exception:
            pass

    def reserve(self, b: int, n_tokens: int) -> None:
        """Give sequence b pages for positions [0, n_tokens) (allocating only the missing blocks)."""
        need = (int(n_tokens) + 31) // 32 - len(self.seq_pages[b])
        if need <= 0:
            return
        if need + len(self.seq_pages[b]) > self._pt_host.shape[1]:
            raise ValueError(f"sequence {b}: {n_tokens} tokens exceed max_seq {self.cfg.max_seq}")
        got = self.pool.allocate_pages(need)
        if len(got) != need:
            raise RuntimeError(f"KV page pool exhausted ({self.pool.num_free_pages()} free, {need} needed)")
        self.seq_pages[b] = np.concatenate([self.seq_pages[b], got])
        self._pt_host[b, :len(self.seq_pages[b])] = self.seq_pages[b]
        self.page_table[b].copy_(torch.from_numpy(self._pt_host[b]))

    def map_pages(self, b: int, pages) -> None:
        """Point sequence b's 32-token blocks at `pages` (block j -> pages[j]): pages a caller allocated
        from this decoder's pool itself, e.g. through sgl_kernel.kvcache.KVCacheManager(backing=self),
        the reference's paged-KV API over the same pool (tests/test_kv_cache_cpp.py:283-373). The
        decoder releases them with the sequence (release)."""
        pg = np.asarray(pages, dtype=np.int32).reshape(-1)
        if not self.paged:
            raise ValueError("map_pages needs a paged decoder (num_pages > 0)")
        if len(pg) > self._pt_host.shape[1] or ((pg < 0) | (pg >= self.pool.num_pages)).any():
            raise ValueError(f"sequence {b}: bad page list ({len(pg)} pages, pool of {self.pool.num_pages})")
        self.seq_pages[b] = pg.copy()
        self._pt_host[b] = 0
        self._pt_host[b, :len(pg)] = pg
        self.page_table[b].copy_(torch.from_numpy(self._pt_host[b]))

    def release(self, b: int) -> None:
        """Return sequence b's pages to the pool (a finished request)."""
        self.pool.free_pages(self.seq_pages[b])
        self.seq_pages[b] = np.zeros(0, dtype=np.int32)
        self._pt_host[b] = 0
        self.page_table[b].zero_()

    def prefill(self, seqs, chunk_rows: int = 4096) -> None:
        """Prompt pass (include/wf_bitnet.h wf_model_prefill): `seqs` = iterable of (slot, tokens,
        start); token i of a slot is processed at position start + i and its K/V lands in the
        slot's cache (pages reserved on demand). Rows are packed per slot, padded to a multiple of
        WF_PREFILL_ROW_GROUP by repeating the slot's last token, and run `chunk_rows` at a time. The decode state
        (tokens / positions / logits) is left alone: see admit()."""
        seqs = [(int(b), [int(t) for t in toks], int(start)) for b, toks, start in seqs]
        for b, toks, start in seqs:
            if start + len(toks) > self.cfg.max_seq:
                raise ValueError(f"slot {b}: positions up to {start + len(toks)} exceed max_seq {self.cfg.max_seq}")
            if self.paged and toks:
                self.reserve(b, start + len(toks))
        tok, slot, pos = pack_prefill_rows(seqs)
        rows = len(tok)
        if rows == 0:
            return
        g = _lib.WF_PREFILL_ROW_GROUP
        chunk_rows = max(g, chunk_rows // g * g)
        call("wf_model_prefill_reserve", self._h, min(rows, chunk_rows))
        t = torch.tensor(tok, dtype=torch.int32, device=self.dev)
        sl = torch.tensor(slot, dtype=torch.int32, device=self.dev)
        ps = torch.tensor(pos, dtype=torch.int32, device=self.dev)
        st = torch.cuda.current_stream().cuda_stream
        for r0 in range(0, rows, chunk_rows):
            n = min(rows - r0, chunk_rows)
            call("wf_model_prefill", self._h, t[r0:].data_ptr(), sl[r0:].data_ptr(), ps[r0:].data_ptr(), n, st)
        self._pf_keep = (t, sl, ps)  # alive until the stream has consumed them

    def prefill_view(self, rows: int):
        """The last prefill call's last layer (include/wf_bitnet.h wf_model_prefill_view): q rows
        after RoPE and the causal attention output rows, [rows, Hq, D] bf16 copies on the device."""
        qp, ap = C.c_void_p(), C.c_void_p()
        call("wf_model_prefill_view", self._h, C.byref(qp), C.byref(ap))
        cfg = self.cfg
        out = []
        for p in (qp, ap):
            t = torch.empty(rows, cfg.n_heads, cfg.head_dim, dtype=torch.bfloat16, device=self.dev)
            ops.device_copy(t.data_ptr(), p.value, t.numel() * 2)
            out.append(t)
        return out[0], out[1]

    def admit(self, b: int, prompt) -> None:
        """Start sequence `prompt` in slot b: prefill all but its last token, then the next decode
        step runs the last token at position len - 1 (scripts/direct_inference_full.py's loop)."""
        prompt = [int(x) for x in prompt]
        if not prompt:
            raise ValueError("empty prompt")
        self.prefill([(b, prompt[:-1], 0)])
        if self.paged:
            self.reserve(b, len(prompt))
        self.tokens[b] = prompt[-1]
        self.positions[b] = len(prompt) - 1

    def set_state(self, tokens, positions) -> None:
        self.tokens.copy_(torch.as_tensor(tokens, dtype=torch.int32))
        self.positions.copy_(torch.as_tensor(positions, dtype=torch.int32))

    def fill_kv_random(self, ctx: int, seed: int = 0) -> None:
        """Synthetic context: random bf16 K/V for positions [0, ctx) of every sequence (storage
        order; in the tile layouts whole 32-key blocks)."""
        g = torch.Generator(device=self.dev).manual_seed(seed)
        D = self.cfg.head_dim
        if self.kv_fp8:  # random finite codes (the whole store: stale rows are never read)
            enc = KV_CODES[self.kv_dtype][0]
            for l in range(self.cfg.layers):
                for j, c in enumerate((self.k_cache, self.v_cache)):
                    c[l].copy_(enc(torch.randn(c[l].shape, generator=g, device=self.dev), float(self.kv_scale[l, j])))
            return
        for l in range(self.cfg.layers):
            for c in (self.k_cache, self.v_cache):
                if self.paged:
                    c[l].normal_(generator=g)
                elif self.kv_tiled:
                    B, H, S, _ = c[l].shape
                    c[l].view(B, H, S * D)[..., :(ctx + 31) // 32 * 32 * D].normal_(generator=g)
                else:
                    c[l, :, :, :ctx].normal_(generator=g)

    def load_kv(self, layer: int, k: torch.Tensor, v: torch.Tensor, lengths=None) -> None:
        """Write logical K/V [B, Hkv, n, D] into positions [0, n) of a layer (any storage layout).
        Paged: only the first lengths[b] (default n) positions of sequence b, on pages reserved for them."""
        n = k.shape[2]
        if self.kv_fp8:  # the stored codes, as the step's cache epilogue writes them
            ks, vs = (float(x) for x in self.kv_scale[layer])
            enc = KV_CODES[self.kv_dtype][0]
            k = enc(k, ks)
            v = enc(v, vs)
        if self.paged:
            B, H, _, D = k.shape
            nblk = (n + 31) // 32
            kp = torch.zeros(B, H, nblk * 32, D, dtype=k.dtype, device=self.dev)
            vp = torch.zeros_like(kp)
            kp[:, :, :n].copy_(k)
            vp[:, :, :n].copy_(v)
            kt, vt = to_kv_tiles(kp, vp)
            for b in range(B):
                nb = (min(n, int(lengths[b]) if lengths is not None else n) + 31) // 32
                if nb == 0:
                    continue
                self.reserve(b, 32 * nb)
                ids = torch.from_numpy(self.seq_pages[b][:nb].astype(np.int64)).to(self.dev)
                self.k_cache[layer].index_copy_(0, ids, kt[b].reshape(H, nblk, 32 * D)[:, :nb].transpose(0, 1))
                self.v_cache[layer].index_copy_(0, ids, vt[b].reshape(H, nblk, 32 * D)[:, :nb].transpose(0, 1))
            return
        if not self.kv_tiled:
            self.k_cache[layer, :, :, :n].copy_(k)
            self.v_cache[layer, :, :, :n].copy_(v)
            return
        kl, vl = from_kv_tiles(self.k_cache[layer], self.v_cache[layer])
        kl[:, :, :n].copy_(k)
        vl[:, :, :n].copy_(v)
        kt, vt = to_kv_tiles(kl, vl)
        self.k_cache[layer].copy_(kt)
        self.v_cache[layer].copy_(vt)

    def step(self, graph: bool = True) -> None:
        """One decode token for every sequence (stream-ordered; no host sync)."""
        st = torch.cuda.current_stream().cuda_stream
        call("wf_model_graph_launch" if graph else "wf_model_step", self._h, st)

    def check(self) -> None:
        """Raise RuntimeError if a decode attention launched so far gave up on its in-launch exchange
        (include/wf_bitnet.h wf_model_check; synchronise the stream first to cover every step)."""
        call("wf_model_check", self._h)

    def debug_stall_attention(self, on: bool) -> None:
        """Test hook (wf_model_debug_stall_attention): the next eager attention launches poll for a tag
        no workgroup publishes and take the bounded-spin timeout path."""
        call("wf_model_debug_stall_attention", self._h, 1 if on else 0)

    def attention_records(self):
        """The last WF_OP_QKV / WF_OP_ATTN hand-off (include/wf_bitnet.h wf_model_attn_view) as torch
        tensors on the device: q [B, Hq, D] bf16, ml [B, Hq, R, 2] (m, l), o [B, Hq, R, D] float
        (unnormalised, logical dim order). For kernel-level checks; copies, not views."""
        v = _lib.WFAttnView()
        call("wf_model_attn_view", self._h, C.addressof(v))
        cfg, B = self.cfg, self.batch
        Hq, D, R = cfg.n_heads, cfg.head_dim, int(v.records)
        if D != 128:
            raise ValueError("attention records need head_dim 128")

        q = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=self.dev)
        ml = torch.empty(B, Hq, R, 2, dtype=torch.float32, device=self.dev)
        o = torch.empty(B * Hq * R * D, dtype=torch.float32, device=self.dev)
        ops.device_copy(q.data_ptr(), v.q, q.numel() * 2)
        ops.device_copy(ml.data_ptr(), v.part_ml, ml.numel() * 4)
        ops.device_copy(o.data_ptr(), v.part_o, o.numel() * 4)
        # record layout: element d at ((d >> 2) & 1) * 64 + (d >> 3) * 4 + (d & 3)
        d = torch.arange(D, device=self.dev)
        idx = ((d >> 2) & 1) * 64 + (d >> 3) * 4 + (d & 3)
        o = o.view(B, Hq, R, D)[..., idx]
        return q, ml, o

    def attention_row(self):
        """The bf16 attention output the O projection reads after WF_OP_ATTN ([B, Hq, D];
        include/wf_bitnet.h wf_attn_records.attn_row): every attention path writes it (batch < 16 /
        untiled caches: the head's merging block; batch >= 16 tile layout: the batched kernel)."""
        v = _lib.WFAttnView()
        call("wf_model_attn_view", self._h, C.addressof(v))
        if not v.attn_row:
            return None
        cfg = self.cfg
        row = torch.empty(self.batch, cfg.n_heads, cfg.head_dim, dtype=torch.bfloat16, device=self.dev)
        ops.device_copy(row.data_ptr(), v.attn_row, row.numel() * 2)
        return row

    @property
    def fused_norm(self) -> tuple:
        """(QKV, O, gate|up, down): which batched GEMMs normalise their input rows inside the GEMM
        launch (include/wf_bitnet.h wf_model_fused_norm)."""
        f = (C.c_int * 4)()
        call("wf_model_fused_norm", self._h, C.addressof(f))
        return tuple(bool(x) for x in f)

    def load_attention_q(self, q: torch.Tensor) -> None:
        """Overwrite the q hand-off of the last WF_OP_QKV with q [B, Hq, D] bf16 (kernel-level checks:
        the next WF_OP_ATTN reads it)."""
        v = _lib.WFAttnView()
        call("wf_model_attn_view", self._h, C.addressof(v))
        cfg, B = self.cfg, self.batch
        if tuple(q.shape) != (B, cfg.n_heads, cfg.head_dim) or q.dtype != torch.bfloat16 or not q.is_cuda:
            raise ValueError("q must be [batch, n_heads, head_dim] bf16 on the decoder's device")
        q = q.contiguous()
        ops.device_copy(v.q, q.data_ptr(), q.numel() * 2)

    @property
    def weight_bytes(self) -> int:
        return sum(t.numel() for t in (self.w_qkv, self.w_o, self.w_gu, self.w_d)) + self.embed.numel() * 2

    def launch_op(self, layer: int, op: int) -> None:
        """Launch one op of the decode step (WF_OP_*), for per-kernel timing/profiling."""
        call("wf_model_launch_op", self._h, int(layer), int(op), torch.cuda.current_stream().cuda_stream)

    def op_bytes(self, op: int, ctx: int = 0) -> int:
        """Algorithmic HBM bytes of one launch of `op` at batch `self.batch` (weights once, activations
        and outputs per sequence, K/V rows per cached position)."""
        cfg, B = self.cfg, self.batch
        h, i, kv, D = cfg.hidden, cfg.inter, cfg.kv_dim, cfg.head_dim
        per_layer = {
            _lib.WF_OP_QKV: self.w_qkv[0].numel() + B * (2 * h + 2 * (h + 2 * kv)),
            _lib.WF_OP_O: self.w_o[0].numel() + B * (2 * h + 4 * h),
            _lib.WF_OP_GATE_UP: self.w_gu[0].numel() + B * (2 * h + 2 * i),
            _lib.WF_OP_DOWN: self.w_d[0].numel() + B * (2 * i + 4 * h),
            _lib.WF_OP_ATTN: B * (2 * kv * (1 if self.kv_fp8 else 2) * ctx + 2 * 2 * h),
            _lib.WF_OP_LM_HEAD: self.embed.numel() * 2 + B * (2 * h + 2 * cfg.vocab),
        }
        return int(per_layer.get(op, 0))
