"""sgl_kernel.kvcache drop-in: paged KV pool with a free list (API: tests/test_kv_cache_cpp.py:270-373;
Python twin PythonKVCacheReference :20-127).

Standalone (the reference's form): storage [max_pages, num_layers, 2, num_heads, head_dim] in HBM;
scatter_kv/gather_kv run as HIP copy kernels (one 4-byte-vectorised row copy per token and K/V).
One token per page; `slots` is accepted and unused, as in the reference.

Backed by a decode engine (`backing=` a paged wfamd.model.BitNetDecoder): ONE pool behind both APIs.
The manager allocates from, frees to and stores into the decoder's own page pool -- 32-token pages
of every kv head in the tile layouts the batched attention reads (include/wf_bitnet.h
wf_model_desc.page_table) -- so page_size is 32 and `slots` is the position within a page (the
reference's slot_indices); scatter_kv/gather_kv translate token rows [T, H*D] to and from the tile
layouts (C-ABI wf_kv_scatter_tiles / wf_kv_gather_tiles). A sequence whose pages the caller maps with
BitNetDecoder.map_pages is decoded by BitNetDecoder.step from exactly those pages.
"""
from __future__ import annotations

import torch

from wfamd import _lib
from wfamd import ops as _ops


def check_kernel_available() -> bool:
    return _ops.check_kernel_available()


class KVCacheManager:
    def __init__(self, num_layers: int, num_heads: int, head_dim: int, page_size: int, max_pages: int,
                 dtype: torch.dtype = torch.float32, device=None, backing=None):
        self.num_layers, self.num_heads, self.head_dim = num_layers, num_heads, head_dim
        self.page_size, self.max_pages, self.dtype = page_size, max_pages, dtype
        self.backing = backing
        if backing is not None:
            cfg = backing.cfg
            if not getattr(backing, "paged", False) or backing.kv_dtype != "bf16":
                raise ValueError("backing= needs a paged bf16 BitNetDecoder (num_pages > 0, kv_dtype 'bf16')")
            if (num_layers, num_heads, head_dim, page_size, max_pages, dtype) != (
                    cfg.layers, cfg.n_kv_heads, cfg.head_dim, 32, backing.pool.num_pages, torch.bfloat16):
                raise ValueError("backing=: the manager's geometry must be the decoder's (layers, n_kv_heads, head_dim, "
                                 "page_size 32, its pool's pages, bfloat16)")
            self.device = backing.dev
            self.cache_storage = None  # the decoder's k_cache / v_cache [layers, pages, H, 32 * D]
            self._pool = backing.pool  # one free list for both APIs
        else:
            self.device = torch.device(device) if device is not None else _ops._device()
            self.cache_storage = torch.zeros(max_pages, num_layers, 2, num_heads, head_dim, dtype=dtype,
                                             device=self.device)
            # LIFO free list, allocation order 0, 1, 2, ... like the reference twin (:46-59)
            self._free = list(range(max_pages - 1, -1, -1))
        self._bad = torch.zeros(1, dtype=torch.int32, device=self.device)

    @classmethod
    def from_decoder(cls, dec) -> "KVCacheManager":
        """The manager over a paged decoder's own pool (backing=dec with the decoder's geometry)."""
        cfg = dec.cfg
        return cls(cfg.layers, cfg.n_kv_heads, cfg.head_dim, 32, dec.pool.num_pages, torch.bfloat16, backing=dec)

    # -- allocation (host bookkeeping, :48-73) --------------------------------------------------
    def allocate_page(self) -> int:
        if self.backing is not None:
            got = self._pool.allocate_pages(1)
            return int(got[0]) if len(got) else -1
        return self._free.pop() if self._free else -1

    def allocate_pages(self, num_pages: int) -> torch.Tensor:
        if self.backing is not None:
            got = self._pool.allocate_pages(int(num_pages))
            return torch.from_numpy(got.astype("int32")) if len(got) == num_pages else torch.empty(0, dtype=torch.int32)
        if len(self._free) < num_pages:
            return torch.empty(0, dtype=torch.int32)
        return torch.tensor([self._free.pop() for _ in range(num_pages)], dtype=torch.int32)

    def free_page(self, page_id: int) -> None:
        if self.backing is not None:
            self._pool.free_pages([int(page_id)])
        elif 0 <= page_id < self.max_pages:
            self._free.append(int(page_id))

    def free_pages(self, page_ids) -> None:
        for p in torch.as_tensor(page_ids).tolist():
            self.free_page(p)

    free_pages_batch = free_pages

    def num_free_pages(self) -> int:
        return self._pool.num_free_pages() if self.backing is not None else len(self._free)

    # -- data movement ---------------------------------------------------------------------------
    def _prep(self, pages, t: torch.Tensor):
        if self.device.type != "cuda":
            raise RuntimeError("KVCacheManager data movement runs on the HIP device; this pool was built on the host")
        pg = torch.as_tensor(pages, dtype=torch.int32).to(self.device).contiguous()
        if t.dtype != self.dtype:
            raise ValueError(f"dtype {t.dtype} does not match the cache dtype {self.dtype}")
        if t.shape[0] != pg.shape[0] or t[0].numel() != self.num_heads * self.head_dim:
            raise ValueError(f"expected [{pg.shape[0]}, {self.num_heads * self.head_dim}] K/V rows, got {tuple(t.shape)}")
        return pg

    def _tiles(self, name, k, v, pages, slots, layer_id):
        """Token rows <-> the backing decoder's tile-layout pages (wf_kv_scatter_tiles / _gather_tiles)."""
        if not 0 <= int(layer_id) < self.num_layers:
            raise ValueError(f"layer {layer_id} out of range [0, {self.num_layers})")
        pg = torch.as_tensor(pages, dtype=torch.int32).to(self.device).contiguous()
        sl = torch.as_tensor(slots, dtype=torch.int32).to(self.device).contiguous()
        if sl.shape != pg.shape or k.shape[0] != pg.shape[0] or k[0].numel() != self.num_heads * self.head_dim:
            raise ValueError(f"expected pages / slots [{pg.shape[0]}] and [{pg.shape[0]}, {self.num_heads * self.head_dim}] rows")
        if k.dtype != torch.bfloat16 or v.dtype != torch.bfloat16:
            raise ValueError("the engine pool stores bfloat16 K/V")
        dec = self.backing
        _lib.call(name, dec.k_cache[layer_id].data_ptr(), dec.v_cache[layer_id].data_ptr(), dec.pool.num_pages,
                  self.num_heads, self.head_dim, k.data_ptr(), v.data_ptr(), pg.data_ptr(), sl.data_ptr(), pg.shape[0],
                  self._bad.data_ptr(), _ops._stream())

    def scatter_kv(self, k_in: torch.Tensor, v_in: torch.Tensor, pages, slots, layer_id: int) -> None:
        if self.backing is not None:
            k, v = _ops._on_device(k_in).contiguous(), _ops._on_device(v_in).contiguous()
            self._tiles("wf_kv_scatter_tiles", k, v, pages, slots, layer_id)
            return
        pg = self._prep(pages, k_in)
        k, v = _ops._on_device(k_in), _ops._on_device(v_in)
        _lib.call("wf_kv_scatter", self.cache_storage.data_ptr(), self.cache_storage.element_size(), self.max_pages,
                  self.num_layers, self.num_heads, self.head_dim, k.data_ptr(), v.data_ptr(), pg.data_ptr(),
                  pg.shape[0], int(layer_id), self._bad.data_ptr(), _ops._stream())

    def gather_kv(self, k_out: torch.Tensor, v_out: torch.Tensor, pages, slots, layer_id: int) -> None:
        """Writes into the caller's buffers (tests/test_kv_cache_cpp.py:331-335)."""
        if self.backing is not None:
            dev_k = k_out if k_out.is_cuda and k_out.is_contiguous() else torch.empty_like(k_out, device=self.device)
            dev_v = v_out if v_out.is_cuda and v_out.is_contiguous() else torch.empty_like(v_out, device=self.device)
            self._tiles("wf_kv_gather_tiles", dev_k, dev_v, pages, slots, layer_id)
            if dev_k is not k_out:
                k_out.copy_(dev_k)
                v_out.copy_(dev_v)
            return
        pg = self._prep(pages, k_out)
        dev_k = k_out if k_out.is_cuda else torch.empty_like(k_out, device=self.device)
        dev_v = v_out if v_out.is_cuda else torch.empty_like(v_out, device=self.device)
        _lib.call("wf_kv_gather", self.cache_storage.data_ptr(), self.cache_storage.element_size(), self.max_pages,
                  self.num_layers, self.num_heads, self.head_dim, dev_k.data_ptr(), dev_v.data_ptr(), pg.data_ptr(),
                  pg.shape[0], int(layer_id), self._bad.data_ptr(), _ops._stream())
        if not k_out.is_cuda:
            k_out.copy_(dev_k)
            v_out.copy_(dev_v)

    def invalid_page_count(self) -> int:
        return int(self._bad.item())
