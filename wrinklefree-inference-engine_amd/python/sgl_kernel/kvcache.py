"""sgl_kernel.kvcache drop-in: paged KV pool with a free list (API: tests/test_kv_cache_cpp.py:270-373;
Python twin PythonKVCacheReference :20-127).

Storage [max_pages, num_layers, 2, num_heads, head_dim] lives in HBM; scatter_kv/gather_kv run as
HIP copy kernels (one 4-byte-vectorised row copy per token and K/V). One token per page; `slots` is
accepted and unused, as in the reference.
"""
from __future__ import annotations

import torch

from wfamd import _lib
from wfamd import ops as _ops


def check_kernel_available() -> bool:
    return _ops.check_kernel_available()


class KVCacheManager:
    def __init__(self, num_layers: int, num_heads: int, head_dim: int, page_size: int, max_pages: int,
                 dtype: torch.dtype = torch.float32, device=None):
        self.num_layers, self.num_heads, self.head_dim = num_layers, num_heads, head_dim
        self.page_size, self.max_pages, self.dtype = page_size, max_pages, dtype
        self.device = torch.device(device) if device is not None else _ops._device()
        self.cache_storage = torch.zeros(max_pages, num_layers, 2, num_heads, head_dim, dtype=dtype,
                                         device=self.device)
        # LIFO free list, allocation order 0, 1, 2, ... like the reference twin (:46-59)
        self._free = list(range(max_pages - 1, -1, -1))
        self._bad = torch.zeros(1, dtype=torch.int32, device=self.device)

    # -- allocation (host bookkeeping, :48-73) --------------------------------------------------
    def allocate_page(self) -> int:
        return self._free.pop() if self._free else -1

    def allocate_pages(self, num_pages: int) -> torch.Tensor:
        if len(self._free) < num_pages:
            return torch.empty(0, dtype=torch.int32)
        return torch.tensor([self._free.pop() for _ in range(num_pages)], dtype=torch.int32)

    def free_page(self, page_id: int) -> None:
        if 0 <= page_id < self.max_pages:
            self._free.append(int(page_id))

    def free_pages(self, page_ids) -> None:
        for p in torch.as_tensor(page_ids).tolist():
            self.free_page(p)

    free_pages_batch = free_pages

    def num_free_pages(self) -> int:
        return len(self._free)

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

    def scatter_kv(self, k_in: torch.Tensor, v_in: torch.Tensor, pages, slots, layer_id: int) -> None:
        pg = self._prep(pages, k_in)
        k, v = _ops._on_device(k_in), _ops._on_device(v_in)
        _lib.call("wf_kv_scatter", self.cache_storage.data_ptr(), self.cache_storage.element_size(), self.max_pages,
                  self.num_layers, self.num_heads, self.head_dim, k.data_ptr(), v.data_ptr(), pg.data_ptr(),
                  pg.shape[0], int(layer_id), self._bad.data_ptr(), _ops._stream())

    def gather_kv(self, k_out: torch.Tensor, v_out: torch.Tensor, pages, slots, layer_id: int) -> None:
        """Writes into the caller's buffers (tests/test_kv_cache_cpp.py:331-335)."""
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
