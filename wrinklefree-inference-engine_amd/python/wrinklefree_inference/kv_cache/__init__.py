"""KV cache drop-in (reference src/wrinklefree_inference/kv_cache/__init__.py:8-24)."""
from wrinklefree_inference.kv_cache.kv_cache import (  # noqa: F401
    KVCache,
    KVCacheConfig,
    KVCacheDtype,
    KVCacheValidator,
    attention_with_kv_cache,
    compute_kv_cache_memory,
)

__all__ = [
    "KVCache",
    "KVCacheConfig",
    "KVCacheDtype",
    "KVCacheValidator",
    "attention_with_kv_cache",
    "compute_kv_cache_memory",
]
