"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every symbol that
include/wf_bitnet.h declares, the Python bindings cover them, the reference-facing modules import
with the reference's names, and the host-side logic (layouts, numpy helpers, bookkeeping) matches
the reference. No kernel is launched here (no GPU in this container)."""
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden

HEADER = ROOT / "include" / "wf_bitnet.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wf_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from wfamd import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in wf_bitnet.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"
    assert lib.wf_abi_version() == 1


def test_library_has_gfx950_code_object():
    so = ROOT / "wrinklefree-inference-engine_amd" / "lib" / "libwfbitnet.so"
    blob = so.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle entry of the gfx950 code object


def test_no_device_means_not_available():
    from sgl_kernel.quantization import bitnet_check_kernel_available
    from sgl_kernel.quantization.bitnet import check_kernel_available
    if not torch.cuda.is_available():
        assert bitnet_check_kernel_available() is False
        assert check_kernel_available() is False


def test_reference_surface_names():
    import sgl_kernel
    from sgl_kernel import quantization as q
    from sgl_kernel.quantization import bitnet as qb
    for n in ("bitnet_gemv", "bitnet_gemm", "bitnet_quantize_activations", "bitnet_check_kernel_available",
              "BITNET_BLOCK_SIZE", "quantize_activations_i8"):
        assert hasattr(q, n), n
    for n in ("bitnet_gemv", "quantize_activations_i8", "check_kernel_available", "auto_tune_tiles"):
        assert hasattr(qb, n), n
    assert q.BITNET_BLOCK_SIZE == 128
    from sgl_kernel.kvcache import KVCacheManager, check_kernel_available  # noqa: F401
    from wrinklefree_inference.kernels import (NATIVE_KERNELS_AVAILABLE, BitNetLinearNative,  # noqa: F401
                                               benchmark_kernels, patch_model_with_native_kernels)
    from wrinklefree_inference.kernels.bitnet_patch import extract_packed_weight_and_scale, pack_ternary_weights  # noqa
    from wrinklefree_inference.kernels.native import (build_kernel, get_kernel, pack_weights,  # noqa: F401
                                                      quantize_activations, repack_hf_weights, unpack_weights)
    from wrinklefree_inference.kv_cache import (KVCache, KVCacheConfig, KVCacheDtype,  # noqa: F401
                                                attention_with_kv_cache, compute_kv_cache_memory)
    assert hasattr(torch.ops.sgl_kernel, "bitnet_gemv_cpu")
    assert hasattr(torch.ops.sgl_kernel, "bitnet_gemm_cpu")
    assert hasattr(torch.ops.sgl_kernel, "bitnet_quantize_activations_cpu")
    assert hasattr(torch.ops.sgl_kernel, "bitnet_qkv_forward_cpu")
    assert hasattr(torch.ops.sgl_kernel, "bitnet_mlp_forward_cpu")


def test_torch_op_fake_impls():
    """torch.compile shape propagation (docs/research/sglang_optimization_plan.md:61-74)."""
    import sgl_kernel  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        w = torch.empty(640, 640, dtype=torch.uint8)
        a = torch.empty(2560, dtype=torch.int8)
        assert torch.ops.sgl_kernel.bitnet_gemv_cpu(w, a, 0.5).shape == (640,)
        a2 = torch.empty(4, 2560, dtype=torch.int8)
        assert torch.ops.sgl_kernel.bitnet_gemm_cpu(w, a2, 0.5).shape == (4, 640)
        q, s = torch.ops.sgl_kernel.bitnet_quantize_activations_cpu(torch.empty(3, 2560))
        assert q.dtype == torch.int8 and q.shape == (3, 2560)
        x = torch.empty(2, 3, 2560, dtype=torch.bfloat16)
        wqkv = torch.empty(3840, 640, dtype=torch.uint8)
        yq, yk, yv = torch.ops.sgl_kernel.bitnet_qkv_forward_cpu(x, wqkv, 2560, 640, 640, 0.5, 0.5, 0.5)
        assert (yq.shape, yk.shape, yv.shape) == ((2, 3, 2560), (2, 3, 640), (2, 3, 640)) and yq.dtype == torch.bfloat16
        y = torch.ops.sgl_kernel.bitnet_mlp_forward_cpu(x, torch.empty(13824, 640, dtype=torch.uint8),
                                                        torch.empty(2560, 1728, dtype=torch.uint8), 0.5, 0.5, 0.5,
                                                        torch.empty(6912, dtype=torch.bfloat16))
        assert y.shape == (2, 3, 2560) and y.dtype == torch.bfloat16


def test_native_numpy_helpers_match_reference():
    from wrinklefree_inference.kernels.native import pack_weights, quantize_activations, repack_hf_weights, unpack_weights
    g = load_golden("packing")
    assert np.array_equal(pack_weights(g["lsb_w"].astype(np.float32)), g["lsb_p"])
    assert np.array_equal(unpack_weights(g["lsb_p"]).astype(np.int8), g["lsb_w"])
    assert np.array_equal(repack_hf_weights(g["hf2lsb_in"]), g["hf2lsb_out"])
    q = load_golden("quant")
    for i in range(8):
        qi, si = quantize_activations(q[f"x{i}"])
        assert np.array_equal(qi, q[f"qt{i}"]) and np.float32(si) == q[f"st{i}"]


def test_lsb_pack_matches_reference():
    from wrinklefree_inference.kernels.bitnet_patch import pack_ternary_weights
    g = load_golden("packing")
    p, s = pack_ternary_weights(torch.from_numpy(g["lsb_w"].astype(np.float32)))
    assert np.array_equal(p.numpy(), g["lsb_p"])


def test_kv_memory_calc_matches_reference():
    from wrinklefree_inference.kv_cache import KVCacheDtype, compute_kv_cache_memory
    g = load_golden("kv")
    mem = compute_kv_cache_memory({"num_layers": 30, "num_heads": 5, "head_dim": 128}, 4096, KVCacheDtype.BF16)
    assert mem["total_mb"] == float(g["mem_total_mb"]) and mem["per_token_kb"] == float(g["mem_per_token_kb"])


def test_kv_manager_allocation_semantics():
    """tests/test_kv_cache_cpp.py:20-73 allocation order / failure behaviour (host bookkeeping)."""
    from sgl_kernel.kvcache import KVCacheManager
    g = load_golden("kv")
    m = KVCacheManager(num_layers=3, num_heads=2, head_dim=8, page_size=16, max_pages=10, device="cpu")
    a = m.allocate_pages(4)
    m.free_pages(a[1:3])
    b = m.allocate_pages(3)
    single = m.allocate_page()
    too_many = m.allocate_pages(100)
    assert np.array_equal(a.numpy(), g["pg_a"]) and np.array_equal(b.numpy(), g["pg_b"])
    assert single == int(g["pg_single"]) and too_many.numel() == int(g["pg_too_many"])
    assert m.num_free_pages() == int(g["pg_free_after"])
    with pytest.raises(RuntimeError):
        m.scatter_kv(torch.zeros(1, 16), torch.zeros(1, 16), torch.tensor([0]), None, 0)


def test_decoder_page_pool_semantics():
    """The paged decoder's host allocator follows the same allocation / failure order as
    KVCacheManager (tests/test_kv_cache_cpp.py:20-73 golden)."""
    from wfamd.model import PagePool
    g = load_golden("kv")
    m = PagePool(10)
    a = m.allocate_pages(4)
    m.free_pages(a[1:3])
    b = m.allocate_pages(3)
    single = m.allocate_pages(1)
    too_many = m.allocate_pages(100)
    assert np.array_equal(a, g["pg_a"]) and np.array_equal(b, g["pg_b"])
    assert int(single[0]) == int(g["pg_single"]) and too_many.size == int(g["pg_too_many"])
    assert m.num_free_pages() == int(g["pg_free_after"])
    m.free_pages([-1, 10])  # ignored
    assert m.num_free_pages() == int(g["pg_free_after"])
    s = PagePool(64, seed=3)  # scattered placement: a permutation of the pool
    ids = s.allocate_pages(64)
    assert sorted(ids.tolist()) == list(range(64)) and ids.tolist() != list(range(64))


def test_prefill_row_packing():
    """wf_model_prefill's row contract (include/wf_bitnet.h): every aligned group of
    WF_PREFILL_ROW_GROUP rows is one slot, positions consecutive from `start`, pads repeat the last row."""
    from wfamd import _lib
    from wfamd.model import pack_prefill_rows
    g = _lib.WF_PREFILL_ROW_GROUP
    seqs = [(3, [5, 6, 7], 0), (0, [], 4), (7, list(range(100, 100 + g + 1)), 10), (1, [9] * g, 2)]
    tok, slot, pos = pack_prefill_rows(seqs)
    assert len(tok) == len(slot) == len(pos) == 4 * g
    for r0 in range(0, len(tok), g):
        assert len(set(slot[r0:r0 + g])) == 1
    assert tok[:3] == [5, 6, 7] and pos[:3] == [0, 1, 2] and set(tok[3:g]) == {7} and set(pos[3:g]) == {2}
    assert slot[g:3 * g] == [7] * 2 * g and pos[g:2 * g + 1] == list(range(10, 10 + g + 1))
    assert pos[2 * g + 1:3 * g] == [10 + g] * (g - 1) and tok[3 * g:] == [9] * g and pos[3 * g:] == list(range(2, 2 + g))


def test_model_layout_permutations():
    from wfamd.model import gate_up_interleave, qkv_row_permutation
    p = qkv_row_permutation(3, 128)
    assert sorted(p.tolist()) == list(range(384))
    # block t of head h holds dims 8t..8t+7 and 64+8t..64+8t+7
    blk = p[16 * 9:16 * 10].tolist()  # head 1, tile 1
    assert blk == [128 + 8 + i for i in range(8)] + [128 + 72 + i for i in range(8)]
    gu = gate_up_interleave(32)
    assert sorted(gu.tolist()) == list(range(64))
    assert gu[:16].tolist() == list(range(8)) + list(range(32, 40))


def test_bytes_accounting():
    from wfamd.model import BITNET_2B
    assert BITNET_2B.ternary_weights() == 2_084_044_800
    assert BITNET_2B.kv_bytes_per_token(1) == 76_800


def test_kv_tile_layout_matches_device_offsets():
    """wfamd.model.to_kv_tiles / from_kv_tiles agree with the device offsets k_tile_off /
    v_tile_off (csrc/wf_norm.h) the batched decode writes and reads."""
    import torch
    from wfamd.model import from_kv_tiles, to_kv_tiles
    S, D = 96, 128
    k = torch.arange(S * D, dtype=torch.float32).reshape(1, S, D)
    v = k + 0.5
    kt, vt = to_kv_tiles(k, v)

    def koff(t, d):
        blk, o = t >> 5, t & 31
        return ((((blk * 2 + ((o >> 2) & 1)) * 16 + (d >> 3)) * 16 + 4 * (o >> 3) + (o & 3)) * 8 + (d & 7))

    def voff(t, d):
        blk, o = t >> 5, t & 31
        return ((((blk * 8 + (d >> 4)) * 4 + (o >> 3)) * 16 + (d & 15)) * 8 + (o & 7))
    kf, vf = kt.reshape(-1), vt.reshape(-1)
    for t in range(S):
        for d in range(0, D, 5):
            assert kf[koff(t, d)] == k[0, t, d] and vf[voff(t, d)] == v[0, t, d]
    k2, v2 = from_kv_tiles(kt, vt)
    assert torch.equal(k2, k) and torch.equal(v2, v)


def test_sglang_backend_surface():
    from wrinklefree_inference.sglang_backend import BITNET_QUANT_TYPES, BitNetConfig
    from wrinklefree_inference.sglang_backend import bitnet_quantization as bq
    for n in ("BitNetQuantType", "BITNET_BLOCK_SIZE", "BitNetWeightSpec", "quantize_to_bitnet", "dequantize_bitnet",
              "dequantize_bitnet_reference", "bitnet_matmul_reference", "BitNetLinearMethod", "validate_bitnet_model"):
        assert hasattr(bq, n), n
    assert bq.BITNET_BLOCK_SIZE == 128 and len(BITNET_QUANT_TYPES) == 3 and int(bq.BitNetQuantType.I2_S) == 30
    assert BitNetConfig.get_name() == "bitnet" and "I2_S" in repr(BitNetConfig())
    spec = bq.BitNetWeightSpec((8, 128), bq.BitNetQuantType.I2_S, 1.0, (8, 32))
    assert spec.compression_ratio == pytest.approx(16 / 1.58)
    r = bq.validate_bitnet_model("/nonexistent/model-i2_s.gguf")
    assert not r["valid"] and r["errors"]
    meth = bq.BitNetLinearMethod()
    assert meth.compute_dtype == torch.bfloat16 and meth.get_sparsity_stats() == {"enabled": False}


def test_fused_projection_and_mlp_argument_errors():
    """wf_bitnet_linear_fused / wf_bitnet_mlp validate their arguments on the host before any HIP
    call (WF_EINVAL + wf_last_error), so the boundary's error behaviour is checkable without a GPU;
    workspace sizes are host arithmetic."""
    import ctypes as C
    from wfamd import _lib
    lib = _lib.load()
    x = (C.c_uint16 * 4096)()
    w = (C.c_uint8 * 4096)()
    y0, y1 = (C.c_uint16 * 4096)(), (C.c_uint16 * 4096)()
    ys = (C.c_void_p * 2)(C.addressof(y0), C.addressof(y1))
    n = (C.c_int * 2)(256, 256)
    ws = (C.c_float * 2)(1.0, 1.0)
    ld = (C.c_int64 * 2)(256, 256)

    def fused(nseg, K=256, nn=n, ldy=ld):
        return lib.wf_bitnet_linear_fused(0, C.addressof(w), nseg, C.addressof(nn), C.addressof(ws), C.addressof(x),
                                          K, 1, K, C.addressof(ys), C.addressof(ldy), None, None)
    assert fused(0) == _lib.WF_EINVAL and b"segments" in lib.wf_last_error()
    assert fused(4) == _lib.WF_EINVAL
    assert fused(2, K=200) == _lib.WF_EINVAL and b"K % 128" in lib.wf_last_error()
    bad_n = (C.c_int * 2)(256, 0)
    assert fused(2, nn=bad_n) == _lib.WF_EINVAL and b"segment 1" in lib.wf_last_error()
    bad_ld = (C.c_int64 * 2)(256, 100)
    assert fused(2, ldy=bad_ld) == _lib.WF_EINVAL and b"segment 1" in lib.wf_last_error()
    assert lib.wf_bitnet_mlp(0, C.addressof(w), C.addressof(w), 1.0, 1.0, 1.0, C.addressof(x), 1e-5, C.addressof(x),
                             256, 1, 256, 200, C.addressof(y0), 256, None, None) == _lib.WF_EINVAL
    assert lib.wf_bitnet_mlp_ws_bytes(0, 2560, 6912) == 0
    ws_b = lib.wf_bitnet_mlp_ws_bytes(4, 2560, 6912)
    assert ws_b >= 2 * 4 * 6912 * 2 + lib.wf_bitnet_linear_ws_bytes(4, 6912)
