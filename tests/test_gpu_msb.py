"""GPU parity of the SGLang BitNet linear method (sglang_backend/bitnet_quantization.py)
through the C-ABI: ternarise/pack and dequantise are bit-exact against the reference's golden
vectors; the linear (direct 2-bit kernel for <= 16 rows, cached dequantised matrix + GEMM above)
matches the reference's outputs and the CPU oracle within one rounding of the compute dtype, and
passes the reference's own accuracy bar (cosine > 0.9999 vs fp32, tests/test_sglang_bitnet.py:243-283)."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

DT = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from wfamd import _lib
    assert _lib.kernel_available(), "gfx950 kernels must load on the GPU box (no fallback)"
    torch.cuda.set_device(0)


def f32(t: torch.Tensor) -> np.ndarray:
    return t.float().cpu().numpy()


def within_one_rounding(got: np.ndarray, ref: np.ndarray, dtype: torch.dtype, ws: float, bias=None) -> None:
    """One rounding of the pre-bias product (its magnitude is at most |y| + |bias|) plus the final one."""
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10
    pre = np.abs(ref) + (0.0 if bias is None else np.abs(np.asarray(bias, np.float32)))
    err = np.abs(got - ref)
    assert np.all(err <= ulp * (np.abs(ref) + pre) + 1e-3 * ws), float(err.max())
    assert np.mean(got == ref) > 0.85


def test_quantize_and_dequantize_golden_bitexact():
    from wrinklefree_inference.sglang_backend import bitnet_quantization as bq
    g = load_golden("msb")
    for name in ("w32", "wb", "wh", "wz", "wt"):
        w = torch.from_numpy(g[f"{name}_in"]).to(DT[int(g[f"{name}_dtype"])])
        packed, scale = bq.quantize_to_bitnet(w.cuda())
        assert packed.is_cuda and scale == float(g[f"{name}_scale"]), name
        assert np.array_equal(packed.cpu().numpy(), g[f"{name}_packed"]), name
        hp, hs = bq.quantize_to_bitnet(w)  # host tensors in, host tensors out (staged through the GPU)
        assert not hp.is_cuda and hs == scale and np.array_equal(hp.numpy(), g[f"{name}_packed"])
        n, k = w.shape
        deq = bq.dequantize_bitnet(packed, scale, n, k)
        assert deq.dtype == torch.float32 and np.array_equal(deq.cpu().numpy(), g[f"{name}_deq"]), name
        assert np.array_equal(bq.dequantize_bitnet_reference(hp, hs, n, k).numpy(), g[f"{name}_deq"])
    with pytest.raises(AssertionError):
        bq.quantize_to_bitnet(torch.randn(4, 96, device="cuda"))


@pytest.mark.parametrize("tag,dtype", [("bf", torch.bfloat16), ("h", torch.float16)])
def test_apply_golden(tag, dtype):
    from wrinklefree_inference.sglang_backend import bitnet_quantization as bq
    g = load_golden("msb")
    packed, scale = torch.from_numpy(g["lin_packed"]), float(g["lin_scale"])
    bias = torch.from_numpy(g["lin_bias"])
    ws = float(torch.tensor(scale).to(dtype).float())
    for m in (1, 3, 32):  # 1, 3: direct 2-bit kernel; 32: dequantised matrix + GEMM
        x = torch.from_numpy(g[f"lin_x{m}"])
        meth = bq.BitNetLinearMethod(compute_dtype=dtype)
        for key, b in ((f"lin_y{m}_{tag}", None), (f"lin_yb{m}_{tag}", bias)):
            ref = torch.from_numpy(g[key].view(np.int16)).view(dtype).float().numpy()
            y = meth.apply(packed, scale, x, 192, 1024, bias=b)
            assert not y.is_cuda and y.dtype == dtype and y.shape == (m, 192)
            within_one_rounding(f32(y), ref, dtype, ws, None if b is None else b.to(dtype).float().numpy())
            yd = meth.apply(packed.cuda(), scale, x.cuda(), 192, 1024, bias=None if b is None else b.cuda())
            assert yd.is_cuda and np.array_equal(f32(yd), f32(y))


@pytest.mark.parametrize("n,k", [(2560, 2560), (6912, 2560), (2560, 6912), (4096, 11008), (1024, 16384),
                                 (640, 2624), (100, 64)])
def test_direct_linear_vs_oracle(orc, n, k):
    from wfamd import ops
    rng = np.random.default_rng(n + 3 * k)
    packed = rng.integers(0, 256, size=(n, k // 4), dtype=np.uint8)  # includes code 3 (-> +2, as dequantised)
    pd = torch.from_numpy(packed).cuda()
    scale = 1.7
    for dtype, dt in ((torch.bfloat16, "bfloat16"), (torch.float16, "float16")):
        ws = float(torch.tensor(scale).to(dtype).float())
        bias = torch.randn(n).to(dtype)
        for m in (1, 2, 4, 5, 16):
            x = torch.randn(m, k).to(dtype)
            y = ops.msb_linear(pd, scale, x.cuda(), n, k, bias.cuda())
            ref = orc.msb_linear(packed, ws, x.float().numpy(), bias.float().numpy(), dt)
            within_one_rounding(f32(y), ref, dtype, ws, bias.float().numpy())


@pytest.mark.parametrize("size", [(4096, 4096), (11008, 4096), (4096, 11008)])
@pytest.mark.parametrize("m", [4, 32])
def test_reference_accuracy_bar(size, m):
    """tests/test_sglang_bitnet.py:243-305 on the GPU: cosine > 0.9999 and mean relative error < 5%
    against the fp32 product, for the direct kernel (m = 4) and the GEMM path (m = 32)."""
    from wrinklefree_inference.sglang_backend import bitnet_quantization as bq
    out_dim, in_dim = size
    g = torch.Generator(device="cuda").manual_seed(out_dim + in_dim + m)
    w = torch.randn(out_dim, in_dim, device="cuda", generator=g)
    packed, scale = bq.quantize_to_bitnet(w)
    w32 = bq.dequantize_bitnet(packed, scale, out_dim, in_dim)
    x = torch.randn(m, in_dim, device="cuda", generator=g)
    y_ref = x @ w32.T
    for dtype in (torch.bfloat16, torch.float16):
        y = bq.BitNetLinearMethod(compute_dtype=dtype).apply(packed, scale, x, out_dim, in_dim).float()
        cos = torch.nn.functional.cosine_similarity(y_ref.flatten()[None], y.flatten()[None]).item()
        assert cos > 0.9999, (dtype, cos)
        rel = ((y_ref - y).abs() / (y_ref.abs() + 1e-8)).mean().item()
        # The reference asserts the 5 % bar at 4096x4096, m = 32 only (:289-305). Elsewhere the mean
        # relative error is dominated by a few near-zero outputs, so the bar there is: no worse than
        # the reference's own computation (dequantised weight and input cast to dtype, torch matmul).
        y_t = (x.to(dtype) @ w32.to(dtype).T).float()
        rel_t = ((y_ref - y_t).abs() / (y_ref.abs() + 1e-8)).mean().item()
        assert rel < max(0.05, 1.25 * rel_t), (dtype, rel, rel_t)


def test_sparsity_on_device_and_fp32_compute():
    from wrinklefree_inference.sglang_backend import activation_sparsity as sp
    from wrinklefree_inference.sglang_backend import bitnet_quantization as bq
    g = load_golden("msb")
    xs = torch.from_numpy(g["sp_x"]).cuda()
    y, _ = sp.apply_top_k_sparsity(xs, 0.4)
    assert np.array_equal(y.cpu().numpy(), g["sp_topk"])
    packed, scale = torch.from_numpy(g["lin_packed"]).cuda(), float(g["lin_scale"])
    x = torch.from_numpy(g["lin_x3"]).cuda()
    meth = bq.BitNetLinearMethod(compute_dtype=torch.bfloat16, sparsity_config=sp.get_qsparse_config())
    y = meth.apply(packed, scale, x, 192, 1024)
    xk, _ = sp.apply_top_k_sparsity(x.to(torch.bfloat16), 0.4)
    y2 = bq.BitNetLinearMethod(compute_dtype=torch.bfloat16).apply(packed, scale, xk, 192, 1024)
    assert torch.equal(y, y2) and meth.get_last_sparsity() == pytest.approx(0.6)
    y32 = bq.BitNetLinearMethod(compute_dtype=torch.float32).apply(packed, scale, x, 192, 1024)
    ref = x @ bq.dequantize_bitnet(packed, scale, 192, 1024).T
    assert torch.allclose(y32, ref, rtol=1e-5, atol=1e-4)
