"""One-byte K/V codes on the host (CPU, no GPU): the int8 codes the decode step stores
(wfamd.model.to_int8_codes, wf_decode.hip to_kv8) against the reference's KVCache INT8 / "FP8"
quantizer (kv_cache/kv_cache.py:159-185: (x * 127 / absmax).round().clamp(-127, 127), int8 codes),
and the oracle's dequantiser (oracle.int8_codes_to_bf16) against the codes."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "wrinklefree-inference-engine_amd" / "python"))


def test_int8_codes_match_reference_formula():
    from wfamd.model import from_int8_codes, to_int8_codes
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(4096, generator=g) * 2.5).to(torch.bfloat16)
    absmax = float(x.float().abs().max())
    ref = (x.float() * (127.0 / absmax)).round().clamp(-127, 127).to(torch.int8)
    got = to_int8_codes(x, absmax / 127.0).view(torch.int8)
    # x / (absmax / 127) and x * (127 / absmax) round apart only at exact half-integer ties
    diff = (got.int() - ref.int()).abs()
    assert int(diff.max()) <= 1 and int((diff > 0).sum()) <= 2
    back = from_int8_codes(to_int8_codes(x, absmax / 127.0), absmax / 127.0)
    assert float((back - x.float()).abs().max()) <= absmax / 127.0 / 2 + 1e-6


def test_int8_codes_saturate_and_round_half_even():
    from wfamd.model import to_int8_codes
    x = torch.tensor([1000.0, -1000.0, 0.5, 1.5, 2.5, -0.5, -2.5, 126.6, -127.4], dtype=torch.float32)
    c = to_int8_codes(x, 1.0).view(torch.int8).tolist()
    assert c == [127, -127, 0, 2, 2, 0, -2, 127, -127]


def test_oracle_dequantiser_matches_codes():
    from oracle import oracle as orc
    from wfamd.model import from_int8_codes, to_int8_codes
    x = torch.linspace(-3, 3, 997)
    s = 3.0 / 127
    codes = to_int8_codes(x, s)
    want = orc.f32_to_bf16(from_int8_codes(codes, s).numpy().astype(np.float32))
    assert np.array_equal(orc.int8_codes_to_bf16(codes.numpy(), s), want)
