"""The decode prologue's fast exact arithmetic (wf_device.h: div_rn, act_scale_f, quant8 --
Markstein quotients instead of the IEEE divide sequences and the former per-element branch) agrees
bit for bit with the IEEE forms it replaces: a host restatement with a correctly rounded fma
(tools/check_fast_arith.c) over random numerators, every positive bf16 scale numerator and
constructed half-integer quantizer ties. The GPU parity tests then check the kernels end to end."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host C compiler")
def test_fast_exact_arithmetic_matches_ieee(tmp_path):
    exe = tmp_path / "check_fast_arith"
    subprocess.run(["gcc", "-O2", "-mfma", "-o", str(exe), str(ROOT / "tools" / "check_fast_arith.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "0.02"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert "act scale: 0 mismatches" in r.stdout
