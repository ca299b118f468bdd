"""pytest configuration: markers, import paths, shared fixtures."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_PY = ROOT / "wrinklefree-inference-engine_amd" / "python"
for p in (str(ROOT), str(PKG_PY)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels through the C-ABI)")


def pytest_collection_modifyitems(session, config, items):
    """The replica test starts GPU child processes: run it before any test of this process touches
    the GPU (tests/test_gpu_replicas.py)."""
    items.sort(key=lambda it: 0 if it.nodeid.startswith("tests/test_gpu_replicas.py") else 1)


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as o
    o.build()
    return o
