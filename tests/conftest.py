import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "nightcore-to-flac-analyzer_amd"
for p in (str(PKG), str(REPO), str(REPO / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libncgpu.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from nightcore_analyzer import _native
    ctx = _native.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def golden_units():
    import json
    return json.loads((REPO / "tests" / "golden" / "units.json").read_text())


@pytest.fixture(scope="session")
def golden_pipeline():
    import json
    return json.loads((REPO / "tests" / "golden" / "pipeline.json").read_text())
