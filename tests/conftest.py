"""Test configuration.

`-m gpu` tests need an MI355X (run through gpurun); everything else runs on
the CPU: the oracle against the reference's known-answer tests and the golden
fixtures, the host logic, and the C ABI surface (no compute calls).
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "symbolicregression.jl_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def gpu_ctx():
    import srhip

    n = srhip.device_count()
    if n == 0:
        pytest.fail("gpu test selected but no HIP device is visible")
    return srhip.get_context(0)
