"""pytest setup: markers, import paths, shared fixtures.

`-m "not gpu"` runs here (no GPU): oracle vs the reference's known-answer vectors,
host logic, ABI surface.  `-m gpu` runs on an MI355X: parity of the HIP path
(called through the C ABI) against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "gsm-renderer_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def gsm():
    import gsm_amd
    gsm_amd._lib()  # raises if libgsm_amd.so is missing: no silent fallback
    return gsm_amd


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test requested but no HIP device is visible")
    return torch
