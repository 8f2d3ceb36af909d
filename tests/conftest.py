import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the native kernel library")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "allow_vendor: a GPU test that exercises a vendor-library fallback on purpose")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _strict_native_on_gpu(request, monkeypatch):
    """GPU tests run in strict native mode: an op that would leave the hand-written kernels for a
    vendor library (torch.matmul / _scaled_mm on a GPU tensor) raises instead (ops.vendor_fallback).
    A test that exercises such a path on purpose marks itself ``allow_vendor``."""
    if "gpu" in request.keywords and "allow_vendor" not in request.keywords:
        monkeypatch.setenv("VWA_STRICT_NATIVE", "1")
    yield


def pytest_sessionstart(session):
    """Build the CPU runtime library (grammar engine) in-tree if this checkout has no .so yet."""
    native = os.path.join(ROOT, "voice_enabled_browser_automation_amd", "ops", "_vwa_native.so")
    if not os.path.exists(native):
        from voice_enabled_browser_automation_amd.ops.build import build_native

        build_native()
