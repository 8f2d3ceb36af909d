import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU and the native kernel library")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def pytest_sessionstart(session):
    """Build the CPU runtime library (grammar engine) in-tree if this checkout has no .so yet."""
    native = os.path.join(ROOT, "voice_enabled_browser_automation_amd", "ops", "_vwa_native.so")
    if not os.path.exists(native):
        from voice_enabled_browser_automation_amd.ops.build import build_native

        build_native()
