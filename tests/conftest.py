import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3dg-vol-renderer_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLDEN, "scenes")
RENDERS = os.path.join(GOLDEN, "renders")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvr_hip.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


@pytest.fixture
def device_options():
    """Set vr_set_option values on the cuda:0 context for one test; restored afterwards."""
    import vr_amd as vr
    dev = vr.Device.get(0)
    saved = {}

    def set_opt(name, value):
        if name not in saved:
            saved[name] = dev.get_option(name)
        dev.set_option(name, value)

    yield set_opt
    for name, value in saved.items():
        dev.set_option(name, value)
