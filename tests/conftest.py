import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librbc_gpu.so on the device)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "rbc_golden.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def ref():
    import rbc_ref
    return rbc_ref


@pytest.fixture(scope="session")
def gpu():
    """The HIP library on a real GPU: fails (never skips) when absent."""
    import cleisthenes_amd as ca
    assert ca.device_count() > 0, "gpu test run without a visible GPU"
    return ca


def pytest_sessionfinish(session, exitstatus):
    """A GPU session must have run on the ROCm runtime librbc_gpu.so links:
    torch (if something imported it) maps its own libamdhip64 / librccl."""
    if "torch" in sys.modules and session.config.getoption("-m") == "gpu":
        print("\nWARNING: torch was imported in a GPU test session")
