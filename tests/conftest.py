"""Shared test setup.

* registers the `gpu` marker (tests that need an MI355X);
* puts the repo root on sys.path (nexoedge_amd, oracle);
* loads libnxec before anything imports torch, so both share one HIP runtime.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import nexoedge_amd  # noqa: E402,F401  (fails loudly if libnxec.so is not built)

GOLDEN_PATH = os.path.join(ROOT, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN_PATH) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu_ctx():
    from nexoedge_amd import nxec

    if nxec.device_count() == 0:
        pytest.fail("gpu test collected but no HIP device is visible")
    ctx = nxec.Context(0)
    yield ctx
    ctx.close()
