import asyncio
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs the MI355X box (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running soak/bench style test")


@pytest.fixture(scope="session", autouse=True)
def _native_extension():
    """Build the C++ extension once per session if it is missing or stale."""
    from k8s_watcher_amd.ops import native
    native.ensure_built(quiet=True)
    yield


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))
