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


@pytest.fixture(autouse=True)
def _keep_cpu_affinity():
    """A test that starts a WatcherService without shutting it down must not
    leave the test runner's thread pinned (watcher.thread_pinning / decode_affinity)."""
    import os
    try:
        before = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        yield
        return
    yield
    try:
        if os.sched_getaffinity(0) != before:
            os.sched_setaffinity(0, before)
    except OSError:
        pass
