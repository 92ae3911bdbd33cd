"""Memory accounting and release: the C heap gauges (glibc mallinfo2) and the
periodic malloc_trim of the native engine (watcher.malloc_trim_seconds)."""

import asyncio
import os

import pytest

from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.utils.config import ConfigError, load_settings


def test_malloc_info_and_trim():
    kw = load()
    blocks = [bytearray(1 << 16) for _ in range(256)]  # 16 MiB through the C heap
    info = kw.malloc_info()
    assert set(info) == {"in_use_bytes", "free_bytes", "arena_bytes", "mmap_bytes"}
    if "asan" in os.environ.get("LD_PRELOAD", "") and info["in_use_bytes"] == 0:
        pytest.skip("the sanitizer replaced glibc's allocator: mallinfo2 sees nothing")
    assert info["in_use_bytes"] >= 16 << 20
    del blocks
    assert kw.malloc_trim() in (True, False)
    after = kw.malloc_info()
    assert after["in_use_bytes"] < info["in_use_bytes"]


def test_malloc_trim_setting():
    assert load_settings("production", environ={}).watcher.malloc_trim_seconds == 60.0
    s = load_settings("production", overrides={"watcher": {"malloc_trim_seconds": 0}}, environ={})
    assert s.watcher.malloc_trim_seconds == 0.0
    with pytest.raises(ConfigError):
        load_settings("production", overrides={"watcher": {"malloc_trim_seconds": -1}}, environ={})


def _trim_stub(min_free_mb, monkeypatch):
    import types

    from k8s_watcher_amd.engine import service
    from k8s_watcher_amd.metrics import Metrics
    monkeypatch.setattr(service, "MALLOC_TRIM_MIN_FREE", int(min_free_mb * (1 << 20)))
    return types.SimpleNamespace(metrics=Metrics(), log=__import__("logging").getLogger("test"))


def test_service_trims_periodically(monkeypatch):
    """The service's trim loop runs the trim off the event loop, counts and times it."""
    from k8s_watcher_amd.engine.service import WatcherService

    async def body():
        stub = _trim_stub(0.0, monkeypatch)
        task = asyncio.ensure_future(WatcherService._malloc_trim_loop(stub, 0.01))
        await asyncio.sleep(1.4)  # each trim waits for a quiet half second first
        task.cancel()
        return stub.metrics

    m = asyncio.run(body())
    assert m.c.get("malloc_trims", 0) >= 2
    assert m.c["malloc_trim_us"] > 0 and m.gauges["malloc_trim_max_ms"]() >= m.gauges["malloc_trim_last_ms"]() > 0


def test_service_skips_trim_below_free_threshold(monkeypatch):
    """service.MALLOC_TRIM_MIN_FREE: no trim (no arena walk under their
    locks) while the heap retains less free memory than that."""
    from k8s_watcher_amd.engine.service import WatcherService

    async def body():
        stub = _trim_stub(1e6, monkeypatch)  # a terabyte: never reached
        task = asyncio.ensure_future(WatcherService._malloc_trim_loop(stub, 0.01))
        await asyncio.sleep(0.15)
        task.cancel()
        return stub.metrics

    m = asyncio.run(body())
    assert m.c.get("malloc_trims", 0) == 0 and m.c["malloc_trims_skipped"] >= 2


def test_service_defers_trim_under_load(monkeypatch):
    """Under sustained traffic the trim waits for a quiet moment (the freed
    pages would be reused at once, and a trim stalls allocating threads)."""
    from k8s_watcher_amd.engine.service import WatcherService

    async def body():
        stub = _trim_stub(0.0, monkeypatch)
        task = asyncio.ensure_future(WatcherService._malloc_trim_loop(stub, 0.05))
        t_end = asyncio.get_running_loop().time() + 1.2
        while asyncio.get_running_loop().time() < t_end:  # ~20k events/s
            stub.metrics.c["events_received"] += 100
            await asyncio.sleep(0.005)
        task.cancel()
        return stub.metrics

    m = asyncio.run(body())
    assert m.c.get("malloc_trims", 0) == 0 and m.c["malloc_trims_deferred"] >= 1


_TUNE_PROBE = r"""
import sys
from k8s_watcher_amd.ops.native import load
kw = load()
if sys.argv[1] == "tune":
    assert kw.malloc_tune(512 << 10, 4 << 20) is True
big = bytearray(8 << 20)  # freed: a sliding threshold would rise to 8 MiB
del big
held = bytearray(1 << 20)  # 1 MiB: its own mapping only under a fixed threshold
print(kw.malloc_info()["mmap_bytes"])
"""


@pytest.mark.parametrize("mode", ["tune", "default"])
def test_malloc_tune_keeps_transients_off_the_arenas(mode):
    """kwcore.malloc_tune fixes glibc's mmap threshold: after an 8 MiB block
    is freed, a 1 MiB block still gets its own mapping (returned to the kernel
    when freed) instead of a hole in the arena; glibc's default slides the
    threshold up to 8 MiB and carves the 1 MiB block from the heap."""
    import subprocess
    import sys
    if "asan" in os.environ.get("LD_PRELOAD", ""):
        pytest.skip("the sanitizer replaced glibc's allocator")
    out = subprocess.run([sys.executable, "-c", _TUNE_PROBE, mode], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    mmapped = int(out.stdout.split()[-1])
    if mode == "tune":
        assert mmapped >= 1 << 20
    else:
        assert mmapped < 1 << 20


def test_malloc_tune_rejects_out_of_range():
    kw = load()
    with pytest.raises(ValueError):
        kw.malloc_tune(0, 1 << 20)
    with pytest.raises(ValueError):
        kw.malloc_tune(64 << 20, 1 << 20)
