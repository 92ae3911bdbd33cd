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
    config.addinivalue_line("markers", "perf: wall-clock rate comparison (box tier only: also marked gpu)")


@pytest.fixture(scope="session", autouse=True)
def _native_extension():
    """Build the C++ extension once per session if it is missing or stale."""
    from k8s_watcher_amd.ops import native
    native.ensure_built(quiet=True)
    yield


HEADLINE_MAX_BYTES = 4096  # the driver keeps ~8 KB of output; the headline must fit with room to spare


def bench_result(proc, json_out: str) -> dict:
    """bench.py's full record (``--json-out``) after checking its stdout:
    exactly one JSON line (rank 0's), the last line, under HEADLINE_MAX_BYTES.
    The headline dict is returned under ``"_headline"``."""
    import json
    assert proc.returncode == 0, (proc.stdout[-2000:], proc.stderr[-3000:])
    lines = proc.stdout.strip().splitlines()
    heads = [ln for ln in lines if ln.startswith("{")]
    assert len(heads) == 1 and lines[-1] == heads[0], proc.stdout[-3000:]
    assert len(heads[0].encode()) < HEADLINE_MAX_BYTES, len(heads[0])
    head = json.loads(heads[0])
    with open(json_out) as fh:
        detail = json.load(fh)
    assert head["value"] == detail["value"] and head["detail_json"] == json_out
    detail["_headline"] = head
    return detail


def run_bench(args, tmp_dir=None, timeout=600, env=None, torchrun_ranks=0, port=None) -> dict:
    """Run bench.py (or ``torchrun`` of it with ``torchrun_ranks``) with
    ``args`` and return :func:`bench_result`."""
    import subprocess
    import tempfile
    out = os.path.join(str(tmp_dir or tempfile.gettempdir()), f"bench-{next(tempfile._get_candidate_names())}.json")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    if torchrun_ranks:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(torchrun_ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py")]
    proc = subprocess.run(cmd + list(args) + ["--json-out", out], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)
    return bench_result(proc, out)


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
