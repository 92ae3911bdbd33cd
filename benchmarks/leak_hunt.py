#!/usr/bin/env python3
"""Memory growth per step of an in-process watcher (what the long soak flags, in minutes).

    python -m benchmarks.leak_hunt [--steps 60] [--pods 2000] [--variant base|nonotify|nocheckpoint|python]

One :class:`WatcherService` (production profile: critical + namespace filter,
checkpoints) watches ``testing/replay_server.py`` (``churn``) and notifies the
stub clusterapi; steps are streamed back to back. Every ``--every`` steps the
RSS and the Python heap (``tracemalloc``) are sampled; at the end the growth
after warm-up is split into Python-heap and native (RSS minus Python heap)
bytes per step, with the top Python allocation sites that grew.
"""

from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import sys
import tempfile
import time
import tracemalloc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TARGETS = ["default", "production", "monitoring", "kube-system"]


def rss_kb() -> int:
    with open("/proc/self/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return 0


async def amain(a) -> dict:
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.utils.config import load_settings

    replay = await asyncio.create_subprocess_exec(
        sys.executable, "-m", "k8s_watcher_amd.testing.replay_server", "--template", "churn", "--pods", str(a.pods),
        stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE, cwd=ROOT)
    ready = (await replay.stdout.readline()).decode().split()
    port, per_step = int(ready[1]), int(ready[2])
    with __import__("socket").socket() as so:
        so.bind(("127.0.0.1", 0))
        sink_port = so.getsockname()[1]
    sink = await asyncio.create_subprocess_exec(  # out of process: it keeps what it receives
        sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port", str(sink_port), "--workers", "1",
        stdout=asyncio.subprocess.PIPE, cwd=ROOT)
    await sink.stdout.readline()
    sink_url = f"http://127.0.0.1:{sink_port}"
    state = tempfile.mkdtemp(prefix="kw-leak-")
    watcher = {"namespaces": TARGETS, "retry": {"max_attempts": 0, "delay_seconds": 0.05},
               "engine": "python" if a.variant == "python" else "native"}
    if a.variant != "nocheckpoint":
        watcher["checkpoint"] = {"path": os.path.join(state, "ckpt.bin"), "interval_seconds": 1}
    settings = load_settings("production", overrides={
        "clusterapi": {"base_url": sink_url, "enabled": a.variant != "nonotify", "health_check_on_start": False,
                       "pool": {"connections": 4, "pipeline_depth": 32}},
        "watcher": watcher,
        **({"metrics": {"enabled": True, "host": "127.0.0.1", "port": a.scrape}} if a.scrape else {})})
    metrics = Metrics()
    svc = WatcherService(settings, endpoint=KubeEndpoint(server=f"http://127.0.0.1:{port}"), metrics=metrics)
    await svc.start()
    c = metrics.c

    async def cmd(line: str) -> None:
        replay.stdin.write((line + "\n").encode())
        await replay.stdin.drain()
        await replay.stdout.readline()

    tracemalloc.start(25)
    samples = []
    snap0 = None
    target = c["events_received"]
    for k in range(a.steps):
        if a.mix and k % 11 == 10:  # compaction mid-step: 410, relist (events after it are gone)
            await cmd(f"STEP {k} expire={per_step // 2}")
            await asyncio.sleep(a.pause)
        elif a.mix and k % 7 == 6:  # every watch dropped mid-step: resume from the resourceVersion
            await cmd(f"STEP {k} drop={per_step // 2}")
            target += per_step
        else:
            await cmd(f"STEP {k}")
            target += per_step
        if a.mix and k % 3 == 2:
            await cmd("BOOKMARK")
        target = max(target, c["events_received"]) if a.mix and k % 11 == 10 else target
        t_end = time.monotonic() + 60
        while (c["events_received"] < target or svc.notifier.outstanding() > 0) and time.monotonic() < t_end:
            await asyncio.sleep(0.002)
        if a.scrape:
            import urllib.request
            await asyncio.get_running_loop().run_in_executor(None, lambda: urllib.request.urlopen(
                f"http://127.0.0.1:{a.scrape}/metrics").read())
        if a.pause:
            await asyncio.sleep(a.pause)
        if k % a.every == a.every - 1:
            gc.collect()
            await asyncio.sleep(0.05)
            py_cur, _ = tracemalloc.get_traced_memory()
            samples.append({"step": k + 1, "rss_kb": rss_kb(), "py_heap_kb": py_cur // 1024,
                            "cached": c.get("cached_pods")})
            print(json.dumps(samples[-1]), file=sys.stderr, flush=True)
            if k + 1 == a.warmup:
                snap0 = tracemalloc.take_snapshot()
    snap1 = tracemalloc.take_snapshot()
    top = []
    if snap0 is not None:
        for st in snap1.compare_to(snap0, "traceback")[:8]:
            top.append({"kb": st.size_diff // 1024, "count": st.count_diff,
                        "where": [f"{f.filename.replace(ROOT, '')}:{f.lineno}" for f in st.traceback[-4:]]})
    svc.stop()
    await svc.shutdown()
    sink.terminate()
    await sink.wait()
    replay.stdin.write(b"QUIT\n")
    await replay.wait()
    after = [s for s in samples if s["step"] >= a.warmup]
    out = {"variant": a.variant, "pods_per_step": a.pods, "events_per_step": per_step, "samples": samples,
           "top_python_growth": top}
    if len(after) >= 2:
        n = after[-1]["step"] - after[0]["step"]
        out["rss_bytes_per_step"] = round((after[-1]["rss_kb"] - after[0]["rss_kb"]) * 1024 / n)
        out["py_heap_bytes_per_step"] = round((after[-1]["py_heap_kb"] - after[0]["py_heap_kb"]) * 1024 / n)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--pods", type=int, default=2000)
    ap.add_argument("--mix", action="store_true", help="drop / expire / bookmark steps as in benchmarks.soak")
    ap.add_argument("--scrape", type=int, default=0, help="serve /metrics on this port and scrape it every step")
    ap.add_argument("--pause", type=float, default=0.0, help="idle seconds after each step")
    ap.add_argument("--variant", default="base", choices=["base", "nonotify", "nocheckpoint", "python"])
    a = ap.parse_args(argv)
    res = asyncio.run(amain(a))
    print(json.dumps({k: v for k, v in res.items() if k != "samples"}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
