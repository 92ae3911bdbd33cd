#!/usr/bin/env python3
"""All five BASELINE.json configurations, this framework vs the reference-equivalent pipeline.

    python -m benchmarks.suite [--scale 1.0] [--only 1,3] [--out benchmarks/RESULTS.json]

| # | BASELINE.json config | how it is run here |
|---|---|---|
| 1 | mocked API, 10 pod ADDED events, stub sink | development profile; 10 pods served by the initial LIST |
| 2 | development.yaml, 100-pod create/delete churn | `createdelete` template: 100 pods × ADDED/MODIFIED/DELETED per round, 1,000 rounds streamed back to back (sustained rate), DEBUG logging |
| 3 | staging.yaml, single namespace, 1k pods steady, 10 ev/s MODIFIED | `steady` template: 1000 listed pods; throughput = 300 unthrottled MODIFIED rounds streamed back to back, latency at 10 ev/s |
| 4 | production.yaml, all namespaces, 10k-pod churn, 100 ev/s | `churn` template, 10k lifecycles per step; latency at 100 ev/s (same as bench.py) |
| 5 | soak: RV bookmark/resume across API-server restarts, 1M events | 20 × 50k churn events with connection drops mid-step (resume), bookmarks and 410 compactions; the sink checks exactly-once |

Each config runs the real :class:`WatcherService` against a replay API server
child process and a stub clusterapi child process. The reference-equivalent
pipeline (``benchmarks/reference_equiv.py``) then runs against the same
servers. Logs go to a file in both cases, so the two do the same logging work.
"""

from __future__ import annotations

import argparse
import asyncio
import glob
import json
import logging
import os
import signal
import socket
import sys
import tempfile
import threading
import time
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from k8s_watcher_amd.engine.service import WatcherService  # noqa: E402
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint  # noqa: E402
from k8s_watcher_amd.metrics import Metrics  # noqa: E402
from k8s_watcher_amd.utils.config import deep_merge, load_settings  # noqa: E402
from k8s_watcher_amd.utils.logsetup import setup_logging  # noqa: E402


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Servers:
    """Replay API server + stub clusterapi, as child processes."""

    def __init__(self, template: str, pods: int, prerender: int = 0, namespaces: Optional[str] = None,
                 sink_workers: int = 4, verify: bool = False) -> None:
        self.args = ["--template", template, "--pods", str(pods), "--prerender", str(prerender)]
        if namespaces:
            self.args += ["--namespaces", namespaces]
        self.sink_workers = sink_workers
        self.verify_dir = tempfile.mkdtemp(prefix="kw-verify-") if verify else None

    async def __aenter__(self) -> "Servers":
        spawn = lambda *a: asyncio.create_subprocess_exec(  # noqa: E731
            *a, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            stderr=asyncio.subprocess.DEVNULL, start_new_session=True, cwd=ROOT)
        self.replay = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.replay_server", *self.args)
        self.sink_port = free_port()
        sink_args = ["--port", str(self.sink_port), "--workers", str(self.sink_workers)]
        if self.verify_dir:
            sink_args += ["--verify-dir", self.verify_dir]
        self.sink = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", *sink_args)
        ready = (await self.replay.stdout.readline()).decode().split()
        assert ready and ready[0] == "READY", ready
        self.api_port, self.events_per_step = int(ready[1]), int(ready[2])
        await self.sink.stdout.readline()
        await asyncio.sleep(0.3)
        return self

    async def cmd(self, line: str) -> int:
        self.replay.stdin.write((line + "\n").encode())
        await self.replay.stdin.drain()
        return int((await self.replay.stdout.readline()).decode().split()[2])

    async def wait_watchers(self, n: int, timeout: float = 20) -> None:
        deadline = time.monotonic() + timeout
        while await self.cmd("WATCHERS") != n:
            if time.monotonic() > deadline:
                raise TimeoutError(f"expected {n} watch streams")
            await asyncio.sleep(0.01)

    def sink_keys(self) -> Dict[str, int]:
        merged: Dict[str, int] = {}
        for path in glob.glob(os.path.join(self.verify_dir, "sink-*.json")):
            with open(path) as fh:
                for k, v in json.load(fh)["keys"].items():
                    merged[k] = merged.get(k, 0) + v
        return merged

    async def __aexit__(self, *exc) -> None:
        for p in (self.replay, self.sink):
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        for p in (self.replay, self.sink):
            try:
                await asyncio.wait_for(p.wait(), 300 if (self.verify_dir and p is self.sink) else 10)
            except asyncio.TimeoutError:
                os.killpg(p.pid, signal.SIGKILL)
            t = getattr(p, "_transport", None)
            if t is not None:
                t.close()
        if self.verify_dir:
            # every worker writes its dump on SIGTERM (renamed into place when complete)
            deadline = time.monotonic() + 300
            while (len(glob.glob(os.path.join(self.verify_dir, "sink-*.json"))) < self.sink_workers
                   and time.monotonic() < deadline):
                await asyncio.sleep(0.1)


EXTRA_OVERRIDES: dict = {}  # --set key.path=value, applied to every config


async def run_ours(srv: Servers, profile: str, overrides: dict, steps: List[str], warm_steps: List[str],
                   pace: Optional[str], expect_watchers: int = 1, step_timeout: float = 300) -> dict:
    settings = load_settings(profile, overrides=deep_merge(deep_merge(
        {"clusterapi": {"base_url": f"http://127.0.0.1:{srv.sink_port}"},
         "watcher": {"retry": {"max_attempts": 0, "delay_seconds": 0.02}}}, overrides), EXTRA_OVERRIDES))
    m = Metrics(record_samples=True)
    t_start = time.perf_counter()
    svc = WatcherService(settings, endpoint=KubeEndpoint(server=f"http://127.0.0.1:{srv.api_port}"), metrics=m)
    await svc.start()
    await srv.wait_watchers(expect_watchers)
    c = m.c

    async def until_idle(base: int, n: int) -> None:
        deadline = time.monotonic() + step_timeout
        while c["events_received"] < base + n or svc.notifier.outstanding() > 0:
            if time.monotonic() > deadline:
                raise TimeoutError(f"{c['events_received'] - base}/{n} events")
            await asyncio.sleep(0.0005)

    await until_idle(0, 0)
    list_p50 = m.latency.percentile_ns(50)
    startup = {"delivered": c["notify_delivered"], "seconds": time.perf_counter() - t_start,
               "p50_ms": (list_p50 / 1e6) if list_p50 else None}
    def settle() -> None:
        # the notifier's I/O thread hands latency samples over in blocks: take
        # what it holds at a phase's end, so they do not land in the next phase
        # (they had put the saturated phase's tail into config #3's paced p50)
        flush = getattr(svc.notifier, "flush", None)
        if flush is not None:
            flush()

    for s in warm_steps:
        await until_idle(c["events_received"], await srv.cmd(s))
    settle()
    m.latency.reset()
    n0, d0 = c["events_received"], c["notify_delivered"]
    t0 = time.perf_counter()
    for s in steps:
        base = c["events_received"]
        n = await srv.cmd(s)
        if s.startswith("STEP") and ("drop=" in s or "expire=" in s):
            await asyncio.sleep(0.05)
            await srv.wait_watchers(expect_watchers)
            await srv.cmd("BOOKMARK")
        # after a 410 the relist reconciles instead of replaying, so count by the stream's RV
        deadline = time.monotonic() + step_timeout
        while True:
            rvs_done = all(r.rv is not None and int(r.rv) >= _last_rv(srv, s) for r in svc.reflectors)
            if (c["events_received"] >= base + n or rvs_done) and svc.notifier.outstanding() == 0:
                break
            if time.monotonic() > deadline:
                raise TimeoutError(f"step {s}: {c['events_received'] - base}/{n}")
            await asyncio.sleep(0.0005)
    elapsed = time.perf_counter() - t0
    events = c["events_received"] - n0
    settle()
    sat_p50 = m.latency.percentile_ns(50)
    out = {"events": events, "seconds": elapsed, "events_per_s": events / elapsed if elapsed else None,
           "notified": c["notify_delivered"] - d0,
           "saturated_p50_ms": sat_p50 / 1e6 if sat_p50 else None, "startup": startup}
    if pace:
        m.latency.reset()
        await until_idle(c["events_received"], await srv.cmd(pace))
        settle()
        p50, p99 = m.latency.percentile_ns(50), m.latency.percentile_ns(99)
        out.update({"p50_ms": p50 / 1e6 if p50 else None, "p99_ms": p99 / 1e6 if p99 else None,
                    "latency_samples": m.latency.n})
    out["counters"] = {k: v for k, v in c.items() if v}
    import resource
    out["max_rss_mb"] = round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1)  # watcher process
    out["cached_pods_at_end"] = len(svc.pipeline.cache) if svc.pipeline is not None else None
    svc.stop()
    await svc.shutdown()
    return out


_STEP_RV: Dict[str, int] = {}


def _last_rv(srv: Servers, s: str) -> int:
    parts = s.split()
    if parts[0] == "STEPS":
        return 10_000_000 + int(parts[2]) * srv.events_per_step - 1
    step = int(parts[1])
    n = srv.events_per_step if parts[0] == "STEP" else int(parts[3])
    return 10_000_000 + step * srv.events_per_step + n - 1


async def run_reference(srv: Servers, profile: str, namespaces: List[str], critical: bool, n_events: int,
                        warm: int, start_cmd: Optional[str], pace: Optional[str]) -> dict:
    from benchmarks.reference_equiv import RefEquivWatcher
    loop = asyncio.get_running_loop()
    ref = RefEquivWatcher(profile, namespaces, critical, f"http://127.0.0.1:{srv.sink_port}")
    connected = loop.create_future()
    warmed = loop.create_future()
    res = {}

    def work() -> None:
        res["elapsed"] = ref.run(f"http://127.0.0.1:{srv.api_port}", warm + n_events,
                                 on_connected=lambda: loop.call_soon_threadsafe(connected.set_result, None),
                                 warm_events=warm,
                                 on_warm=lambda: loop.call_soon_threadsafe(warmed.set_result, None))

    await srv.wait_watchers(0)
    th = threading.Thread(target=work, daemon=True)
    th.start()
    await connected
    await srv.wait_watchers(1)
    if warm:
        await warmed
    if start_cmd:
        await srv.cmd(start_cmd)
    deadline = time.monotonic() + 900
    while th.is_alive():
        if time.monotonic() > deadline:
            raise TimeoutError(f"reference-equivalent run stuck at {ref.processed}/{warm + n_events} events")
        await asyncio.sleep(0.01)
    lat = sorted(ref.latencies_ns)
    out = {"events": ref.processed - warm, "seconds": res["elapsed"],
           "events_per_s": (ref.processed - warm) / res["elapsed"] if res.get("elapsed") else None,
           "notified": ref.notified, "saturated_p50_ms": lat[len(lat) // 2] / 1e6 if lat else None}
    if pace:
        ref2 = RefEquivWatcher(profile, namespaces, critical, f"http://127.0.0.1:{srv.sink_port}")
        connected2 = loop.create_future()
        warmed2 = loop.create_future()
        n = int(pace.split()[3])
        th2 = threading.Thread(target=lambda: ref2.run(
            f"http://127.0.0.1:{srv.api_port}", warm + n,
            on_connected=lambda: loop.call_soon_threadsafe(connected2.set_result, None),
            warm_events=warm, on_warm=lambda: loop.call_soon_threadsafe(warmed2.set_result, None)),
            daemon=True)
        await srv.wait_watchers(0)
        th2.start()
        await connected2
        await srv.wait_watchers(1)
        if warm:
            await warmed2
        await srv.cmd(pace)
        while th2.is_alive():
            await asyncio.sleep(0.01)
        lat = sorted(ref2.latencies_ns)
        out["p50_ms"] = lat[len(lat) // 2] / 1e6 if lat else None
        out["p99_ms"] = lat[min(len(lat) - 1, int(len(lat) * 0.99))] / 1e6 if lat else None
    return out


# ----------------------------------------------------------------------------- configs


async def config1(a) -> dict:
    async with Servers("steady", 10, namespaces="default,kube-system") as srv:
        ours = await run_ours(srv, "development", {}, [], [], None)
        ref = await run_reference(srv, "development", ["default", "kube-system"], False, 10, 0, None, None)
    ok = ours["startup"]["delivered"] == 10 and ref["notified"] == 10
    return {"ours": ours, "reference_equiv": ref, "all_10_delivered": ok}


async def config2(a) -> dict:
    steps = max(2, int(1000 * a.scale))  # 300 events per step: 300k events, a stable sustained rate
    async with Servers("createdelete", 100, prerender=steps + 1) as srv:
        e = srv.events_per_step
        # one stream of `steps` rounds: the sustained rate, not a stop-and-wait per 300-event round
        ours = await run_ours(srv, "development", {}, [f"STEPS 1 {steps + 1}"],
                              ["STEP 0"], f"PACE {steps + 1} 100 {min(e, 200)}")
        ref = await run_reference(srv, "development", ["default", "kube-system"], False, e, 0,
                                  f"STEP {steps + 2}", f"PACE {steps + 3} 100 {min(e, 200)}")
    return {"ours": ours, "reference_equiv": ref}


async def config3(a) -> dict:
    steps = max(2, int(300 * a.scale))  # 1,000 events per step: 300k events
    ov = {"watcher": {"namespaces": ["default"], "namespace_scope": "server"}}
    async with Servers("steady", 1000, prerender=steps + 1, namespaces="default") as srv:
        ours = await run_ours(srv, "staging", ov, [f"STEPS 1 {steps + 1}"], ["STEP 0"],
                              f"PACE {steps + 1} 10 {max(10, int(30 * a.scale))}")
        ref = await run_reference(srv, "staging", ["default"], False, 1000, 1000, f"STEP {steps + 2}",
                                  f"PACE {steps + 3} 10 {max(10, int(30 * a.scale))}")
    return {"ours": ours, "reference_equiv": ref}


async def config4(a) -> dict:
    steps = max(2, int(10 * a.scale))
    pods = max(1000, int(10000 * a.scale))
    async with Servers("churn", pods, prerender=steps + 1) as srv:
        e = srv.events_per_step
        ours = await run_ours(srv, "production", {}, [f"STEP {k}" for k in range(1, steps + 1)], ["STEP 0"],
                              f"PACE {steps + 1} 100 300")
        ref = await run_reference(srv, "production", ["default", "production", "monitoring", "kube-system"],
                                  True, min(e, 10000), 0, f"STEP {steps + 2}",
                                  f"PACE {steps + 3} 100 300")
    return {"ours": ours, "reference_equiv": ref}


async def config5(a) -> dict:
    steps = max(5, int(20 * a.scale))
    pods = max(1000, int(10000 * a.scale))
    ov = {"watcher": {"log_level": "WARNING"}}
    plan = []
    for k in range(1, steps + 1):
        if k % 5 == 0:
            plan.append(f"STEP {k} expire={pods * 5 * 4 // 5}")
        elif k % 2 == 0:
            plan.append(f"STEP {k} drop={pods * 5 // 2}")
        else:
            plan.append(f"STEP {k}")
    async with Servers("churn", pods, prerender=0, verify=True) as srv:
        ours = await run_ours(srv, "staging", ov, plan, ["STEP 0"], None)
        e = srv.events_per_step
    keys = srv.sink_keys()
    dup = sum(v - 1 for v in keys.values() if v > 1)
    by_step: Dict[int, List[str]] = {}
    for k in keys:
        by_step.setdefault(int(k[:8], 16), []).append(k)
    complete, deleted_ok = [], True
    for k, s in enumerate(plan, start=1):
        ks = by_step.get(k, [])
        uids = {x.split("|")[0] for x in ks}
        dels = {x.split("|")[0] for x in ks if x.split("|")[1] == "DELETED"}
        deleted_ok &= uids == dels
        if "expire" not in s:
            complete.append(len(ks) == e)
    return {"ours": ours, "events_replayed": steps * e, "notifications_checked": sum(keys.values()),
            "duplicates": dup, "drop_only_steps_complete": all(complete),
            "every_pod_ends_deleted": deleted_ok, "restarts": sum("drop=" in s for s in plan),
            "compactions_410": sum("expire=" in s for s in plan),
            "reference_equiv": "n/a: the reference cannot resume (410 exits the process, SURVEY §5.3)"}


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}


def markdown(results: dict) -> str:
    rows = ["| # | config | ours: events/s | ref-equiv: events/s | speedup | ours p50 ms | ref p50 ms | notes |",
            "|---|---|---|---|---|---|---|---|"]
    names = {1: "mock API, 10 ADDED", 2: "dev, 100-pod create/delete churn", 3: "staging, 1 ns, 1k steady MODIFIED",
             4: "prod, all ns, 10k churn", 5: "soak: restarts + 410, exactly-once"}
    for k in sorted(results, key=int):
        r = results[k]
        o = r["ours"]
        ref = r["reference_equiv"] if isinstance(r.get("reference_equiv"), dict) else None
        f = lambda v, d=1: ("%.*f" % (d, v)) if isinstance(v, (int, float)) else "–"  # noqa: E731
        if int(k) == 1:
            rows.append(f"| 1 | {names[1]} | – | – | – | {f(o['startup']['p50_ms'], 3)} | "
                        f"{f(ref.get('saturated_p50_ms') if ref else None, 3)} | "
                        f"all 10 delivered (both): {r['all_10_delivered']}; p50 = list read → 2xx |")
            continue
        ours_eps = o.get("events_per_s")
        ref_eps = ref.get("events_per_s") if ref else None
        sp = (ours_eps / ref_eps) if ours_eps and ref_eps else None
        note = ""
        if int(k) == 5:
            note = (f"{r['events_replayed']} events, {r['restarts']} restarts, {r['compactions_410']} × 410; "
                    f"duplicates={r['duplicates']}, drop-only steps complete={r['drop_only_steps_complete']}, "
                    f"every pod ends DELETED={r['every_pod_ends_deleted']}")
        rows.append(f"| {k} | {names[int(k)]} | {f(ours_eps)} | {f(ref_eps)} | {f(sp)}× | {f(o.get('p50_ms'), 3)} | "
                    f"{f(ref.get('p50_ms') if ref else None, 3)} | {note} |")
    return "\n".join(rows)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--only", default="1,2,3,4,5")
    ap.add_argument("--scale", type=float, default=1.0, help="shrink step counts / sizes (tests use 0.1)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="config override for every run, e.g. clusterapi.pool.pipeline_depth=8")
    a = ap.parse_args(argv)
    from k8s_watcher_amd.utils.config import parse_override
    for expr in a.set:
        EXTRA_OVERRIDES.update(deep_merge(EXTRA_OVERRIDES, parse_override(expr)))
    log_path = os.path.join(tempfile.gettempdir(), f"kw-suite-{os.getpid()}.log")
    results = {}
    for k in [int(x) for x in a.only.split(",") if x]:
        profile = {1: "development", 2: "development", 3: "staging", 4: "production", 5: "staging"}[k]
        # config 5 is a soak of the resume machinery: per-event INFO lines are off there
        level = "WARNING" if k == 5 else load_settings(profile).watcher.log_level
        setup_logging(profile, level, log_file=log_path)
        logging.getLogger("watcher.pod_watcher").setLevel(logging.NOTSET)
        t = time.time()
        results[str(k)] = asyncio.run(CONFIGS[k](a))
        print(f"config {k} done in {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    md = markdown(results)
    print(md)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(results, fh, indent=1, default=str)
    return 0


if __name__ == "__main__":
    sys.exit(main())
