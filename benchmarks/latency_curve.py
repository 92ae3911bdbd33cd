#!/usr/bin/env python3
"""Event→notify latency vs offered load, this framework and the reference-equivalent pipeline.

    python -m benchmarks.latency_curve [--rates 100,1000,10000,100000,500000]
        [--profile staging] [--min-samples 5000] [--ref-rates 100,1000] [--out f.json]

BASELINE.json's metric pairs throughput with "p50 event→notify latency" and
its target is "p50 ≤ reference". The reference notifies with one synchronous
``requests`` POST per event on the watch thread
(``/root/reference/watcher/clusterapi_client.py:36``, call site
``pod_watcher.py:236``), so its latency is one round trip as long as the
offered load stays below ~1/RTT and grows without bound above it. This tool
measures both pipelines at each offered load on the same fixture
(``testing/cluster_replay.py``: events paced by the API-server side) and the
same stub clusterapi:

* latency = socket read of the watch bytes holding the event → 2xx from
  clusterapi, per notified event (``Metrics.latency`` samples / the
  reference-equivalent's own clock, measured the same way);
* at each rate the pace runs until at least ``--min-samples`` notifications
  (and at least ``--min-seconds``) — the profile decides which events notify
  (staging: every event; production: DELETED + terminal phases in the target
  namespaces, ~20%);
* the reference-equivalent runs only at the rates it can sustain
  (``--ref-rates``): above ~1/RTT its queue — the watch socket — grows for as
  long as the run lasts, so a percentile there measures the run length.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import sys
import threading
import time
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(samples: List[int], q: float) -> Optional[float]:
    if not samples:
        return None
    s = sorted(samples)
    return s[max(0, min(len(s) - 1, int(-(-q * len(s) // 100)) - 1))] / 1e6


class Fixture:
    async def start(self, pods: int, namespaces: int, targets: str, sink_workers: int) -> None:
        from bench import free_port, spawn
        from k8s_watcher_amd.testing.cluster_replay import namespace_names
        self.names = namespace_names(namespaces)
        self.targets = ([n for i, n in enumerate(self.names) if i % 2 == 0] if targets == "even"
                        else list(self.names))
        self.replay = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.cluster_replay",
                                  "--pods", str(pods), "--namespace-list", ",".join(self.names),
                                  "--targets", ",".join(self.targets), "--workers", "2")
        self.sink_port = free_port()
        self.sink = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port",
                                str(self.sink_port), "--workers", str(sink_workers))
        line = (await asyncio.wait_for(self.replay.stdout.readline(), 600)).decode()
        self.info = json.loads(line[6:])
        await asyncio.wait_for(self.sink.stdout.readline(), 60)
        await asyncio.sleep(0.3)

    async def cmd(self, line: str) -> list:
        self.replay.stdin.write((line + "\n").encode())
        await self.replay.stdin.drain()
        return (await self.replay.stdout.readline()).decode().split()

    async def watchers(self, n: int) -> None:
        for _ in range(3000):
            if int((await self.cmd("WATCHERS"))[2]) == n:
                return
            await asyncio.sleep(0.01)
        raise TimeoutError(f"expected {n} watch streams")

    async def close(self) -> None:
        for p in (self.replay, self.sink):
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            try:
                await asyncio.wait_for(p.wait(), 5)
            except asyncio.TimeoutError:
                os.killpg(p.pid, signal.SIGKILL)
            t = getattr(p, "_transport", None)
            if t is not None:
                t.close()


def plan(rate: float, fraction: float, min_samples: int, min_seconds: float, max_events: int,
         max_seconds: float = 90.0) -> int:
    """Events to pace so that ~min_samples notify and the run lasts >= min_seconds
    (and at most max_seconds: a 20%-notifying profile at 100 ev/s would need 5 min)."""
    n = max(int(min_samples / max(fraction, 1e-6) * 1.1), int(rate * min_seconds))
    return max(1, min(n, max_events, int(rate * max_seconds)))


async def paced(fx: "Fixture", line: str, progress) -> None:
    """Run a PACE command, printing progress every 10 s (a silent minute looks hung)."""
    task = asyncio.ensure_future(fx.cmd(line))
    while True:
        done, _ = await asyncio.wait([task], timeout=10.0)
        if done:
            task.result()
            return
        print(f"  ... {line}: {progress()}", file=sys.stderr, flush=True)


async def ours(fx: Fixture, a, rates: List[float], step0: int) -> list:
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.utils.config import load_settings
    from k8s_watcher_amd.utils.logsetup import setup_logging
    import tempfile
    log_path = os.path.join(tempfile.gettempdir(), f"kw-latency-{os.getpid()}.log")
    setup_logging(a.profile, load_settings(a.profile).watcher.log_level, log_file=log_path)
    s = load_settings(a.profile, overrides={
        "clusterapi": {"base_url": f"http://127.0.0.1:{fx.sink_port}", "health_check_on_start": False},
        "watcher": {"namespaces": fx.targets, "retry": {"max_attempts": 0, "delay_seconds": 0.05}}})
    m = Metrics(record_samples=True)
    svc = WatcherService(s, endpoint=KubeEndpoint(server=f"http://127.0.0.1:{fx.info['port']}"), metrics=m)
    await svc.start()
    await fx.watchers(1)
    c = m.c
    fraction = fx.info["notifiable_per_step"] / fx.info["events_per_step"] if a.profile == "production" else 1.0
    out = []
    for i, rate in enumerate(rates):
        n = plan(rate, fraction, a.min_samples, a.min_seconds, fx.info["events_per_step"], a.max_seconds)
        m.latency.reset()
        base = c["events_received"]
        t0 = time.perf_counter()
        await paced(fx, f"PACE {step0 + i} {rate} {n}", lambda: f"{c['events_received'] - base}/{n} events")
        deadline = time.monotonic() + 600
        while c["events_received"] < base + n or svc.notifier.outstanding() > 0:
            if time.monotonic() > deadline:
                raise TimeoutError(f"rate {rate}: {c['events_received'] - base}/{n}")
            await asyncio.sleep(0.001)
        elapsed = time.perf_counter() - t0
        lat = list(m.latency.samples or [])
        row = {"offered_ev_s": rate, "events": n, "seconds": round(elapsed, 3),
               "achieved_ev_s": round(n / elapsed, 1), "samples": len(lat),
               "p50_ms": pct(lat, 50), "p90_ms": pct(lat, 90), "p99_ms": pct(lat, 99), "p999_ms": pct(lat, 99.9)}
        print(f"ours  {rate:>9.0f} ev/s: {row}", file=sys.stderr, flush=True)
        out.append(row)
    svc.stop()
    await svc.shutdown()
    return out


async def reference(fx: Fixture, a, rates: List[float], step0: int) -> list:
    from benchmarks.reference_equiv import RefEquivWatcher
    from k8s_watcher_amd.utils.config import load_settings
    s = load_settings(a.profile)
    fraction = fx.info["notifiable_per_step"] / fx.info["events_per_step"] if a.profile == "production" else 1.0
    out = []
    loop = asyncio.get_running_loop()
    for i, rate in enumerate(rates):
        n = plan(rate, fraction, a.min_samples, a.min_seconds, fx.info["events_per_step"], a.max_seconds)
        await fx.watchers(0)
        ref = RefEquivWatcher(a.profile, fx.targets, s.watcher.critical_events_only,
                              f"http://127.0.0.1:{fx.sink_port}")
        connected = loop.create_future()
        res = {}
        th = threading.Thread(target=lambda: res.update(elapsed=ref.run(
            f"http://127.0.0.1:{fx.info['port']}", n,
            on_connected=lambda: loop.call_soon_threadsafe(connected.set_result, None))), daemon=True)
        th.start()
        await connected
        await fx.watchers(1)
        t0 = time.perf_counter()
        await paced(fx, f"PACE {step0 + i} {rate} {n}", lambda: f"{ref.processed}/{n} events")
        while th.is_alive():
            await asyncio.sleep(0.01)
        elapsed = time.perf_counter() - t0
        lat = ref.latencies_ns
        row = {"offered_ev_s": rate, "events": ref.processed, "seconds": round(elapsed, 3),
               "achieved_ev_s": round(ref.processed / elapsed, 1), "samples": len(lat),
               "p50_ms": pct(lat, 50), "p90_ms": pct(lat, 90), "p99_ms": pct(lat, 99), "p999_ms": pct(lat, 99.9)}
        print(f"ref   {rate:>9.0f} ev/s: {row}", file=sys.stderr, flush=True)
        out.append(row)
    return out


def markdown(res: dict) -> str:
    ref = {r["offered_ev_s"]: r for r in res["reference_equiv"]}
    lines = [f"profile `{res['profile']}`; latency = socket read of the watch bytes → 2xx from clusterapi", "",
             "| offered ev/s | ours achieved | ours samples | ours p50 ms | p90 | p99 | p99.9 | ref-equiv achieved | "
             "ref samples | ref p50 ms | ref p99 ms |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    f = lambda v: f"{v:.3f}" if isinstance(v, float) else "–"  # noqa: E731
    for r in res["ours"]:
        q = ref.get(r["offered_ev_s"], {})
        lines.append(f"| {r['offered_ev_s']:,.0f} | {r['achieved_ev_s']:,.0f} | {r['samples']:,} | {f(r['p50_ms'])} | "
                     f"{f(r['p90_ms'])} | {f(r['p99_ms'])} | {f(r['p999_ms'])} | "
                     f"{q.get('achieved_ev_s', '–') if not q else format(q['achieved_ev_s'], ',.0f')} | "
                     f"{q.get('samples', '–')} | {f(q.get('p50_ms'))} | {f(q.get('p99_ms'))} |")
    return "\n".join(lines)


async def amain(a) -> dict:
    rates = [float(x) for x in a.rates.split(",") if x]
    ref_rates = [float(x) for x in a.ref_rates.split(",") if x]
    fx = Fixture()
    await fx.start(a.pods, a.namespaces, "even" if a.profile == "production" else "all", a.sink_workers)
    try:
        res = {"profile": a.profile, "ours": await ours(fx, a, rates, 0),
               "reference_equiv": await reference(fx, a, ref_rates, len(rates)) if ref_rates else []}
    finally:
        await fx.close()
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--rates", default="100,1000,10000,100000,500000")
    ap.add_argument("--ref-rates", default="100,1000")
    ap.add_argument("--profile", default="staging", choices=["development", "staging", "production"])
    ap.add_argument("--min-samples", type=int, default=5000)
    ap.add_argument("--min-seconds", type=float, default=2.0)
    ap.add_argument("--max-seconds", type=float, default=90.0, help="cap per rate (fewer samples at low rates)")
    ap.add_argument("--pods", type=int, default=120000, help="lifecycles per fixture step (caps events per rate)")
    ap.add_argument("--namespaces", type=int, default=64)
    ap.add_argument("--sink-workers", type=int, default=4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    res = asyncio.run(amain(a))
    md = markdown(res)
    print(md)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
