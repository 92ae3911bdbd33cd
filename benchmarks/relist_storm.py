#!/usr/bin/env python3
"""Relist storm: every pod watch of a large cluster expires at once.

The reference's only recovery is a process restart that re-lists the whole
cluster (``/root/reference/watcher/pod_watcher.py:264,273-275``; SURVEY §5.3
item 5). This watcher relists per scope and diffs against its cache
(``ops/csrc/relist.inc``); this benchmark measures that path at cluster scale:

1. ``testing/storm_server.py`` serves ``--namespaces`` × (``--pods`` / N)
   running pods; the watcher (staging profile: every event notified, native
   engine and notifier) syncs — ``--scope discover`` is one watch per
   namespace, ``cluster`` the reference's single all-namespaces watch — and
   every pod must reach the stub clusterapi exactly once (ADDED);
2. while the watches are still open the cluster changes *silently*:
   ``--churn`` pods finish, ``--churn`` are deleted, ``--churn`` created;
3. every pod watch gets ``ERROR 410`` (a compaction past all their
   resourceVersions) and must relist; the sink must then receive exactly the
   churn — each finished pod MODIFIED/Succeeded, each deleted pod DELETED, each
   new pod ADDED, once — and nothing for the unchanged pods.

Reported: the storm's wall time (410 → every scope re-synced and every
notification acknowledged), the watcher's CPU seconds over it, the longest
single relist slice on the loop thread (the "stall" one scope's relist can
cause), the event loop's worst scheduling lag (all scopes together), and the
exactly-once verdict. ``--json-out`` writes the line.
"""

from __future__ import annotations

import argparse
import asyncio
import glob
import json
import os
import shutil
import signal
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--namespaces", type=int, default=1000)
    ap.add_argument("--pods", type=int, default=100000, help="pods in the whole cluster")
    ap.add_argument("--scope", default="discover", choices=["discover", "cluster"])
    ap.add_argument("--churn", type=int, default=1000, help="pods finished, deleted and created while expired")
    ap.add_argument("--slice-ms", type=float, default=4.0, help="engine/reflector.py RELIST_SLICE_MS (loop time per relist slice)")
    ap.add_argument("--concurrency", type=int, default=16, help="watcher.relist_concurrency")
    ap.add_argument("--page", type=int, default=500, help="watcher.list_page_size")
    ap.add_argument("--decode-threads", default="auto")
    ap.add_argument("--initial-sync", default="list", choices=["list", "watch_list"],
                    help="watcher.initial_sync: LIST pages, or a WatchList stream (sendInitialEvents) — "
                         "both the initial sync and the post-410 resync")
    ap.add_argument("--sink-workers", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--fixture-placement", default="apart", choices=["apart", "any"],
                    help="apart: the fixtures run on other L3 domains than the watcher (off its loop core)")
    ap.add_argument("--slow-ms", type=float, default=10.0,
                    help="name the loop turns (and collector pauses) longer than this in loop_lag.slow_turns (0: off)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


def fixture_cpus(placement: str):
    """CPUs for the storm and sink fixtures: ``apart`` = the other L3 domains
    of this host (the watcher keeps the one it runs on, and its event-loop
    core is not shared with a fixture's busy process); ``any`` = unpinned."""
    if placement != "apart":
        return None
    from k8s_watcher_amd.utils.cpus import l3_domain_cpus, l3_domains
    doms = l3_domains()
    here = l3_domain_cpus()
    if len(doms) < 2 or not here:
        return None
    allowed = os.sched_getaffinity(0)
    rest = set().union(*(d for d in doms if d != frozenset(here))) & allowed
    return rest or None


async def spawn(*cmd, cpus=None):
    def pin():
        if cpus:
            os.sched_setaffinity(0, cpus)
    return await asyncio.create_subprocess_exec(*cmd, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
                                                stderr=asyncio.subprocess.DEVNULL, start_new_session=True, cwd=ROOT,
                                                preexec_fn=pin if cpus else None)


async def command(proc, line: str) -> dict:
    proc.stdin.write((line + "\n").encode())
    await proc.stdin.drain()
    out = (await proc.stdout.readline()).decode()
    assert out.startswith("OK "), out
    return json.loads(out[3:])


async def sink_keys(sinks, verify_dir: str, workers: int, sig=signal.SIGUSR1) -> dict:
    for f in glob.glob(os.path.join(verify_dir, "sink-*.json")):
        os.unlink(f)
    for s in sinks:
        os.killpg(s.pid, sig)
    deadline = time.monotonic() + 60
    files = []
    while time.monotonic() < deadline:
        files = glob.glob(os.path.join(verify_dir, "sink-*.json"))
        if len(files) >= workers:
            break
        await asyncio.sleep(0.05)
    keys: dict = {}
    for f in files:
        with open(f) as fh:
            for k, v in json.load(fh)["keys"].items():
                keys[k] = keys.get(k, 0) + v
    return keys


class LagMonitor:
    """Event-loop scheduling lag: a 1 ms timer, how late it fires. With
    ``slow_ms`` it also names the loop turns that took longer (the callback or
    task step that ran, where it stood) and the collector pauses, so a lag
    outlier has a cause in the JSON."""

    def __init__(self, slow_ms: float = 0.0) -> None:
        self.max_s = 0.0
        self.samples = []
        self._task = None
        self.slow_s = slow_ms / 1e3
        self.slow: list = []
        self._orig = None
        self._t0 = 0.0
        self._gc_t = 0.0

    async def _run(self) -> None:
        while True:
            t = time.perf_counter()
            await asyncio.sleep(0.001)
            lag = time.perf_counter() - t - 0.001
            self.samples.append(lag)
            if lag > self.max_s:
                self.max_s = lag

    @staticmethod
    def _name(handle) -> str:
        cb = handle._callback
        task = getattr(cb, "__self__", None)
        if isinstance(task, asyncio.Task):
            coro = task.get_coro()
            fr = getattr(coro, "cr_frame", None)
            where = f"{os.path.basename(fr.f_code.co_filename)}:{fr.f_lineno}" if fr else "done"
            return f"task {getattr(coro, '__qualname__', coro)} @ {where}"
        return getattr(cb, "__qualname__", repr(cb))[:80]

    def _gc_cb(self, phase: str, info: dict) -> None:
        if phase == "start":
            self._gc_t = time.perf_counter()
        else:
            dt = time.perf_counter() - self._gc_t
            if dt > self.slow_s:
                self.slow.append((dt, self._gc_t - self._t0, f"gc gen {info['generation']} "
                                                             f"(collected {info['collected']})", None))

    def _watch(self, loop_tid: int) -> None:
        # a thread that samples the loop thread's Python stack while a turn
        # runs long: it gets the GIL only if the loop released it (blocked in
        # C code or descheduled outside a GIL section), so a stack here says
        # which call the loop sat in; none says it held the GIL throughout
        import sys
        import traceback
        while not self._stop_watch:
            time.sleep(0.005)
            t = self._turn_t
            if t and time.perf_counter() - t > self.slow_s:
                fr = sys._current_frames().get(loop_tid)
                if fr is not None:
                    st = traceback.extract_stack(fr)[-6:]
                    key = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st))
                    self.stacks[key] = self.stacks.get(key, 0) + 1

    def start(self) -> None:
        self.max_s, self.samples, self.slow = 0.0, [], []
        self.stacks = {}
        self._turn_t = 0.0
        self._stop_watch = False
        self._t0 = time.perf_counter()
        if self.slow_s > 0:
            import asyncio.events as ev
            import gc
            orig = self._orig = ev.Handle._run
            mon = self

            thread_time = time.thread_time

            def _run(handle):
                c = thread_time()
                t = mon._turn_t = time.perf_counter()
                try:
                    return orig(handle)
                finally:
                    mon._turn_t = 0.0
                    dt = time.perf_counter() - t
                    if dt > mon.slow_s:  # with the loop thread's CPU time over it: work, or waiting
                        mon.slow.append((dt, t - mon._t0, mon._name(handle), thread_time() - c))

            ev.Handle._run = _run
            gc.callbacks.append(self._gc_cb)
            import threading
            self._watcher = threading.Thread(target=self._watch, args=(threading.get_ident(),), daemon=True)
            self._watcher.start()
        self._task = asyncio.ensure_future(self._run())

    def stop(self) -> dict:
        self._task.cancel()
        if self._orig is not None:
            import asyncio.events as ev
            import gc
            ev.Handle._run = self._orig
            self._orig = None
            gc.callbacks.remove(self._gc_cb)
            self._stop_watch = True
            self._watcher.join()
        s = sorted(self.samples) or [0.0]
        out = {"max_ms": round(self.max_s * 1e3, 2), "p99_ms": round(s[int(0.99 * (len(s) - 1))] * 1e3, 2),
               "p50_ms": round(s[len(s) // 2] * 1e3, 3), "samples": len(s)}
        if self.slow_s > 0:  # the longest turns, with when (s from the phase's start) and what ran
            out["slow_turns"] = [{"ms": round(dt * 1e3, 1), "cpu_ms": None if cpu is None else round(cpu * 1e3, 1),
                                  "at_s": round(at, 3), "what": what}
                                 for dt, at, what, cpu in sorted(self.slow, key=lambda x: -x[0])[:12]]
            # where the loop thread stood while a turn ran long (5 ms samples)
            out["slow_turn_stacks"] = [{"samples": n, "stack": k}
                                       for k, n in sorted(self.stacks.items(), key=lambda kv: -kv[1])[:8]]
        return out


async def wait_quiet(svc, c, relists_target: int, timeout: float) -> None:
    deadline = time.monotonic() + timeout
    while c["relists"] < relists_target or svc.notifier.outstanding() > 0:
        if time.monotonic() > deadline:
            raise TimeoutError(f"relists {c['relists']}/{relists_target}, outstanding {svc.notifier.outstanding()}")
        await asyncio.sleep(0.002)


async def main_async(args) -> dict:
    from k8s_watcher_amd.engine import reflector as _reflector
    from k8s_watcher_amd.engine.service import WatcherService
    _reflector.RELIST_SLICE_MS = args.slice_ms  # (a fixed choice since round 6: the A/B knob of this benchmark)
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.testing.stub_sink import _GEN  # noqa: F401  (same key format as payload_key)
    from k8s_watcher_amd.utils.config import load_settings
    from k8s_watcher_amd.utils.logsetup import setup_logging

    verify_dir = tempfile.mkdtemp(prefix="storm-verify-")
    out_dir = tempfile.mkdtemp(prefix="storm-out-")
    server = sinks = None
    try:
        t_fix = time.perf_counter()
        fx_cpus = fixture_cpus(args.fixture_placement)
        server = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.storm_server", "--namespaces",
                             str(args.namespaces), "--pods", str(args.pods), "--out-dir", out_dir, cpus=fx_cpus)
        line = (await asyncio.wait_for(server.stdout.readline(), 600)).decode()
        assert line.startswith("READY "), line
        info = json.loads(line[6:])
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            sink_port = s.getsockname()[1]
        sinks = [await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port", str(sink_port),
                             "--workers", str(args.sink_workers), "--engine", "native", "--verify-dir", verify_dir, cpus=fx_cpus)]
        await asyncio.wait_for(sinks[0].stdout.readline(), 60)
        await asyncio.sleep(0.3)
        fixture_s = time.perf_counter() - t_fix

        setup_logging("staging", "WARNING", log_file=os.path.join(out_dir, "watcher.log"))
        settings = load_settings("staging", overrides={
            "clusterapi": {"base_url": f"http://127.0.0.1:{sink_port}", "timeout": 30},
            "watcher": {"engine": "native", "log_level": "WARNING", "retry": {"max_attempts": 0, "delay_seconds": 0.05},
                        "namespace_scope": "discover" if args.scope == "discover" else "client",
                        "list_page_size": args.page,
                        "relist_concurrency": args.concurrency, "decode_threads": args.decode_threads,
                        "initial_sync": args.initial_sync}},
            environ={})
        metrics = Metrics()
        c = metrics.c
        svc = WatcherService(settings, endpoint=KubeEndpoint(server=f"http://127.0.0.1:{info['port']}"),
                             metrics=metrics, serve_metrics=False)
        lag = LagMonitor(args.slow_ms)

        # ---- initial sync: every pod ADDED once
        lag.start()
        cpu0, t0 = os.times(), time.perf_counter()
        await asyncio.wait_for(svc.start(), args.timeout)
        scopes = len(svc.reflectors)
        await wait_quiet(svc, c, scopes, args.timeout)
        initial_s = time.perf_counter() - t0
        cpu1 = os.times()
        initial_lag = lag.stop()
        initial_slices = [r.last_relist for r in svc.reflectors if r.last_relist]
        keys0 = await sink_keys(sinks, verify_dir, args.sink_workers, signal.SIGUSR2)  # dump and reset
        initial_ok = (len(keys0) == info["pods"] and all(v == 1 for v in keys0.values())
                      and all(k.split("|")[1] == "ADDED" for k in keys0))

        # ---- the storm
        churn = await command(server, f"CHURN {args.churn} 7")
        with open(churn["expected"]) as fh:
            expected = set(json.load(fh))
        relists_before = c["relists"]
        for r in svc.reflectors:
            r.last_relist = None
        lag.start()
        prof = None
        if os.environ.get("STORM_PROFILE"):  # cProfile of the storm phase only
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        cpu2, t2 = os.times(), time.perf_counter()
        expired = await command(server, "EXPIRE")
        await wait_quiet(svc, c, relists_before + scopes, args.timeout)
        storm_s = time.perf_counter() - t2
        if prof is not None:
            prof.disable()
            prof.dump_stats(os.environ["STORM_PROFILE"])
        cpu3 = os.times()
        storm_lag = lag.stop()
        storm = [r.last_relist for r in svc.reflectors if r.last_relist]
        keys = await sink_keys(sinks, verify_dir, args.sink_workers)
        stats = await command(server, "STATS")
        got = set(keys)
        dup = {k: v for k, v in keys.items() if v > 1}
        svc.stop()
        await svc.shutdown()

        def cpu(a, b):
            return round((b.user - a.user) + (b.system - a.system), 3)

        def slices(rs):
            return {"scopes": len(rs), "max_slice_ms": round(max((r["max_step_s"] for r in rs), default=0) * 1e3, 2),
                    "busy_s": round(sum(r["busy_s"] for r in rs), 3),
                    "listed": sum(r["listed"] for r in rs), "added": sum(r["added"] for r in rs),
                    "modified": sum(r["modified"] for r in rs), "unchanged": sum(r["unchanged"] for r in rs),
                    "deleted": sum(r["deleted"] for r in rs), "slices": sum(r["steps"] for r in rs),
                    "pages": sum(r["pages"] for r in rs)}

        return {
            "benchmark": "relist_storm",
            "config": {"namespaces": args.namespaces, "pods": info["pods"], "scope": args.scope, "scopes": scopes,
                       "churn": args.churn, "relist_slice_ms": args.slice_ms, "relist_concurrency": args.concurrency,
                       "list_page_size": args.page, "profile": "staging", "engine": "native",
                       "initial_sync": args.initial_sync,
                       "fixture_cpus": len(fx_cpus) if fx_cpus else "any"},
            "fixture_setup_s": round(fixture_s, 2),
            "initial": {"wall_s": round(initial_s, 3), "watcher_cpu_s": cpu(cpu0, cpu1), "loop_lag": initial_lag,
                        "relist": slices(initial_slices), "exactly_once": initial_ok, "notified": len(keys0)},
            "storm": {"expired_watches": expired["expired"], "wall_s": round(storm_s, 3),
                      "watcher_cpu_s": cpu(cpu2, cpu3), "loop_lag": storm_lag, "relist": slices(storm),
                      "expected": len(expected), "received_unique": len(got), "missing": len(expected - got),
                      "unexpected": len(got - expected), "duplicates": len(dup),
                      "exactly_once": got == expected and not dup},
            "server": stats,
        }
    finally:
        for p in [server] + (sinks or []):
            if p is None:
                continue
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
            try:
                await asyncio.wait_for(p.wait(), 10)
            except asyncio.TimeoutError:
                os.killpg(p.pid, signal.SIGKILL)
        shutil.rmtree(verify_dir, ignore_errors=True)
        shutil.rmtree(out_dir, ignore_errors=True)


def main(argv=None) -> int:
    args = parse_args(argv)
    # what the service does at start() in a deployment, where its process is
    # still single-threaded then; here asyncio's child watcher has started a
    # thread per fixture by the time the service starts (utils/fds.py)
    from k8s_watcher_amd.utils.fds import reserve_fd_table
    reserve_fd_table(16384)
    res = asyncio.run(main_async(args))
    line = json.dumps(res)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as fh:
            fh.write(line + "\n")
    return 0 if res["initial"]["exactly_once"] and res["storm"]["exactly_once"] else 1


if __name__ == "__main__":
    sys.exit(main())
