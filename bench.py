#!/usr/bin/env python3
"""Headline benchmark: sustained pod-events/s + p50 event→notify latency.

BASELINE.json metric: "pod-events/sec sustained + p50 event→notify latency
(single process, mock API)"; its throughput config is #4: ``production.yaml``,
all-namespaces watch, 10k-pod churn, async HTTP notifier pool. The reference
publishes no numbers, so the reference-equivalent pipeline
(``benchmarks/reference_equiv.py``) is measured on the same replay in the same
run and ``vs_baseline`` is the ratio to it.

Per rank (one watcher process per rank; ``torchrun`` ranks = independent
namespace shards, weak scaling):

* a replay API server child (``testing/replay_server.py``) streams one *step* =
  ``--pods-per-step`` pod lifecycles (ADDED → 3×MODIFIED → DELETED, ≈4 KB of
  real-shaped Pod JSON per event, one HTTP chunk per event);
* a stub clusterapi child (``testing/stub_sink.py``) acks every POST;
* this process runs the real :class:`WatcherService` (production profile:
  critical-events filter, namespace filter, notifier pool) and a step ends when
  every event of the step has been decoded, filtered and — if it survived the
  filters — POSTed and acknowledged (2xx) by the sink.

``W`` warmup steps run untimed, then exactly ``K`` steps are timed between
barriers; the slowest rank's time is used. Latency (socket read of the watch
chunk → 2xx from clusterapi) is measured afterwards at the config's nominal
rate (``--latency-rate``, default 100 ev/s as in config #4).

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]`` (one JSON line on
rank 0). There is no device work in this workload — see SURVEY.md §2.2 — so
there is nothing to ``torch.cuda.synchronize()``; the barrier (gloo, for N>1)
brackets the timed region.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "pod-events/sec sustained + p50 event→notify latency (single process, mock API)"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one watcher process each)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods-per-step", type=int, default=10000, help="pod lifecycles per step (5 events each)")
    ap.add_argument("--profile", default="production", choices=["development", "staging", "production"])
    ap.add_argument("--engine", default="native", choices=["native", "python"])
    ap.add_argument("--connections", type=int, default=None, help="notifier pool connections")
    ap.add_argument("--pipeline-depth", type=int, default=None)
    ap.add_argument("--decode-threads", default=None, help="watcher.decode_threads (int or auto)")
    ap.add_argument("--decode-affinity", default=None, choices=["auto", "none", "l3"])
    ap.add_argument("--watch-read-bytes", type=int, default=None, help="watcher.watch_read_bytes")
    ap.add_argument("--no-placement", dest="placement", action="store_false",
                    help="no per-rank L3 domain assignment (each watcher still pins per watcher.decode_affinity)")
    ap.add_argument("--python-pool", action="store_true", help="asyncio notifier pool instead of the C++ core")
    ap.add_argument("--io-thread", action="store_true",
                    help="serve the C++ notifier core's sockets on its own thread (clusterapi.pool.io_thread)")
    ap.add_argument("--tls", action="store_true",
                    help="https clusterapi (as production.yaml): the stub sink serves TLS with a throw-away CA")
    ap.add_argument("--sink-workers", type=int, default=4)
    ap.add_argument("--latency-rate", type=float, default=100.0)
    ap.add_argument("--latency-seconds", type=float, default=3.0)
    ap.add_argument("--ref-events", type=int, default=10000,
                    help="events for the reference-equivalent run (0 = skip, vs_baseline null)")
    ap.add_argument("--step-timeout", type=float, default=300.0)
    ap.add_argument("--json-out", default=None, help="also write the result line to this file")
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Dist:
    """gloo process group when launched by torchrun with WORLD_SIZE > 1."""

    def __init__(self) -> None:
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self) -> None:
        if self.world > 1:
            self.dist.barrier()

    def all_gather(self, obj) -> list:
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def reduce(self, value: float, op: str) -> float:
        if self.world == 1:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def close(self) -> None:
        if self.world > 1:
            self.dist.destroy_process_group()


async def spawn(*cmd: str):
    return await asyncio.create_subprocess_exec(
        *cmd, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
        stderr=asyncio.subprocess.DEVNULL, start_new_session=True, cwd=ROOT)


def cpu_ranges(cpus) -> "str | None":
    if not cpus:
        return None
    out, run = [], []
    for c in sorted(cpus):
        if run and c != run[-1] + 1:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
            run = []
        run.append(c)
    out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def placement(d: "Dist"):
    """L3 domain for this rank's watcher on a chiplet host (None elsewhere).

    Every rank keeps the domain it is already running on — its memory is
    local there; measured on the MI355X host, moving the watcher and its
    fixtures to other chiplets after start-up cost ~30% — unless a lower rank
    holds it, in which case it takes a free domain on the same socket.
    The replay and sink fixtures are not pinned."""
    from k8s_watcher_amd.utils.cpus import assign_domains, l3_domain_cpus, l3_domains
    doms = l3_domains()
    if len(doms) < 2:
        return None
    cur = l3_domain_cpus()
    here = next((i for i, x in enumerate(doms) if cur and x == frozenset(cur)), 0)
    wanted = d.all_gather(here)
    return set(doms[assign_domains(wanted, doms)[d.rank]])


async def rank_main(args, d: Dist) -> dict:
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.utils.config import load_settings
    from k8s_watcher_amd.utils.logsetup import setup_logging

    watcher_cpus = placement(d) if args.placement else None
    if watcher_cpus:
        os.sched_setaffinity(0, watcher_cpus)  # the decode workers inherit it
    replay = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.replay_server",
                         "--pods-per-step", str(args.pods_per_step), "--seed", str(d.rank),
                         "--prerender", str(args.warmup + args.steps))
    sink_port = free_port()
    tls_args, pki = [], None
    if args.tls:
        import tempfile
        from k8s_watcher_amd.testing.certs import make_pki
        pki = make_pki(tempfile.mkdtemp(prefix="bench-pki-"))
        tls_args = ["--tls-cert", pki.server_crt, "--tls-key", pki.server_key]
    scheme = "https" if args.tls else "http"
    sink = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port", str(sink_port),
                       "--workers", str(args.sink_workers), *tls_args)
    try:
        ready = (await asyncio.wait_for(replay.stdout.readline(), 600)).decode().split()
        assert ready and ready[0] == "READY", ready
        api_port, events_per_step = int(ready[1]), int(ready[2])
        await asyncio.wait_for(sink.stdout.readline(), 60)
        await asyncio.sleep(0.3)  # let every SO_REUSEPORT worker bind

        async def cmd(line: str) -> int:
            replay.stdin.write((line + "\n").encode())
            await replay.stdin.drain()
            reply = (await replay.stdout.readline()).decode().split()
            return int(reply[2])

        log_path = os.path.join("/tmp", f"k8s-watcher-bench-{os.getpid()}.log")
        setup_logging(args.profile, "WARNING" if args.profile == "production" else "INFO", log_file=log_path)
        overrides = {
            "clusterapi": {"base_url": f"{scheme}://127.0.0.1:{sink_port}", "timeout": 30,
                           **({"ca_file": pki.ca_crt} if pki else {}),
                           "enabled": not os.environ.get("BENCH_NO_NOTIFY")},
            "watcher": {"engine": args.engine, "retry": {"max_attempts": 0, "delay_seconds": 0.05},
                        **({"decode_threads": args.decode_threads} if args.decode_threads is not None else {}),
                        **({"watch_read_bytes": args.watch_read_bytes} if args.watch_read_bytes else {}),
                        # placement already pinned this thread (the decode workers inherit it)
                        **({"decode_affinity": args.decode_affinity or ("none" if watcher_cpus else "auto")})},
        }
        pool = {}
        if args.connections:
            pool["connections"] = args.connections
        if args.pipeline_depth:
            pool["pipeline_depth"] = args.pipeline_depth
        if args.python_pool:
            pool["native"] = False
        if args.io_thread:
            pool["io_thread"] = True
        if pool:
            overrides["clusterapi"]["pool"] = pool
        settings = load_settings(args.profile, overrides=overrides)
        if settings.watcher.log_level:
            setup_logging(args.profile, settings.watcher.log_level, log_file=log_path)
        metrics = Metrics(record_samples=True)
        svc = WatcherService(settings, endpoint=KubeEndpoint(server=f"http://127.0.0.1:{api_port}"),
                             metrics=metrics)
        await svc.start()
        for _ in range(200):
            if await cmd("WATCHERS 0") >= 1:
                break
            await asyncio.sleep(0.01)

        c = metrics.c
        native_pl = svc.pipeline.native if svc.pipeline is not None else None
        decode_threads = native_pl.decode_threads() if native_pl is not None else None

        debug = bool(os.environ.get("BENCH_DEBUG"))

        async def run_step(k: int, pace: str = "") -> None:
            base = c["events_received"]
            t_start = time.perf_counter()
            n = await cmd(f"PACE {k} {pace}" if pace else f"STEP {k}")
            t_sent = time.perf_counter()
            t_ingest = None
            deadline = time.monotonic() + args.step_timeout
            while c["events_received"] < base + n or svc.notifier.outstanding() > 0:
                if t_ingest is None and c["events_received"] >= base + n:
                    t_ingest = time.perf_counter()
                if time.monotonic() > deadline:
                    raise TimeoutError(f"step {k}: {c['events_received'] - base}/{n} events, "
                                       f"{svc.notifier.outstanding()} notifications outstanding")
                await asyncio.sleep(0.0005)
            if debug:
                t_end = time.perf_counter()
                print(f"step {k}: sent {t_sent - t_start:.3f}s ingest "
                      f"{(t_ingest or t_end) - t_start:.3f}s done {t_end - t_start:.3f}s", file=sys.stderr)

        for k in range(args.warmup):
            await run_step(k)
        metrics.latency.reset()
        d.barrier()
        n0, s0 = c["events_received"], c["notify_delivered"]
        cpu0 = cpu_snapshot(replay.pid, sink.pid)
        t0 = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            await run_step(k)
        elapsed = time.perf_counter() - t0
        cpu1 = cpu_snapshot(replay.pid, sink.pid)
        d.barrier()
        events = c["events_received"] - n0
        notified = c["notify_delivered"] - s0
        sat_p50 = metrics.latency.percentile_ns(50)

        # latency at the nominal rate (untimed)
        metrics.latency.reset()
        count = max(1, int(args.latency_rate * args.latency_seconds))
        await run_step(args.warmup + args.steps, f"{args.latency_rate} {count}")
        p50 = metrics.latency.percentile_ns(50)
        p99 = metrics.latency.percentile_ns(99)
        lat_n = metrics.latency.n
        failed = c["notify_failed"]
        svc.stop()
        await svc.shutdown()

        ref = None
        if args.ref_events > 0 and d.rank == 0:
            ref = await run_reference(args, api_port, f"{scheme}://127.0.0.1:{sink_port}", cmd,
                                      args.warmup + args.steps + 1, pki.ca_crt if pki else None)
        replay.stdin.write(b"QUIT\n")
        await replay.stdin.drain()
        return {"elapsed": elapsed, "events": events, "notified": notified, "events_per_step": events_per_step,
                "p50_ns": p50, "p99_ns": p99, "lat_samples": lat_n, "sat_p50_ns": sat_p50,
                "failed": failed, "ref": ref,
                "cpu_util": {k: round((cpu1[k] - cpu0[k]) / elapsed, 2) for k in cpu0
                             if not k.startswith("thread_") or k == "thread_loop"},
                "cpu_threads": sorted((round((cpu1[k] - cpu0[k]) / elapsed, 2) for k in cpu0
                                       if k.startswith("thread_") and k != "thread_loop" and k in cpu1),
                                      reverse=True)[:8],
                "decode_threads": decode_threads,
                "placement": {"watcher": cpu_ranges(watcher_cpus)}}
    finally:
        for p in (replay, sink):
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            try:
                await asyncio.wait_for(p.wait(), 5)
            except asyncio.TimeoutError:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
            transport = getattr(p, "_transport", None)
            if transport is not None:
                transport.close()  # close pipes while the loop is alive (no __del__ noise)


def cpu_snapshot(replay_pid: int, sink_pid: int) -> dict:
    """CPU seconds (user+system) of this watcher process and of the replay and
    sink process trees — which side saturates a core tells what bounds a run."""
    import psutil

    def tree(pid: int) -> float:
        try:
            root = psutil.Process(pid)
            procs = [root] + root.children(recursive=True)
        except psutil.NoSuchProcess:
            return 0.0
        tot = 0.0
        for pr in procs:
            try:
                t = pr.cpu_times()
                tot += t.user + t.system
            except psutil.NoSuchProcess:
                pass
        return tot

    t = os.times()
    out = {"watcher": t.user + t.system, "replay": tree(replay_pid), "sink": tree(sink_pid)}
    main = threading.get_native_id()
    for th in psutil.Process().threads():  # per thread: the event loop vs the decode workers
        out["thread_loop" if th.id == main else f"thread_{th.id}"] = th.user_time + th.system_time
    return out


async def run_reference(args, api_port: int, sink_url: str, cmd, step: int, ca_file=None) -> dict:
    from benchmarks.reference_equiv import RefEquivWatcher
    from k8s_watcher_amd.utils.config import load_settings

    s = load_settings(args.profile)
    ref = RefEquivWatcher(args.profile, s.watcher.namespaces, s.watcher.critical_events_only,
                          sink_url, ca_file=ca_file)
    loop = asyncio.get_running_loop()
    connected = loop.create_future()
    result = {}

    def work() -> None:
        result["elapsed"] = ref.run(f"http://127.0.0.1:{api_port}", args.ref_events,
                                    on_connected=lambda: loop.call_soon_threadsafe(connected.set_result, None))

    for _ in range(500):
        if await cmd("WATCHERS 0") == 0:
            break
        await asyncio.sleep(0.01)
    th = threading.Thread(target=work, daemon=True)
    th.start()
    await connected
    for _ in range(200):
        if await cmd("WATCHERS 0") >= 1:
            break
        await asyncio.sleep(0.01)
    await cmd(f"PACE {step} 0 {args.ref_events}")
    while th.is_alive():
        await asyncio.sleep(0.01)
    lat = sorted(ref.latencies_ns)
    p50 = lat[len(lat) // 2] if lat else None
    return {"events": ref.processed, "elapsed": result.get("elapsed"), "notified": ref.notified,
            "events_per_s": ref.processed / result["elapsed"] if result.get("elapsed") else None,
            "sat_p50_ns": p50}


def main(argv=None) -> int:
    args = parse_args(argv)
    d = Dist()
    res = asyncio.run(rank_main(args, d))
    elapsed = d.reduce(res["elapsed"], "MAX")
    events = d.reduce(float(res["events"]), "SUM")
    notified = d.reduce(float(res["notified"]), "SUM")
    p50 = d.reduce(res["p50_ns"] or 0.0, "MAX")
    p99 = d.reduce(res["p99_ns"] or 0.0, "MAX")
    d.close()
    if d.rank != 0:
        return 0
    value = events / elapsed
    ref = res["ref"]
    ref_rate = ref["events_per_s"] if ref else None
    per_rank = value / d.world
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "pod-events/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1000, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(per_rank / ref_rate, 2) if ref_rate else None,
        "dtype": "n/a",
        "data": "synthetic",
        "config": {
            "model": f"k8s-watcher {args.profile} profile (BASELINE config #4: all-namespaces watch, "
                     f"{args.pods_per_step}-pod churn, async notifier pool)",
            "global_batch": int(res["events_per_step"] * d.world),
            "seq_len": None,
            "parallelism": f"shard{d.world}" if d.world > 1 else "single-process",
            "engine": args.engine,
            "decode_threads": res["decode_threads"],
            "clusterapi": "https" if args.tls else "http",
        },
        "p50_latency_ms": round(p50 / 1e6, 3) if p50 else None,
        "p99_latency_ms": round(p99 / 1e6, 3) if p99 else None,
        "latency_rate_ev_s": args.latency_rate,
        "latency_samples": res["lat_samples"],
        "notified_per_s": round(notified / elapsed, 1),
        "notify_failed": res["failed"],
        "cpu_util_rank0": res["cpu_util"],
        "cpu_other_threads_rank0": res["cpu_threads"],
        # the watcher's own efficiency (the rate is bound by the replay fixture's core when it hits 1.0)
        "events_per_watcher_cpu_second": (round(res["events"] / (res["cpu_util"]["watcher"] * res["elapsed"]), 1)
                                          if res["cpu_util"].get("watcher") else None),
        "placement_rank0": res["placement"],
        "saturated_p50_latency_ms": round(res["sat_p50_ns"] / 1e6, 3) if res["sat_p50_ns"] else None,
        "reference_equiv": ({"events_per_s": round(ref_rate, 1), "events": ref["events"],
                             "notified": ref["notified"],
                             "saturated_p50_latency_ms": round(ref["sat_p50_ns"] / 1e6, 3)
                             if ref["sat_p50_ns"] else None} if ref else None),
        "baseline_source": "reference-equivalent pipeline measured in this run on the same replay "
                           "(BASELINE.md: reference publishes no numbers)",
    }
    line = json.dumps(out)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as fh:
            fh.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
