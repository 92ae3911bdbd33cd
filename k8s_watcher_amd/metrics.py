"""Counters, latency histogram and Prometheus exposition.

The reference has no metrics at all — only log lines. The watcher counts
every stage of the pipeline and records the event→notify latency (socket read
of the watch chunk → 2xx from clusterapi) in a log-bucketed histogram; when
``record_samples`` is on (benchmarks) the raw samples are kept too so exact
percentiles can be reported.

Exposition uses the Prometheus text format directly (no client library
needed); :func:`start_metrics_server` serves ``/metrics``, ``/healthz`` and
``/readyz`` on a small asyncio HTTP server.
"""

from __future__ import annotations

import array
import asyncio
import bisect
import math
import time
from typing import Callable, Dict, List, Optional

COUNTERS = (
    "events_received",      # decoded watch events (incl. list-synthesised)
    "events_filtered_critical",
    "events_filtered_namespace",
    "events_unchanged",     # dropped by notify_on=phase_change
    "events_invalid",
    "events_other_shard",
    "bookmarks",
    "notify_submitted",
    "notify_delivered",
    "notify_failed",
    "notify_retried",
    "notify_retry_after_waits",  # retries delayed to clusterapi's Retry-After
    "notify_superseded",
    "notify_coalesced",
    "notify_spooled",       # owed notifications written to the spool (parallel/spool.py)
    "spool_replayed",
    "spool_stale_skipped",
    "spool_dropped",
    "watch_restarts",
    "short_watches",        # watches the server ended at once with nothing in them (backed off)
    "auth_refreshes",       # 401 answers that made the watcher re-read its token / re-run the exec plugin
    "api_throttled",        # 429 answers from the API server (not counted against watcher.retry)
    "retry_after_waits",    # retries delayed to the API server's Retry-After
    "relists",
    "relist_items",         # pods in the LISTs of relists
    "relist_unchanged",     # ... whose resourceVersion matched the cache (nothing sent)
    "relist_deleted",       # cached pods a relist no longer found: notified DELETED from the cache
    "watches_hub_dispatch",  # watches the reader hub fed to the native pipeline directly (hub_dispatch)
    "list_continue_expired",  # paginated LISTs whose continue token expired (redone unpaginated)
    "watch_list_syncs",     # initial state via WatchList (sendInitialEvents) instead of LIST
    "expired_410",
    "expired_relist_backoffs",  # 410s right after a relist (no progress): the next relist waited
    "checkpoints_written",
    "malloc_trims",         # times the C heap's free pages were handed back (watcher.malloc_trim_seconds)
    "malloc_trims_skipped",  # ... periods with less free heap than watcher.malloc_trim_min_free_mb (no trim)
    "malloc_trims_deferred",  # ... periods without a quiet half second (trimmed later; at the latest every 10th)
    "malloc_trim_us",       # time spent in those trims (every arena locked meanwhile), microseconds
    "checkpoint_owed_resent",  # owed notifications a format-2 checkpoint re-submitted on start
    "namespace_changes",    # namespace set changes seen by watcher.namespace_scope: discover
    "scopes_started",       # per-namespace pod watches opened after start-up (new or handed-over namespaces)
    "scopes_stopped",       # ... and closed (namespace deleted or now owned by another shard)
    "shard_handovers_out",  # namespaces handed to another shard with their cached pods (shard.handover_dir)
    "shard_handover_pods_out",
    "shard_handovers_in",   # ... taken over from another shard's record
    "shard_handover_pods_in",
    "shard_handover_timeouts",  # a moved namespace's record never came (its pods re-announced)
    "shard_handover_errors",    # a record could not be written
    "shard_handover_owed_late",  # notifications still owed for a namespace when its record went out anyway
    "notify_io_switches",   # clusterapi.pool.io_thread: auto — sockets handed between loop and I/O thread
    "namespace_deleted_synthesized",  # pods of a deleted namespace notified DELETED from the cache (no event came)
    "leader_acquired",      # leadership terms started (engine/leader.py)
    "leader_lost",
    "lease_update_conflicts",
    "lease_update_errors",
)

# 1 µs .. ~100 s, 4 buckets per decade (upper bounds in ns)
_BUCKETS_NS = [int(10 ** (3 + i / 4)) for i in range(0, 33)]


class LatencyHistogram:
    """Log-bucketed histogram. Besides direct observations it can pull from
    *sources* — callables returning cumulative ``(counts, total_ns, n)`` kept
    elsewhere (the native notifier core buckets in C++) — merged lazily when the
    histogram is read, so the hot path does no per-notification Python work."""

    def __init__(self, record_samples: bool = False) -> None:
        self._counts = [0] * (len(_BUCKETS_NS) + 1)
        self._total_ns = 0
        self._n = 0
        self.samples: Optional[array.array] = array.array("q") if record_samples else None
        self._sources: List[list] = []  # [fn, last counts, last total, last n]

    def add_source(self, fn: Callable[[], tuple]) -> None:
        counts, total, n = fn()
        self._sources.append([fn, list(counts), total, n])  # start from the current totals

    def sync(self) -> None:
        for src in self._sources:
            counts, total, n = src[0]()
            if n == src[3]:
                continue
            c, last = self._counts, src[1]
            for i, v in enumerate(counts):
                if v != last[i]:
                    c[i] += v - last[i]
            self._total_ns += total - src[2]
            self._n += n - src[3]
            src[1], src[2], src[3] = list(counts), total, n

    @property
    def counts(self) -> List[int]:
        self.sync()
        return self._counts

    @property
    def total_ns(self) -> int:
        self.sync()
        return self._total_ns

    @property
    def n(self) -> int:
        self.sync()
        return self._n

    def observe_ns(self, ns: int) -> None:
        self._counts[bisect.bisect_left(_BUCKETS_NS, ns)] += 1
        self._total_ns += ns
        self._n += 1
        if self.samples is not None:
            self.samples.append(ns)

    def observe_many(self, values: "array.array") -> None:
        """Bulk observe (int64 nanoseconds), e.g. latencies reported by the native notifier."""
        counts = self._counts
        bl = bisect.bisect_left
        for ns in values:
            counts[bl(_BUCKETS_NS, ns)] += 1
        self._total_ns += sum(values)
        self._n += len(values)
        if self.samples is not None:
            self.samples.extend(values)

    def add_samples(self, values: "array.array") -> None:
        if self.samples is not None:
            self.samples.extend(values)

    def reset(self) -> None:
        self.sync()  # sources restart from their current totals
        self._counts = [0] * (len(_BUCKETS_NS) + 1)
        self._total_ns = 0
        self._n = 0
        if self.samples is not None:
            self.samples = array.array("q")

    def percentile_ns(self, q: float) -> Optional[float]:
        """Exact when samples are recorded, otherwise bucket upper bound."""
        n = self.n  # syncs
        if n == 0:
            return None
        if self.samples is not None and len(self.samples):
            s = sorted(self.samples)
            k = max(0, min(len(s) - 1, int(math.ceil(q / 100.0 * len(s))) - 1))
            return float(s[k])
        target = q / 100.0 * n
        acc = 0
        for i, c in enumerate(self._counts):
            acc += c
            if acc >= target:
                return float(_BUCKETS_NS[i] if i < len(_BUCKETS_NS) else _BUCKETS_NS[-1])
        return float(_BUCKETS_NS[-1])


class Metrics:
    def __init__(self, record_samples: bool = False) -> None:
        self.c: Dict[str, int] = {k: 0 for k in COUNTERS}
        self.latency = LatencyHistogram(record_samples)  # socket read of the event -> 2xx from clusterapi
        self.rtt = LatencyHistogram()  # request on the wire -> 2xx (clusterapi + network share)
        self.record_samples = record_samples
        self.started = time.time()
        self.ready = False
        self.gauges: Dict[str, Callable[[], float]] = {}

    def inc(self, name: str, n: int = 1) -> None:
        self.c[name] = self.c.get(name, 0) + n

    def snapshot(self) -> Dict[str, float]:
        out: Dict[str, float] = dict(self.c)
        for k, fn in self.gauges.items():
            out[k] = fn()
        p50 = self.latency.percentile_ns(50)
        p99 = self.latency.percentile_ns(99)
        out["notify_latency_p50_ms"] = p50 / 1e6 if p50 is not None else float("nan")
        out["notify_latency_p99_ms"] = p99 / 1e6 if p99 is not None else float("nan")
        return out

    def prometheus_text(self) -> str:
        lines: List[str] = []
        for k, v in self.c.items():
            name = f"k8s_watcher_{k}_total"
            lines.append(f"# TYPE {name} counter")
            lines.append(f"{name} {v}")
        for k, fn in self.gauges.items():
            name = f"k8s_watcher_{k}"
            lines.append(f"# TYPE {name} gauge")
            lines.append(f"{name} {fn()}")
        for name, h in (("k8s_watcher_notify_latency_seconds", self.latency),
                        ("k8s_watcher_notify_rtt_seconds", self.rtt)):
            lines.append(f"# TYPE {name} histogram")
            acc = 0
            for ub, c in zip(_BUCKETS_NS, h.counts):
                acc += c
                lines.append(f'{name}_bucket{{le="{ub / 1e9:.9g}"}} {acc}')
            lines.append(f'{name}_bucket{{le="+Inf"}} {h.n}')
            lines.append(f"{name}_sum {h.total_ns / 1e9:.9f}")
            lines.append(f"{name}_count {h.n}")
        return "\n".join(lines) + "\n"


def memory_census(top: int = 40) -> Dict[str, object]:
    """``/debug/memory`` (``metrics.debug``): what the interpreter holds —
    live objects per type (the collector's view; the most numerous ``top``),
    the allocator's block count, and with ``tracemalloc`` running
    (``PYTHONTRACEMALLOC=1``) the ``top`` allocation sites by size. A soak
    diffs two of these, an hour apart, to name what grows outside the C heap."""
    import gc
    import sys
    import tracemalloc
    # live objects only: without a collection first the counts include cyclic
    # garbage the collector has not reached yet (a closed connection's
    # transport <-> protocol cycle waits for a gen-2 pass: 23 "extra"
    # transports in a soak's census diff were exactly that)
    # (watcher.gc_freeze) frozen objects are invisible to get_objects() and
    # never collected: thaw them for the count, report how many there were and
    # how much of them had become garbage (the freeze's one-time cost), and
    # freeze what is still live again
    frozen = gc.get_freeze_count()
    if frozen:
        gc.unfreeze()
    collected = gc.collect()
    counts: Dict[str, int] = {}
    for o in gc.get_objects():
        t = type(o)
        k = f"{t.__module__}.{t.__qualname__}"
        counts[k] = counts.get(k, 0) + 1
    if frozen:
        gc.freeze()
    out: Dict[str, object] = {
        "gc_objects": sum(counts.values()), "garbage_collected": collected, "frozen_before": frozen,
        "allocated_blocks": sys.getallocatedblocks(),
        "types": dict(sorted(counts.items(), key=lambda kv: -kv[1])[:top]), "gc_counts": list(gc.get_count())}
    try:  # the C heap per glibc arena (0: main, the loop's): where retained free bytes sit
        from .ops.native import load as _load_native
        out["malloc_arenas"] = [{"arena": a, "free_bytes": f, "system_bytes": sz}
                                for a, f, sz in _load_native().malloc_arenas()]
    except Exception:  # noqa: BLE001 - no native extension (python engine): not part of the census
        pass
    if tracemalloc.is_tracing():
        snap = tracemalloc.take_snapshot().filter_traces(
            [tracemalloc.Filter(False, tracemalloc.__file__)])
        stats = snap.statistics("lineno")
        out["tracemalloc"] = {
            "traced_bytes": tracemalloc.get_traced_memory()[0],
            "top": [{"site": f"{s.traceback[0].filename}:{s.traceback[0].lineno}", "bytes": s.size,
                     "blocks": s.count} for s in stats[:top]]}
    return out


async def start_metrics_server(metrics: Metrics, host: str, port: int, debug: bool = False) -> asyncio.AbstractServer:
    """Tiny HTTP/1.1 server: ``/metrics``, ``/healthz``, ``/readyz`` (one request per connection);
    with ``debug`` also ``/debug/memory`` (:func:`memory_census`, JSON)."""

    async def handle(reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            line = await asyncio.wait_for(reader.readline(), 10)
            while True:
                h = await asyncio.wait_for(reader.readline(), 10)
                if h in (b"\r\n", b"\n", b""):
                    break
            parts = line.decode("latin-1").split()
            path = parts[1] if len(parts) > 1 else "/"
            if path.startswith("/metrics"):
                status, body, ctype = "200 OK", metrics.prometheus_text(), "text/plain; version=0.0.4"
            elif path.startswith("/healthz"):
                status, body, ctype = "200 OK", "ok\n", "text/plain"
            elif path.startswith("/readyz"):
                status = "200 OK" if metrics.ready else "503 Service Unavailable"
                body, ctype = ("ready\n" if metrics.ready else "not ready\n"), "text/plain"
            elif debug and path.startswith("/debug/memory"):
                import json
                status, body, ctype = "200 OK", json.dumps(memory_census()), "application/json"
            else:
                status, body, ctype = "404 Not Found", "not found\n", "text/plain"
            data = body.encode()
            writer.write(f"HTTP/1.1 {status}\r\nContent-Type: {ctype}\r\nContent-Length: {len(data)}\r\n"
                         f"Connection: close\r\n\r\n".encode() + data)
            await writer.drain()
        except (asyncio.TimeoutError, ConnectionError):
            pass
        finally:
            writer.close()

    return await asyncio.start_server(handle, host, port)
