"""Watcher service orchestrator (SURVEY C6 + C7, layer L4).

Reference: ``PodWatcher.setup_k8s_client`` + ``start_watching``
(``/root/reference/watcher/pod_watcher.py:110-157,243-277``). The same log
messages (§2.4) are emitted in the same order; the behavioural fixes are:

* the connectivity probe is ``GET /version`` (``CoreV1Api.get_api_version``
  at ``:140`` does not exist and makes the reference fail setup);
* the namespace sample is bounded (``limit=5``) instead of listing them all;
* setup failure is an error the CLI turns into exit status 1 (the reference
  returns and exits 0, ``:245-247``);
* the clusterapi notifier is enabled and health-checked (``:14,236,250-253``
  are commented out in the reference);
* SIGTERM and SIGINT both stop the watch, drain the notifier and write a
  final checkpoint.

With ``watcher.namespace_scope: server`` one reflector per target namespace
watches ``/api/v1/namespaces/<ns>/pods``, so the API server only sends the
pods the watcher cares about (the reference always watches the whole cluster
and filters client-side). With ``namespace_scope: discover`` the
namespace set itself is watched (``engine/namespaces.py``) and one reflector
runs per namespace this shard owns — the sharded form of the reference's
all-namespaces watch: reflectors start and stop as namespaces come and go.
"""

from __future__ import annotations

import asyncio
import gc
import logging
import os
import time
from typing import Dict, List, Optional, Set

from ..kube.api import ApiError, KubeApi
from ..kube.kubeconfig import ConfigException, KubeEndpoint, load_incluster_config, load_kube_config
from ..metrics import Metrics, start_metrics_server
from ..net.http import HttpError
from ..ops.cache import CORE, NAME, NS, PHASE, RV, make_pod_cache
from ..ops.decode import make_decoder
from ..parallel.native_notifier import NativeNotifierPool
from ..parallel.notifier import NotifierPool, NullNotifier
from ..parallel.shard import ShardFilter, layout_of, owner_of, record_layout, take_handover, write_handover
from ..parallel.spool import Spool, SpoolReplayer
from ..utils.config import Settings
from ..utils.fastlog import EventLog
from ..utils.logsetup import SERVICE_LOGGER
from .checkpoint import load_checkpoint, native_snapshot, save_checkpoint, write_native
from .namespaces import NamespaceWatcher
from .pipeline import EventPipeline
from .reflector import Reflector, WatchFailed


# Fixed choices that were settings until round 6 (each one's A/B is in
# BENCHMARKS.md; tests monkeypatch these module attributes):
# the descriptor table grown once at start to hold this many fds (a watch per
# namespace opens two each; growing it later, with threads running, waits an
# RCU grace period per doubling: utils/fds.py)
FD_TABLE_RESERVE = 16384
# once every scope has synced, collect and freeze what start-up left
# (gc.freeze): later full collections walk only objects made since, not the
# service's long-lived ones (a 1,000-scope relist storm's gen-2 pauses);
# unfrozen at shutdown. Start-up objects that later become cyclic garbage stay
# until shutdown. Skipped when something is already frozen (an embedding
# application's own freeze)
GC_FREEZE = True
# the reader hub's thread de-chunks and splits watch bodies (readerhub.inc
# HubFramer): auto = with several watch scopes (namespace watches: the reader
# has time, the loop has per-stream work), not for the one cluster-wide
# watch, whose reader thread is the bound (profiles/r5/framing_ab,
# r5/framing_many); on | off for tests
HUB_FRAMING = "auto"
# reader-hub threads (net/reader.py; readerhub.inc set_readers): 0 = auto
# (utils/cpus.py auto_reader_threads: two for several watch scopes on a CPU
# share of 12+, else one)
HUB_READERS = 0
# read-ahead over all streams when there are several watch scopes and
# watcher.watch_reader_max_bytes is 0: with the whole pool (256 MiB) the
# namespace watches' buffers waited 13-28 ms for the loop and were out of the
# L3 by then, and the pool ran short (starved streams); 8 MiB keeps them young.
# 64 namespaces, interleaved on the box: 2.45-2.54M (one reader, the pool),
# 2.59-2.94M (one reader, 8 MiB), 3.05-3.13M (two readers, 8 MiB)
# (profiles/r6/readers/final). One cluster-wide watch keeps the pool: its two
# buffers of 4 MiB are its read-ahead anyway.
HUB_MULTI_READ_AHEAD = 8 << 20
MALLOC_TRIM_MIN_FREE = 16 << 20  # a periodic malloc_trim runs only when the C heap keeps this much free
SPOOL_REPLAY_BATCH = 1000  # owed notifications re-submitted from the spool per replay pass


class SetupError(Exception):
    """The Kubernetes client could not be set up (reference ``:246``)."""


def required_permissions(s: Settings) -> List[tuple]:
    """``(verb, resource, api group, namespace or None, name or None)`` this
    configuration needs — what ``--check`` asks the API server about and what
    ``deploy/k8s/rbac.yaml`` must grant (``tests/test_deploy.py`` holds them equal).

    The reference needs list/watch on pods cluster-wide and list on namespaces
    (``pod_watcher.py:146,264``); server-side scopes need them per namespace,
    namespace discovery also watches namespaces, leader election its Lease."""
    w = s.watcher
    wanted = []
    scopes = w.namespaces if w.namespace_scope == "server" and w.namespaces else [None]
    for ns in scopes:
        wanted += [("list", "pods", "", ns, None), ("watch", "pods", "", ns, None)]
    wanted.append(("list", "namespaces", "", None, None))
    if w.namespace_scope == "discover":
        wanted.append(("watch", "namespaces", "", None, None))
    le = w.leader_election
    if le.enabled:
        from .leader import default_lease_namespace, shard_lease
        lease = shard_lease(s)
        ns = lease.lease_namespace or default_lease_namespace()
        wanted += [("get", "leases", "coordination.k8s.io", ns, lease.lease_name),
                   ("update", "leases", "coordination.k8s.io", ns, lease.lease_name),
                   ("create", "leases", "coordination.k8s.io", ns, None)]
    return wanted


class WatcherService:
    def __init__(self, settings: Settings, endpoint: Optional[KubeEndpoint] = None,
                 metrics: Optional[Metrics] = None, notifier_factory=None, serve_metrics: bool = True) -> None:
        self.settings = settings
        self.serve_metrics = serve_metrics  # False when an outer runner owns the metrics server
        self.endpoint = endpoint
        self.metrics = metrics or Metrics()
        self.notifier_factory = notifier_factory
        self.log = logging.getLogger(SERVICE_LOGGER)
        self.api: Optional[KubeApi] = None
        self.notifier = None
        self.pipeline: Optional[EventPipeline] = None
        self._decode_pool = None
        self._gc_frozen = False
        self._reader_hub = None
        self.thread_placement = None
        self._loop_affinity = None
        self.reflectors: List[Reflector] = []
        self.decoder = None
        self._stop = asyncio.Event()
        self._tasks: List[asyncio.Task] = []
        self._metrics_server = None
        self.started = asyncio.Event()
        self.server_version: Optional[str] = None
        self.spool = None
        self.spool_replayer = None
        self.ns_watcher: Optional[NamespaceWatcher] = None
        self._scope_tasks: Dict[str, asyncio.Task] = {}
        # namespaces gained from another shard, waiting for its hand-over record
        # before their watch starts (watcher.shard.handover_dir)
        self._gaining: Dict[str, asyncio.Task] = {}
        # namespaces handed to another shard whose record waits for this shard's
        # owed notifications of them to be acknowledged (_handover_out)
        self._handing: Dict[str, asyncio.Task] = {}
        self._layout_since = 0.0  # when the shard layout in handover_dir's history began (record_layout)
        self._ns_seen: Set[str] = set()  # the namespace set the last ownership decision used
        self._retiring: Dict[str, asyncio.TimerHandle] = {}  # deleted namespaces draining their pod watch
        self._failure: Optional[asyncio.Future] = None
        self._saved_rvs: Dict[str, Optional[str]] = {}
        self._multi = False  # several (or dynamic) watch scopes, each with its own pipeline
        self.last_checkpoint: Optional[dict] = None
        self._live = False  # scopes follow namespace changes once start() has built the first set
        self._list_gate: Optional[asyncio.Semaphore] = None  # watcher.relist_concurrency
        self._ck_lock = asyncio.Lock()  # one checkpoint snapshot+write at a time, in cut order
        self._ck_inflight: Optional[asyncio.Future] = None  # a format-2 write on its executor thread

    # ------------------------------------------------------------------ setup
    def load_endpoint(self) -> KubeEndpoint:
        k = self.settings.kubernetes
        if self.endpoint is not None:
            return self.endpoint
        if k.use_incluster_config:
            self.log.info("Using in-cluster configuration")
            return load_incluster_config()
        if k.config_file:
            self.log.info(f"Loading kubeconfig from: {k.config_file}")
            if not os.path.exists(k.config_file):
                self.log.error(f"Kubeconfig file not found: {k.config_file}")
                raise SetupError(f"kubeconfig not found: {k.config_file}")
            return load_kube_config(config_file=k.config_file, context=k.context)
        self.log.info("Using default kubeconfig")
        return load_kube_config(context=k.context)

    async def setup_k8s_client(self) -> bool:
        """Reference-compatible setup: returns False (after logging) on failure."""
        try:
            ep = self.load_endpoint()
            self.endpoint = ep
            self.api = KubeApi(ep, timeout=self.settings.kubernetes.request_timeout,
                               compression=self.settings.kubernetes.compression,
                               keepalive=self.settings.kubernetes.tcp_keepalive_seconds)
            ver = await self.api.get_version()
            self.server_version = ver.get("gitVersion") or f"{ver.get('major')}.{ver.get('minor')}"
            self.log.info(f"Successfully connected to Kubernetes API version: {self.server_version}")
            try:
                nss = await self.api.list_namespaces(limit=5)
                names = [(i.get("metadata") or {}).get("name") for i in (nss.get("items") or [])[:5]]
                self.log.info(f"Sample namespaces: {names}")
            except ApiError as exc:
                # RBAC may not grant namespace list; the watch itself only needs pods.
                self.log.warning(f"Could not list namespaces: {exc}")
            return True
        except ConfigException as exc:
            self.log.error(f"Kubernetes config error: {exc}")
        except SetupError:
            pass
        except (ApiError, HttpError, OSError, ValueError) as exc:
            self.log.error(f"Error setting up k8s client: {exc}")
        if self.api is not None:
            await self.api.close()
            self.api = None
        return False

    async def preflight(self) -> bool:
        """``--check``: the RBAC permissions this configuration needs (SelfSubjectAccessReview)
        and the clusterapi health endpoint. Logs one line per item; True if all pass."""
        assert self.api is not None
        s = self.settings
        wanted = required_permissions(s)
        ok = True
        for verb, res, group, ns, name in wanted:
            what = f"{verb} {group + '/' if group else ''}{res}" + (f" in {ns}" if ns else " (cluster-wide)")
            try:
                allowed, reason = await self.api.can_i(verb, res, group, ns, name)
            except (ApiError, HttpError) as exc:
                self.log.warning(f"Permission check for {what} unavailable: {exc}")
                continue
            if allowed:
                self.log.info(f"Permission OK: {what}")
            else:
                ok = False
                self.log.error(f"Permission missing: {what}" + (f" ({reason})" if reason else ""))
        if s.clusterapi.enabled:
            self.event_log = EventLog(self.log)
            notifier = self._make_notifier()
            try:
                if await notifier.health_check():
                    self.log.info(f"ClusterAPI health check passed: {s.clusterapi.base_url}{s.clusterapi.health}")
                else:
                    ok = False
                    self.log.error(f"ClusterAPI health check failed: {s.clusterapi.base_url}{s.clusterapi.health}")
            finally:
                await notifier.close()
        return ok

    def _make_notifier(self):
        c = self.settings.clusterapi
        w = self.settings.watcher
        if self.notifier_factory is not None:
            return self.notifier_factory(self)
        if not c.enabled:
            return NullNotifier(self.metrics)
        log_events = w.log_events if w.log_events is not None else self.log.isEnabledFor(logging.INFO)
        if w.engine == "native" and c.pool.native:
            # per-request work in C++ (ops/csrc/engine.inc), TLS included
            return NativeNotifierPool(c, self.metrics, ts_mode=w.event_timestamp, log_events=log_events,
                                      on_saturation=self._on_saturation, event_log=self.event_log)
        return NotifierPool(c, self.metrics, ts_mode=w.event_timestamp, log_events=log_events,
                            on_saturation=self._on_saturation, native=w.engine == "native",
                            event_log=self.event_log)

    def _on_saturation(self, saturated: bool) -> None:
        for r in self.reflectors:
            r.set_paused(saturated)

    # ------------------------------------------------------------------ run
    async def start(self) -> None:
        """Setup + start background tasks; returns once every scope has synced."""
        s = self.settings
        # before the decode pool, reader and I/O threads exist: growing a
        # shared descriptor table later stalls the opening thread ~150 ms
        # per doubling on a 256-CPU host (utils/fds.py)
        from ..utils.fds import reserve_fd_table
        reserve_fd_table(FD_TABLE_RESERVE)
        if self._native_pipeline() and s.watcher.malloc_trim_seconds > 0:
            # fixed glibc thresholds before the cache and the buffers exist:
            # blocks >= 512 KiB on their own mappings (unmapped when freed),
            # so multi-MiB transients leave no holes in the arenas (round-5
            # soak: RSS grew with retained free bytes; kwcore.cpp malloc_tune)
            from ..ops.native import load as _load_kw
            _load_kw().malloc_tune(512 << 10, 4 << 20)
        if GC_FREEZE and gc.get_freeze_count() == 0:
            # what import and configuration made is permanent: the full
            # collections that starting a thousand scopes triggers then walk
            # only the scopes' own objects (70-140 ms gen-2 pauses otherwise).
            # Only when nothing is frozen yet: an embedding application that
            # froze its own objects keeps control of the permanent generation
            # (shutdown's unfreeze would thaw its objects too)
            gc.freeze()
            self._gc_frozen = True
        if not await self.setup_k8s_client():
            self.log.error("Failed to setup Kubernetes client")
            raise SetupError("Failed to setup Kubernetes client")
        assert self.api is not None
        self.event_log = EventLog(self.log)  # after logging is configured: picks the fast path
        self.notifier = self._make_notifier()
        if s.clusterapi.enabled and s.clusterapi.health_check_on_start:
            if await self.notifier.health_check():
                self.log.info("ClusterAPI health check passed")
            else:
                self.log.warning("ClusterAPI health check failed, but continuing...")
        if s.clusterapi.enabled and hasattr(self.notifier, "warm_up"):
            await self.notifier.warm_up()
        sp = s.clusterapi.spool
        if s.clusterapi.enabled and sp.path and hasattr(self.notifier, "attach_spool"):
            self.spool = Spool(sp.path, sp.max_bytes, sp.segment_bytes, sp.fsync, self.metrics)
            self.notifier.attach_spool(self.spool)
            self.metrics.gauges["spool_records"] = lambda: float(len(self.spool))
            self.metrics.gauges["spool_bytes"] = lambda: float(self.spool.bytes)
            if len(self.spool):
                self.log.warning(f"Spool {sp.path} holds {len(self.spool)} notifications from an earlier run")
            self.spool_replayer = SpoolReplayer(self.spool, self.notifier, self.metrics,
                                                sp.replay_interval_seconds, SPOOL_REPLAY_BATCH)
            self._tasks.append(asyncio.ensure_future(self.spool_replayer.run()))
        self.decoder = make_decoder(s.watcher.engine, s.environment, s.watcher.state_format,
                                    s.watcher.payload_extra, s.watcher.validate)
        self._failure = asyncio.get_running_loop().create_future()
        scope_mode = s.watcher.namespace_scope
        if scope_mode == "discover":
            self.ns_watcher = NamespaceWatcher(self.api, s, self.metrics, self._on_namespaces)
            ns_task = asyncio.ensure_future(self.ns_watcher.run())
            self._tasks.append(ns_task)
            synced = asyncio.ensure_future(self.ns_watcher.synced.wait())
            await asyncio.wait([synced, ns_task], return_when=asyncio.FIRST_COMPLETED)
            if not synced.done():
                synced.cancel()
                if ns_task.exception() is not None:
                    raise ns_task.exception()  # type: ignore[misc]
                raise SetupError("namespace watch ended before the initial list")
            self._ns_seen = set(self.ns_watcher.names)
            scopes: List[Optional[str]] = list(self._owned(self._ns_seen))
        elif scope_mode == "server" and s.watcher.namespaces:
            scopes = list(ShardFilter(s.watcher.shard).namespaces(s.watcher.namespaces))
        else:
            scopes = [None]
        self._multi = scope_mode == "discover" or len(scopes) > 1
        if s.watcher.shard.count > 1:
            self.log.info(f"Shard {s.watcher.shard.index}/{s.watcher.shard.count} "
                          f"(key={s.watcher.shard.key}); watch scopes: {[x or '*' for x in scopes]}")
        cache = make_pod_cache(self._native_pipeline())
        saved_rvs = {}
        owed: list = []
        ck = s.watcher.checkpoint.path
        if ck:
            loaded = load_checkpoint(ck, native_cache=self._native_pipeline())
            if loaded is not None:
                saved_rvs, cache, _, owed = loaded
                self.log.info(f"Resuming from checkpoint {ck}: {len(cache)} cached pods"
                              + (f", {len(owed)} owed notifications" if owed else ""))
        self._saved_rvs = saved_rvs
        self.pipeline = EventPipeline(s, self.decoder, self.notifier, self.metrics, cache, self.event_log,
                                      event_sharding=self._event_sharding())
        if self._native_pipeline():
            from ..ops.native import load as _load_native
            _kw = _load_native()
            _kw.set_partitioned_apply(True)
            # which apply path ran, and how much of it (cumulative, process-wide)
            for _key in ("partitioned_batches", "partitioned_lines", "tail_serial_lines", "tail_submits",
                         "tail_lock_runs", "serial_batches", "serial_lines"):
                self.metrics.gauges["apply_" + _key] = (lambda k=_key: float(_kw.apply_stats()[k]))
            self._decode_pool = self._make_decode_pool()
            self.pipeline.attach_native(self._decode_pool)
            http = self.api.http
            if s.watcher.watch_reader == "native" and (http.ssl_context is None
                                                       or getattr(http.ssl_context, "kw_tls", None) is not None):
                # watch bodies read (and, for https, decrypted) on a native thread (net/reader.py)
                from ..net.reader import WatchReaderHub
                from ..utils.cpus import auto_reader_threads, auto_tls_threads
                self._reader_hub = WatchReaderHub(s.watcher.watch_read_bytes or (4 << 20),
                                                  s.watcher.watch_reader_buffers,
                                                  max_bytes=(s.watcher.watch_reader_max_bytes or
                                                             (HUB_MULTI_READ_AHEAD if self._multi else 0)),
                                                  frame=(HUB_FRAMING == "on" or
                                                         (HUB_FRAMING == "auto" and self._multi)),
                                                  readers=HUB_READERS or auto_reader_threads(self._multi),
                                                  tls_records=s.watcher.watch_tls_records == "native",
                                                  tls_threads=(s.watcher.watch_tls_threads
                                                               if s.watcher.watch_tls_threads >= 0
                                                               else auto_tls_threads()))
                self.api.http.reader_hub = self._reader_hub
                hub = self._reader_hub
                self.metrics.gauges["watch_reader_streams"] = lambda: float(len(hub.protos))
                self.metrics.gauges["watch_reader_reads"] = lambda: float(hub.stats().get("reads", 0))
                self.metrics.gauges["watch_reader_wakeups"] = lambda: float(hub.stats().get("signals", 0))
                # reads whose chunk framing and line split ran on the reader thread (watcher.hub_framing)
                self.metrics.gauges["watch_reader_framed_reads"] = lambda: float(hub.stats().get("framed_reads", 0))
                # memory accounting: read buffers allocated (up to watch_reader_buffers x watch_read_bytes)
                self.metrics.gauges["watch_reader_allocated_bytes"] = \
                    lambda: float(hub.stats().get("allocated_bytes", 0))
                self.metrics.gauges["watch_reader_held_bytes"] = lambda: float(hub.stats().get("held_bytes", 0))
                # https watches on the hub's own TLS 1.3 record layer (ops/csrc/tls13.inc):
                # ciphertext rings (inside watch_reader_allocated_bytes), streams taken
                # over / left on SSL_read, records opened and key updates followed
                for key, name in (("tls_ring_bytes", "watch_reader_tls_ring_bytes"),
                                  ("tls_taken", "watch_tls_streams_native"), ("tls_kept", "watch_tls_streams_openssl"),
                                  ("tls_records", "watch_tls_records"), ("tls_key_updates", "watch_tls_key_updates")):
                    self.metrics.gauges[name] = lambda key=key: float(hub.stats().get(key, 0))
            self._pin_threads()
        gains: Set[str] = set()
        if s.watcher.shard.handover_dir and self._multi and s.watcher.shard.key == "namespace":
            gains, owed = self._reshard_on_start(scopes, saved_rvs, owed)
        if owed:
            # the checkpoint's cut: clusterapi never acknowledged these; send them
            # (in their original order) before anything newer — the watches that
            # resume after them, and the DELETEDs synthesized just below, which
            # must be the last word for their pods
            self._resubmit_owed(owed)
        if saved_rvs and None not in scopes:
            if self.ns_watcher is not None:
                # namespaces deleted while the watcher was down: their pods get
                # DELETED from the cache, as _retire_scope and a relist would
                # (only this shard had them cached: each shard's checkpoint is its own)
                self._notify_deleted_namespaces(set(self.ns_watcher.names))
            # pods of namespaces this shard no longer watches would never be reconciled
            self._forget_namespaces_except(set(scopes))
        self.metrics.gauges["cached_pods"] = lambda: float(len(cache))
        if hasattr(cache, "memory"):  # native cache: bytes held (cores + keys), for memory accounting
            self.metrics.gauges["cache_bytes"] = lambda: float(sum(v for k, v in cache.memory().items()
                                                                   if k.endswith("_bytes")))
        if self._native_pipeline():  # memory accounting: the C heap (glibc), in use vs retained free
            from ..ops.native import load as _load_native
            _mi = _load_native().malloc_info
            self.metrics.gauges["malloc_in_use_bytes"] = lambda: float(_mi()["in_use_bytes"])
            self.metrics.gauges["malloc_free_bytes"] = lambda: float(_mi()["free_bytes"])
            self.metrics.gauges["malloc_arenas"] = lambda: float(len(_load_native().malloc_arenas()))
        self.metrics.gauges["notify_outstanding"] = lambda: float(self.notifier.outstanding())
        if hasattr(self.notifier, "outstanding_bytes"):
            self.metrics.gauges["notify_outstanding_bytes"] = lambda: float(self.notifier.outstanding_bytes())
        self.metrics.gauges["watch_scopes"] = lambda: float(len(self.reflectors))
        self.log.info(f"Starting Pod watcher in {s.environment} environment...")
        if s.watcher.namespaces:
            self.log.info(f"Monitoring namespaces: {s.watcher.namespaces}")
        else:
            self.log.info("Monitoring all namespaces")
        for i, ns in enumerate(scopes):
            if ns in gains:  # another shard's under the previous layout: its record first
                self._gain_scope(ns)
            else:
                self._start_scope(ns, primed=bool(saved_rvs))
            if i % 64 == 63:  # a thousand namespaces: let the started scopes (and the loop) run meanwhile
                await asyncio.sleep(0)
                if self._stop.is_set():
                    break
        if s.metrics.enabled and self.serve_metrics:
            self._metrics_server = await start_metrics_server(self.metrics, s.metrics.host, s.metrics.port,
                                                              debug=s.metrics.debug)
        if ck:
            self._tasks.append(asyncio.ensure_future(self._checkpoint_loop()))
        if self._native_pipeline() and s.watcher.malloc_trim_seconds > 0:
            self._tasks.append(asyncio.ensure_future(self._malloc_trim_loop(s.watcher.malloc_trim_seconds)))
        self._live = True
        if self.ns_watcher is not None:
            self._on_namespaces(self.ns_watcher.names)  # changes seen while the first scopes started
        await self._wait_synced()
        if self._gc_frozen and not self._stop.is_set():
            # the scopes' long-lived objects join the frozen set; only the young
            # generations are collected first (a full pass over a 1,000-scope
            # start's objects would hold the loop ~30 ms; cyclic garbage already
            # in the old generation stays frozen until shutdown unfreezes it)
            gc.collect(1)
            gc.freeze()
        self.metrics.ready = True
        self.started.set()

    # ------------------------------------------------------------------ watch scopes
    def _event_sharding(self) -> bool:
        """Per-event shard filtering: off when the watches themselves are the
        shard's namespaces (server-side scopes keyed by namespace)."""
        w = self.settings.watcher
        scoped = w.namespace_scope == "discover" or (w.namespace_scope == "server" and bool(w.namespaces))
        return not (scoped and w.shard.key == "namespace")

    def _owned(self, names: Set[str]) -> List[str]:
        return ShardFilter(self.settings.watcher.shard).namespaces(sorted(names))

    def _start_scope(self, ns: Optional[str], primed: bool) -> Reflector:
        s = self.settings
        key = ns or "*"
        if self._multi:
            # Each scope decodes its own stream: give it a private decoder.
            dec = make_decoder(s.watcher.engine, s.environment, s.watcher.state_format, s.watcher.payload_extra,
                               s.watcher.validate)
            pipe = self._scope_pipeline(dec)
        else:
            dec, pipe = self.decoder, self.pipeline
        if self._list_gate is None and s.watcher.relist_concurrency > 0:
            self._list_gate = asyncio.Semaphore(s.watcher.relist_concurrency)
        r = Reflector(self.api, s, dec, pipe, self.metrics, namespace=ns,
                      resource_version=self._saved_rvs.get(key), primed=primed, list_gate=self._list_gate)
        if getattr(self.notifier, "saturated", False):
            r.set_paused(True)
        self.reflectors.append(r)
        task = asyncio.ensure_future(r.run())
        self._scope_tasks[key] = task
        task.add_done_callback(lambda t, k=key: self._scope_done(k, t))
        return r

    def _scope_done(self, key: str, task: "asyncio.Task") -> None:
        if self._scope_tasks.get(key) is not task:
            return  # stopped on purpose (namespace gone or handed over)
        if task.cancelled() or self._stop.is_set():
            return
        exc = task.exception()
        if exc is not None and self._failure is not None and not self._failure.done():
            self._failure.set_exception(exc)

    def _stop_scope(self, ns: str, handover_to: Optional[int] = None) -> None:
        timer = self._retiring.pop(ns, None)
        if timer is not None:
            timer.cancel()
        gaining = self._gaining.pop(ns, None)
        if gaining is not None:  # handed on before its watch started: nothing of it is cached here
            gaining.cancel()
        task = self._scope_tasks.pop(ns, None)
        stopped = [r for r in self.reflectors if r.namespace == ns]
        for r in stopped:
            r.stop()
            self.reflectors.remove(r)
        if task is not None and not task.done():
            task.cancel()
        if handover_to is not None and stopped:
            # the namespace's pods stay cached until the record is written
            self._handing[ns] = asyncio.ensure_future(self._handover_out(ns, handover_to))
            return
        self._forget_namespaces({ns})

    def _cached_pods_of(self, cache, ns: str) -> list:
        return [(uid, e[RV], e[PHASE], e[NAME], e[CORE]) for uid, e in cache.items() if e[NS] == ns]

    async def _handover_out(self, ns: str, dst: int) -> None:
        """The old owner's half of a live namespace hand-over: with its watch
        stopped, wait until clusterapi has acknowledged (or this shard has
        given up) every notification still owed for the namespace — a retried
        MODIFIED (clusterapi answering 503, say) must not land after the new
        owner's notifications for the same pod — then write this shard's
        cached pods of ``ns`` to the shared directory for shard ``dst``
        (parallel/shard.py) and forget them. The wait is bounded by half of
        ``shard.handover_wait_seconds`` (the new owner's patience): past it the
        record goes out anyway and the late notifications are counted
        (``shard_handover_owed_late``)."""
        sh = self.settings.watcher.shard
        loop = asyncio.get_running_loop()
        try:
            deadline = loop.time() + sh.handover_wait_seconds / 2
            pending_in = getattr(self.notifier, "pending_in", None)
            late = 0
            while pending_in is not None and not self._stop.is_set():
                late = pending_in(ns)
                if late == 0 or loop.time() >= deadline:
                    break
                await asyncio.sleep(0.05)
            if late:
                self.metrics.c["shard_handover_owed_late"] += late
                self.log.warning(f"Handing namespace {ns} over with {late} notification(s) for it still owed "
                                 f"to clusterapi: they may arrive after shard {dst}'s")
            cache = self.pipeline.cache if self.pipeline is not None else None
            if cache is None:
                return
            pods = self._cached_pods_of(cache, ns)
            try:
                # (json + fsync on a shared volume: off the loop)
                await loop.run_in_executor(None, write_handover, sh.handover_dir, ns, sh.index, dst, pods, None,
                                           layout_of(sh))
            except OSError as exc:
                self.metrics.c["shard_handover_errors"] += 1
                self.log.error(f"Could not write the hand-over of namespace {ns} to shard {dst} "
                               f"({exc}): its new owner will re-announce its pods")
            else:
                self.metrics.c["shard_handovers_out"] += 1
                self.metrics.c["shard_handover_pods_out"] += len(pods)
                self.log.info(f"Handed namespace {ns} ({len(pods)} cached pods) over to shard {dst}")
            if self._handing.get(ns) is asyncio.current_task():
                self._forget_namespaces({ns})
        finally:
            if self._handing.get(ns) is asyncio.current_task():
                del self._handing[ns]

    def _reshard_on_start(self, scopes, saved_rvs: dict, owed: list):
        """A new shard layout (``shard.count`` changed, every shard restarted):
        the hand-over across a restart (parallel/shard.py). Notes the layout in
        ``handover_dir``'s history, writes a record for every namespace this
        shard held (its checkpoint) or owned under the previous layout that
        another shard owns now — with the checkpoint's owed notifications for
        it, which then are not re-sent here — and returns the namespaces this
        shard now owns that were another's, which wait for their record.
        Returns ``(gains, owed left to re-send here)``."""
        sh = self.settings.watcher.shard
        layout = layout_of(sh)
        try:
            prev, self._layout_since = record_layout(sh.handover_dir, layout)
        except OSError as exc:
            self.log.error(f"Could not record the shard layout in {sh.handover_dir} ({exc}): no hand-over")
            return set(), owed
        if self.ns_watcher is not None:
            names = set(self._ns_seen)
        else:
            names = set(self.settings.watcher.namespaces)
        owned = {x for x in scopes if x}
        cache = self.pipeline.cache
        held = {ns for ns in cache.namespaces() if ns is not None} | {k for k in saved_rvs if k != "*"}
        was_mine = set()
        if prev and prev != layout and prev.get("key", "namespace") == "namespace":
            was_mine = {ns for ns in names if owner_of(ns, names, prev["count"], prev["assignment"]) == sh.index}
        out = sorted(ns for ns in (held | was_mine) if ns in names and ns not in owned)
        for ns in out:
            dst = owner_of(ns, names, sh.count, sh.assignment)
            pods = self._cached_pods_of(cache, ns)
            mine = [o for o in owed if o[2] == ns]
            try:
                write_handover(sh.handover_dir, ns, sh.index, dst, pods, mine, layout)
            except OSError as exc:
                self.metrics.c["shard_handover_errors"] += 1
                self.log.error(f"Could not write the hand-over of namespace {ns} to shard {dst} ({exc})")
                continue
            self.metrics.c["shard_handovers_out"] += 1
            self.metrics.c["shard_handover_pods_out"] += len(pods)
            self.log.info(f"New shard layout {layout}: handed namespace {ns} ({len(pods)} cached pods, "
                          f"{len(mine)} owed notifications) over to shard {dst}")
        gone = set(out)
        owed = [o for o in owed if o[2] not in gone]
        gains: Set[str] = set()
        if prev and prev != layout and prev.get("key", "namespace") == "namespace":
            gains = {ns for ns in owned if ns not in saved_rvs
                     and owner_of(ns, names, prev["count"], prev["assignment"]) != sh.index}
            if gains:
                self.log.info(f"New shard layout {layout} (was {prev}): waiting for the hand-over of "
                              f"{len(gains)} namespace(s) from their old owners")
        return gains, owed

    def _gain_scope(self, ns: str) -> None:
        self._gaining[ns] = asyncio.ensure_future(self._await_handover(ns))

    async def _await_handover(self, ns: str) -> None:
        """The new owner's half: wait for the old owner's record, send the
        notifications it still owed for the namespace (before anything of this
        shard's), load its pods into the cache, then start the watch — its
        first LIST reconciles against that state (unchanged pods stay quiet,
        pods gone meanwhile are DELETED), as a relist after a 410 would.
        Records written before this wait could have been meant for it (an
        older move's, whose new owner timed out) or under another layout are
        stale and discarded."""
        sh = self.settings.watcher.shard
        loop = asyncio.get_running_loop()
        deadline = loop.time() + sh.handover_wait_seconds
        # a live move's record is written after the old owner saw the change
        # (seconds around ours); a restart's since the layout began
        not_before = min(time.time() - max(60.0, sh.handover_wait_seconds),
                         self._layout_since - 60.0 if self._layout_since else time.time())
        layout = layout_of(sh)
        while True:
            rec = take_handover(sh.handover_dir, ns, sh.index, not_before=not_before, layout=layout)
            if rec is not None or loop.time() >= deadline or self._stop.is_set():
                break
            await asyncio.sleep(0.05)
        if self._gaining.get(ns) is not asyncio.current_task() or self._stop.is_set():
            return
        del self._gaining[ns]
        if rec is None:
            self.metrics.c["shard_handover_timeouts"] += 1
            self.log.warning(f"No hand-over of namespace {ns} from its old owner after "
                             f"{sh.handover_wait_seconds}s: its pods are announced as ADDED again")
        else:
            if rec.owed:  # the old owner's unacknowledged notifications: first, in their order
                self._resubmit_owed(list(rec.owed))
            cache = self.pipeline.cache
            for uid, rv, phase, name, core in rec.pods:
                cache.put(uid, rv, phase, ns, name, core)
            self.metrics.c["shard_handovers_in"] += 1
            self.metrics.c["shard_handover_pods_in"] += len(rec.pods)
            self.log.info(f"Took over namespace {ns} ({len(rec.pods)} pods, {len(rec.owed)} owed "
                          f"notifications from shard {rec.src})")
        self._start_scope(ns, primed=True)

    def _forget_namespaces(self, namespaces: Set[str]) -> None:
        """Drop cached pods of namespaces this shard stopped watching, silently:
        they are now the business of another shard (or gone with the namespace).
        Both caches index entries by namespace: only those namespaces' pods are touched."""
        cache = self.pipeline.cache if self.pipeline is not None else None
        if cache is None:
            return
        cache.drop_namespaces(namespaces)

    def _forget_namespaces_except(self, keep: Set[str]) -> None:
        cache = self.pipeline.cache if self.pipeline is not None else None
        if cache is None:
            return
        cache.drop_namespaces_except(keep)

    def _notify_deleted_namespaces(self, existing: Set[str]) -> None:
        cache = self.pipeline.cache
        gone = sorted(ns for ns in cache.namespaces() if ns is not None and ns not in existing)
        for ns in gone:
            n = cache.count_namespace(ns)
            self.metrics.c["namespace_deleted_synthesized"] += n
            self.log.warning(f"Namespace {ns} was deleted while the watcher was down: notifying its "
                             f"{n} cached pod(s) as DELETED")
            for ev in self.pipeline.delete_scope(ns, time.monotonic_ns()):
                self.log.warning(f"Skipping undecodable cached entry ({ev[0]}): {ev[8]}")

    def _on_namespaces(self, names: Set[str]) -> None:
        """NamespaceWatcher callback: start/stop reflectors to match the owned set.

        A namespace handed to another shard stops at once (its pods are that
        shard's business now). A *deleted* namespace drains first: the namespace
        watch and the namespace's pod watch are separate streams, read in
        whatever order their bytes arrive, so its pods' DELETED events may still
        be on the way when the namespace's own DELETED is seen (kube-apiserver
        deletes the pods before the namespace, but nothing orders two streams)."""
        if not self._live or self._stop.is_set():
            return
        sh = self.settings.watcher.shard
        prev, self._ns_seen = self._ns_seen, set(names)
        owned = set(self._owned(names))
        current = set(self._scope_tasks) | set(self._gaining)
        for ns in sorted(owned & set(self._retiring)):  # deleted and created again: keep watching
            self._retiring.pop(ns).cancel()
        for ns in sorted(owned - current):
            handing = self._handing.pop(ns, None)
            if handing is not None:  # back before its record went out: still ours, cache and all
                handing.cancel()
            self.metrics.c["scopes_started"] += 1
            self.log.info(f"Watching namespace {ns} (new or now owned by shard {sh.index})")
            if sh.handover_dir and ns in prev and owner_of(ns, prev, sh.count, sh.assignment) != sh.index:
                self._gain_scope(ns)  # moved here from another shard: its state first
            else:
                self._start_scope(ns, primed=True)
        for ns in sorted(current - owned):
            if ns in self._gaining and ns not in names:  # deleted before its hand-over came
                self._gaining.pop(ns).cancel()
                continue
            if ns not in names:
                if ns not in self._retiring:  # already draining: its timer is running
                    self._retire_scope(ns)
                continue
            self.metrics.c["scopes_stopped"] += 1
            self.log.info(f"Stopped watching namespace {ns} (owned by another shard)")
            self._stop_scope(ns, owner_of(ns, names, sh.count, sh.assignment) if sh.handover_dir else None)

    def _cached_in(self, ns: str) -> int:
        cache = self.pipeline.cache if self.pipeline is not None else None
        return 0 if cache is None else cache.count_namespace(ns)

    def _retire_scope(self, ns: str, waited: float = 0.0) -> None:
        """Keep a deleted namespace's pod watch until every pod cached there has
        been seen DELETED, or ``watcher.namespace_drain_seconds`` passed; then
        notify any pod still cached there as DELETED from its cached state (as a
        relist that no longer finds it would) and stop the watch."""
        if self._stop.is_set() or ns not in self._scope_tasks:
            self._retiring.pop(ns, None)
            return
        step = 0.05
        limit = self.settings.watcher.namespace_drain_seconds
        if self._cached_in(ns) and waited < limit:
            old = self._retiring.get(ns)
            if old is not None:
                old.cancel()  # one drain timer per namespace, whoever scheduled it
            self._retiring[ns] = asyncio.get_running_loop().call_later(
                step, self._retire_scope, ns, waited + step)
            return
        self._retiring.pop(ns, None)
        left = [r for r in self.reflectors if r.namespace == ns]
        if left and self._cached_in(ns):
            pipe = left[0].pipeline
            n = self._cached_in(ns)
            self.metrics.c["namespace_deleted_synthesized"] += n
            self.log.warning(f"Namespace {ns} deleted: {n} pod(s) without a DELETED event after "
                             f"{limit:g}s; notifying them as DELETED from the cache")
            for ev in pipe.delete_scope(ns, time.monotonic_ns()):
                left[0]._handle_control(ev)
        self.metrics.c["scopes_stopped"] += 1
        self.log.info(f"Stopped watching namespace {ns} (deleted)")
        self._stop_scope(ns)

    def _scope_pipeline(self, decoder) -> EventPipeline:
        assert self.pipeline is not None
        p = EventPipeline(self.settings, decoder, self.notifier, self.metrics, self.pipeline.cache,
                          self.event_log, event_sharding=self._event_sharding())
        if self._native_pipeline():
            p.attach_native(self._decode_pool)
        return p

    def _make_decode_pool(self):
        """One decode pool for every watch scope (they share the loop thread)."""
        from ..ops.native import load
        from ..utils.cpus import auto_decode_spin_us, auto_decode_threads, pin_to_l3_domain
        w = self.settings.watcher
        n = w.decode_threads if w.decode_threads >= 0 else auto_decode_threads()
        if n > 0:
            # Workers started below inherit the mask. Measured on a chiplet
            # host (BENCHMARKS.md): 3 workers spread over CCDs were slower than
            # none; the same 3 inside the loop thread's L3 ran ~1.6x faster.
            # A process already inside one L3 domain (a launcher placed it)
            # stays where it is.
            dom = pin_to_l3_domain(min_cpus=n + 1, only_if_split=True)
            if dom:
                self.log.info(f"Decode pool pinned to L3 domain CPUs {sorted(dom)}")
        spin = auto_decode_spin_us()
        return load().DecodePool(n, spin) if n > 0 else 0

    def _pin_threads(self) -> None:
        """``watcher.thread_pinning: auto``: keep one physical core of the L3
        domain free for the event-loop thread (which applies every event in
        stream order, the rate's bound): the decode workers and the reader
        thread are pinned to the rest. The loop thread itself stays free to
        move — pinned hard, it could not escape another process scheduled on
        its core, and the latency tail grew to ~10 ms (profiles/latency_curve_*)."""
        mode = self.settings.watcher.thread_pinning
        if mode == "none":
            return
        from ..utils.cpus import loop_core_split, reader_core_split
        try:
            split = loop_core_split(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            return
        if split is None:
            return
        loop_cpus, rest = split
        tids = list(self._decode_pool.thread_ids()) if self._decode_pool else []
        # the hub's TLS pool threads (https watches) were made with the loop
        # thread's whole domain: left there, three of them ran on the loop's
        # core and it waited 5.8 ms/s for a CPU (profiles/r6/tls_timeline)
        if self._reader_hub is not None:
            tids += list(self._reader_hub.core.tls_thread_ids())
            # reader threads past the first run beside the workers (the first
            # gets a core of its own below)
            tids += list(self._reader_hub.core.thread_ids())[1:]
        reader_cpus = None
        reader_tid = self._reader_hub.core.thread_id() if self._reader_hub is not None else 0
        if reader_tid and mode == "auto":
            # the reader thread gets a core of its own too: it copies the watch
            # bodies out of the kernel and bounds the single-stream rate
            rsplit = reader_core_split(rest)
            if rsplit is not None:
                reader_cpus, rest = rsplit
        if reader_tid and reader_cpus is None:
            tids.append(reader_tid)
        try:
            if reader_cpus is not None:
                os.sched_setaffinity(reader_tid, reader_cpus)
            for tid in tids:
                if tid:
                    os.sched_setaffinity(tid, rest)
            # the loop thread moves to the free core now (its caches follow
            # it) but keeps the whole domain to run on
            self._loop_affinity = os.sched_getaffinity(0)
            os.sched_setaffinity(0, loop_cpus)
            os.sched_setaffinity(0, self._loop_affinity)
        except OSError as exc:
            self.log.warning(f"Thread pinning skipped: {exc}")
            return
        self.thread_placement = {"loop": sorted(loop_cpus), "workers": sorted(rest),
                                 **({"reader": sorted(reader_cpus)} if reader_cpus is not None else {})}
        self.log.info(f"CPUs {sorted(loop_cpus)} kept for the event-loop thread; {len(tids)} worker threads on the rest")

    def _native_pipeline(self) -> bool:
        return self.settings.watcher.engine == "native"

    async def _wait_synced(self) -> None:
        synced = asyncio.ensure_future(asyncio.gather(*[r.synced.wait() for r in self.reflectors]))
        runs = list(self._tasks) + list(self._scope_tasks.values())
        done, _ = await asyncio.wait([synced] + runs, return_when=asyncio.FIRST_COMPLETED)
        if synced not in done:
            synced.cancel()
            for t in runs:
                if t.done() and not t.cancelled() and t.exception() is not None:
                    raise t.exception()  # type: ignore[misc]
            raise SetupError("watch ended before the initial sync")

    async def wait(self) -> None:
        """Run until :meth:`stop` or a watch fails permanently."""
        stopper = asyncio.ensure_future(self._stop.wait())
        waits = [t for t in self._tasks] + [stopper]
        if self._failure is not None:
            waits.append(self._failure)
        if not self._multi:
            waits += list(self._scope_tasks.values())  # a lone watch that ends ends the service
        done, _ = await asyncio.wait(waits, return_when=asyncio.FIRST_COMPLETED)
        err = None
        for t in done:
            if t is not stopper and not t.cancelled() and t.exception() is not None:
                err = t.exception()
        if not stopper.done():
            stopper.cancel()
        if err is not None:
            raise err

    def stop(self) -> None:
        self._stop.set()
        if self.ns_watcher is not None:
            self.ns_watcher.stop()
        for r in self.reflectors:
            r.stop()

    async def shutdown(self, drain_timeout: float = 10.0, checkpoint: bool = True) -> None:
        """Stop watching, drain the notifier, write the final checkpoint.

        The checkpoint is written only if every notification was delivered:
        a resourceVersion saved with notifications still queued would skip
        them on restart; the previous (quiescent) checkpoint replays them
        instead. ``checkpoint=False`` (a leader that lost its lease) never
        writes — the new leader owns the file now.

        With a spool, notifications still owed after the drain are written to
        it first (closing the notifier), so the checkpoint can be written
        anyway: a restart resumes exactly and replays the spool. A leader that
        lost its lease drops what it still owes instead of spooling it — the
        new leader relists, and an old record replayed in a later term could
        overwrite newer state.
        """
        self.log.info("Stopping Pod watcher...")
        if self._gc_frozen:  # this service's objects are collectable again (a leader's next term)
            self._gc_frozen = False
            gc.unfreeze()
        if self.ns_watcher is not None:
            self.ns_watcher.stop()
        for r in self.reflectors:
            r.stop()
        for t in self._handing.values():  # records not written yet: their pods stay in the checkpoint,
            t.cancel()                    # and the restart hands them over (_reshard_on_start)
        self._handing.clear()
        drained = True
        closed = False
        if self.notifier is not None:
            if not checkpoint and self.spool is not None:
                self.notifier.detach_spool()
            drained = await self.notifier.drain(drain_timeout)
            if not drained and checkpoint and self.spool is not None:
                await self.notifier.close()  # spools the rest
                closed = drained = True
        if checkpoint and (drained or self._native_checkpoint()):
            # a periodic write cancelled mid-way keeps running on its thread: let
            # it land first, so the final cut is the one that stays on disk
            await self._await_inflight_checkpoint()
            await self._write_checkpoint()  # format 2 carries whatever is still owed
        tasks = list(self._tasks) + list(self._scope_tasks.values()) + list(self._gaining.values())
        for t in tasks:
            if not t.done():
                t.cancel()
        for t in tasks:
            try:
                await t
            except (asyncio.CancelledError, WatchFailed, Exception):  # noqa: BLE001
                pass
        if self._metrics_server is not None:
            self._metrics_server.close()
        if self.notifier is not None and not closed:
            await self.notifier.close()  # with a spool, whatever is still owed is written to it
        if self.spool is not None:
            self.spool.close()
        if self._reader_hub is not None:
            if self.api is not None:
                self.api.http.reader_hub = None
            self._reader_hub.close()
            self._reader_hub = None
        if self._decode_pool:
            # its threads end now, not when the garbage collector frees this
            # service (a leader's every term builds a new one; the shared
            # Metrics gauges keep the old one reachable until the next term)
            self._decode_pool.close()
        if self._loop_affinity is not None:
            try:
                os.sched_setaffinity(0, self._loop_affinity)
            except OSError:
                pass
            self._loop_affinity = None
        if self.api is not None:
            await self.api.close()

    async def run(self) -> None:
        try:
            await self.start()
            await self.wait()
        finally:
            await self.shutdown()

    # ------------------------------------------------------------------ checkpoint
    def _native_checkpoint(self) -> bool:
        """Format 2 (consistent cut, no pause/drain): native cache + native notifier core."""
        return (self._native_pipeline() and self.pipeline is not None
                and hasattr(self.pipeline.cache, "snapshot")
                and (self.notifier is None or hasattr(self.notifier, "core") or not self.settings.clusterapi.enabled))

    def _resubmit_owed(self, owed: list) -> None:
        core = getattr(self.notifier, "core", None)
        if core is None:
            self.log.warning(f"{len(owed)} owed notifications in the checkpoint: no native notifier to resend them")
            return
        now = time.monotonic_ns()
        for uid, etype, ns, name, body in owed:
            core.submit_body(uid, etype, ns, name, body, now)
        self.metrics.c["checkpoint_owed_resent"] += len(owed)
        self.notifier.flush()

    async def _write_checkpoint(self) -> None:
        ck = self.settings.watcher.checkpoint.path
        if not ck or self.pipeline is None:
            return
        if self._native_checkpoint():
            await self._write_snapshot(ck)
            return
        async with self._ck_lock:
            scopes = {r.scope: r.rv for r in self.reflectors}
            save_checkpoint(ck, scopes, self.pipeline.cache, {"written_at": time.time()})
        self.metrics.c["checkpoints_written"] += 1

    async def _await_inflight_checkpoint(self) -> None:
        fut = self._ck_inflight
        if fut is not None and not fut.done():
            try:
                await fut
            except Exception as exc:  # noqa: BLE001 - the final write below reports its own errors
                self.log.warning(f"Checkpoint write in progress at shutdown failed: {exc}")

    async def _write_snapshot(self, ck: str) -> None:
        """Format 2: the consistent cut (a few ms per 100k pods, on the loop
        thread) and its write (executor thread), one at a time — a later cut is
        never overwritten by an earlier one."""
        async with self._ck_lock:
            await self._await_inflight_checkpoint()
            scopes = {r.scope: r.rv for r in self.reflectors}
            meta = {"written_at": time.time()}
            snap = native_snapshot(self.pipeline.cache, getattr(self.notifier, "core", None))
            st = snap.stats()
            loop = asyncio.get_running_loop()
            self._ck_inflight = loop.run_in_executor(None, write_native, snap, ck, scopes, meta)
            nbytes, secs = await asyncio.shield(self._ck_inflight)
        g = self.metrics.gauges
        last = {"checkpoint_stall_ms": st["snapshot_seconds"] * 1e3, "checkpoint_write_ms": secs * 1e3,
                "checkpoint_bytes": float(nbytes), "checkpoint_pods": float(st["entries"]),
                "checkpoint_owed": float(st["owed"]), "checkpoint_written_at": meta["written_at"]}
        for k, v in last.items():
            g[k] = (lambda v=v: v)
        self.last_checkpoint = dict(last)
        self.metrics.c["checkpoints_written"] += 1

    async def checkpoint_now(self, drain_timeout: float = 30.0) -> bool:
        """Write a checkpoint now.

        Native engine + notifier core: a consistent cut taken synchronously on
        the loop thread (``PodCache.snapshot``, a few ms per 100k pods) and
        written on an executor thread — the watches keep running. Otherwise:
        pause readers, drain the notifier, save, resume (format 1)."""
        if self._native_checkpoint():
            ck = self.settings.watcher.checkpoint.path
            if not ck or self.pipeline is None:
                return False
            await self._write_snapshot(ck)
            return True
        for r in self.reflectors:
            r.set_paused(True)
        try:
            ok = await self.notifier.drain(drain_timeout) if self.notifier is not None else True
            if ok:
                await self._write_checkpoint()
            return ok
        finally:
            saturated = getattr(self.notifier, "saturated", False)
            for r in self.reflectors:
                r.set_paused(saturated)

    async def _malloc_trim_loop(self, period: float) -> None:
        """The decode workers, the reader hub and the notifier allocate on
        several threads; glibc keeps what each thread's arena freed. Handing
        the free pages back now and then keeps the RSS at what is in use
        (soak: RSS grew ~1-2 MiB/hour with no growth in use).

        A trim locks each arena while it walks it, and a thread allocating
        from that arena waits: it runs only when the heap retains at least
        ``MALLOC_TRIM_MIN_FREE`` free, and every trim is timed
        (``malloc_trim_last_ms`` / ``malloc_trim_max_ms`` gauges,
        ``malloc_trim_us`` counter) so a latency outlier can be checked
        against it. It waits for half a second
        without events (up to nine periods; then it trims anyway), so a trim
        does not stall notifications in flight."""
        from ..ops.native import load
        kw = load()
        trim, info = kw.malloc_trim, kw.malloc_info
        min_free = MALLOC_TRIM_MIN_FREE
        loop = asyncio.get_running_loop()
        c, g = self.metrics.c, self.metrics.gauges
        last = {"last_ms": 0.0, "max_ms": 0.0}
        g["malloc_trim_last_ms"] = lambda: last["last_ms"]
        g["malloc_trim_max_ms"] = lambda: last["max_ms"]

        def timed_trim() -> float:
            t = time.perf_counter()
            trim()
            return time.perf_counter() - t

        async def quiet_moment() -> bool:
            # a trim makes every allocating thread wait on its arena while it
            # walks it (7.5-15 ms on the MI355X host with the heap the
            # saturated bench leaves): a notification in flight then waits
            # too. Wait, up to one period, for half a second with no event.
            deadline = time.monotonic() + period
            while time.monotonic() < deadline:
                n0 = c["events_received"]
                await asyncio.sleep(0.5)
                if c["events_received"] == n0:
                    return True
            return False

        deferred = 0
        while True:
            await asyncio.sleep(period)
            if min_free > 0 and info()["free_bytes"] < min_free:
                c["malloc_trims_skipped"] += 1
                continue
            # a watcher that is never quiet still trims, every tenth period
            if deferred < 9 and not await quiet_moment():
                deferred += 1
                c["malloc_trims_deferred"] += 1
                continue
            deferred = 0
            try:
                secs = await loop.run_in_executor(None, timed_trim)
            except RuntimeError as exc:  # the executor is going away (shutdown)
                self.log.debug(f"malloc_trim skipped: {exc}")
                continue
            last["last_ms"] = secs * 1e3
            last["max_ms"] = max(last["max_ms"], secs * 1e3)
            c["malloc_trims"] += 1
            c["malloc_trim_us"] += int(secs * 1e6)

    async def _checkpoint_loop(self) -> None:
        period = self.settings.watcher.checkpoint.interval_seconds
        last = None
        while True:
            await asyncio.sleep(period)
            state = (tuple(r.rv for r in self.reflectors), len(self.pipeline.cache) if self.pipeline else 0)
            if state == last:
                continue
            if await self.checkpoint_now():
                last = state
