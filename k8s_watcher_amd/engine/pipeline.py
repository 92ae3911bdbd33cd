"""The per-event pipeline (SURVEY C9 ``handle_pod_event``, §3.2 hot loop).

Order of operations matches ``/root/reference/watcher/pod_watcher.py:214-241``:

1. production ``critical_events_only`` filter — silent drop (``:220-221``);
2. INFO ``Pod event detected: <TYPE> - <ns>/<name>`` (``:223``) — logged
   *before* the namespace filter, as in the reference;
3. client-side namespace filter with DEBUG ``Skipping pod ...`` (``:226-229``);
4. payload build + ``event_type`` (``:232-233``);
5. notify (commented out in the reference, ``:236``; enabled here).

Additions: every event first updates the pod cache (for ``notify_on:
phase_change`` and relist diffs), and events are processed in *batches* —
all events decoded from one socket read share one pass, one timestamp and
one notifier flush, which is what keeps Python overhead per event small.
"""

from __future__ import annotations

import logging
from typing import List, Optional, Tuple

from ..metrics import Metrics
from ..ops.cache import CORE, MISSING, NAME, NS, PHASE, PodCache, make_pod_cache
from ..ops.decode import (ADDED, BOOKMARK, DELETED, E_EXTRA, E_HAS_STATUS, E_NAME, E_NS, E_PHASE,
                          E_RV, E_TYPE, E_UID, INVALID, MODIFIED)
from ..ops.filters import TERMINAL_PHASES
from ..parallel.shard import ShardFilter
from ..utils.config import Settings, ShardSettings
from ..utils.fastlog import EventLog
from ..utils.logsetup import SERVICE_LOGGER
from ..utils.timefmt import event_timestamp

_POD_EVENTS = frozenset({ADDED, MODIFIED, DELETED})


class EventPipeline:
    def __init__(self, settings: Settings, decoder, notifier, metrics: Metrics,
                 cache: Optional[PodCache] = None, event_log: Optional[EventLog] = None,
                 event_sharding: bool = True) -> None:
        w = settings.watcher
        self.settings = settings
        self.decoder = decoder
        self.notifier = notifier
        self.metrics = metrics
        self.cache = cache if cache is not None else PodCache()
        self.log = logging.getLogger(SERVICE_LOGGER)
        self.elog = event_log if event_log is not None else EventLog(self.log)
        self.critical_active = settings.environment == "production" and w.critical_events_only
        self.namespaces = frozenset(w.namespaces)
        self.phase_mode = w.notify_on == "phase_change"
        self.ts_mode = w.event_timestamp
        self.log_events_setting = w.log_events
        # event_sharding=False: the watch scopes are already this shard's
        # namespaces (parallel/shard.py), so every received event is ours
        self.shard = ShardFilter(w.shard if event_sharding else ShardSettings())
        self.last_rv: Optional[str] = None
        self.native = None
        self._native_log = None

    @property
    def log_events(self) -> bool:
        if self.log_events_setting is not None:
            return self.log_events_setting
        return self.log.isEnabledFor(logging.INFO)

    # ------------------------------------------------------------------ native fast path
    def attach_native(self, decode_pool=None) -> None:
        """Run watch batches through ``_kwcore.Pipeline`` (decode + this class's
        per-event logic fused in C++), submitting straight into the native
        notifier core when the pool has one. Relists run natively too
        (``native.relist``, driven by ``Reflector``); :meth:`reconcile` remains
        the Python engine's and the WatchList path's.

        Line decoding fans out over ``decode_pool`` (a ``_kwcore.DecodePool``
        shared by every scope's pipeline) or, without one, a private pool of
        ``watcher.decode_threads`` workers (``auto``: utils/cpus.py).
        """
        from ..ops.native import load
        from ..utils.cpus import auto_decode_threads
        w = self.settings.watcher
        core = getattr(self.notifier, "core", None)
        if isinstance(self.cache, PodCache):  # the fused pipeline keeps the cache in C++
            self.cache = make_pod_cache(True, self.cache.to_records())
        decode = decode_pool if decode_pool is not None else (
            w.decode_threads if w.decode_threads >= 0 else auto_decode_threads())
        self.native = load().Pipeline(
            self.settings.environment, self.cache, self.metrics.c, self.namespaces or None,
            self.critical_active, self.phase_mode, self.shard.count, self.shard.index, self.shard.by_uid,
            w.event_timestamp == "utc", core, False, False, decode)
        if w.payload_extra:
            self.native.set_extra(w.payload_extra)
        from ..ops.decode import VALIDATE_MODES
        self.native.set_validate(VALIDATE_MODES[w.validate])
        if w.state_format == "python_repr":  # str(V1ContainerState) in C++ (ops/csrc/pyrepr.inc)
            from ..models.payload import repr_fallback, utc_tzinfo_repr
            self.native.set_repr(utc_tzinfo_repr(), repr_fallback(self.settings.environment, w.payload_extra))
        if self.elog.native_sink is not None:
            self.native.set_log_sink(self.elog.native_sink)  # per-event lines formatted in C++

    def handle_raw(self, data: bytes, read_ns: int, framed: bool) -> List[tuple]:
        """Native path: raw watch bytes (HTTP-chunk framed or not) → everything
        :meth:`handle_batch` does. Returns the control events."""
        native = self.native
        log_events = self.log_events
        flags = (log_events, log_events and self.elog.enabled(logging.DEBUG))
        if flags != self._native_log:
            native.set_log(*flags)
            self._native_log = flags
        ctrl = self.native_result((native.feed_chunked if framed else native.feed)(data, read_ns), read_ns)
        self.notifier.flush()
        self.elog.flush()
        return ctrl

    def native_result(self, res: tuple, read_ns: int) -> List[tuple]:
        """What Python does with one native feed()'s result — the resume RV,
        log lines, asyncio-pool submissions — short of flushing (the reader
        hub's dispatch flushes once for all its streams: :meth:`flush_outputs`).
        Returns the control events."""
        ctrl, last_rv, logs, submits, ts = res
        if last_rv is not None:
            self.last_rv = last_rv
        if logs:
            elog = self.elog
            for level, msg in logs:
                elog.log(level, msg)
        if submits:
            submit = self.notifier.submit
            for uid, et, ns, name, core, ev_ts in submits:
                submit(uid, et, ns, name, core, read_ns, ev_ts)
        return ctrl

    def flush_outputs(self) -> None:
        """After the reader hub fed bound streams natively: the notifier's and
        the event log's flush, once, and the log flags the native side uses."""
        self.sync_native_log()
        self.notifier.flush()
        self.elog.flush()

    def shared_flush(self):
        """The part of :meth:`flush_outputs` every scope sharing this notifier
        and event log has in common — a closure over those two only, so the
        reader hub's per-notifier flush keeps no scope's pipeline alive."""
        notifier, elog = self.notifier, self.elog

        def flush() -> None:
            notifier.flush()
            elog.flush()
        return flush

    def log_flags_fn(self):
        """A function giving this pipeline's event-log switches (log_events,
        DEBUG on) now — a closure over the setting, the logger and the event
        log only, shared by every scope that has the same three (the reader
        hub evaluates it once per dispatch for all of them: net/reader.py)."""
        setting, log, elog = self.log_events_setting, self.log, self.elog

        def flags() -> tuple:
            on = setting if setting is not None else log.isEnabledFor(logging.INFO)
            return (on, on and elog.enabled(logging.DEBUG))
        return flags

    def sync_native_log(self, flags: Optional[tuple] = None) -> None:
        """Hand the event-log switches (log_events, DEBUG on) to the native side."""
        if flags is None:
            log_events = self.log_events
            flags = (log_events, log_events and self.elog.enabled(logging.DEBUG))
        if flags != self._native_log and self.native is not None:
            self.native.set_log(*flags)
            self._native_log = flags

    def native_slice(self, fn, budget_us: float, read_ns: int) -> Tuple[bool, List[tuple]]:
        """Run one slice of a native relist (``Relist.step`` / ``Relist.sweep``,
        ``ops/csrc/relist.inc``) and hand its log lines and (asyncio pool)
        submissions on, as :meth:`handle_raw` does. Returns ``(done, ctrl)``."""
        log_events = self.log_events
        flags = (log_events, log_events and self.elog.enabled(logging.DEBUG))
        if flags != self._native_log:
            self.native.set_log(*flags)
            self._native_log = flags
        done, ctrl, logs, submits = fn(budget_us, read_ns)
        elog = self.elog
        if logs:
            for level, msg in logs:
                elog.log(level, msg)
        if submits:
            submit = self.notifier.submit
            for uid, et, ns, name, core, ev_ts in submits:
                submit(uid, et, ns, name, core, read_ns, ev_ts)
        self.notifier.flush()
        elog.flush()
        return done, ctrl

    def delete_scope(self, scope_ns: str, read_ns: int) -> List[tuple]:
        """Notify every cached pod of namespace ``scope_ns`` as DELETED (from
        its cached payload) and forget it — what a relist that finds the
        namespace empty does. Synchronous: a namespace's leftovers are few."""
        if self.native is None:
            return self.reconcile([], read_ns, scope_ns=scope_ns)
        rl = self.native.relist(scope_ns, True)
        ctrl: List[tuple] = []
        done = False
        while not done:
            done, c = self.native_slice(rl.sweep, 1e9, read_ns)
            ctrl.extend(c)
        self.metrics.c["relist_deleted"] += rl.stats()["deleted"]
        return ctrl

    def handle_batch(self, events: List[tuple], read_ns: int) -> List[tuple]:
        """Process decoded events; returns control events (ERROR/INVALID) for the reflector."""
        ctrl: List[tuple] = []
        c = self.metrics.c
        observe = self.cache.observe
        set_core = self.cache.set_core
        critical = self.critical_active
        nsset = self.namespaces
        phase_mode = self.phase_mode
        elog = self.elog
        log_events = self.log_events
        log_debug = log_events and elog.enabled(logging.DEBUG)
        decoder = self.decoder
        submit = self.notifier.submit
        shard = self.shard if self.shard.active else None
        for ev in events:
            et = ev[E_TYPE]
            if et not in _POD_EVENTS:
                if et == BOOKMARK:
                    if ev[E_RV]:
                        self.last_rv = ev[E_RV]
                    c["bookmarks"] += 1
                else:
                    ctrl.append(ev)
                continue
            c["events_received"] += 1
            if shard is not None and not shard.owns(ev[E_UID], ev[E_NS]):
                if ev[E_RV]:
                    self.last_rv = ev[E_RV]
                c["events_other_shard"] += 1
                continue
            uid = ev[E_UID]
            rv = ev[E_RV]
            if rv:
                self.last_rv = rv
            phase = ev[E_PHASE]
            ns = ev[E_NS]
            name = ev[E_NAME]
            prev = observe(et, uid, rv, phase, ns, name)
            if critical and not (et == DELETED or not ev[E_HAS_STATUS] or phase in TERMINAL_PHASES):
                c["events_filtered_critical"] += 1
                continue
            if log_events:
                elog.log(logging.INFO, f"Pod event detected: {et} - {ns}/{name}")
            if nsset and ns not in nsset:
                if log_debug:
                    elog.log(logging.DEBUG, f"Skipping pod {ns}/{name} - not in target namespaces")
                c["events_filtered_namespace"] += 1
                continue
            if phase_mode and not (et == DELETED or prev is MISSING or prev != phase):
                c["events_unchanged"] += 1
                continue
            core = ev[E_EXTRA]
            if core is None:
                try:
                    core = decoder.core(ev)
                except ValueError as exc:  # e.g. a container state the library could not represent
                    ctrl.append((INVALID, None, None, None, None, None, False, None, f"{exc}"))
                    continue
            if et != DELETED:
                set_core(uid, core)
            # stamped per event as it is submitted (reference: at payload build, pod_watcher.py:199)
            submit(uid, et, ns, name, core, read_ns, event_timestamp(self.ts_mode))
        self.notifier.flush()
        elog.flush()
        return ctrl

    # ------------------------------------------------------------------ relist
    def reconcile(self, listed: List[tuple], read_ns: int, notify: bool = True,
                  scope_ns: Optional[str] = None) -> List[tuple]:
        """Diff a full LIST against the cache and run the resulting events.

        New uid → ADDED, changed resourceVersion → MODIFIED, cached uid absent
        from the list → DELETED (payload from the last cached core). With
        ``notify=False`` the cache is primed silently (``initial_list: skip``).
        ``scope_ns`` limits deletions to one namespace (server-side scopes).
        """
        cache = self.cache
        out: List[tuple] = []
        seen = set()
        for ev in listed:
            uid = ev[E_UID]
            seen.add(uid)
            ent = cache.get(uid)
            if ent is None:  # a WatchList's MODIFIED of an uncached pod is an ADDED too
                out.append(ev if ev[E_TYPE] == ADDED else (ADDED,) + ev[1:])
            elif ent[0] != ev[E_RV]:
                out.append((MODIFIED,) + ev[1:])
        for uid, ent in cache.items():
            if uid in seen or (scope_ns is not None and ent[NS] != scope_ns):
                continue
            core = ent[CORE]
            if core is None:
                core = self.decoder.core_from_summary(uid, ent[NS], ent[NAME], ent[PHASE])
            out.append((DELETED, uid, ent[NS], ent[NAME], ent[0], ent[PHASE], True, None, core))
        if not notify:
            for ev in out:
                uid = ev[E_UID]
                if self.shard.active and not self.shard.owns(uid, ev[E_NS]):
                    continue
                if ev[E_TYPE] == DELETED:
                    cache.pop(uid, None)
                else:
                    cache.put(uid, ev[E_RV], ev[E_PHASE], ev[E_NS], ev[E_NAME], None)
            return []
        saved_rv = self.last_rv
        ctrl = self.handle_batch(out, read_ns)
        self.last_rv = saved_rv  # the list RV, set by the caller, stays authoritative
        return ctrl
