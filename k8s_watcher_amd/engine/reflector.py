"""List-then-watch reflector with resume, bookmarks and 410 recovery.

Reference: ``self.watch.stream(self.v1.list_pod_for_all_namespaces)``
(``/root/reference/watcher/pod_watcher.py:264``). The library re-issues the
watch from the last seen resourceVersion when the server closes it, gives up
when it never saw one, and raises on the second 410 so the process exits and
Kubernetes restarts it, replaying every pod as ``ADDED``.

This reflector:

* LISTs (paginated, ``watcher.list_page_size``) and diffs the result against
  the pod cache (:meth:`EventPipeline.reconcile`) — on first start this turns
  every existing pod into ``ADDED``, the same thing the reference's watch
  without a resourceVersion produces;
* WATCHes from the list/last resourceVersion with ``allowWatchBookmarks`` and
  a server-side ``timeoutSeconds``; a normal server close resumes from the last
  resourceVersion with no relist;
* on ``410 Gone`` (HTTP status or ``ERROR`` event) relists and reconciles, so
  no state change is lost and unchanged pods are not re-notified;
* with ``watcher.initial_sync: watch_list`` gets the state as a WatchList
  stream (``sendInitialEvents``) instead of a LIST, falling back to LIST on
  API servers without it;
* on transport errors backs off per ``watcher.retry`` and gives up after
  ``max_attempts`` consecutive failures (0 = never), raising
  :class:`WatchFailed`; waits at least the server's ``Retry-After``, and a
  ``429`` (API Priority and Fairness throttling) is waited out without
  counting toward ``max_attempts``;
* pauses its socket while the notifier reports backpressure.
"""

from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Optional

from ..kube.api import ApiError, KubeApi
from ..metrics import Metrics
from ..net.http import HttpError
from ..ops.decode import ADDED, BOOKMARK, DELETED, E_EXTRA, E_RV, E_TYPE, E_UID, ERROR, INVALID, MODIFIED
from ..utils.backoff import Backoff
from ..utils.config import Settings
from ..utils.logsetup import SERVICE_LOGGER
from .pipeline import EventPipeline

# a watch that ends sooner than this without moving the resourceVersion is
# treated like client-go's "very short watch": back off before reconnecting
SHORT_WATCH_SECONDS = 1.0
# native engine: a relist applies its LIST in slices of this much loop time
# (the other scopes' watches and the notifier run between them)
RELIST_SLICE_MS = 4.0
# watch_list: an initial-events stream quiet this long without its
# initial-events-end bookmark falls back to LIST
WATCH_LIST_IDLE_SECONDS = 5.0

class Expired(Exception):
    """The watch resourceVersion is too old (410 Gone)."""


class WatchFailed(Exception):
    """Consecutive watch failures exhausted ``watcher.retry.max_attempts``."""


class WatchListUnsupported(Exception):
    """The API server refused ``sendInitialEvents`` or never ended the initial events."""


class Reflector:
    def __init__(self, api: KubeApi, settings: Settings, decoder, pipeline: EventPipeline,
                 metrics: Metrics, namespace: Optional[str] = None,
                 resource_version: Optional[str] = None, primed: bool = False,
                 list_gate: Optional[asyncio.Semaphore] = None) -> None:
        self.api = api
        self.settings = settings
        self.decoder = decoder
        self.pipeline = pipeline
        self.metrics = metrics
        self.namespace = namespace
        self._rv = resource_version
        self._rv_native = None  # the bound native pipeline's last_rv() while the hub feeds it directly
        self.primed = primed
        self.log = logging.getLogger(SERVICE_LOGGER)
        self.stream = None
        self._paused = False
        self._stop = asyncio.Event()
        self.connected = asyncio.Event()
        self.synced = asyncio.Event()
        self.watch_count = 0
        self.watch_list = settings.watcher.initial_sync == "watch_list"
        self.last_relist: Optional[dict] = None  # native relist stats (items, slices, max slice time)
        # shared by every scope of the service: at most watcher.relist_concurrency
        # LISTs in flight, so a compaction that expires every namespace watch at
        # once does not turn into a LIST storm on the API server (or the loop)
        self.list_gate = list_gate

    @property
    def rv(self) -> Optional[str]:
        """The resume point: the newest resourceVersion seen. While the reader
        hub feeds the watch to the native pipeline directly
        (``StreamResponse.bind_native``) no Python runs per read, so it is read
        from the pipeline."""
        get = self._rv_native
        if get is not None:
            v = get()
            if v is not None:
                return v
        return self._rv

    @rv.setter
    def rv(self, value: Optional[str]) -> None:
        self._rv = value
        if self._rv_native is not None:
            self.pipeline.native.set_last_rv(value)

    @property
    def scope(self) -> str:
        return self.namespace or "*"

    # ------------------------------------------------------------------ control
    def stop(self) -> None:
        self._stop.set()
        if self.stream is not None:
            self.stream.close()

    def set_paused(self, paused: bool) -> None:
        self._paused = paused
        s = self.stream
        if s is not None:
            s._proto.set_reading(not paused)

    # ------------------------------------------------------------------ list
    async def relist(self, notify: bool = True) -> None:
        if self.pipeline.native is not None:
            await self._relist_native(notify)
            return
        w = self.settings.watcher
        events = []
        cont = None
        list_rv = None
        limit: Optional[int] = w.list_page_size
        while True:
            try:
                body = await self.api.list_pods_raw(
                    namespace=self.namespace, limit=limit, continue_token=cont,
                    label_selector=w.label_selector, field_selector=w.field_selector)
            except ApiError as exc:
                if exc.status != 410 or cont is None:
                    raise
                # the continue token outlived etcd's compaction window (a large
                # cluster paged slowly): paging again would likely expire again,
                # so take the state in one unpaginated LIST, as client-go's
                # pager does (FullListIfExpired)
                self.metrics.c["list_continue_expired"] += 1
                self.log.warning("LIST continue token expired (410); retrying as one unpaginated LIST")
                events, cont, list_rv, limit = [], None, None, None
                continue
            page_rv, cont, evs = self.decoder.decode_list(body)
            if list_rv is None:
                list_rv = page_rv
            events.extend(evs)
            if not cont:
                break
        self.metrics.c["relists"] += 1
        read_ns = time.monotonic_ns()
        ctrl = self.pipeline.reconcile(events, read_ns, notify=notify,
                                       scope_ns=self.namespace if self._scoped() else None)
        for ev in ctrl:
            self._handle_control(ev)
        self.rv = list_rv
        self.pipeline.last_rv = list_rv
        self.synced.set()

    async def _relist_native(self, notify: bool) -> None:
        """LIST + reconcile in the native engine (``ops/csrc/relist.inc``).

        Each page is applied as it arrives, in slices of at most
        ``RELIST_SLICE_MS`` of loop time (the other scopes' watches and
        the notifier run between them): decode, compare with the cache and
        notify happen in C++ with no Python object per pod. After the last page
        the scope's cached pods the LIST lacked are notified DELETED, also in
        slices. A namespace scope touches only its namespace's cache entries."""
        w = self.settings.watcher
        pipe = self.pipeline
        rl = pipe.native.relist(self.namespace if self._scoped() else None, notify)
        budget_us = RELIST_SLICE_MS * 1000.0
        cont = None
        list_rv = None
        limit: Optional[int] = w.list_page_size
        t_busy = time.monotonic()
        while True:
            try:
                body = await self.api.list_pods_raw(
                    namespace=self.namespace, limit=limit, continue_token=cont,
                    label_selector=w.label_selector, field_selector=w.field_selector)
            except ApiError as exc:
                if exc.status != 410 or cont is None:
                    raise
                # as in relist(): one unpaginated LIST; what the earlier pages
                # applied stays (a consistent older state), their marks do not
                self.metrics.c["list_continue_expired"] += 1
                self.log.warning("LIST continue token expired (410); retrying as one unpaginated LIST")
                rl.restart()
                cont, list_rv, limit = None, None, None
                continue
            read_ns = time.monotonic_ns()
            rl.page(body)
            del body  # the Relist holds the page until its last item is applied
            while True:
                done, ctrl = pipe.native_slice(rl.step, budget_us, read_ns)
                for ev in ctrl:
                    self._handle_control(ev)
                if done:
                    break
                await asyncio.sleep(0)
            page_rv, cont = rl.page_meta()
            if list_rv is None:
                list_rv = page_rv
            if not cont:
                break
            await asyncio.sleep(0)
        read_ns = time.monotonic_ns()
        while True:
            done, ctrl = pipe.native_slice(rl.sweep, budget_us, read_ns)
            for ev in ctrl:
                self._handle_control(ev)
            if done:
                break
            await asyncio.sleep(0)
        st = rl.stats()
        c = self.metrics.c
        c["relists"] += 1
        c["relist_items"] += st["listed"]
        c["relist_unchanged"] += st["unchanged"]
        c["relist_deleted"] += st["deleted"]
        self.last_relist = dict(st, wall_s=time.monotonic() - t_busy, scope=self.scope)
        self.rv = list_rv
        pipe.last_rv = list_rv
        self.synced.set()

    async def sync(self, notify: bool = True) -> None:
        """Initial / post-410 state: WatchList when configured and supported, else LIST."""
        if self.list_gate is None:
            await self._sync(notify)
            return
        async with self.list_gate:
            await self._sync(notify)

    async def _sync(self, notify: bool) -> None:
        if self.watch_list:
            try:
                await self.watch_list_sync(notify)
                return
            except WatchListUnsupported as exc:
                self.watch_list = False  # do not ask again in this process
                self.log.warning(f"WatchList unavailable ({exc}); falling back to LIST")
        await self.relist(notify=notify)

    async def watch_list_sync(self, notify: bool = True) -> None:
        """Streamed initial state (``sendInitialEvents=true``, KEP-3157).

        The API server serves the current state from its watch cache as
        ``ADDED`` events and closes it with a bookmark annotated
        ``k8s.io/initial-events-end`` — no large LIST response has to be built
        server-side. The events are collected until that bookmark and then
        reconciled against the pod cache exactly like a LIST (unchanged pods
        are not re-notified, vanished ones become ``DELETED``); the stream is
        closed there and the regular watch resumes from the bookmark's
        resourceVersion.
        """
        w = self.settings.watcher
        decoder = self.decoder
        decoder.reset()
        state: dict = {}
        end: list = []
        framed = [False]
        errors: list = []
        pipe = self.pipeline
        native = pipe.native
        rl = wl = None
        t_busy = time.monotonic()
        if native is not None:
            # native: the initial events go into a Relist as they arrive, read
            # by read (ops/csrc/relist.inc, WatchList): no Python object per
            # pod and no whole-state reconcile at the end — only the sweep of
            # the cached pods the stream did not contain, in slices
            from ..ops.native import load
            wl = load().WatchList()
            rl = native.relist(self.namespace if self._scoped() else None, notify)

        def on_mode(is_framed: bool) -> None:
            framed[0] = is_framed

        # native: the sink only cuts each read into segments (C++, no Python
        # object per pod) and queues them; the coroutine below applies them in
        # RELIST_SLICE_MS slices with the loop free in between, and
        # the socket stops being read while more than this is queued
        queue: list = []  # [(segments, read_ns)]
        queued = [0]
        backlog_limit = max(8 << 20, 2 * (w.watch_read_bytes or (4 << 20)))
        wake = asyncio.Event()
        held = [False]
        stream_done = [False]

        def sink_native(data: bytes, read_ns: int) -> None:
            if stream_done[0]:
                return
            segs = wl.feed(data, framed[0])
            queue.append((segs, read_ns))
            for kind, payload in segs:
                if kind <= 1:
                    queued[0] += len(payload)
                elif kind in (2, 3):
                    stream_done[0] = True
            wake.set()
            if stream_done[0] and self.stream is not None:
                self.stream.close()
            elif queued[0] > backlog_limit and not held[0] and self.stream is not None:
                held[0] = True
                self.stream._proto.set_reading(False)

        async def apply_queued() -> None:
            budget_us = RELIST_SLICE_MS * 1000.0
            while queue and not end and not errors:
                segs, read_ns = queue.pop(0)
                for kind, payload in segs:
                    if kind == 0:  # ADDED / MODIFIED objects of one read: a Relist page
                        rl.page(payload)
                        while True:
                            done, ctrl = pipe.native_slice(rl.step, budget_us, read_ns)
                            for ev in ctrl:
                                self._handle_control(ev)
                            if done:
                                break
                            await asyncio.sleep(0)
                        queued[0] -= len(payload)
                    elif kind == 1:  # DELETED during the initial events: the watch path
                        # (cache-only when the sync does not notify, as the Relist's pages)
                        for ev in pipe.native_result(native.feed(payload, read_ns, not notify), read_ns):
                            self._handle_control(ev)
                        queued[0] -= len(payload)
                    elif kind == 2:
                        try:
                            errors.append(json.loads(payload) or {})
                        except ValueError:
                            errors.append({"message": "undecodable ERROR event"})
                    elif kind == 3:
                        end.append(payload)
                    else:
                        self.metrics.c["events_invalid"] += 1
                        self.log.warning(f"Skipping undecodable watch line (INVALID): {payload}")
                    if end or errors:
                        break
                if held[0] and queued[0] <= backlog_limit // 2 and self.stream is not None:
                    held[0] = False
                    if not self._paused:
                        self.stream._proto.set_reading(True)
                await asyncio.sleep(0)

        def sink(data: bytes, read_ns: int) -> None:
            if end or errors:
                return
            evs = decoder.feed_chunked(data) if framed[0] else decoder.feed(data)
            for ev in evs:
                t = ev[E_TYPE]
                if t == ADDED or t == MODIFIED:
                    state[ev[E_UID]] = ev
                elif t == DELETED:
                    state.pop(ev[E_UID], None)
                elif t == BOOKMARK:
                    if ev[E_EXTRA] is True:
                        end.append(ev[E_RV])
                        break
                elif t == ERROR:
                    errors.append(ev[E_EXTRA] or {})
                    break
                else:
                    self._handle_control(ev)
            if (end or errors) and self.stream is not None:
                self.stream.close()

        try:
            self.stream = await self.api.watch_pods(
                sink_native if wl is not None else sink, namespace=self.namespace, send_initial_events=True,
                label_selector=w.label_selector, field_selector=w.field_selector,
                raw_chunked=True, on_mode=on_mode)
        except ApiError as exc:
            # only the answers that mean "no such feature" downgrade to LIST for
            # good; 401 (token rotation), 403, 410 and 429 (APF throttling) go
            # to run() for credential refresh, relist and Retry-After handling
            if exc.status in (400, 404, 405, 415, 422, 501):
                raise WatchListUnsupported(str(exc)) from None
            raise
        try:
            finished = self.stream.finished
            idle = WATCH_LIST_IDLE_SECONDS
            if wl is not None:
                while not end and not errors and not self._stop.is_set():
                    if queue:
                        await apply_queued()
                        continue
                    if finished.done():
                        break
                    wake.clear()
                    waiter = asyncio.ensure_future(wake.wait())
                    await asyncio.wait([finished, waiter], timeout=min(1.0, idle),
                                       return_when=asyncio.FIRST_COMPLETED)
                    waiter.cancel()
                    if (not queue and not finished.done() and not end and not held[0]
                            and time.monotonic() - self.stream.last_activity > idle):
                        raise WatchListUnsupported(f"no initial-events-end bookmark after {idle}s idle")
            while not finished.done() and not end and not errors and not self._stop.is_set():
                await asyncio.wait([finished], timeout=min(1.0, idle))
                if (not finished.done() and not end
                        and time.monotonic() - self.stream.last_activity > idle):
                    # an API server that ignores sendInitialEvents streams the
                    # state and then goes quiet without the end marker
                    raise WatchListUnsupported(f"no initial-events-end bookmark after {idle}s idle")
        finally:
            if self.stream is not None:
                self.stream.close()
            self.stream = None
        if errors:
            st = errors[0]
            if st.get("code") == 410 or st.get("reason") in ("Expired", "Gone"):
                raise Expired()
            raise HttpError(f"watch-list ERROR event: {st.get('message') or st}")
        if not end:
            if self._stop.is_set():
                return
            raise HttpError("watch-list stream ended before the initial events were complete")
        read_ns = time.monotonic_ns()
        if rl is not None:
            # the scope's cached pods the initial events did not contain: DELETED, in slices
            budget_us = RELIST_SLICE_MS * 1000.0
            while True:
                done, ctrl = pipe.native_slice(rl.sweep, budget_us, read_ns)
                for ev in ctrl:
                    self._handle_control(ev)
                if done:
                    break
                await asyncio.sleep(0)
            st = rl.stats()
            c = self.metrics.c
            c["relist_items"] += st["listed"]
            c["relist_unchanged"] += st["unchanged"]
            c["relist_deleted"] += st["deleted"]
            self.last_relist = dict(st, wall_s=time.monotonic() - t_busy, scope=self.scope, watch_list=wl.stats())
        else:
            ctrl = self.pipeline.reconcile(list(state.values()), read_ns, notify=notify,
                                           scope_ns=self.namespace if self._scoped() else None)
            for ev in ctrl:
                self._handle_control(ev)
        # counted once the whole state is applied, sweep included (what waits on them sees a finished sync)
        self.metrics.c["relists"] += 1
        self.metrics.c["watch_list_syncs"] += 1
        self.rv = end[0]
        self.pipeline.last_rv = end[0]
        if native is not None:
            native.set_last_rv(end[0])
        self.synced.set()

    def _scoped(self) -> bool:
        return self.namespace is not None

    # ------------------------------------------------------------------ watch
    def _handle_control(self, ev: tuple) -> None:
        if ev[E_TYPE] != ERROR:  # INVALID line or an event type this watcher does not know
            self.metrics.c["events_invalid"] += 1
            self.log.warning(f"Skipping undecodable watch line ({ev[E_TYPE]}): {ev[E_EXTRA]}")
            return
        status = ev[E_EXTRA] or {}
        code = status.get("code")
        if code == 410 or status.get("reason") in ("Expired", "Gone"):
            self._expired = True
        else:
            self.log.warning(f"Watch ERROR event: {status.get('message') or status}")
            self._error = True
        if self.stream is not None:
            self.stream.close()

    async def watch_once(self) -> None:
        w = self.settings.watcher
        self.decoder.reset()
        self._expired = False
        self._error = False
        pipeline = self.pipeline
        decoder = self.decoder
        framed = [False]

        def on_mode(is_framed: bool) -> None:
            framed[0] = is_framed

        native = pipeline.native
        if native is not None:
            native.reset()

        def sink(data: bytes, read_ns: int) -> None:
            if native is not None:
                ctrl = pipeline.handle_raw(data, read_ns, framed[0])
                if pipeline.last_rv:
                    self.rv = pipeline.last_rv
                for ev in ctrl:
                    self._handle_control(ev)
                if framed[0] and native.body_done() and self.stream is not None:
                    self.stream.close()  # server ended the watch (timeoutSeconds)
                return
            if framed[0]:
                evs = decoder.feed_chunked(data)
                if decoder.body_done() and self.stream is not None:
                    self.stream.close()  # server ended the watch (timeoutSeconds)
            else:
                evs = decoder.feed(data)
            if evs:
                ctrl = pipeline.handle_batch(evs, read_ns)
                if pipeline.last_rv:
                    self.rv = pipeline.last_rv
                for ev in ctrl:
                    self._handle_control(ev)

        def on_native(res: tuple, read_ns: int, body_done: bool) -> None:
            for ev in pipeline.native_result(res, read_ns):
                self._handle_control(ev)
            if body_done and self.stream is not None:
                self.stream.close()  # server ended the watch (timeoutSeconds)

        pipeline.last_rv = self.rv
        if native is not None:
            native.set_last_rv(self.rv)
        self.stream = await self.api.watch_pods(
            sink, namespace=self.namespace, resource_version=self.rv,
            timeout_seconds=w.watch_timeout_seconds or None, allow_bookmarks=True,
            label_selector=w.label_selector, field_selector=w.field_selector,
            raw_chunked=True, on_mode=on_mode, read_size=w.watch_read_bytes,
            zero_copy=native is not None)  # the fused pipeline copies what it keeps (partial lines)
        self.watch_count += 1
        self.connected.set()
        if (native is not None and framed[0]
                and self.stream.bind_native(native, on_native, pipeline.shared_flush(),
                                            (id(pipeline.notifier), id(pipeline.elog)),
                                            sync=pipeline.sync_native_log,
                                            sync_group=((id(pipeline.elog), pipeline.log_events_setting),
                                                        pipeline.log_flags_fn()))):
            self._rv_native = native.last_rv
            pipeline.sync_native_log()
            self.metrics.c["watches_hub_dispatch"] += 1
        if self._stop.is_set():
            self.stream.close()
        if self._paused:
            self.set_paused(True)
        idle_limit = (w.watch_timeout_seconds or 300) + 60
        try:
            finished = self.stream.finished
            while not finished.done():
                # asyncio.wait (not wait_for): never swallows a cancellation on 3.10
                await asyncio.wait([finished], timeout=5.0)
                if (not finished.done() and not self._paused
                        and time.monotonic() - self.stream.last_activity > idle_limit):
                    self.log.warning("Watch stream idle for too long; reconnecting")
                    self.stream.close()
        finally:
            self.stream.close()
            self.stream = None
            if self._rv_native is not None:
                self._rv = self.rv
                self._rv_native = None
                pipeline.last_rv = self._rv
        if self._expired:
            raise Expired()
        if self._error:
            raise HttpError("watch ended with an ERROR event")

    async def run(self) -> None:
        w = self.settings.watcher
        backoff = Backoff(w.retry)
        # consecutive 410 → relist cycles in which the watch never got past the
        # relist's resourceVersion (a lagging watch cache, a relist RV that is
        # already compacted): each further relist waits longer, as client-go's
        # ListAndWatch backoff does, instead of LIST-storming the API server
        expired_backoff = Backoff(w.retry)
        relist_rv: Optional[str] = None
        need_list = self.rv is None
        first = not self.primed
        failures = 0
        while not self._stop.is_set():
            try:
                if need_list:
                    notify = not (first and w.initial_list == "skip")
                    await self.sync(notify=notify)
                    need_list = False
                    first = False
                    relist_rv = self.rv
                else:
                    self.synced.set()
                rv_before, t0 = self.rv, time.monotonic()
                await self.watch_once()
                if self._stop.is_set():
                    break
                self.metrics.c["watch_restarts"] += 1
                if self.rv != relist_rv:
                    expired_backoff.reset()
                if time.monotonic() - t0 < SHORT_WATCH_SECONDS and self.rv == rv_before:
                    # the server ended the watch at once with nothing in it
                    # (proxy or API server misbehaving): back off instead of
                    # reconnecting in a hot loop. Not a failure for
                    # max_attempts — the connection itself worked.
                    self.metrics.c["short_watches"] += 1
                    await self._sleep(backoff.next_delay())
                    continue
                failures = 0
                backoff.reset()
            except (Expired, ApiError) as exc:
                if isinstance(exc, ApiError) and exc.status != 410:
                    if exc.status == 401 and await self.api.endpoint.refresh_credentials():
                        # a rotated service-account token or an expired exec
                        # credential: the next attempt fetches a fresh one
                        self.metrics.c["auth_refreshes"] += 1
                        self.log.warning("API server answered 401; refreshing credentials")
                    if exc.status == 429:
                        # throttled by API Priority and Fairness: wait as asked but
                        # do not count it toward max_attempts — exiting and
                        # relisting would only add load to a busy API server
                        self.metrics.c["api_throttled"] += 1
                        await self._backoff(backoff, 0, exc)
                        continue
                    failures += 1
                    await self._backoff(backoff, failures, exc)
                    continue
                self.metrics.c["expired_410"] += 1
                failures = 0
                if relist_rv is not None and self.rv == relist_rv:
                    # expired again without a single event past the last relist
                    delay = expired_backoff.next_delay()
                    self.metrics.c["expired_relist_backoffs"] += 1
                    self.log.warning(f"Watch resourceVersion {self.rv} expired (410) again right after a "
                                     f"relist; relisting in {delay:.2f}s")
                    await self._sleep(delay)
                else:
                    self.log.warning(f"Watch resourceVersion {self.rv} expired (410); relisting")
                need_list = True
            except HttpError as exc:
                if self._stop.is_set():
                    break
                failures += 1
                await self._backoff(backoff, failures, exc)

    async def _backoff(self, backoff: Backoff, failures: int, exc: Exception) -> None:
        limit = self.settings.watcher.retry.max_attempts
        if limit and failures and failures >= limit:
            self.log.error(f"Error in Pod watcher: {exc}")
            raise WatchFailed(str(exc)) from exc
        delay = backoff.next_delay()
        retry_after = getattr(exc, "retry_after", None)
        if retry_after is not None:
            # the API server named its own wait (429 under API Priority and
            # Fairness, 503 while starting): honour it, never retry sooner
            delay = max(delay, retry_after)
            self.metrics.c["retry_after_waits"] += 1
        if failures:
            self.log.warning(f"Watch failed ({exc}); retry {failures}/{limit or 'inf'} in {delay:.2f}s")
        else:
            self.log.warning(f"Watch throttled ({exc}); retry in {delay:.2f}s")
        self.metrics.c["watch_restarts"] += 1
        await self._sleep(delay)

    async def _sleep(self, delay: float) -> None:
        """Sleep ``delay`` seconds or until :meth:`stop`."""
        waiter = asyncio.ensure_future(self._stop.wait())
        try:
            await asyncio.wait([waiter], timeout=delay)
        finally:
            waiter.cancel()
