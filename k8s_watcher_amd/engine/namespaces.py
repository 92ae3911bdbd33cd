"""Namespace discovery for sharded all-namespace watching (``watcher.namespace_scope: discover``).

The reference watches every namespace through one cluster-wide stream and
filters client-side (``/root/reference/watcher/pod_watcher.py:226-229,264``),
so one process decodes every pod event of the cluster. With ``discover``
the watcher LISTs and WATCHes ``/api/v1/namespaces`` instead and opens one
pod watch per namespace *its shard owns* (``parallel/shard.py``): N shard
processes together still see every namespace — new ones as they appear — but
the API server sends each pod event to exactly one of them. The reference's
client-side filters (critical events, ``watcher.namespaces``) still run
unchanged on what each shard receives.

:class:`NamespaceWatcher` keeps the live namespace set and reports every
change through ``on_change(names)``; the service turns that into started and
stopped pod reflectors. It follows the reflector's resilience rules: resume
from the last resourceVersion, relist on 410, back off per ``watcher.retry``.
"""

from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Callable, Optional, Set

from ..kube.api import ApiError, KubeApi
from ..metrics import Metrics
from ..net.http import HttpError
from ..utils.backoff import Backoff
from ..utils.config import Settings
from ..utils.logsetup import SERVICE_LOGGER
from .reflector import Expired, WatchFailed


class NamespaceWatcher:
    def __init__(self, api: KubeApi, settings: Settings, metrics: Metrics,
                 on_change: Callable[[Set[str]], None]) -> None:
        self.api = api
        self.settings = settings
        self.metrics = metrics
        self.on_change = on_change
        self.log = logging.getLogger(SERVICE_LOGGER)
        self.names: Set[str] = set()
        self.rv: Optional[str] = None
        self.synced = asyncio.Event()
        self._stop = asyncio.Event()
        self.stream = None

    def stop(self) -> None:
        self._stop.set()
        if self.stream is not None:
            self.stream.close()

    def _set(self, names: Set[str]) -> None:
        if names != self.names:
            self.names = names
            self.metrics.c["namespace_changes"] += 1
            self.on_change(set(names))

    async def relist(self) -> None:
        names: Set[str] = set()
        cont = None
        rv = None
        while True:
            doc = await self.api.list_namespaces(limit=self.settings.watcher.list_page_size, continue_token=cont)
            md = doc.get("metadata") or {}
            if rv is None:
                rv = md.get("resourceVersion")
            for item in doc.get("items") or []:
                name = (item.get("metadata") or {}).get("name")
                if name:
                    names.add(name)
            cont = md.get("continue")
            if not cont:
                break
        self.rv = rv
        self._set(names)
        self.synced.set()

    async def watch_once(self) -> None:
        buf = bytearray()
        expired = []

        def sink(data: bytes, _read_ns: int) -> None:
            buf.extend(data)
            while not expired:
                i = buf.find(b"\n")
                if i < 0:
                    return
                line = bytes(buf[:i])
                del buf[:i + 1]
                if not line.strip():
                    continue
                try:
                    ev = json.loads(line)
                    etype = ev["type"]
                    obj = ev.get("object") or {}
                except (ValueError, KeyError, TypeError, AttributeError):
                    self.metrics.c["events_invalid"] += 1
                    continue
                md = obj.get("metadata") or {}
                if etype == "ERROR":
                    if obj.get("code") == 410 or obj.get("reason") in ("Expired", "Gone"):
                        expired.append(True)
                    else:
                        self.log.warning(f"Namespace watch ERROR event: {obj.get('message') or obj}")
                    if self.stream is not None:
                        self.stream.close()
                    return
                if md.get("resourceVersion"):
                    self.rv = md["resourceVersion"]
                name = md.get("name")
                if etype in ("ADDED", "MODIFIED") and name:
                    if name not in self.names:
                        self._set(self.names | {name})
                elif etype == "DELETED" and name in self.names:
                    self._set(self.names - {name})

        w = self.settings.watcher
        self.stream = await self.api.watch_namespaces(sink, resource_version=self.rv,
                                                      timeout_seconds=w.watch_timeout_seconds or None)
        if self._stop.is_set():
            self.stream.close()
        idle_limit = (w.watch_timeout_seconds or 300) + 60
        try:
            finished = self.stream.finished
            while not finished.done():
                await asyncio.wait([finished], timeout=5.0)
                if not finished.done() and time.monotonic() - self.stream.last_activity > idle_limit:
                    self.stream.close()
        finally:
            self.stream.close()
            self.stream = None
        if expired:
            raise Expired()

    async def run(self) -> None:
        w = self.settings.watcher
        backoff = Backoff(w.retry)
        need_list = True
        failures = 0
        while not self._stop.is_set():
            try:
                if need_list:
                    await self.relist()
                    need_list = False
                rv_before, t0 = self.rv, time.monotonic()
                await self.watch_once()
                if self._stop.is_set():
                    break
                if time.monotonic() - t0 < 1.0 and self.rv == rv_before:
                    await self._sleep(backoff.next_delay())  # watch ended at once: no hot loop
                    continue
                failures = 0
                backoff.reset()
            except Expired:
                need_list = True
                await self._sleep(backoff.next_delay())
            except (ApiError, HttpError) as exc:
                if self._stop.is_set():
                    break
                if isinstance(exc, ApiError) and exc.status == 410:
                    need_list = True
                    continue
                if isinstance(exc, ApiError) and exc.status == 401 and await self.api.endpoint.refresh_credentials():
                    self.metrics.c["auth_refreshes"] += 1
                throttled = isinstance(exc, ApiError) and exc.status == 429
                if not throttled:
                    failures += 1
                limit = w.retry.max_attempts
                if limit and failures >= limit:
                    self.log.error(f"Error in namespace watcher: {exc}")
                    raise WatchFailed(str(exc)) from exc
                delay = backoff.next_delay()
                ra = getattr(exc, "retry_after", None)
                if ra is not None:
                    delay = max(delay, ra)
                self.log.warning(f"Namespace watch failed ({exc}); retry in {delay:.2f}s")
                await self._sleep(delay)

    async def _sleep(self, delay: float) -> None:
        waiter = asyncio.ensure_future(self._stop.wait())
        try:
            await asyncio.wait([waiter], timeout=delay)
        finally:
            waiter.cancel()
