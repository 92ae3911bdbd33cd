"""Asynchronous clusterapi notifier pool (SURVEY C11 + §7.1 step 5).

Reference: ``ClusterApiClient.update_pod_status`` does one blocking
``requests`` POST per event with no timeout and no retry, and counts only
HTTP 200 as success (``/root/reference/watcher/clusterapi_client.py:20-53``);
had it been enabled, every event would have stalled the watch stream for a
full round trip.

This pool keeps ``connections`` keep-alive HTTP/1.1 connections to
clusterapi, each carrying up to ``pipeline_depth`` requests in flight, all
driven from the event-loop thread:

* **Per-pod ordering** — a pod's notifications always use the same
  connection (``hash(uid) % connections``), whose requests are sent and
  answered in FIFO order; different pods proceed in parallel.
* **Monotonic delivery under failure** — a failed request is retried (after
  ``clusterapi.retry`` backoff) only while it is still the newest
  notification for its pod; once a newer one exists the stale one is dropped
  as *superseded*, so a retry can never overwrite newer state.
  Delivery is at-least-once.
* **Success** is any 2xx (reference: exactly 200). 408/429/5xx and transport
  errors are retried; other statuses fail at once.
* **Timeout** — ``clusterapi.timeout`` is enforced per request by a
  watchdog that aborts a connection whose oldest request is overdue.
* **Backpressure** — past ``queue_size`` outstanding requests the pool
  reports saturation and the watch reader pauses its socket until half
  the queue has drained; optional latest-state *coalescing* replaces a
  pod's not-yet-sent body instead of queueing another one.
"""

from __future__ import annotations

import asyncio
import collections
import logging
import time
import zlib
from typing import Callable, Deque, Dict, List, Optional
from urllib.parse import urlsplit

from ..metrics import Metrics
from ..models.payload import finish_body
from ..net.http import response_scanner
from ..net.sockopt import tune_socket
from ..utils.backoff import Backoff
from ..utils.config import ClusterApiSettings, RetryPolicy
from ..utils.fastlog import EventLog
from ..utils.logsetup import NOTIFIER_LOGGER, SERVICE_LOGGER
from ..utils.aio import with_timeout

RETRYABLE_STATUS = frozenset({408, 425, 429, 500, 502, 503, 504})


class NotifyRequest:
    __slots__ = ("uid", "seq", "etype", "ns", "name", "body", "read_ns", "attempts", "sent_ns", "conn")

    def __init__(self, uid, seq, etype, ns, name, body, read_ns, conn):
        self.uid = uid
        self.seq = seq
        self.etype = etype
        self.ns = ns
        self.name = name
        self.body = body
        self.read_ns = read_ns
        self.attempts = 0
        self.sent_ns = 0
        self.conn = conn


class _Conn(asyncio.Protocol):
    """One pooled connection. Requests are written in order; responses matched FIFO."""

    IDLE, CONNECTING, UP = range(3)

    def __init__(self, pool: "NotifierPool", index: int) -> None:
        self.pool = pool
        self.index = index
        self.state = self.IDLE
        self.transport: Optional[asyncio.Transport] = None
        self.queue: Deque[NotifyRequest] = collections.deque()
        self.inflight: Deque[NotifyRequest] = collections.deque()
        self.scanner = response_scanner(pool.native)
        self.connect_backoff = Backoff(RetryPolicy(1_000_000, 0.05, 2.0, 5.0, 0.2))
        self.reconnect_handle: Optional[asyncio.TimerHandle] = None

    # ------------------------------------------------------------- asyncio protocol
    def connection_made(self, transport) -> None:  # type: ignore[override]
        self.transport = transport
        tune_socket(transport.get_extra_info("socket"), self.pool.settings.tcp_keepalive_seconds)
        self.state = self.UP
        self.connect_backoff.reset()
        self.scanner.reset()
        self.pump()

    def data_received(self, data: bytes) -> None:  # type: ignore[override]
        try:
            results = self.scanner.feed(data)
        except ValueError as exc:  # protocol violation: drop the connection
            self.pool.log.error(f"Unexpected error calling clusterapi: {exc}")
            if self.transport is not None:
                self.transport.abort()
            return
        if results:
            inflight = self.inflight
            pool = self.pool
            for r in results:
                if not inflight:
                    break  # unsolicited response; ignore
                req = inflight.popleft()
                if r.__class__ is int:
                    pool._delivered(req)
                    continue
                status, keep_alive, body, retry_after = r
                if 200 <= status < 300:
                    pool._delivered(req)
                else:
                    pool._failed(req, status, body[:500].decode("utf-8", "replace"), retry_after)
                if not keep_alive and self.transport is not None:
                    self.transport.close()
                    pool.elog.flush()
                    return
            pool.elog.flush()
            # refill at the end of this loop tick: every response that arrived in
            # the same epoll round frees its slot first, so one write() carries
            # all the follow-up requests of this connection
            pool._defer_pump(self)

    def connection_lost(self, exc) -> None:  # type: ignore[override]
        self.transport = None
        self.state = self.IDLE
        failed = list(self.inflight)
        self.inflight.clear()
        reason = f"Connection error: Unable to connect to clusterapi at {self.pool.endpoint_url}"
        for req in failed:
            self.pool._failed(req, None, reason)
        if self.queue:
            self.schedule_connect()

    # ------------------------------------------------------------- internals
    def schedule_connect(self) -> None:
        if self.state != self.IDLE or self.reconnect_handle is not None or self.pool.closing:
            return
        delay = 0.0 if self.connect_backoff.attempt == 0 else self.connect_backoff.next_delay()
        if self.connect_backoff.attempt == 0:
            self.connect_backoff.attempt = 1
        self.reconnect_handle = self.pool.loop.call_later(delay, self._start_connect)

    def _start_connect(self) -> None:
        self.reconnect_handle = None
        if self.state != self.IDLE or self.pool.closing:
            return
        self.state = self.CONNECTING
        self.pool.loop.create_task(self._connect())

    async def _connect(self) -> None:
        pool = self.pool
        try:
            await with_timeout(
                pool.loop.create_connection(lambda: self, pool.host, pool.port, ssl=pool.ssl_context,
                                            server_hostname=pool.host if pool.ssl_context else None),
                pool.settings.timeout)
        except (OSError, asyncio.TimeoutError) as exc:
            self.state = self.IDLE
            failed = list(self.queue)
            self.queue.clear()
            for req in failed:
                req.attempts += 1  # a refused connection counts as an attempt
                pool._failed(req, None, f"Connection error: Unable to connect to clusterapi at "
                                        f"{pool.endpoint_url} ({exc.__class__.__name__})")
            if self.queue:
                self.schedule_connect()

    def pump(self) -> None:
        """Move queued requests onto the wire up to the pipeline depth."""
        if self.state != self.UP:
            if self.queue:
                self.schedule_connect()
            return
        depth = self.pool.depth
        inflight = self.inflight
        queue = self.queue
        if not queue or len(inflight) >= depth:
            return
        parts: List[bytes] = []
        now = time.monotonic_ns()
        head = self.pool.request_head
        unsent = self.pool.unsent
        pool = self.pool
        while queue and len(inflight) < depth:
            if pool.rl_qps and not pool._take_token(self):
                break  # rate limited: the pool re-pumps this connection when a token is due
            req = queue.popleft()
            if unsent.get(req.uid) is req:
                del unsent[req.uid]
            req.sent_ns = now
            req.attempts += 1
            inflight.append(req)
            parts.append(head)
            parts.append(str(len(req.body)).encode())
            parts.append(b"\r\n\r\n")
            parts.append(req.body)
        assert self.transport is not None
        self.transport.write(b"".join(parts))


class NotifierPool:
    """See module docstring. Create inside a running event loop."""

    def __init__(self, settings: ClusterApiSettings, metrics: Optional[Metrics] = None,
                 ts_mode: str = "local", log_events: bool = False, ssl_context=None,
                 on_saturation: Optional[Callable[[bool], None]] = None, native: Optional[bool] = None,
                 event_log: Optional[EventLog] = None) -> None:
        self.settings = settings
        if native is None:
            from ..ops.native import available
            native = available()
        self.native = native  # response framing in _kwcore.ResponseScanner
        self.metrics = metrics or Metrics()
        self.loop = asyncio.get_running_loop()
        self.log = logging.getLogger(NOTIFIER_LOGGER)
        self.svc_log = logging.getLogger(SERVICE_LOGGER)
        self.elog = event_log if event_log is not None else EventLog(self.svc_log)
        self.log_events = log_events
        self.ts_mode = ts_mode
        u = urlsplit(settings.base_url)
        self.host = u.hostname or "localhost"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        if u.scheme == "https" and ssl_context is None:
            import ssl
            ssl_context = ssl.create_default_context(cafile=settings.ca_file)
            if settings.cert_file:  # mutual TLS
                ssl_context.load_cert_chain(settings.cert_file, settings.key_file)
            if not settings.verify_tls:
                ssl_context.check_hostname = False
                ssl_context.verify_mode = ssl.CERT_NONE
        self.ssl_context = ssl_context if u.scheme == "https" else None
        path = (u.path.rstrip("/") + settings.pod_update) or "/"
        self.endpoint_url = settings.base_url + settings.pod_update
        default_port = 443 if u.scheme == "https" else 80
        host_hdr = self.host if self.port == default_port else f"{self.host}:{self.port}"
        head = (f"POST {path} HTTP/1.1\r\nHost: {host_hdr}\r\nContent-Type: application/json\r\n"
                f"User-Agent: k8s-watcher-amd/1.0\r\n")
        if settings.api_key:
            head += f"Authorization: Bearer {settings.api_key}\r\n"
        head += "Content-Length: "
        self.request_head = head.encode("latin-1")
        self.depth = settings.pool.pipeline_depth
        self.conns = [_Conn(self, i) for i in range(settings.pool.connections)]
        self.latest: Dict[str, int] = {}
        self.unsent: Dict[str, NotifyRequest] = {}
        self.seq = 0
        self.pending = 0
        self.pending_bytes = 0
        self.high_water = settings.pool.queue_size
        self.low_water = max(1, settings.pool.queue_size // 2)
        self.high_bytes = settings.pool.max_queued_bytes
        self.low_bytes = settings.pool.max_queued_bytes // 2
        self.saturated = False
        self.on_saturation = on_saturation
        self.closing = False
        self._idle_event = asyncio.Event()
        self._idle_event.set()
        self._dirty: List[_Conn] = []
        self._flush_scheduled = False
        self.retry_policy = settings.retry
        # clusterapi.rate_limit: token bucket over all connections
        self.rl_qps = settings.rate_limit_qps
        self.rl_burst = settings.rate_limit_burst
        self.rl_tokens = self.rl_burst
        self.rl_last = time.monotonic()
        self._throttled: List[_Conn] = []
        self._throttle_timer: Optional[asyncio.TimerHandle] = None
        # spool (parallel/spool.py): uid -> seq of the newest live submit, for uids with spooled records
        self.spool = None
        self.spool_watch: Dict[str, int] = {}
        self.replaying: Dict[int, NotifyRequest] = {}
        self.retrying: Dict[int, NotifyRequest] = {}
        self._watchdog = self.loop.create_task(self._watchdog_loop())

    # ------------------------------------------------------------------ spool
    def attach_spool(self, spool) -> None:
        """Owed notifications go to ``spool`` instead of being dropped."""
        self.spool = spool
        for uid in spool.uid_counts:
            self.spool_watch.setdefault(uid, 0)

    def detach_spool(self) -> None:
        """Stop spooling: what fails or is left at close is dropped again."""
        self.spool = None

    def replay(self, records) -> int:
        """Resubmit spooled records that are not stale; returns how many were submitted."""
        n = 0
        now = time.monotonic_ns()
        for r in records:
            if self.spool_watch.get(r.uid, 0) > r.seq:
                continue
            self.seq += 1
            conn = self.conns[zlib.crc32(r.uid.encode()) % len(self.conns)] if r.uid else self.conns[0]
            req = NotifyRequest(r.uid, self.seq, r.etype, r.ns, r.name, r.body, now, conn)
            self.latest[r.uid] = req.seq
            self.replaying[req.seq] = req
            conn.queue.append(req)
            self._dirty.append(conn)
            self.metrics.c["notify_submitted"] += 1
            self._add_pending(1, len(r.body))
            n += 1
        return n

    def replay_pending(self) -> int:
        return len(self.replaying)

    def spool_unwatch(self, uid: str) -> None:
        self.spool_watch.pop(uid, None)

    def _finish(self, req: NotifyRequest) -> None:
        if self.replaying:
            self.replaying.pop(req.seq, None)
        self._add_pending(-1, -len(req.body))

    # ------------------------------------------------------------------ public API
    def submit(self, uid: str, etype: str, ns: Optional[str], name: Optional[str], core: bytes,
               read_ns: int, ts: str) -> None:
        """Queue one notification; call :meth:`flush` once per batch to send."""
        body = finish_body(core, etype, ts)
        m = self.metrics.c
        m["notify_submitted"] += 1
        if self.spool_watch and uid in self.spool_watch:
            self.spool_watch[uid] = self.seq + 1  # the seq this submit gets (or coalesces into)
        if self.settings.pool.coalesce:
            old = self.unsent.get(uid)
            if old is not None:
                self._add_pending(0, len(body) - len(old.body))
                old.body = body
                old.etype = etype
                self.seq += 1
                old.seq = self.seq
                self.latest[uid] = old.seq
                old.read_ns = read_ns
                m["notify_coalesced"] += 1
                return
        self.seq += 1
        conn = self.conns[zlib.crc32(uid.encode()) % len(self.conns)] if uid else self.conns[0]
        req = NotifyRequest(uid, self.seq, etype, ns, name, body, read_ns, conn)
        self.latest[uid] = req.seq
        self.unsent[uid] = req
        conn.queue.append(req)
        if len(conn.queue) == 1 or conn.state != _Conn.UP:
            self._dirty.append(conn)
        self._add_pending(1, len(body))

    def _take_token(self, conn: "_Conn") -> bool:
        now = time.monotonic()
        self.rl_tokens = min(self.rl_burst, self.rl_tokens + (now - self.rl_last) * self.rl_qps)
        self.rl_last = now
        if self.rl_tokens >= 1.0:
            self.rl_tokens -= 1.0
            return True
        self._throttled.append(conn)
        if self._throttle_timer is None and not self.closing:
            self._throttle_timer = self.loop.call_later((1.0 - self.rl_tokens) / self.rl_qps, self._unthrottle)
        return False

    def _unthrottle(self) -> None:
        self._throttle_timer = None
        conns, self._throttled = self._throttled, []
        for c in dict.fromkeys(conns):
            c.pump()

    def flush(self) -> None:
        dirty = self._dirty
        if not dirty:
            return
        self._dirty = []
        for conn in dirty:
            conn.pump()

    def _defer_pump(self, conn: "_Conn") -> None:
        self._dirty.append(conn)
        if not self._flush_scheduled:
            self._flush_scheduled = True
            self.loop.call_soon(self._deferred_flush)

    def _deferred_flush(self) -> None:
        self._flush_scheduled = False
        self.flush()

    async def health_check(self, timeout: float = 5.0) -> bool:
        """``GET <health>``; True on 2xx (reference: ``clusterapi_client.py:55-61``)."""
        from ..net.http import HttpClient
        client = HttpClient(self.settings.base_url, self.ssl_context, timeout=timeout)
        try:
            resp = await client.request("GET", self.settings.health)
            return resp.ok
        except Exception:  # noqa: BLE001 - parity: any failure -> False
            return False
        finally:
            await client.close()

    async def warm_up(self, timeout: float = 2.0) -> int:
        """Open every pooled connection now, so the first events do not pay for TCP/TLS setup.

        Returns the number of connections up; failures are not errors (the
        pool reconnects on demand).
        """
        for c in self.conns:
            if c.state == _Conn.IDLE:
                c.schedule_connect()
        deadline = self.loop.time() + timeout
        while self.loop.time() < deadline and any(c.state != _Conn.UP for c in self.conns):
            if all(c.state == _Conn.IDLE and c.reconnect_handle is None for c in self.conns):
                break  # every attempt failed; do not wait out the timeout
            await asyncio.sleep(0.005)
        return sum(c.state == _Conn.UP for c in self.conns)

    async def drain(self, timeout: Optional[float] = None) -> bool:
        self.flush()
        try:
            await with_timeout(self._idle_event.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    async def close(self) -> None:
        self.closing = True
        self._watchdog.cancel()
        if self._throttle_timer is not None:
            self._throttle_timer.cancel()
        owed: List[NotifyRequest] = list(self.retrying.values())
        self.retrying.clear()
        for c in self.conns:
            if c.reconnect_handle is not None:
                c.reconnect_handle.cancel()
            owed.extend(c.inflight)
            owed.extend(c.queue)
            c.inflight.clear()
            c.queue.clear()
            if c.transport is not None:
                c.transport.close()
        for req in owed:  # still outstanding: fail (or spool) them, as the native core does
            self._give_up(req, spoolable=True)
        await asyncio.sleep(0)

    def outstanding(self) -> int:
        return self.pending

    def outstanding_bytes(self) -> int:
        return self.pending_bytes

    def pending_in(self, namespace: str) -> int:
        """Outstanding notifications (queued, in flight, retrying) for pods of ``namespace``."""
        n = sum(1 for r in self.retrying.values() if r.ns == namespace)
        for c in self.conns:
            n += sum(1 for r in c.inflight if r.ns == namespace) + sum(1 for r in c.queue if r.ns == namespace)
        return n

    # ------------------------------------------------------------------ bookkeeping
    def _add_pending(self, n: int, nbytes: int = 0) -> None:
        self.pending += n
        self.pending_bytes += nbytes
        if self.pending > 0:
            self._idle_event.clear()
        else:
            self._idle_event.set()
        if not self.saturated and (self.pending >= self.high_water or self.pending_bytes >= self.high_bytes):
            self.saturated = True
            if self.on_saturation:
                self.on_saturation(True)
        elif self.saturated and self.pending <= self.low_water and self.pending_bytes <= self.low_bytes:
            self.saturated = False
            if self.on_saturation:
                self.on_saturation(False)

    def _delivered(self, req: NotifyRequest) -> None:
        m = self.metrics
        m.c["notify_delivered"] += 1
        now = time.monotonic_ns()
        m.latency.observe_ns(now - req.read_ns)
        m.rtt.observe_ns(now - req.sent_ns)
        if self.latest.get(req.uid) == req.seq:
            del self.latest[req.uid]
        if self.log_events:
            self.elog.log(logging.INFO,
                          f"Successfully notified clusterapi about {req.etype} event for {req.ns}/{req.name}")
        self._finish(req)

    def _failed(self, req: NotifyRequest, status: Optional[int], detail: str,
                retry_after: float = -1.0) -> None:
        if status is not None:
            self.log.error(f"Failed to update pod data. Status: {status}, Response: {detail}")
        else:
            self.log.error(detail)
        retryable = status is None or status in RETRYABLE_STATUS
        if self.latest.get(req.uid) != req.seq:
            self.metrics.c["notify_superseded"] += 1
            self._finish(req)
            return
        if retryable and req.attempts < self.retry_policy.max_attempts and not self.closing:
            self.metrics.c["notify_retried"] += 1
            delay = self.retry_policy.delay(req.attempts)
            if retry_after > delay:  # clusterapi named its own wait (429/503): never retry sooner
                delay = retry_after
                self.metrics.c["notify_retry_after_waits"] += 1
            self.retrying[req.seq] = req
            self.loop.call_later(delay, self._retry_fire, req)
            return
        self._give_up(req, spoolable=retryable)

    def _give_up(self, req: NotifyRequest, spoolable: bool = False) -> None:
        if self.latest.get(req.uid) == req.seq:
            del self.latest[req.uid]
        if self.spool is not None and spoolable:
            self.metrics.c["notify_spooled"] += 1
            for uid in self.spool.append([(req.uid, req.etype, req.ns if req.ns is not None else "None",
                                           req.name if req.name is not None else "None", req.body, req.seq)]):
                self.spool_watch.setdefault(uid, 0)
        else:
            self.metrics.c["notify_failed"] += 1
            self.svc_log.error(f"Failed to notify clusterapi about {req.etype} event for {req.ns}/{req.name}")
        self._finish(req)

    def _retry_fire(self, req: NotifyRequest) -> None:
        if self.retrying.pop(req.seq, None) is None:
            return  # already given up (pool closed)
        if self.latest.get(req.uid) != req.seq:
            self.metrics.c["notify_superseded"] += 1
            self._finish(req)
            return
        if self.closing:
            self._give_up(req, spoolable=True)
            return
        conn = req.conn
        conn.queue.appendleft(req)
        conn.pump()

    async def _watchdog_loop(self) -> None:
        timeout_ns = int(self.settings.timeout * 1e9)
        period = max(0.05, min(1.0, self.settings.timeout / 4))
        while True:
            await asyncio.sleep(period)
            now = time.monotonic_ns()
            for c in self.conns:
                if c.inflight and now - c.inflight[0].sent_ns > timeout_ns and c.transport is not None:
                    self.log.error(f"Timeout error: Request to {self.endpoint_url} timed out")
                    c.transport.abort()


class NullNotifier:
    """Used when ``clusterapi.enabled: false``: payloads are built and counted, not sent.

    This is the reference as shipped (the POST is commented out,
    ``pod_watcher.py:236``).
    """

    def __init__(self, metrics: Optional[Metrics] = None) -> None:
        self.metrics = metrics or Metrics()
        self.saturated = False

    def submit(self, uid, etype, ns, name, core, read_ns, ts) -> None:
        finish_body(core, etype, ts)
        self.metrics.c["notify_submitted"] += 1
        self.metrics.c["notify_delivered"] += 1
        self.metrics.latency.observe_ns(time.monotonic_ns() - read_ns)

    def flush(self) -> None:
        pass

    async def health_check(self, timeout: float = 5.0) -> bool:
        return True

    async def drain(self, timeout: Optional[float] = None) -> bool:
        return True

    async def close(self) -> None:
        pass

    def outstanding(self) -> int:
        return 0

    def pending_in(self, namespace: str) -> int:
        return 0
