"""clusterapi notifier pool on the native core (``_kwcore.Notifier``).

Same contract and semantics as :class:`.notifier.NotifierPool` — per-pod
ordering on a ``crc32(uid)``-chosen connection, pipelined keep-alive
requests, any-2xx success, retries only while still the pod's newest
notification (else *superseded*), optional coalescing, per-request timeout,
backpressure — with the per-request work moved to C++ (``ops/csrc/engine.inc``):
request framing, the send buffers, ``send``/``recv`` on non-blocking sockets,
HTTP response framing, the in-flight windows and the retry decisions.

This wrapper owns the asyncio side only: it connects sockets
(``loop.sock_connect``) and hands their fds to the core, registers
``add_reader``/``add_writer`` callbacks that call straight into C++, turns
the core's retry decisions into ``call_later`` timers, writes the log lines
the core reports and feeds its latency samples into :class:`Metrics`.

For an ``https`` clusterapi the core also runs TLS (OpenSSL, non-blocking,
handshake driven by socket readiness; certificate and hostname/IP checks
per ``clusterapi.verify_tls`` / ``ca_file``), so the production profile's
https endpoint gets the same per-request path.
"""

from __future__ import annotations

import array
import asyncio
import logging
import os
import socket
import time
from typing import Callable, Dict, Optional
from urllib.parse import urlsplit

from ..metrics import _BUCKETS_NS, Metrics
from ..net.http import HttpClient
from ..net.sockopt import tune_socket
from ..ops.native import load
from ..utils.aio import with_timeout
from ..utils.backoff import Backoff
from ..utils.config import ClusterApiSettings, RetryPolicy
from ..utils.fastlog import EventLog
from ..utils.logsetup import NOTIFIER_LOGGER, SERVICE_LOGGER
from .notifier import RETRYABLE_STATUS


class NativeNotifierPool:
    # io_thread: auto — notifications/s above which the I/O thread takes the
    # sockets, below which they come back to the loop (measured:
    # profiles/io_thread_auto_gpu_box.md)
    IO_THREAD_ON_RATE = 50000.0
    IO_THREAD_OFF_RATE = 5000.0

    def __init__(self, settings: ClusterApiSettings, metrics: Optional[Metrics] = None,
                 ts_mode: str = "local", log_events: bool = False,
                 on_saturation: Optional[Callable[[bool], None]] = None,
                 event_log: Optional[EventLog] = None, **_ignored) -> None:
        u = urlsplit(settings.base_url)
        if u.scheme not in ("http", "https"):
            raise ValueError(f"unsupported clusterapi URL scheme in {settings.base_url!r}")
        self.tls = u.scheme == "https"
        self.settings = settings
        self.metrics = metrics or Metrics()
        self.loop = asyncio.get_running_loop()
        self.log = logging.getLogger(NOTIFIER_LOGGER)
        self.svc_log = logging.getLogger(SERVICE_LOGGER)
        self.elog = event_log if event_log is not None else EventLog(self.svc_log)
        self.log_events = log_events
        self.host = u.hostname or "localhost"
        default_port = 443 if self.tls else 80
        self.port = u.port or default_port
        self.endpoint_url = settings.base_url + settings.pod_update
        path = (u.path.rstrip("/") + settings.pod_update) or "/"
        host_hdr = self.host if self.port == default_port else f"{self.host}:{self.port}"
        head = (f"POST {path} HTTP/1.1\r\nHost: {host_hdr}\r\nContent-Type: application/json\r\n"
                f"User-Agent: k8s-watcher-amd/1.0\r\n")
        if settings.api_key:
            head += f"Authorization: Bearer {settings.api_key}\r\n"
        head += "Content-Length: "
        r = settings.retry
        self.core = load().Notifier(
            head.encode("latin-1"), settings.pool.connections, settings.pool.pipeline_depth, r.max_attempts,
            r.delay_seconds, r.multiplier, r.max_delay_seconds, settings.pool.coalesce, log_events,
            sorted(RETRYABLE_STATUS), self.metrics.c)
        if self.elog.native_sink is not None:
            self.core.set_log_sink(self.elog.native_sink)  # delivery lines formatted in C++
        # histograms accumulate in C++; raw samples only when the Metrics keep them (benchmarks)
        self.core.set_histograms(_BUCKETS_NS, self.metrics.record_samples)
        self.metrics.latency.add_source(lambda: self._hist(0))
        self.metrics.rtt.add_source(lambda: self._hist(1))
        if settings.rate_limit_qps > 0:
            self.core.set_rate_limit(settings.rate_limit_qps, settings.rate_limit_burst)
        self._throttle_timer: Optional[asyncio.TimerHandle] = None
        if self.tls:  # TLS runs inside the core (OpenSSL on the same non-blocking sockets)
            self.core.enable_tls(self.host, settings.ca_file, settings.verify_tls, settings.cert_file,
                                 settings.key_file)
        self.n = settings.pool.connections
        self.socks: Dict[int, socket.socket] = {}
        self.connecting: set = set()
        self.writers: set = set()
        self.backoff = [Backoff(RetryPolicy(1_000_000, 0.05, 2.0, 5.0, 0.2)) for _ in range(self.n)]
        self.reconnect: Dict[int, asyncio.TimerHandle] = {}
        self.addr = None
        self.high_water = settings.pool.queue_size
        self.low_water = max(1, settings.pool.queue_size // 2)
        self.high_bytes = settings.pool.max_queued_bytes
        self.low_bytes = settings.pool.max_queued_bytes // 2
        self.saturated = False
        self.on_saturation = on_saturation
        self.closing = False
        self.spool = None
        # clusterapi.pool.io_thread: the core serves the sockets on its own
        # thread (epoll) and signals this eventfd when Python has work to do
        self.threaded = settings.pool.io_thread == "on"
        self._py_fd = -1
        if self.threaded:
            self._py_fd = self.core.start_io()
            self.loop.add_reader(self._py_fd, self._on_io_signal)
        self._watchdog = self.loop.create_task(self._watchdog_loop())
        # io_thread: auto — the loop serves the sockets while notifications are
        # few (lowest latency: no cross-thread hand-off per request); above
        # IO_THREAD_ON_RATE the I/O thread takes them (the loop keeps its time
        # for decoding and applying events), below IO_THREAD_OFF_RATE they
        # come back (requests still in flight are answered on the loop). Sampled
        # every 100 ms; switching needs two samples in a row.
        self._auto = None
        if settings.pool.io_thread == "auto":
            self._auto = self.loop.create_task(self._auto_io_loop())

    # ------------------------------------------------------------------ spool (parallel/spool.py)
    def attach_spool(self, spool) -> None:
        """Owed notifications go to ``spool`` instead of being dropped."""
        self.spool = spool
        self.core.spool_control(True)
        for uid in spool.uid_counts:
            self.core.spool_watch(uid, True)

    def detach_spool(self) -> None:
        """Stop spooling: what fails or is left at close is dropped again."""
        self.spool = None
        self.core.spool_control(False)

    def replay(self, records) -> int:
        """Resubmit spooled records that are not stale; returns how many were submitted."""
        n = 0
        now = time.monotonic_ns()
        core = self.core
        for r in records:
            if core.spool_stale(r.uid, r.seq):
                continue
            core.submit_body(r.uid, r.etype, r.ns, r.name, r.body, now)
            n += 1
        return n

    def replay_pending(self) -> int:
        return self.core.replay_pending()

    def spool_unwatch(self, uid: str) -> None:
        self.core.spool_watch(uid, False)

    # ------------------------------------------------------------------ API (NotifierPool-compatible)
    def submit(self, uid, etype, ns, name, core: bytes, read_ns: int, ts: str) -> None:
        self.core.submit(uid, etype, ns, name, core, ts, read_ns)

    def flush(self) -> None:
        self.core.flush()
        self._after()

    def outstanding(self) -> int:
        return self.core.pending()

    def pending_in(self, namespace: str) -> int:
        """Outstanding notifications (queued, in flight, retrying) for pods of ``namespace``."""
        return self.core.pending_in(namespace)

    def outstanding_bytes(self) -> int:
        return self.core.pending_bytes()

    async def health_check(self, timeout: float = 5.0) -> bool:
        client = HttpClient(self.settings.base_url, self._health_ssl_context(), timeout=timeout)
        try:
            return (await client.request("GET", self.settings.health)).ok
        except Exception:  # noqa: BLE001 - parity: any failure -> False
            return False
        finally:
            await client.close()

    def _health_ssl_context(self):
        if not self.tls:
            return None
        import ssl
        ctx = ssl.create_default_context(cafile=self.settings.ca_file)
        if self.settings.cert_file:
            ctx.load_cert_chain(self.settings.cert_file, self.settings.key_file)
        if not self.settings.verify_tls:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        return ctx

    async def warm_up(self, timeout: float = 2.0) -> int:
        await asyncio.gather(*[self._connect(i) for i in range(self.n) if i not in self.socks],
                             return_exceptions=True)
        return len(self.socks)

    async def drain(self, timeout: Optional[float] = None) -> bool:
        self.flush()
        deadline = None if timeout is None else self.loop.time() + timeout
        while self.core.pending() > 0:
            if deadline is not None and self.loop.time() > deadline:
                self._after()
                return False
            await asyncio.sleep(0.001)
        self._after()  # counters, logs and samples of the last responses (I/O thread mode)
        return True

    async def close(self) -> None:
        self.closing = True
        self._watchdog.cancel()
        if self._auto is not None:
            self._auto.cancel()
        if self._throttle_timer is not None:
            self._throttle_timer.cancel()
        for h in self.reconnect.values():
            h.cancel()
        for i in list(self.socks):
            self.core.detach(i, "closing")  # deregisters the fd before the socket is closed
            self._drop_socket(i)
        self.core.give_up_all()
        self._after()
        if self.threaded:
            self.loop.remove_reader(self._py_fd)
            self.core.stop_io()
            self.threaded = False
        await asyncio.sleep(0)

    # ------------------------------------------------------------------ sockets
    async def _resolve(self):
        if self.addr is None:
            infos = await self.loop.getaddrinfo(self.host, self.port, type=socket.SOCK_STREAM)
            self.addr = infos[0]
        return self.addr

    async def _connect(self, i: int) -> None:
        if i in self.socks or i in self.connecting or self.closing:
            return
        self.connecting.add(i)
        sock = None
        try:
            family, stype, proto, _, sa = await self._resolve()
            sock = socket.socket(family, stype, proto)
            sock.setblocking(False)
            tune_socket(sock, self.settings.tcp_keepalive_seconds)
            await with_timeout(self.loop.sock_connect(sock, sa), self.settings.timeout)
        except (OSError, asyncio.TimeoutError) as exc:
            if sock is not None:
                sock.close()
            self.connecting.discard(i)
            self.core.connect_failed(i, f"Connection error: Unable to connect to clusterapi at "
                                        f"{self.endpoint_url} ({exc.__class__.__name__})")
            self._after(connect_failed=i)
            return
        self.connecting.discard(i)
        if self.closing:
            sock.close()
            return
        self.socks[i] = sock
        self.backoff[i].reset()
        self.core.attach(i, sock.fileno())
        if not self.threaded:
            self.loop.add_reader(sock.fileno(), self._readable, i)
        self.core.flush()
        self._after()

    def _schedule_connect(self, i: int, failed: bool = False) -> None:
        if i in self.socks or i in self.connecting or i in self.reconnect or self.closing:
            return
        delay = self.backoff[i].next_delay() if failed else 0.0

        def fire() -> None:
            self.reconnect.pop(i, None)
            self.loop.create_task(self._connect(i))

        self.reconnect[i] = self.loop.call_later(delay, fire)

    def _drop_socket(self, i: int) -> None:
        sock = self.socks.pop(i, None)
        if sock is None:
            return
        fd = sock.fileno()
        if not self.threaded:
            self.loop.remove_reader(fd)
        if i in self.writers:
            self.loop.remove_writer(fd)
            self.writers.discard(i)
        sock.close()

    def set_io_thread(self, on: bool) -> None:
        """Hand the sockets to the core's I/O thread (``on``) or back to the loop."""
        if on == self.threaded or self.closing:
            return
        if on:
            for sock in self.socks.values():
                self.loop.remove_reader(sock.fileno())
            for i in list(self.writers):
                sock = self.socks.get(i)
                if sock is not None:
                    self.loop.remove_writer(sock.fileno())
            self.writers.clear()
            self._py_fd = self.core.start_io()  # registers every attached socket with the thread
            self.loop.add_reader(self._py_fd, self._on_io_signal)
            self.threaded = True
            if self.saturated:  # the thread wakes us once the queue has drained enough
                self.core.signal_below(self.low_water, self.low_bytes)
        else:
            self.loop.remove_reader(self._py_fd)
            self.core.stop_io()  # joins the thread; sockets stay attached
            self._py_fd = -1
            self.threaded = False
            for i, sock in self.socks.items():
                self.loop.add_reader(sock.fileno(), self._readable, i)
        self.metrics.c["notify_io_switches"] += 1
        self._after()  # writers for unsent bytes, counters

    async def _auto_io_loop(self) -> None:
        on, off = self.IO_THREAD_ON_RATE, self.IO_THREAD_OFF_RATE
        period = 0.1
        c = self.metrics.c
        last = c["notify_submitted"]
        streak = 0
        while True:
            await asyncio.sleep(period)
            if self.threaded:
                self._after()  # counters the I/O thread has not signalled yet
            now = c["notify_submitted"]
            rate = (now - last) / period
            last = now
            want = rate >= on if not self.threaded else rate >= off
            streak = streak + 1 if want != self.threaded else 0
            if streak >= 2:
                streak = 0
                self.set_io_thread(want)

    # ------------------------------------------------------------------ loop callbacks
    def _on_io_signal(self) -> None:
        try:
            os.read(self._py_fd, 8)
        except BlockingIOError:
            pass
        self._after()

    def _readable(self, i: int) -> None:
        self.core.on_readable(i)
        self._after()

    def _writable(self, i: int) -> None:
        if not self.core.on_writable(i):
            sock = self.socks.get(i)
            if sock is not None:
                self.loop.remove_writer(sock.fileno())
            self.writers.discard(i)
        self._after()

    def _hist(self, which: int):
        h_lat, s_lat, h_rtt, s_rtt, n = self.core.histograms()
        return (array.array("Q", h_rtt if which else h_lat), s_rtt if which else s_lat, n)

    def _unthrottle(self) -> None:
        self._throttle_timer = None
        self.flush()

    def _requeue(self, seq: int) -> None:
        self.core.requeue(seq, self.closing)
        self._after()

    def _after(self, connect_failed: Optional[int] = None) -> None:
        retries, logs, need_connect, want_write, lost, lat, spooled, throttle = self.core.take()
        if throttle >= 0 and self._throttle_timer is None and not self.closing:
            self._throttle_timer = self.loop.call_later(throttle, self._unthrottle)
        if spooled and self.spool is not None:
            for uid in self.spool.append(spooled):
                self.core.spool_watch(uid, True)
        for i in lost:
            self._drop_socket(i)
        for seq, delay in retries:
            self.loop.call_later(delay, self._requeue, seq)
        if logs:
            elog = self.elog
            for level, msg in logs:
                if level == logging.INFO:
                    elog.log(level, msg)
                elif msg.startswith("Failed to notify"):
                    self.svc_log.error(msg)
                else:
                    self.log.error(msg)
            elog.flush()
        elif self.elog.native_sink is not None:
            self.elog.flush()  # delivery lines the core wrote into the native sink
        if lat:
            self.metrics.latency.add_samples(array.array("q", lat))
        for i in need_connect:
            self._schedule_connect(i, failed=(i == connect_failed))
        for i in want_write:
            sock = self.socks.get(i)
            if sock is not None and i not in self.writers:
                self.writers.add(i)
                self.loop.add_writer(sock.fileno(), self._writable, i)
        pending = self.core.pending()
        pbytes = self.core.pending_bytes()
        if not self.saturated and (pending >= self.high_water or pbytes >= self.high_bytes):
            self.saturated = True
            if self.threaded:  # the I/O thread wakes us when the queue has drained enough
                self.core.signal_below(self.low_water, self.low_bytes)
            if self.on_saturation:
                self.on_saturation(True)
        elif self.saturated and pending <= self.low_water and pbytes <= self.low_bytes:
            self.saturated = False
            if self.on_saturation:
                self.on_saturation(False)

    async def _watchdog_loop(self) -> None:
        timeout_ns = int(self.settings.timeout * 1e9)
        period = max(0.05, min(1.0, self.settings.timeout / 4))
        while True:
            await asyncio.sleep(period)
            for i in self.core.check_timeouts(timeout_ns):
                self.log.error(f"Timeout error: Request to {self.endpoint_url} timed out")
                self.core.detach(i, f"Timeout error: Request to {self.endpoint_url} timed out")
                self._drop_socket(i)
            self._after()
