"""Minimal asyncio HTTP/1.1 client used for every network link.

The reference delegates transport to ``kubernetes`` → urllib3 (watch stream)
and ``requests`` (clusterapi POST), both blocking. Here one
small ``asyncio.Protocol`` client serves both links so that

* the watch stream hands *raw de-chunked bytes plus their socket-read
  timestamp* straight to the event decoder (no line iterator, no model
  classes), and
* the notifier can keep many keep-alive connections busy from one thread.

Supported: keep-alive pooling, ``Content-Length`` / ``chunked`` /
read-until-close bodies, TLS through an ``ssl.SSLContext``, per-request
timeouts and streaming responses.
"""

from __future__ import annotations

import asyncio
import socket
import ssl as _ssl
import time
import zlib
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import urlencode, urlsplit
from ..utils.aio import with_timeout
from .sockopt import DEFAULT_KEEPALIVE_SECONDS, tune_socket


class HttpError(Exception):
    """Transport-level failure (connect, reset, protocol violation, timeout)."""


class HttpStatusError(HttpError):
    """Non-success HTTP status where the caller asked for one to raise."""

    def __init__(self, status: int, reason: str, body: bytes) -> None:
        super().__init__(f"HTTP {status} {reason}: {body[:300]!r}")
        self.status = status
        self.reason = reason
        self.body = body


class Response:
    __slots__ = ("status", "reason", "headers", "body")

    def __init__(self, status: int, reason: str, headers: Dict[str, str], body: bytes) -> None:
        self.status = status
        self.reason = reason
        self.headers = headers
        self.body = body

    @property
    def ok(self) -> bool:
        return 200 <= self.status < 300

    def text(self) -> str:
        return bytes(self.body).decode("utf-8", "replace")

    def json(self):
        import json
        return json.loads(json_input(self.body))


def json_input(body):
    """``body`` as something ``json.loads`` takes: a large body is an anonymous
    mapping (:func:`_body_buffer`), which it does not (only str, bytes and
    bytearray). The copy happens only for those bodies."""
    return body if isinstance(body, (bytes, bytearray, str)) else bytes(body)


def _body_buffer(n: int):
    """A writable buffer for an ``n``-byte body. Past a few MiB an anonymous
    mapping: its pages are zero-filled by the kernel as the socket reads touch
    them, where ``bytearray(n)`` zeroes all of them up front on the loop thread
    (275 ms for a 400 MB unpaginated LIST of 100k pods)."""
    if n >= (4 << 20):
        import mmap
        return mmap.mmap(-1, n)
    return bytearray(n)


class ResponseParser:
    """Incremental HTTP/1.1 response parser.

    ``feed(data)`` consumes bytes; body bytes go to ``on_body`` (if set) or are
    accumulated. ``on_head`` fires once the status line + headers are parsed;
    ``on_complete`` when the message is done. ``no_body`` must be set for
    responses to HEAD requests.
    """

    HEAD, LENGTH, CHUNK_SIZE, CHUNK_DATA, CHUNK_CRLF, TRAILER, UNTIL_CLOSE, DONE, RAW = range(9)
    DIRECT_MIN = 64 * 1024  # Content-Length bodies this large are read straight into one buffer

    def __init__(self) -> None:
        self.reset()

    def reset(self, no_body: bool = False, raw_chunked: bool = False) -> None:
        self.state = self.HEAD
        self.buf = bytearray()
        # a large Content-Length body (a LIST page): one buffer of that size,
        # filled in place — by feed() and, through direct_window(), by the
        # socket reads themselves — and returned whole by body(): no per-read
        # bytes objects and no final join
        self.direct: Optional[bytearray] = None
        self.direct_off = 0
        self.status = 0
        self.reason = ""
        self.headers: Dict[str, str] = {}
        self.remaining = 0
        self.body_parts: List[bytes] = []
        self.keep_alive = True
        self.no_body = no_body
        # raw_chunked: hand a 2xx chunked body to on_body *with* its chunk framing
        # (RAW state); the consumer de-chunks natively (``_kwcore``) and owns EOF.
        self.raw_chunked = raw_chunked
        self.chunked = False
        self.on_head: Optional[Callable[["ResponseParser"], None]] = None
        self.on_body: Optional[Callable[[bytes], None]] = None
        self.on_complete: Optional[Callable[["ResponseParser"], None]] = None

    # ------------------------------------------------------------------ helpers
    def _emit(self, data: bytes) -> None:
        if data:
            self.body_parts.append(data)

    def _flush_body(self) -> None:
        # One callback per feed(): all chunks that arrived in one socket read
        # reach the consumer together (the watch decoder batches on this).
        if self.on_body is not None and self.body_parts:
            parts = self.body_parts
            self.body_parts = []
            self.on_body(parts[0] if len(parts) == 1 else b"".join(parts))

    def body(self) -> bytes:
        if self.direct is not None:
            return self.direct  # type: ignore[return-value]  (a bytearray: json and the decoder take it)
        return b"".join(self.body_parts)

    def direct_window(self) -> Optional[memoryview]:
        """Where the next socket read of a direct body goes (None: not in one)."""
        if self.direct is None or self.state != self.LENGTH or self.buf:
            return None
        return memoryview(self.direct)[self.direct_off:]

    def direct_filled(self, n: int) -> None:
        """``n`` bytes were read into :meth:`direct_window`."""
        self.direct_off += n
        self.remaining -= n
        if self.remaining == 0:
            self._finish()

    def _finish(self) -> None:
        self._flush_body()
        self.state = self.DONE
        if self.on_complete is not None:
            self.on_complete(self)

    def _parse_head(self, head: bytes) -> None:
        lines = head.split(b"\r\n")
        status_line = lines[0].decode("latin-1")
        parts = status_line.split(" ", 2)
        if len(parts) < 2 or not parts[0].startswith("HTTP/"):
            raise HttpError(f"malformed status line {status_line!r}")
        version = parts[0]
        self.status = int(parts[1])
        self.reason = parts[2] if len(parts) > 2 else ""
        hdrs: Dict[str, str] = {}
        for raw in lines[1:]:
            if not raw:
                continue
            k, _, v = raw.decode("latin-1").partition(":")
            k = k.strip().lower()
            v = v.strip()
            if k in hdrs:
                hdrs[k] = hdrs[k] + ", " + v
            else:
                hdrs[k] = v
        self.headers = hdrs
        conn = hdrs.get("connection", "").lower()
        if version == "HTTP/1.0":
            self.keep_alive = "keep-alive" in conn
        else:
            self.keep_alive = "close" not in conn
        if self.no_body or self.status in (204, 304) or 100 <= self.status < 200:
            self.state = self.DONE
        elif "chunked" in hdrs.get("transfer-encoding", "").lower():
            self.chunked = True
            self.state = self.RAW if (self.raw_chunked and 200 <= self.status < 300) else self.CHUNK_SIZE
        elif "content-length" in hdrs:
            self.remaining = int(hdrs["content-length"])
            self.state = self.LENGTH if self.remaining > 0 else self.DONE
        else:
            self.state = self.UNTIL_CLOSE
            self.keep_alive = False

    # ------------------------------------------------------------------ feeding
    def feed(self, data: bytes) -> bytes:
        """Consume ``data``; returns bytes left over after a complete message."""
        if self.state == self.RAW and not self.buf:
            if self.on_body is not None:  # hot path: framed watch bytes straight through
                self.on_body(data)
            else:
                self.body_parts.append(data)
            return b""
        buf = self.buf
        buf += data
        pos = 0
        n = len(buf)
        while True:
            st = self.state
            if st == self.HEAD:
                idx = buf.find(b"\r\n\r\n", pos)
                if idx < 0:
                    break
                self._parse_head(bytes(buf[pos:idx]))
                pos = idx + 4
                if self.on_head is not None:
                    self.on_head(self)
                if self.state == self.LENGTH and self.on_body is None and self.remaining >= self.DIRECT_MIN:
                    self.direct = _body_buffer(self.remaining)
                if self.state == self.DONE:
                    self._finish()
                    break
            elif st == self.LENGTH:
                take = min(self.remaining, n - pos)
                if take <= 0:
                    break
                if self.direct is not None:
                    self.direct[self.direct_off:self.direct_off + take] = buf[pos:pos + take]
                    self.direct_off += take
                else:
                    self._emit(bytes(buf[pos:pos + take]))
                pos += take
                self.remaining -= take
                if self.remaining == 0:
                    self._finish()
                    break
            elif st == self.CHUNK_SIZE:
                idx = buf.find(b"\r\n", pos)
                if idx < 0:
                    break
                line = bytes(buf[pos:idx]).split(b";", 1)[0].strip()
                try:
                    size = int(line, 16)
                except ValueError:
                    raise HttpError(f"bad chunk size line {line!r}") from None
                pos = idx + 2
                if size == 0:
                    self.state = self.TRAILER
                else:
                    self.remaining = size
                    self.state = self.CHUNK_DATA
            elif st == self.CHUNK_DATA:
                take = min(self.remaining, n - pos)
                if take <= 0:
                    break
                self._emit(bytes(buf[pos:pos + take]))
                pos += take
                self.remaining -= take
                if self.remaining == 0:
                    self.state = self.CHUNK_CRLF
            elif st == self.CHUNK_CRLF:
                if n - pos < 2:
                    break
                pos += 2
                self.state = self.CHUNK_SIZE
            elif st == self.TRAILER:
                idx = buf.find(b"\r\n", pos)
                if idx < 0:
                    break
                empty = idx == pos
                pos = idx + 2
                if empty:
                    self._finish()
                    break
            elif st == self.UNTIL_CLOSE or st == self.RAW:
                if pos < n:
                    self._emit(bytes(buf[pos:]))
                    pos = n
                break
            else:  # DONE
                break
        self._flush_body()
        rest = b""
        if self.state == self.DONE:
            rest = bytes(buf[pos:])
            self.buf = bytearray()
        else:
            del buf[:pos]
        return rest

    def feed_eof(self) -> None:
        if self.state in (self.UNTIL_CLOSE, self.RAW):
            self._finish()
        elif self.state != self.DONE:
            raise HttpError("connection closed mid-response")


def parse_retry_after(value: Optional[str], cap: float = 300.0) -> Optional[float]:
    """``Retry-After: <delta-seconds>`` → float, capped at ``cap`` (HTTP-dates are ignored)."""
    if not value:
        return None
    try:
        secs = float(value.strip())
    except ValueError:
        return None
    if secs != secs or secs < 0:
        return None
    return min(secs, cap)


class PyResponseScanner:
    """Python twin of ``_kwcore.ResponseScanner`` (same results, used without the extension).

    ``feed(data)`` returns one item per complete response: the int status for
    a 2xx keep-alive response, else ``(status, keep_alive, body, retry_after)``
    with ``retry_after`` in seconds, ``-1.0`` without a ``Retry-After`` header.
    """

    def __init__(self) -> None:
        self.parser = ResponseParser()
        self._done: List[object] = []
        self._arm()

    def _arm(self) -> None:
        self.parser.reset()
        self.parser.on_complete = self._complete

    def _complete(self, p: ResponseParser) -> None:
        if 200 <= p.status < 300 and p.keep_alive:
            self._done.append(p.status)
        else:
            self._done.append((p.status, p.keep_alive, p.body(), _retry_after(p)))

    def reset(self) -> None:
        self._done = []
        self._arm()

    def feed(self, data: bytes) -> list:
        try:
            while data:
                data = self.parser.feed(data)
                if self.parser.state == ResponseParser.DONE:
                    self._arm()
        except HttpError as exc:
            raise ValueError(str(exc)) from None
        if self.parser.state == ResponseParser.UNTIL_CLOSE and self.parser.body_parts:
            p = self.parser
            self._done.append((p.status, False, p.body(), _retry_after(p)))
            self._arm()
        out, self._done = self._done, []
        return out


def _retry_after(p: "ResponseParser") -> float:
    ra = parse_retry_after(p.headers.get("retry-after"))
    return -1.0 if ra is None else ra


def response_scanner(native: bool = True):
    """``_kwcore.ResponseScanner`` when requested and built, else :class:`PyResponseScanner`."""
    if native:
        from ..ops.native import load
        return load().ResponseScanner()
    return PyResponseScanner()


_BUF_POOL: Dict[int, List[bytearray]] = {}
_BUF_POOL_BYTES = [0]
_BUF_POOL_CAP = 64 << 20


def _take_buf(n: int) -> bytearray:
    """A read buffer of ``n`` bytes: a recycled one if any. Allocating one of
    256 KiB - 4 MiB means an mmap, zeroed pages and an munmap later — ~0.6 ms
    of loop time per connection, which a 1,000-namespace relist storm paid
    thousands of times (benchmarks/relist_storm.py)."""
    free = _BUF_POOL.get(n)
    if free:
        _BUF_POOL_BYTES[0] -= n
        return free.pop()
    return bytearray(n)


def _give_buf(b: bytearray) -> None:
    if _BUF_POOL_BYTES[0] + len(b) <= _BUF_POOL_CAP:
        _BUF_POOL.setdefault(len(b), []).append(b)
        _BUF_POOL_BYTES[0] += len(b)


class _ClientProtocol(asyncio.BufferedProtocol):
    """One TCP/TLS connection; at most one outstanding request (no pipelining here).

    A buffered protocol: the transport ``recv_into``s a buffer owned here
    (``read_size`` bytes, reused). With ``zero_copy`` set (a stream whose sink
    does not keep the data past the call — the native watch pipeline), body
    bytes in RAW mode reach the sink as a ``memoryview`` of that buffer: no
    per-read allocation or copy on the event-loop thread. Everything else gets
    ``bytes`` as before.
    """

    read_size = 256 * 1024

    def __init__(self, loop: asyncio.AbstractEventLoop) -> None:
        self.loop = loop
        self._rbuf: Optional[bytearray] = None
        self._direct_read = False  # the last get_buffer handed out the parser's direct body window
        self._want = 65536  # read buffer size now (grows while reads fill it)
        self.zero_copy = False
        self.transport: Optional[asyncio.Transport] = None
        self.parser = ResponseParser()
        self.waiter: Optional[asyncio.Future] = None
        self.closed = loop.create_future()
        self.busy = False
        self.stream_sink: Optional[Callable[[bytes, int], None]] = None
        self.stream_head: Optional[asyncio.Future] = None
        self.last_activity = time.monotonic()
        self.read_stamp = 0
        self.hub = None  # net/reader.WatchReaderHub that reads this socket, once adopted
        self.hub_sid = 0
        self.hub_result: Optional[Callable[[tuple, int, bool], None]] = None  # bind_native
        self.hub_sync: Optional[Callable[[], None]] = None  # bind_native: the bound pipeline's log switches

    def deliver(self, data: bytes) -> None:
        """``parser.on_body`` for streams: body bytes + the socket-read timestamp."""
        sink = self.stream_sink
        if sink is not None:
            sink(data, self.read_stamp)

    # asyncio callbacks
    def connection_made(self, transport) -> None:  # type: ignore[override]
        self.transport = transport

    def get_buffer(self, sizehint: int):  # type: ignore[override]
        p = self.parser
        win = p.direct_window()
        if win is not None:  # a LIST page: read straight into its body buffer
            self._direct_read = True
            return win
        self._direct_read = False
        # 64 KiB until reads fill it, then 4x per full read up to read_size (a
        # watch's 4 MiB): a head — all a hub-read watch ever reads here — or a
        # short reply never allocates the big one
        want = min(self.read_size, self._want)
        b = self._rbuf
        if b is None or len(b) != want:
            if b is not None:
                _give_buf(b)
            b = self._rbuf = _take_buf(want)
        return b

    def buffer_updated(self, nbytes: int) -> None:  # type: ignore[override]
        p = self.parser
        if self._direct_read:
            now = time.monotonic_ns()
            self.read_stamp = now
            self.last_activity = now * 1e-9
            try:
                p.direct_filled(nbytes)
            except Exception as exc:  # noqa: BLE001
                self._fail(exc)
                if self.transport is not None:
                    self.transport.close()
            return
        if nbytes >= len(self._rbuf) and self._want < self.read_size:
            self._want *= 4  # the socket had more: read more per call from now on
        if self.zero_copy and p.state == ResponseParser.RAW and not p.buf and p.on_body is not None:
            now = time.monotonic_ns()
            self.read_stamp = now
            self.last_activity = now * 1e-9
            try:
                p.on_body(memoryview(self._rbuf)[:nbytes])
            except Exception as exc:  # noqa: BLE001
                self._fail(exc)
                if self.transport is not None:
                    self.transport.close()
            return
        self.data_received(bytes(memoryview(self._rbuf)[:nbytes]))

    def data_received(self, data: bytes) -> None:  # type: ignore[override]
        now = time.monotonic_ns()
        self.read_stamp = now
        self.last_activity = now * 1e-9
        try:
            self.parser.feed(data)
        except Exception as exc:  # noqa: BLE001
            self._fail(exc)
            if self.transport is not None:
                self.transport.close()

    # net/reader.WatchReaderHub callbacks (event-loop thread)
    def hub_data(self, view: memoryview, read_ns: int) -> None:
        self.read_stamp = read_ns
        self.last_activity = time.monotonic()
        p = self.parser
        try:
            if p.state == ResponseParser.RAW and not p.buf and p.on_body is not None:
                p.on_body(view)
            else:
                p.feed(bytes(view))
        except Exception as exc:  # noqa: BLE001
            self._fail(exc)
            self.close()

    def hub_native(self, result, read_ns: int, body_done: bool) -> None:
        """A read the hub fed to a bound native pipeline needs Python
        (:meth:`StreamResponse.bind_native`): ``result`` is the pipeline's
        feed() tuple, or the exception it raised."""
        self.read_stamp = read_ns
        if isinstance(result, BaseException):
            self._fail(result)
            self.close()
            return
        cb = self.hub_result
        if cb is not None:
            try:
                cb(result, read_ns, body_done)
            except Exception as exc:  # noqa: BLE001  (as a sink raising in hub_data)
                self._fail(exc)
                self.close()

    def hub_eof(self, err: int) -> None:
        """The hub saw the peer close (err 0) or the socket / TLS session fail:
        end the connection through the transport, as a read of EOF would."""
        why = self.hub.error_text(self.hub_sid) if err and self.hub is not None else ""
        self._unhub()
        if why:
            self._fail(HttpError(why))
        if self.transport is not None:
            self.transport.close()

    def _unhub(self) -> None:
        hub, self.hub = self.hub, None
        if hub is not None:
            hub.forget(self.hub_sid)

    def set_reading(self, on: bool) -> None:
        """Flow control for whoever reads the socket (the hub or asyncio)."""
        if self.hub is not None:
            self.hub.pause(self.hub_sid, not on)
        elif self.transport is not None and not self.transport.is_closing():
            if on:
                self.transport.resume_reading()
            else:
                self.transport.pause_reading()

    def connection_lost(self, exc) -> None:  # type: ignore[override]
        self._unhub()
        if self._rbuf is not None:  # up to watch_read_bytes (4 MiB): the next connection's
            _give_buf(self._rbuf)
            self._rbuf = None
        try:
            self.parser.feed_eof()
        except Exception as err:  # noqa: BLE001
            self._fail(err if exc is None else HttpError(str(exc)))
        if not self.closed.done():
            self.closed.set_result(None)
        self._fail(HttpError("connection closed"))

    def _fail(self, exc: BaseException) -> None:
        for fut in (self.stream_head, self.waiter):
            if fut is not None and not fut.done():
                fut.set_exception(exc if isinstance(exc, HttpError) else HttpError(repr(exc)))

    # request helpers
    def is_reusable(self) -> bool:
        return (self.transport is not None and not self.transport.is_closing()
                and not self.busy and self.parser.keep_alive)

    def close(self) -> None:
        self._unhub()  # the hub's dup of the socket goes first, or the peer never sees the close
        if self.transport is not None:
            self.transport.close()


def build_request(method: str, target: str, host_header: str, headers: Dict[str, str],
                  body: Optional[bytes]) -> bytes:
    lines = [f"{method} {target} HTTP/1.1", f"Host: {host_header}"]
    for k, v in headers.items():
        lines.append(f"{k}: {v}")
    if body is not None:
        lines.append(f"Content-Length: {len(body)}")
    head = ("\r\n".join(lines) + "\r\n\r\n").encode("latin-1")
    return head + body if body else head


class StreamResponse:
    """A response whose body is delivered incrementally to a sink callback."""

    def __init__(self, proto: _ClientProtocol, status: int, reason: str, headers: Dict[str, str]) -> None:
        self._proto = proto
        self.status = status
        self.reason = reason
        self.headers = headers

    @property
    def finished(self) -> "asyncio.Future":
        """Resolves when the server ends the body or the connection closes."""
        return self._proto.closed

    @property
    def last_activity(self) -> float:
        p = self._proto
        hub = getattr(p, "hub", None)
        if hub is not None and getattr(p, "hub_sid", None) is not None:
            # a hub-read stream: its reads are timed by the hub (bound ones
            # never pass through Python per read)
            return max(p.last_activity, hub.last_read(p.hub_sid))
        return p.last_activity

    def bind_native(self, pipeline_core, on_result, flush, flush_key, sync=None, sync_group=None) -> bool:
        """A hub-read watch body (net/reader.py) goes straight from the hub's
        buffers into the fused native ``pipeline_core`` — no Python call per
        socket read; ``on_result(result, read_ns, body_done)`` gets only the
        reads that need Python. False (nothing changed) when the stream is
        not hub-read or not at a clean pass-through point."""
        p = self._proto
        hub = p.hub
        parser = p.parser
        if (hub is None or parser.state != ResponseParser.RAW or parser.buf or p.stream_sink is None
                or p.closed.done()):
            return False
        hub.bind(p, pipeline_core, parser.raw_chunked, on_result, flush, flush_key, sync, sync_group)
        return p.hub_result is not None

    def close(self) -> None:
        self._proto.stream_sink = None
        self._proto.hub_result = None
        self._proto.hub_sync = None
        self._proto.close()


class HttpClient:
    """Pooled keep-alive HTTP/1.1 client for one origin (scheme://host:port)."""

    def __init__(self, base_url: str, ssl_context: Optional[_ssl.SSLContext] = None,
                 headers: Optional[Dict[str, str]] = None, timeout: float = 30.0,
                 header_provider: Optional[Callable[[], Dict[str, str]]] = None,
                 max_idle: int = 8, server_name: Optional[str] = None,
                 keepalive: float = DEFAULT_KEEPALIVE_SECONDS) -> None:
        u = urlsplit(base_url)
        if u.scheme not in ("http", "https"):
            raise ValueError(f"unsupported URL scheme in {base_url!r}")
        self.scheme = u.scheme
        self.host = u.hostname or "localhost"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.base_path = u.path.rstrip("/")
        default_port = 443 if u.scheme == "https" else 80
        self.host_header = self.host if self.port == default_port else f"{self.host}:{self.port}"
        if ":" in self.host and not self.host.startswith("["):  # IPv6 literal
            self.host_header = f"[{self.host}]" + ("" if self.port == default_port else f":{self.port}")
        if u.scheme == "https" and ssl_context is None:
            ssl_context = _ssl.create_default_context()
        self.ssl_context = ssl_context if u.scheme == "https" else None
        # SNI and certificate host name (kubeconfig ``tls-server-name``); the URL host otherwise
        self.server_name = server_name or self.host
        self.headers = dict(headers or {})
        self.header_provider = header_provider
        self.timeout = timeout
        self.max_idle = max_idle
        self.keepalive = keepalive  # TCP keep-alive / user timeout, seconds (net/sockopt.py)
        # net/reader.WatchReaderHub: zero-copy raw streams on plain TCP are read
        # by its native thread once their response head is in (None: asyncio)
        self.reader_hub = None
        self._idle: List[_ClientProtocol] = []
        self._all: List[_ClientProtocol] = []

    # ------------------------------------------------------------------ plumbing
    def url_target(self, path: str, query: Optional[Dict[str, object]] = None) -> str:
        target = self.base_path + path
        if query:
            q = {k: ("true" if v is True else "false" if v is False else v)
                 for k, v in query.items() if v is not None}
            if q:
                target += "?" + urlencode(q)
        return target

    def _merged_headers(self, extra: Optional[Dict[str, str]]) -> Dict[str, str]:
        h = dict(self.headers)
        if self.header_provider is not None:
            h.update(self.header_provider())
        if extra:
            h.update(extra)
        return h

    async def _connect(self, timeout: float) -> _ClientProtocol:
        loop = asyncio.get_running_loop()
        try:
            transport, proto = await with_timeout(
                loop.create_connection(lambda: _ClientProtocol(loop), self.host, self.port,
                                       ssl=self.ssl_context,
                                       server_hostname=self.server_name if self.ssl_context else None),
                timeout)
        except asyncio.TimeoutError:
            raise HttpError(f"connect to {self.host}:{self.port} timed out") from None
        except OSError as exc:
            raise HttpError(f"connect to {self.host}:{self.port} failed: {exc}") from None
        tune_socket(transport.get_extra_info("socket"), self.keepalive)
        self._all.append(proto)
        # a closed connection leaves the client's books, whoever closed it (a
        # watch ending, the server hanging up an idle keep-alive socket): every
        # watch reconnect used to leave its protocol — and read buffer — here
        proto.closed.add_done_callback(lambda _f, p=proto: self._forget(p))
        return proto

    async def _connect_for_hub(self, timeout: float):
        """A connected plain socket and a protocol whose transport is a
        :class:`~.reader.HubTransport`, for :meth:`WatchReaderHub.open_tls`."""
        from .reader import HubTransport
        loop = asyncio.get_running_loop()
        sock = None
        try:
            infos = await with_timeout(loop.getaddrinfo(self.host, self.port, type=socket.SOCK_STREAM), timeout)
            family, stype, proto_num, _, addr = infos[0]
            sock = socket.socket(family, stype, proto_num)
            sock.setblocking(False)
            await with_timeout(loop.sock_connect(sock, addr), timeout)
        except asyncio.TimeoutError:
            if sock is not None:
                sock.close()
            raise HttpError(f"connect to {self.host}:{self.port} timed out") from None
        except OSError as exc:
            if sock is not None:
                sock.close()
            raise HttpError(f"connect to {self.host}:{self.port} failed: {exc}") from None
        tune_socket(sock, self.keepalive)
        proto = _ClientProtocol(loop)
        proto.connection_made(HubTransport(loop, proto, self.ssl_context))
        self._all.append(proto)
        proto.closed.add_done_callback(lambda _f, p=proto: self._forget(p))
        return proto, sock

    async def _acquire(self, timeout: float) -> _ClientProtocol:
        while self._idle:
            proto = self._idle.pop()
            if proto.is_reusable():
                return proto
        return await self._connect(timeout)

    def _release(self, proto: _ClientProtocol) -> None:
        proto.busy = False
        if proto.is_reusable() and len(self._idle) < self.max_idle:
            self._idle.append(proto)
        else:
            proto.close()
            self._forget(proto)

    def _forget(self, proto: _ClientProtocol) -> None:
        for group in (self._all, self._idle):
            try:
                group.remove(proto)
            except ValueError:
                pass

    # ------------------------------------------------------------------ API
    async def request(self, method: str, path: str, query: Optional[Dict[str, object]] = None,
                      headers: Optional[Dict[str, str]] = None, body: Optional[bytes] = None,
                      timeout: Optional[float] = None) -> Response:
        tmo = self.timeout if timeout is None else timeout
        target = self.url_target(path, query)
        raw = build_request(method, target, self.host_header, self._merged_headers(headers), body)
        for attempt in (0, 1):
            proto = await self._acquire(tmo)
            reused = attempt == 0 and proto in self._all and proto.parser.state == ResponseParser.DONE
            loop = asyncio.get_running_loop()
            proto.busy = True
            proto.parser.reset(no_body=(method == "HEAD"))
            fut = loop.create_future()
            proto.waiter = fut
            proto.stream_sink = None

            def _done(p: ResponseParser, f=fut) -> None:
                if not f.done():
                    body = p.body()
                    if body and p.headers.get("content-encoding", "").lower() == "gzip":
                        try:
                            body = zlib.decompress(body, 16 + zlib.MAX_WBITS)
                        except zlib.error as exc:
                            f.set_exception(HttpError(f"bad gzip response body: {exc}"))
                            return
                    f.set_result(Response(p.status, p.reason, p.headers, body))

            proto.parser.on_complete = _done
            assert proto.transport is not None
            proto.transport.write(raw)
            try:
                resp = await with_timeout(fut, tmo)
            except asyncio.TimeoutError:
                proto.close()
                self._forget(proto)
                raise HttpError(f"{method} {target} timed out after {tmo}s") from None
            except HttpError:
                proto.close()
                self._forget(proto)
                if reused and method in ("GET", "HEAD"):
                    continue  # stale keep-alive socket: retry once on a fresh one
                raise
            self._release(proto)
            return resp
        raise HttpError("unreachable")

    async def stream(self, method: str, path: str, sink: Callable[[bytes, int], None],
                     query: Optional[Dict[str, object]] = None,
                     headers: Optional[Dict[str, str]] = None,
                     timeout: Optional[float] = None, raw_chunked: bool = False,
                     on_mode: Optional[Callable[[bool], None]] = None,
                     read_size: int = 0, zero_copy: bool = False) -> Tuple[StreamResponse, Optional[bytes]]:
        """Start a request whose body is streamed to ``sink(data, read_ns)``.

        With ``raw_chunked`` a 2xx chunked body is passed through *with* its
        chunk framing; ``on_mode(framed)`` is called once, before any body
        byte, to tell the consumer which form it will receive.

        Returns ``(stream, error_body)``: for a non-2xx status the whole body
        is read and returned as ``error_body`` and the connection is closed.

        ``read_size`` raises the bytes taken per socket read (default 256
        KiB): a busy watch then costs fewer event-loop iterations and fewer
        decoder calls per event. ``zero_copy`` hands RAW body bytes to
        ``sink`` as a ``memoryview`` of the protocol's reused read buffer; the
        sink must not keep it past the call.
        """
        tmo = self.timeout if timeout is None else timeout
        target = self.url_target(path, query)
        raw = build_request(method, target, self.host_header, self._merged_headers(headers), None)
        hub = self.reader_hub
        material = getattr(self.ssl_context, "kw_tls", None) if self.ssl_context is not None else None
        hub_tls = hub is not None and zero_copy and raw_chunked and material is not None
        sock = None
        if hub_tls:
            # https watch: the reader hub owns the connection from the start
            # (handshake, request, decryption on its thread; net/reader.py)
            proto, sock = await self._connect_for_hub(tmo)
        else:
            proto = await self._connect(tmo)
        if read_size > 0 and not hub_tls:
            proto.read_size = read_size  # plain TCP: recv_into this many bytes per readiness event
            if hasattr(proto.transport, "max_size"):
                proto.transport.max_size = read_size
        proto.zero_copy = zero_copy
        loop = asyncio.get_running_loop()
        proto.busy = True
        head_fut = loop.create_future()
        proto.stream_head = head_fut
        parser = proto.parser
        parser.reset(raw_chunked=raw_chunked)
        err_parts: List[bytes] = []

        def _on_head(p: ResponseParser) -> None:
            if not (200 <= p.status < 300):
                proto.stream_sink = None
                p.on_body = err_parts.append
                p.on_complete = lambda _p: (not head_fut.done()) and head_fut.set_result(False)
                return
            if on_mode is not None:
                on_mode(p.state == ResponseParser.RAW)
            p.on_body = proto.deliver
            if not head_fut.done():
                head_fut.set_result(True)

        def _on_complete(_p: ResponseParser) -> None:
            proto.close()

        parser.on_head = _on_head
        parser.on_complete = _on_complete
        proto.stream_sink = sink
        assert proto.transport is not None
        if hub_tls:
            try:
                hub.open_tls(proto, sock, material, self.server_name, raw)
            except OSError as exc:
                proto.close()
                self._forget(proto)
                raise HttpError(f"TLS setup for {self.host}:{self.port} failed: {exc}") from None
        else:
            proto.transport.write(raw)
        try:
            good = await with_timeout(head_fut, tmo)
        except asyncio.TimeoutError:
            proto.close()
            self._forget(proto)
            raise HttpError(f"{method} {target}: no response head within {tmo}s") from None
        except HttpError:
            proto.close()
            self._forget(proto)
            raise
        sr = StreamResponse(proto, parser.status, parser.reason, parser.headers)
        if not good:
            proto.close()
            self._forget(proto)
            return sr, b"".join(err_parts)
        if (hub is not None and not hub_tls and zero_copy and parser.state == ResponseParser.RAW
                and self.ssl_context is None and not proto.closed.done()):
            hub.adopt(proto)
        return sr, None

    async def close(self) -> None:
        for proto in list(self._all):
            proto.close()
        self._all.clear()
        self._idle.clear()
        await asyncio.sleep(0)
