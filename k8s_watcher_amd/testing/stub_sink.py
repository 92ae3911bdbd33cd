"""Stub clusterapi sink (the receiving end of ``POST /api/pods/update``).

The reference ships no clusterapi stub. This one:

* answers ``POST <pod_update>`` (default ``/api/pods/update``) and
  ``GET /health``; keep-alive and HTTP/1.1 pipelining are supported, with
  responses kept in request order per connection;
* records bodies (``record=True``) with their receive time so tests can
  check schema, per-pod order and exactly-once delivery;
* injects latency (fixed seconds) and failures (a status for a fraction of
  requests, or for the next N requests, or an outage with ``state.down``);
* is a raw ``asyncio.Protocol`` so that, in benchmarks, it is not the
  bottleneck; :func:`run_sink_process` runs several SO_REUSEPORT workers.
"""

from __future__ import annotations

import argparse
import asyncio
import collections
import json
import os
import random
import socket
import time
from typing import Deque, Dict, List, Optional, Tuple
from ..utils.aio import with_timeout

_OK = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: 15\r\n\r\n{\"status\":\"ok\"}"


def _resp(status: int, body: bytes = b"{}", retry_after: Optional[float] = None) -> bytes:
    reason = {200: "OK", 201: "Created", 204: "No Content", 400: "Bad Request", 404: "Not Found",
              429: "Too Many Requests", 500: "Internal Server Error",
              503: "Service Unavailable"}.get(status, "Status")
    if status == 204:
        return b"HTTP/1.1 204 No Content\r\n\r\n"
    extra = b"" if retry_after is None else b"Retry-After: %s\r\n" % f"{retry_after:g}".encode()
    return b"HTTP/1.1 %d %s\r\nContent-Type: application/json\r\n%sContent-Length: %d\r\n\r\n%s" % (
        status, reason.encode(), extra, len(body), body)


class SinkState:
    def __init__(self, path: str = "/api/pods/update", record: bool = True, latency: float = 0.0,
                 fail_rate: float = 0.0, fail_status: int = 500, success_status: int = 200,
                 seed: int = 0) -> None:
        self.path = path.encode()
        self.record = record
        self.latency = latency
        self.fail_rate = fail_rate
        self.fail_status = fail_status
        self.success_status = success_status
        self.fail_next: List[int] = []
        self.retry_after: Optional[float] = None  # Retry-After header on injected failures
        self.rng = random.Random(seed)
        self.received: List[Tuple[int, bytes]] = []
        self.heads: List[bytes] = []
        self.count = 0
        self.failed = 0
        self.health_checks = 0
        self.connections = 0
        self.waiters: List[Tuple[int, asyncio.Future]] = []
        self.down = False  # outage: /health and every POST answer 503

    def payloads(self) -> List[Dict]:
        return [json.loads(b) for _, b in self.received]

    def note(self, body: bytes) -> None:
        """Hook for every accepted payload (see ``_VerifyingState``)."""

    def _notify_waiters(self) -> None:
        if not self.waiters:
            return
        keep = []
        for n, fut in self.waiters:
            if self.count >= n and not fut.done():
                fut.set_result(self.count)
            elif not fut.done():
                keep.append((n, fut))
        self.waiters = keep

    async def wait_for(self, n: int, timeout: float = 10.0) -> int:
        if self.count >= n:
            return self.count
        fut = asyncio.get_running_loop().create_future()
        self.waiters.append((n, fut))
        return await with_timeout(fut, timeout)


class _SinkProtocol(asyncio.Protocol):
    def __init__(self, state: SinkState) -> None:
        self.st = state
        self.buf = bytearray()
        self.transport: Optional[asyncio.Transport] = None
        self.out: Deque[List] = collections.deque()  # [ready, bytes]

    def connection_made(self, transport) -> None:  # type: ignore[override]
        self.transport = transport
        self.st.connections += 1

    def data_received(self, data: bytes) -> None:  # type: ignore[override]
        buf = self.buf
        buf += data
        st = self.st
        pos = 0
        responses: List[bytes] = []
        now = time.monotonic_ns()
        while True:
            he = buf.find(b"\r\n\r\n", pos)
            if he < 0:
                break
            head = bytes(buf[pos:he])
            cl = 0
            i = head.lower().find(b"content-length:")
            if i >= 0:
                j = head.find(b"\r\n", i)
                cl = int(head[i + 15:j if j >= 0 else len(head)].strip())
            if len(buf) - (he + 4) < cl:
                break
            body = bytes(buf[he + 4:he + 4 + cl])
            pos = he + 4 + cl
            sp1 = head.find(b" ")
            sp2 = head.find(b" ", sp1 + 1)
            method, path = head[:sp1], head[sp1 + 1:sp2]
            if method == b"GET" and path.startswith(b"/health"):
                st.health_checks += 1
                responses.append(_resp(503, b'{"status":"down"}') if st.down
                                 else _resp(200, b'{"status":"healthy"}'))
                continue
            if method != b"POST" or path != st.path:
                responses.append(_resp(404, b'{"error":"not found"}'))
                continue
            fail = None
            if st.down:
                fail = 503
            elif st.fail_next:
                fail = st.fail_next.pop(0)
            elif st.fail_rate and st.rng.random() < st.fail_rate:
                fail = st.fail_status
            if fail is not None:
                st.failed += 1
                responses.append(_resp(fail, b'{"error":"injected"}', st.retry_after))
                continue
            st.count += 1
            st.note(body)
            if st.record:
                st.received.append((now, body))
                st.heads.append(head)
            responses.append(_OK if st.success_status == 200 else _resp(st.success_status))
        if pos:
            del buf[:pos]
        if responses:
            st._notify_waiters()
            payload = b"".join(responses)
            if st.latency > 0:
                item = [False, payload]
                self.out.append(item)
                asyncio.get_running_loop().call_later(st.latency, self._release, item)
            else:
                if self.out:
                    self.out.append([True, payload])
                    self._flush()
                else:
                    assert self.transport is not None
                    self.transport.write(payload)

    def _release(self, item: List) -> None:
        item[0] = True
        self._flush()

    def _flush(self) -> None:
        parts = []
        while self.out and self.out[0][0]:
            parts.append(self.out.popleft()[1])
        if parts and self.transport is not None and not self.transport.is_closing():
            self.transport.write(b"".join(parts))


class StubSink:
    def __init__(self, **kwargs) -> None:
        self.state = SinkState(**kwargs)
        self.server: Optional[asyncio.AbstractServer] = None
        self.port = 0

    async def start(self, host: str = "127.0.0.1", port: int = 0, reuse_port: bool = False,
                    sock: Optional[socket.socket] = None, ssl_context=None) -> int:
        loop = asyncio.get_running_loop()
        self.scheme = "https" if ssl_context is not None else "http"
        if sock is not None:
            self.server = await loop.create_server(lambda: _SinkProtocol(self.state), sock=sock, ssl=ssl_context)
        else:
            self.server = await loop.create_server(lambda: _SinkProtocol(self.state), host, port,
                                                   reuse_port=reuse_port or None, ssl=ssl_context)
        self.port = self.server.sockets[0].getsockname()[1]
        return self.port

    @property
    def url(self) -> str:
        return f"{getattr(self, 'scheme', 'http')}://127.0.0.1:{self.port}"

    async def stop(self) -> None:
        if self.server is not None:
            self.server.close()
            try:
                await with_timeout(self.server.wait_closed(), 2)
            except asyncio.TimeoutError:
                pass


_GEN = b'"k8s-watcher.test/generation":"'


def payload_key(body: bytes) -> bytes:
    """``uid|event_type|phase`` of a payload without a JSON parse (soak verification),
    plus ``|<generation>`` when the pod carries the replay fixture's
    ``k8s-watcher.test/generation`` annotation (steady pods MODIFIED every round).

    The first ``"uid":`` in a payload is the top-level one (``name`` and
    ``namespace`` precede it and are plain strings)."""
    i = body.find(b'"uid":"') + 7
    uid = body[i:body.find(b'"', i)]
    j = body.rfind(b'"event_type":"') + 14
    et = body[j:body.find(b'"', j)]
    k = body.find(b'"status":{"phase":') + 18
    phase = body[k:body.find(b",", k)].strip(b'"')
    g = body.find(_GEN)
    if g >= 0:
        g += len(_GEN)
        return b"|".join((uid, et, phase, body[g:body.find(b'"', g)]))
    return b"|".join((uid, et, phase))


class _VerifyingState(SinkState):
    """Counts every payload key; dumped as JSON when the worker is told to stop."""

    def __init__(self, **kw) -> None:
        super().__init__(record=False, **kw)
        self.keys: Dict[bytes, int] = {}

    def note(self, body: bytes) -> None:
        k = payload_key(body)
        self.keys[k] = self.keys.get(k, 0) + 1


def _native_sink(port: int, verify: bool, reserve: int = 0):
    """A ``_kwcore.SinkServer`` on a SO_REUSEPORT socket bound to ``port``
    (``reserve``: distinct keys expected in verify mode; the table is sized
    for them instead of rehashing while it serves)."""
    from ..ops.native import load
    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind(("127.0.0.1", port))
    sock.listen(1024)
    try:
        return load().SinkServer(sock.fileno(), b"/api/pods/update", verify, reserve)  # serves a dup of the socket
    finally:
        sock.close()


def run_sink_process(port: int, workers: int = 1, latency: float = 0.0,
                     verify_dir: Optional[str] = None, tls: Optional[Tuple[str, str]] = None,
                     engine: str = "auto", expect_keys: int = 0) -> None:
    """Blocking: serve on ``port`` with ``workers`` SO_REUSEPORT processes (bench helper).

    With ``verify_dir`` every worker records ``uid|event_type|phase`` counts and
    writes them to ``verify_dir/sink-<pid>.json`` on SIGTERM (and, without
    stopping, on SIGUSR1; SIGUSR2 also clears them after the dump).

    ``engine``: ``native`` serves requests with ``_kwcore.SinkServer`` (one
    epoll thread per worker, ~5x less CPU per notification than the asyncio
    protocol: the fixture takes less of the CPU the watchers are measured on);
    ``python`` the asyncio protocol; ``auto`` native unless TLS or latency
    injection is asked for (only the asyncio sink does those).
    """
    import signal as _signal
    if engine == "auto":
        engine = "python" if (tls or latency > 0) else "native"
    if engine == "native" and (tls or latency > 0):
        raise ValueError("the native sink serves plain http without injected latency")
    pids = []
    for _ in range(workers - 1):
        pid = os.fork()
        if pid == 0:
            pids = []
            break
        pids.append(pid)

    async def serve_native() -> None:
        srv = _native_sink(port, bool(verify_dir), expect_keys)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()

        def dump(reset: bool = False) -> None:
            count, keys = srv.snapshot(reset)
            final = os.path.join(verify_dir, f"sink-{os.getpid()}.json")
            with open(final + ".tmp", "w") as fh:  # renamed when complete: readers never see a partial dump
                json.dump({"count": count, "keys": keys, "stalls": srv.stalls()}, fh)
            os.replace(final + ".tmp", final)

        loop.add_signal_handler(_signal.SIGTERM, stop.set)
        if verify_dir:
            loop.add_signal_handler(_signal.SIGUSR1, dump)
            loop.add_signal_handler(_signal.SIGUSR2, lambda: dump(True))
        await stop.wait()
        srv.stop()
        if verify_dir:
            dump()
        srv.close()

    async def serve() -> None:
        sink = StubSink(record=False, latency=latency)
        if verify_dir:
            sink.state = _VerifyingState(latency=latency)
        ctx = None
        if tls:
            import ssl
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.load_cert_chain(*tls)
        await sink.start("127.0.0.1", port, reuse_port=True, ssl_context=ctx)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()

        def dump() -> None:
            st = sink.state
            final = os.path.join(verify_dir, f"sink-{os.getpid()}.json")
            with open(final + ".tmp", "w") as fh:  # renamed when complete: readers never see a partial dump
                json.dump({"count": st.count, "keys": {k.decode(): v for k, v in st.keys.items()}}, fh)
            os.replace(final + ".tmp", final)

        loop.add_signal_handler(_signal.SIGTERM, stop.set)
        if verify_dir:
            loop.add_signal_handler(_signal.SIGUSR1, dump)  # a snapshot while still serving

            def dump_and_reset() -> None:  # long soaks: hand the keys over, keep memory flat
                dump()
                sink.state.keys.clear()
                sink.state.count = 0
            loop.add_signal_handler(_signal.SIGUSR2, dump_and_reset)
        await stop.wait()
        if verify_dir:
            dump()

    try:
        asyncio.run(serve_native() if engine == "native" else serve())
    except KeyboardInterrupt:
        pass
    # the workers got the same SIGTERM (one process group) and may still be
    # writing their final dump: the parent outlives them, so whoever waits for
    # it waits for the whole sink (nothing is left behind for init to reap)
    for pid in pids:
        try:
            os.waitpid(pid, 0)
        except ChildProcessError:
            pass


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description="stub clusterapi sink")
    ap.add_argument("--port", type=int, default=3000)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--latency", type=float, default=0.0)
    ap.add_argument("--verify-dir", default=None, help="record payload keys, dump on SIGTERM")
    ap.add_argument("--expect-keys", type=int, default=0,
                    help="native sink, verify mode: distinct keys per worker to size the key table for")
    ap.add_argument("--tls-cert", default=None, help="serve https with this certificate (and --tls-key)")
    ap.add_argument("--tls-key", default=None)
    ap.add_argument("--engine", default="auto", choices=["auto", "native", "python"],
                    help="request loop: native (_kwcore.SinkServer) or the asyncio protocol")
    ap.add_argument("--no-thp", action="store_true",
                    help="no transparent huge pages for this process and its workers (PR_SET_THP_DISABLE)")
    args = ap.parse_args(argv)
    if args.no_thp:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(41, 1, 0, 0, 0)  # PR_SET_THP_DISABLE, inherited by the forks
    tls = (args.tls_cert, args.tls_key) if args.tls_cert else None
    print(f"stub clusterapi listening on {'https' if tls else 'http'}://127.0.0.1:{args.port}", flush=True)
    run_sink_process(args.port, args.workers, args.latency, args.verify_dir, tls, args.engine, args.expect_keys)


if __name__ == "__main__":
    main()
