"""Plain-TCP watch bodies read on a native thread (``watcher.watch_reader: native``).

asyncio reads a watch socket on the event-loop thread: the kernel's copy of
every watch byte then competes with decoding and applying the events it
carries. :class:`WatchReaderHub` wraps ``_kwcore.ReaderHub`` (see
``ops/csrc/readerhub.inc``): once a watch's response head has been parsed by
asyncio (status, headers, the switch to raw chunked pass-through), the
connection is *adopted* — asyncio stops reading it and a dup of its socket is
polled by the hub's thread, which recv()s into pooled buffers. The event loop
wakes on one eventfd per batch and hands each buffer to the stream's sink
exactly as ``_ClientProtocol.buffer_updated`` would (zero copy, the sink must
not keep the view).

The asyncio transport stays the owner of the connection: closing the stream,
a lost connection and the server's end of the body all go through it, so
``StreamResponse.finished`` / ``close()`` behave as before.

An https watch cannot be adopted mid-stream (its TLS session lives in
Python's ``ssl`` object), so :meth:`open_tls` gives the hub the connection
from the start: a connected socket, a ``_kwcore.TlsContext`` built from the
kubeconfig's trust material (``ssl.SSLContext.kw_tls``), the SNI / verified
host name and the request; the hub runs the handshake and decrypts on its
thread. A :class:`HubTransport` stands in for the asyncio transport.
"""

from __future__ import annotations

import asyncio
import os
import time
from typing import Dict, Optional

from ..ops import native


class WatchReaderHub:
    DISPATCH_SLICE_S = 0.004  # longest delivery of hub reads in one loop turn

    def __init__(self, buf_bytes: int, nbufs: int = 64,
                 loop: Optional[asyncio.AbstractEventLoop] = None, max_bytes: int = 0, frame: bool = True,
                 depth: int = 2, tls_records: bool = True, tls_threads: int = 0, readers: int = 1) -> None:
        self.loop = loop or asyncio.get_running_loop()
        # max_bytes: read-ahead over all streams (0: the whole pool); frame: the
        # hub's thread de-chunks and splits bound bodies (watcher.hub_framing)
        self.frame = bool(frame)
        self.core = native.load().ReaderHub(max(64 * 1024, int(buf_bytes)), max(2, int(nbufs)),
                                            max(0, int(max_bytes)), frame=self.frame)
        # depth: buffers read ahead per stream
        if depth != 2:
            self.core.set_depth(int(depth))
        # readers: threads polling the streams (each stream stays with one)
        if readers > 1:
            self.core.set_readers(int(readers))
        # https watches: the hub opens TLS 1.3 records itself, on a pool of
        # tls_threads besides the reader thread (watcher.watch_tls_records /
        # watch_tls_threads; ops/csrc/tls13.inc)
        self.core.set_tls(bool(tls_records), max(0, int(tls_threads)))
        self.protos: Dict[int, object] = {}
        self._tls: Dict[tuple, object] = {}
        self._flush: Dict[object, object] = {}  # bind(): once per dispatch
        self._pending = None  # (items, touched) a dispatch's delivery left for the next turn
        # bind()'s sync groups: key -> [flags(), the flags the group's streams
        # have]. After each dispatch the flags are evaluated once per group,
        # and the streams' hooks run only when they changed — not once per
        # touched stream per dispatch (64 namespace watches: ~60-90 us of the
        # loop per dispatch)
        self._groups: Dict[object, list] = {}
        self._soon = None  # the loop turn scheduled to deliver it
        self._fd = self.core.fileno()
        self.loop.add_reader(self._fd, self._on_ready)
        self.closed = False

    def adopt(self, proto) -> bool:
        """Take over reading ``proto``'s socket; False (nothing changed) for TLS
        or a transport without a socket."""
        if self.closed:
            return False
        t = proto.transport
        if t is None or t.is_closing() or t.get_extra_info("sslcontext") is not None:
            return False
        sock = t.get_extra_info("socket")
        if sock is None:
            return False
        t.pause_reading()
        sid = self.core.add(os.dup(sock.fileno()))
        self.protos[sid] = proto
        proto.hub, proto.hub_sid = self, sid
        return True

    def tls_context(self, material: dict):
        """``_kwcore.TlsContext`` for an ``ssl.SSLContext``'s ``kw_tls`` material (cached)."""
        key = (material.get("ca_pem"), material.get("cert_pem"), material.get("key_pem"), material.get("verify"))
        ctx = self._tls.get(key)
        if ctx is None:
            ctx = self._tls[key] = native.load().TlsContext(
                ca_pem=material.get("ca_pem"), cert_pem=material.get("cert_pem"),
                key_pem=material.get("key_pem"), verify=bool(material.get("verify", True)))
        return ctx

    def open_tls(self, proto, sock, material: dict, host: str, request: bytes) -> None:
        """A connected TCP socket for an https watch: the hub owns it from here
        on — TLS handshake, the request, then decrypted bytes to ``proto``."""
        ctx = self.tls_context(material)
        sid = self.core.add_tls(sock.detach(), ctx, host, request)
        self.protos[sid] = proto
        proto.hub, proto.hub_sid = self, sid

    def error_text(self, sid: int) -> str:
        return "" if self.closed else self.core.error_text(sid)

    def bind(self, proto, pipeline_core, framed: bool, on_result, flush, flush_key, sync=None,
             sync_group=None) -> None:
        """Feed ``proto``'s body straight to a fused ``_kwcore.Pipeline`` on
        the hub's dispatch (no Python call per read): only reads whose result
        needs Python — control events, log lines, submissions, the end of the
        body, an error — come back, through ``on_result(result, read_ns,
        body_done)``. ``flush`` runs once per dispatch that fed a bound stream
        (one per distinct ``flush_key``: streams sharing a notifier flush it
        once; it should hold only what they share, so a retired stream's
        pipeline is not kept alive by it). ``sync`` is this stream's own
        per-dispatch hook (its pipeline's log switches): it runs after every
        dispatch that touched the stream, and goes away with the stream.
        ``sync_group`` = ``(key, flags)``: streams whose hook takes the value
        of one shared ``flags()`` — it is evaluated once per dispatch for the
        group, and the group's hooks run (``sync(value)``) only when it
        changed."""
        if self.closed or proto.hub is not self:
            return
        self.core.bind(proto.hub_sid, pipeline_core, framed)
        proto.hub_result = on_result
        proto.hub_sync = sync
        proto.hub_group = None
        if sync is not None and sync_group is not None:
            key, flags = sync_group
            proto.hub_group = key
            g = self._groups.get(key)
            if g is None:
                self._groups[key] = [flags, flags()]
        self._flush[flush_key] = flush

    def last_read(self, sid: int) -> float:
        """time.monotonic() of stream ``sid``'s last read with bytes (0.0: none)."""
        return 0.0 if self.closed else self.core.last_read(sid)

    def forget(self, sid: int) -> None:
        if self.protos.pop(sid, None) is not None and not self.closed:
            self.core.remove(sid)

    def pause(self, sid: int, paused: bool) -> None:
        if not self.closed:
            self.core.pause(sid, paused)

    def _continue(self) -> None:
        self._soon = None
        self._on_ready()

    def _on_ready(self) -> None:
        core = self.core
        if self._pending is not None:  # the rest of the last dispatch first: no newer read may pass it
            if self._soon is not None:
                return  # the eventfd, still readable: the turn scheduled for the rest delivers it
            items, touched = self._pending
            self._pending = None
        else:
            # (a bound stream's activity is the hub's: last_read, not a
            # Python attribute set per dispatch)
            items, touched = core.take_dispatch()
        try:
            self._deliver(core, items, touched)
        finally:
            if touched:
                protos = self.protos
                for key, g in self._groups.items():
                    now = g[0]()
                    if now != g[1]:  # (rare: a runtime log-level change) every stream of the group
                        g[1] = now
                        for proto in list(protos.values()):
                            if getattr(proto, "hub_group", None) == key and proto.hub_sync is not None:
                                proto.hub_sync(now)
                for sid in touched:  # streams outside a group: their own hook, as before
                    proto = protos.get(sid)
                    if (proto is not None and getattr(proto, "hub_group", None) is None
                            and getattr(proto, "hub_sync", None) is not None):
                        proto.hub_sync()
                for flush in list(self._flush.values()):
                    flush()

    def _deliver(self, core, items, touched=()) -> None:
        # one loop turn delivers for at most DISPATCH_SLICE_S: a storm hands the
        # loop hundreds of reads that need Python at once (every watch of a
        # 1,000-namespace cluster answering 410 together: ~50 us each); the rest
        # waits for the next turn, ahead of anything newer (take_dispatch is not
        # called while a rest is pending, so a bound stream's later reads stay
        # queued behind its attention read)
        deadline = time.perf_counter() + self.DISPATCH_SLICE_S
        last = len(items) - 1
        for i, (sid, buf, view, read_ns, err) in enumerate(items):
            if buf == -2:  # a bound stream's read that needs Python (take_dispatch)
                proto = self.protos.get(sid)
                if proto is not None:
                    proto.hub_native(view, read_ns, bool(err))
            else:
                self._deliver_read(core, sid, buf, view, read_ns, err)
            if i < last and not self.closed and time.perf_counter() > deadline:
                self._pending = (items[i + 1:], touched)
                self._soon = self.loop.call_soon(self._continue)
                return

    def _deliver_read(self, core, sid, buf, view, read_ns, err) -> None:
        try:
            proto = self.protos.get(sid)
            if proto is not None:
                if view is not None:
                    proto.hub_data(view, read_ns)
                else:
                    proto.hub_eof(err)
        finally:
            if view is not None:
                try:
                    view.release()
                except BufferError:  # a consumer kept a slice: never reuse under it
                    buf = -1
            if buf >= 0 and not self.closed:
                core.release(buf)

    def stats(self) -> dict:
        return {} if self.closed else dict(self.core.stats(), streams=len(self.protos))

    def close(self) -> None:
        if self.closed:
            return
        self.closed = True
        try:
            self.loop.remove_reader(self._fd)
        except (RuntimeError, ValueError):
            pass
        for proto in list(self.protos.values()):
            proto.hub = None
            proto.close()
        self.protos.clear()
        self._flush.clear()
        self._groups.clear()
        self._pending = None
        if self._soon is not None:
            self._soon.cancel()
            self._soon = None
        self.core.close()


class HubTransport(asyncio.BaseTransport):
    """Transport stand-in for a connection the hub owns from the start (TLS):
    ``close()`` ends it like an asyncio transport would (``connection_lost``
    on the next loop iteration); reading is flow-controlled through the hub."""

    def __init__(self, loop: asyncio.AbstractEventLoop, proto, sslcontext) -> None:
        super().__init__()
        self._loop = loop
        self._proto = proto
        self._closing = False
        self._ssl = sslcontext

    def is_closing(self) -> bool:
        return self._closing

    def close(self) -> None:
        if self._closing:
            return
        self._closing = True
        self._loop.call_soon(self._proto.connection_lost, None)

    def get_extra_info(self, name, default=None):
        if name == "sslcontext":
            return self._ssl
        return default

    def write(self, data) -> None:  # the request went to the hub with the socket
        raise RuntimeError("HubTransport: the request is written by the reader hub")

    def pause_reading(self) -> None:
        self._proto.set_reading(False)

    def resume_reading(self) -> None:
        self._proto.set_reading(True)
