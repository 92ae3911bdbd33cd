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
"""

from __future__ import annotations

import asyncio
import os
from typing import Dict, Optional

from ..ops import native


class WatchReaderHub:
    def __init__(self, buf_bytes: int, nbufs: int = 64,
                 loop: Optional[asyncio.AbstractEventLoop] = None) -> None:
        self.loop = loop or asyncio.get_running_loop()
        self.core = native.load().ReaderHub(max(64 * 1024, int(buf_bytes)), max(2, int(nbufs)))
        self.protos: Dict[int, object] = {}
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

    def forget(self, sid: int) -> None:
        if self.protos.pop(sid, None) is not None and not self.closed:
            self.core.remove(sid)

    def pause(self, sid: int, paused: bool) -> None:
        if not self.closed:
            self.core.pause(sid, paused)

    def _on_ready(self) -> None:
        core = self.core
        for sid, buf, view, read_ns, err in core.take():
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
                        continue
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
        self.core.close()
