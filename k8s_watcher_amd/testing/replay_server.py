"""High-rate watch replay server for benchmarks (the "mock API" of BASELINE.json).

:class:`~.fake_apiserver.FakeApiServer` serialises every event as it happens,
which caps it far below the watcher's speed. This server instead renders a
churn *template* once (``pods_per_step`` pod lifecycles = 5 events each, see
:func:`.podgen.churn_events`) and, per step, re-stamps it with fresh
resourceVersions and pod uids — a byte splice, no JSON work — then streams it
as one HTTP chunk per event, exactly like kube-apiserver, as fast as the
client reads (``STEP``) or at a fixed rate (``PACE``).

Control is line-based on stdin, replies on stdout::

    READY <port> <events_per_step>
    STEP <k>                 -> SENT <k> <n>     (whole step, unthrottled)
    PACE <k> <rate> <count>  -> SENT <k> <n>     (first <count> events at <rate>/s)
    QUIT

HTTP surface: ``/version``, ``/api/v1/namespaces``, an empty ``PodList`` for
``/api/v1/pods``, and ``?watch=true`` streams that receive every step.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
from typing import List, Optional, Tuple

from .podgen import churn_events

_HDR = (b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
        b"Transfer-Encoding: chunked\r\n\r\n")


class Template:
    def __init__(self, pods_per_step: int, seed: int, namespaces: Optional[List[str]] = None) -> None:
        # each event: (segments, uid-tail) where the line is
        # seg0 + RV + seg1 + UID + seg2 + UID + ... and UID = <8-hex step tag> + uid-tail
        self.events: List[Tuple[List[bytes], bytes]] = []
        for etype, obj in churn_events(pods_per_step, seed=seed, namespaces=namespaces):
            uid = obj["metadata"]["uid"].encode()
            obj["metadata"]["resourceVersion"] = "@@RV@@"
            line = json.dumps({"type": etype, "object": obj}, separators=(",", ":"),
                              ensure_ascii=False).encode("utf-8") + b"\n"
            pre, post = line.split(b"@@RV@@", 1)
            segs = [pre] + post.split(uid)
            self.events.append((segs, uid[8:]))

    def __len__(self) -> int:
        return len(self.events)

    def render(self, step: int, start: int, stop: int, rv_base: int) -> bytes:
        tag = b"%08x" % (step & 0xFFFFFFFF)
        out = []
        for i in range(start, stop):
            segs, tail = self.events[i]
            body = (tag + tail).join(segs[1:])
            n = len(segs[0]) + len(body) + len(str(rv_base + i))
            out.append(b"%x\r\n%s%d%s\r\n" % (n, segs[0], rv_base + i, body))
        return b"".join(out)


class ReplayServer:
    def __init__(self, template: Template, prerender: int = 0) -> None:
        self.t = template
        self.watchers: List[asyncio.StreamWriter] = []
        self.rv = 1000
        # Whole steps rendered ahead of time so that, during a timed step, this
        # process only issues send() calls and can never be the bottleneck.
        self.rendered = {k: self.t.render(k, 0, len(self.t), self.rv_base(k)) for k in range(prerender)}

    def rv_base(self, step: int) -> int:
        return 10_000_000 + step * len(self.t)

    async def handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                line = await reader.readline()
                if not line:
                    return
                while True:
                    h = await reader.readline()
                    if h in (b"\r\n", b"\n", b""):
                        break
                target = line.split()[1].decode()
                low = target.lower()
                if "watch=true" in low or "watch=1" in low:
                    writer.write(_HDR)
                    self.watchers.append(writer)
                    await reader.read()  # hold until the client goes away
                    return
                if target.startswith("/version"):
                    body = b'{"major":"1","minor":"33","gitVersion":"v1.33.1-replay"}'
                elif target.startswith("/api/v1/namespaces") and "/pods" not in target:
                    body = json.dumps({"kind": "NamespaceList", "apiVersion": "v1", "metadata": {},
                                       "items": [{"metadata": {"name": "default"}}]}).encode()
                else:
                    body = json.dumps({"kind": "PodList", "apiVersion": "v1",
                                       "metadata": {"resourceVersion": str(self.rv)}, "items": []}).encode()
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
                             % (len(body), body))
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            if writer in self.watchers:
                self.watchers.remove(writer)
            writer.close()

    async def send(self, step: int, rate: Optional[float] = None, count: Optional[int] = None) -> int:
        n = len(self.t) if count is None else min(count, len(self.t))
        rv_base = self.rv_base(step)
        pre = self.rendered.pop(step, None)
        if pre is not None and count is None:
            view = memoryview(pre)
            piece = 1 << 22
            for a in range(0, len(view), piece):
                for w in list(self.watchers):
                    w.write(view[a:a + piece])
                    await w.drain()
        elif rate:
            t0 = time.monotonic()
            for i in range(n):
                data = self.t.render(step, i, i + 1, rv_base)
                for w in list(self.watchers):
                    w.write(data)
                delay = t0 + (i + 1) / rate - time.monotonic()
                if delay > 0:
                    await asyncio.sleep(delay)
        else:
            slice_ = 256
            for a in range(0, n, slice_):
                data = self.t.render(step, a, min(n, a + slice_), rv_base)
                for w in list(self.watchers):
                    w.write(data)
                    await w.drain()
        self.rv = rv_base + n
        return n


async def amain(args) -> None:
    tmpl = Template(args.pods_per_step, args.seed, args.namespaces.split(",") if args.namespaces else None)
    srv = ReplayServer(tmpl, args.prerender)
    server = await asyncio.start_server(srv.handle, "127.0.0.1", args.port)
    port = server.sockets[0].getsockname()[1]
    print(f"READY {port} {len(tmpl)}", flush=True)
    loop = asyncio.get_running_loop()
    reader = asyncio.StreamReader()
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), sys.stdin)
    while True:
        line = await reader.readline()
        if not line:
            break
        parts = line.decode().split()
        if not parts:
            continue
        cmd = parts[0].upper()
        if cmd == "QUIT":
            break
        if cmd == "STEP":
            n = await srv.send(int(parts[1]))
        elif cmd == "PACE":
            n = await srv.send(int(parts[1]), float(parts[2]), int(parts[3]))
        elif cmd == "WATCHERS":
            n = sum(1 for w in srv.watchers if not w.is_closing())
        else:
            n = -1
        print(f"SENT {parts[1] if len(parts) > 1 else '-'} {n}", flush=True)
    server.close()


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--pods-per-step", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--namespaces", default=None)
    ap.add_argument("--prerender", type=int, default=0, help="render steps [0, N) before READY")
    asyncio.run(amain(ap.parse_args(argv)))


if __name__ == "__main__":
    main()
