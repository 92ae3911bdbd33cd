"""High-rate watch replay server for benchmarks (the "mock API" of BASELINE.json).

:class:`~.fake_apiserver.FakeApiServer` serialises every event as it happens,
which caps it far below the watcher's speed. This server renders a *template*
once and, per step, re-stamps it with fresh resourceVersions (and, for churn,
fresh pod uids) by splicing bytes — no JSON work — then streams it as one HTTP
chunk per event, like kube-apiserver, as fast as the client reads (``STEP``)
or at a fixed rate (``PACE``).

Templates (``--template``):

* ``churn`` — ``--pods`` lifecycles per step: ADDED → 3×MODIFIED → DELETED
  (BASELINE config #4, #5);
* ``createdelete`` — ADDED → MODIFIED(Running) → DELETED (config #2);
* ``steady`` — ``--pods`` pods exist from the start (served by LIST); each step
  MODIFIES every pod once (config #3).

It keeps enough state to behave like an API server across restarts: a
LIST returns the live pods at the current resourceVersion; a watch with
``resourceVersion=X`` first receives every event after ``X`` (re-rendered from
the template); ``X`` older than the last compaction gets an ``ERROR`` 410 event.

Control is line-based on stdin, replies on stdout::

    READY <port> <events_per_step>
    STEP <k> [drop=<n>] [expire=<n>]  -> SENT <k> <n>  whole step; optionally abort every
                                          watch (drop) or compact + 410 them (expire) after n events
    STEPS <a> <b>                     -> SENT <b-1> <n>  steps a..b-1 back to back (sustained stream)
    PACE <k> <rate> <count>           -> SENT <k> <n>  first <count> events at <rate>/s (rate 0 = max)
    DROP | EXPIRE | BOOKMARK          -> SENT - <watchers>
    WATCHERS                          -> SENT - <open watch streams>
    QUIT
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import re
import sys
import time
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

from .podgen import PodFactory, churn_events

_HDR = (b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
        b"Transfer-Encoding: chunked\r\n\r\n")
_PH = re.compile(rb"@@(RV|UID|STEP)@@")
RV0 = 10_000_000
_TYPES = {"ADDED": b'{"type":"ADDED","object":', "MODIFIED": b'{"type":"MODIFIED","object":',
          "DELETED": b'{"type":"DELETED","object":'}


def _compile(obj: dict, uid: str) -> List:
    raw = json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode("utf-8")
    raw = raw.replace(uid.encode(), b"@@UID@@")
    return _PH.split(raw)  # [lit, name, lit, name, ..., lit]


class Template:
    def __init__(self, kind: str, pods: int, seed: int = 0, namespaces: Optional[List[str]] = None) -> None:
        self.kind = kind
        self.events: List[Tuple[str, List, str]] = []   # (etype, segments, uid)
        self.initial: List[Tuple[List, str]] = []       # steady: pods present before step 0
        if kind == "churn":
            for et, obj in churn_events(pods, seed=seed, namespaces=namespaces):
                obj["metadata"]["resourceVersion"] = "@@RV@@"
                uid = obj["metadata"]["uid"]
                self.events.append((et, _compile(obj, uid), uid))
        elif kind == "createdelete":
            f = PodFactory(seed, namespaces)
            for _ in range(pods):
                p0 = f.new_pod()
                p1 = f.running(p0)
                p2 = f.deleting(p1)
                for et, obj in (("ADDED", p0), ("MODIFIED", p1), ("DELETED", p2)):
                    obj["metadata"]["resourceVersion"] = "@@RV@@"
                    self.events.append((et, _compile(obj, p0["metadata"]["uid"]), p0["metadata"]["uid"]))
        elif kind == "steady":
            f = PodFactory(seed, namespaces)
            for _ in range(pods):
                p = f.running(f.new_pod())
                p["metadata"]["resourceVersion"] = "@@RV@@"
                p["metadata"]["annotations"]["k8s-watcher.test/generation"] = "@@STEP@@"
                uid = p["metadata"]["uid"]
                segs = _compile(p, uid)
                self.initial.append((segs, uid))
                self.events.append(("MODIFIED", segs, uid))
        else:
            raise ValueError(f"unknown template {kind!r}")

    def __len__(self) -> int:
        return len(self.events)

    def uid(self, step: int, uid: str) -> str:
        if self.kind == "steady":
            return uid
        return f"{step & 0xFFFFFFFF:08x}" + uid[8:]

    def obj(self, segs: List, rv: int, uid: str, step: int) -> bytes:
        sub = {b"RV": str(rv).encode(), b"UID": uid.encode(), b"STEP": str(step).encode()}
        out = [segs[0]]
        for j in range(1, len(segs), 2):
            out.append(sub[segs[j]])
            out.append(segs[j + 1])
        return b"".join(out)

    def line(self, step: int, i: int) -> bytes:
        et, segs, uid = self.events[i]
        body = _TYPES[et] + self.obj(segs, RV0 + step * len(self) + i, self.uid(step, uid), step) + b"}\n"
        return b"%x\r\n%s\r\n" % (len(body), body)

    def render(self, step: int, start: int, stop: int) -> Tuple[bytes, List[int]]:
        """Chunked bytes for events [start, stop) and each event's byte offset."""
        parts, offsets, pos = [], [], 0
        for i in range(start, stop):
            b = self.line(step, i)
            offsets.append(pos)
            pos += len(b)
            parts.append(b)
        return b"".join(parts), offsets


class ReplayServer:
    def __init__(self, template: Template, prerender: int = 0) -> None:
        self.t = template
        self.E = len(template)
        self.watchers: List[asyncio.StreamWriter] = []
        self.rv = RV0 - 1 if template.kind != "steady" else RV0 - 1
        self.compacted_rv = RV0 - 1
        # live objects: uid -> (step, event index | -1 for the initial state)
        self.live: Dict[str, Tuple[int, int]] = {}
        self._pending: List[List[int]] = []  # [step, start, stop) ranges sent but not yet applied to live
        self._lists: Dict[str, Tuple[int, List[bytes], int]] = {}  # continue token -> (rv, items, offset)
        self._list_seq = 0
        if template.kind == "steady":
            self.live = {uid: (-1, j) for j, (_, uid) in enumerate(template.initial)}
        # Whole steps rendered ahead of time into memory files so that, during
        # a timed step, this process only issues sendfile() calls: the kernel
        # moves the bytes (no user-space copy), which keeps this fixture well
        # ahead of the watcher it feeds.
        self.rendered = {k: self._to_memfile(*self.t.render(k, 0, self.E)) for k in range(prerender)}

    @staticmethod
    def _to_memfile(data: bytes, offsets: List[int]):
        if not hasattr(os, "memfd_create"):
            return data, offsets
        fd = os.memfd_create("replay-step")
        view = memoryview(data)
        while view:
            view = view[os.write(fd, view):]
        return open(fd, "rb"), offsets

    # ------------------------------------------------------------------ state
    def pos_of(self, rv: int) -> Tuple[int, int]:
        return (rv - RV0) // self.E, (rv - RV0) % self.E

    def _advance(self, step: int, start: int, stop: int) -> None:
        """Record that events [start, stop) of ``step`` went out. Only the
        range is noted here — per-event bookkeeping in this process would
        cost ~0.5 µs per event on the one core that feeds the watcher; the
        live set is brought up to date when a LIST or a fresh watch needs it."""
        p = self._pending
        if p and p[-1][0] == step and p[-1][2] == start:
            p[-1][2] = stop
        else:
            p.append([step, start, stop])
        self.rv = RV0 + step * self.E + stop - 1

    def _materialize(self) -> None:
        for step, start, stop in self._pending:
            self._apply(step, start, stop)
        self._pending.clear()

    def _apply(self, step: int, start: int, stop: int) -> None:
        t = self.t
        for i in range(start, stop):
            et, _, uid = t.events[i]
            u = t.uid(step, uid)
            if et == "DELETED":
                self.live.pop(u, None)
            else:
                self.live[u] = (step, i)

    def _live_items(self) -> List[bytes]:
        self._materialize()
        items = []
        t = self.t
        for u, (step, i) in self.live.items():
            if step < 0:
                segs, _ = t.initial[i]
                items.append(t.obj(segs, RV0 - 1, u, 0))
            else:
                _, segs, _ = t.events[i]
                items.append(t.obj(segs, RV0 + step * self.E + i, u, step))
        return items

    def list_body(self, limit: int = 0, cont: Optional[str] = None) -> bytes:
        """A PodList; with ``limit`` paginated like kube-apiserver: every page of
        one LIST comes from the snapshot taken for its first page (same RV),
        linked by an opaque ``continue`` token."""
        if cont:
            snap = self._lists.get(cont)
            if snap is None:
                return b""  # unknown/expired token: the caller answers 410
            rv, items, off = snap
            del self._lists[cont]
        else:
            rv, items, off = self.rv, self._live_items(), 0
        end = len(items) if not limit else min(len(items), off + limit)
        meta = b'"resourceVersion":"%d"' % rv
        if end < len(items):
            self._list_seq += 1
            token = f"r{self._list_seq}"
            self._lists[token] = (rv, items, end)
            meta += b',"continue":"%s","remainingItemCount":%d' % (token.encode(), len(items) - end)
        return (b'{"kind":"PodList","apiVersion":"v1","metadata":{%s},"items":[%s]}'
                % (meta, b",".join(items[off:end])))

    def backlog(self, since: int) -> bytes:
        """Every event with resourceVersion in (since, self.rv]."""
        out = []
        rv = max(since, RV0 - 1) + 1
        while rv <= self.rv:
            step, i = self.pos_of(rv)
            out.append(self.t.line(step, i))
            rv += 1
        return b"".join(out)

    # ------------------------------------------------------------------ HTTP
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
                u = urlsplit(target)
                q = {k: v[-1] for k, v in parse_qs(u.query).items()}
                if q.get("watch", "").lower() in ("true", "1"):
                    self.start_watch(writer, q.get("resourceVersion"))
                    await reader.read()  # hold until the client goes away
                    return
                if u.path == "/version":
                    body = b'{"major":"1","minor":"33","gitVersion":"v1.33.1-replay"}'
                elif u.path == "/api/v1/namespaces":
                    body = json.dumps({"kind": "NamespaceList", "apiVersion": "v1", "metadata": {},
                                       "items": [{"metadata": {"name": "default"}}]}).encode()
                else:
                    body = self.list_body(int(q.get("limit") or 0), q.get("continue"))
                    if not body:
                        body = json.dumps({"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                           "reason": "Expired", "code": 410,
                                           "message": "The provided continue parameter is too old"}).encode()
                        writer.write(b"HTTP/1.1 410 Gone\r\nContent-Type: application/json\r\n"
                                     b"Content-Length: %d\r\n\r\n" % len(body) + body)
                        await writer.drain()
                        continue
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
                             % len(body) + body)
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            if writer in self.watchers:
                self.watchers.remove(writer)
            writer.close()

    def start_watch(self, writer: asyncio.StreamWriter, rv_param: Optional[str]) -> None:
        """Synchronous: the backlog and the registration happen between two sends."""
        writer.write(_HDR)
        if rv_param not in (None, "", "0"):
            since = int(rv_param)
            if since < self.compacted_rv:
                err = json.dumps({"type": "ERROR", "object": {
                    "kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": "Expired", "code": 410,
                    "message": f"too old resource version: {since} ({self.compacted_rv})"}}).encode() + b"\n"
                writer.write(b"%x\r\n%s\r\n0\r\n\r\n" % (len(err), err))
                writer.close()
                return
            writer.write(self.backlog(since))
        else:
            # no resourceVersion: synthetic ADDED for every live pod, then live events
            # (what kube-apiserver does, and what the reference's watch relies on)
            t = self.t
            self._materialize()
            for u, (step, i) in self.live.items():
                if step < 0:
                    segs, _ = t.initial[i]
                    obj = t.obj(segs, RV0 - 1, u, 0)
                else:
                    obj = t.obj(t.events[i][1], RV0 + step * self.E + i, u, step)
                body = _TYPES["ADDED"] + obj + b"}\n"
                writer.write(b"%x\r\n%s\r\n" % (len(body), body))
        self.watchers.append(writer)

    def drop(self) -> int:
        n = len(self.watchers)
        for w in list(self.watchers):
            w.transport.abort()
        self.watchers.clear()
        return n

    def expire(self) -> int:
        self.compacted_rv = self.rv
        n = len(self.watchers)
        err = json.dumps({"type": "ERROR", "object": {
            "kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": "Expired", "code": 410,
            "message": "too old resource version"}}).encode() + b"\n"
        for w in list(self.watchers):
            w.write(b"%x\r\n%s\r\n0\r\n\r\n" % (len(err), err))
            w.close()
        self.watchers.clear()
        return n

    def bookmark(self) -> int:
        line = (b'{"type":"BOOKMARK","object":{"kind":"Pod","apiVersion":"v1","metadata":'
                b'{"resourceVersion":"%d"}}}\n' % self.rv)
        for w in self.watchers:
            w.write(b"%x\r\n%s\r\n" % (len(line), line))
        return len(self.watchers)

    # ------------------------------------------------------------------ streaming
    async def _broadcast(self, data) -> None:
        for w in list(self.watchers):
            w.write(data)
        for w in list(self.watchers):
            try:
                await w.drain()
            except ConnectionError:
                pass

    async def send(self, step: int, rate: Optional[float] = None, count: Optional[int] = None,
                   drop_at: Optional[int] = None, expire_at: Optional[int] = None) -> int:
        n = self.E if count is None else min(count, self.E)
        cut = drop_at if drop_at is not None else expire_at
        pre = self.rendered.pop(step, None)
        if rate:
            t0 = time.monotonic()
            for i in range(n):
                self._advance(step, i, i + 1)
                await self._broadcast(self.t.line(step, i))
                delay = t0 + (i + 1) / rate - time.monotonic()
                if delay > 0:
                    await asyncio.sleep(delay)
            return n
        if pre is not None and count is None:
            data, offsets = pre
        else:
            data, offsets = self.t.render(step, 0, n)
        if not isinstance(data, bytes):  # a prerendered memory file
            try:
                return await self._send_file(step, n, data, offsets, drop_at, expire_at)
            finally:
                data.close()
        offsets = offsets + [len(data)]
        view = memoryview(data)
        i = 0
        while i < n:
            j = min(n, i + 1024)
            if cut is not None and i < cut <= j:
                j = cut
            # advance first: _broadcast writes before its first await, so a watch
            # that joins while we wait for drains gets exactly the events after this slice
            self._advance(step, i, j)
            await self._broadcast(view[offsets[i]:offsets[j]])
            i = j
            if cut is not None and i == cut:
                if drop_at is not None:
                    self.drop()
                else:
                    self.expire()
                cut = None
                await asyncio.sleep(0)
        return n


    async def _send_file(self, step: int, n: int, f, offsets: List[int], drop_at: Optional[int],
                         expire_at: Optional[int]) -> int:
        """``send`` for a prerendered step: same slicing, drop/expire points and
        watcher bookkeeping, but each slice goes out with sendfile()."""
        loop = asyncio.get_running_loop()
        size = os.fstat(f.fileno()).st_size
        offsets = offsets + [size]
        cut = drop_at if drop_at is not None else expire_at
        i = 0
        while i < n:
            j = min(n, i + 1024)
            if cut is not None and i < cut <= j:
                j = cut
            # advance before the first await (as _broadcast): a watch that joins
            # while this slice is in flight gets it from its backlog instead
            self._advance(step, i, j)
            targets = list(self.watchers)
            if targets:
                res = await asyncio.gather(*(loop.sendfile(w.transport, f, offsets[i], offsets[j] - offsets[i])
                                             for w in targets), return_exceptions=True)
                for w, r in zip(targets, res):
                    if isinstance(r, BaseException) and not isinstance(r, (ConnectionError, RuntimeError)):
                        raise r
            i = j
            if cut is not None and i == cut:
                if drop_at is not None:
                    self.drop()
                else:
                    self.expire()
                cut = None
                await asyncio.sleep(0)
        return n


async def amain(args) -> None:
    tmpl = Template(args.template, args.pods, args.seed, args.namespaces.split(",") if args.namespaces else None)
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
        opts = dict(p.split("=", 1) for p in parts[2:] if "=" in p)
        if cmd == "QUIT":
            break
        if cmd == "STEP":
            n = await srv.send(int(parts[1]), drop_at=int(opts["drop"]) if "drop" in opts else None,
                               expire_at=int(opts["expire"]) if "expire" in opts else None)
        elif cmd == "STEPS":
            n = 0
            for k in range(int(parts[1]), int(parts[2])):
                n += await srv.send(k)
            parts[1] = str(int(parts[2]) - 1)
        elif cmd == "PACE":
            rate = float(parts[2])
            n = await srv.send(int(parts[1]), rate or None, int(parts[3]))
        elif cmd == "WATCHERS":
            n = sum(1 for w in srv.watchers if not w.is_closing())
        elif cmd == "DROP":
            n = srv.drop()
        elif cmd == "EXPIRE":
            n = srv.expire()
        elif cmd == "BOOKMARK":
            n = srv.bookmark()
        else:
            n = -1
        print(f"SENT {parts[1] if len(parts) > 1 and cmd in ('STEP', 'STEPS', 'PACE') else '-'} {n}", flush=True)
    server.close()


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--template", default="churn", choices=["churn", "createdelete", "steady"])
    ap.add_argument("--pods", "--pods-per-step", dest="pods", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--namespaces", default=None)
    ap.add_argument("--prerender", type=int, default=0, help="render steps [0, N) before READY")
    asyncio.run(amain(ap.parse_args(argv)))


if __name__ == "__main__":
    main()
