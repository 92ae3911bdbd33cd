"""API-server fixture for relist storms (``benchmarks/relist_storm.py``).

Serves a large, mostly static cluster — N namespaces × P running pods — to
watchers in any scope shape (``/api/v1/pods``, ``/api/v1/namespaces/<ns>/pods``,
the namespace list and its watch), and on command makes every pod watch
expire at once, the way an etcd compaction past all their resourceVersions
does: each open watch gets ``ERROR 410`` and ends, and any watch resumed from
an older resourceVersion gets the same. The watchers' answer is a relist of
every scope — the recovery path of the reference, whose restart re-lists the
whole cluster (``/root/reference/watcher/pod_watcher.py:264,273-275``).

What the cluster does while the watches are down is scripted (``CHURN``):
some pods finish (``MODIFIED`` to ``Succeeded``), some are deleted, some are
created — with no watch event, so only the relist diff can deliver them. The
fixture writes the ``uid|event_type|phase`` keys a correct watcher must then
notify, for the sink's exactly-once check.

Pods are kept pre-serialised (one prototype per pod shape, name/uid/namespace
and resourceVersion spliced in), so a LIST page is a join of bytes: the
fixture's cost stays far below the watcher's and the relist is measured on
the watcher side. Control (stdin → one stdout line each)::

    READY {"port": p, "pods": n, "namespaces": n}
    CHURN <n> <seed>   n finish + n delete + n create, silently -> OK {"expected": file, "keys": k}
    EXPIRE             every pod watch: ERROR 410 + end; older RVs now 410 -> OK {"expired": w}
    STATS              -> OK {"lists": ..., "list_bytes": ..., "pod_watches": ..., "rv": ...}
    QUIT
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

from .podgen import PodFactory

_HDR = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n"
_NS, _NAME, _UID, _RV = b"@@NS@@", b"@@NAME@@", b"@@UID@@", b"@@RV@@"


def _chunk(data: bytes) -> bytes:
    return b"%x\r\n%s\r\n" % (len(data), data)


class Cluster:
    def __init__(self, namespaces: int, pods: int, seed: int = 0, prototypes: int = 64) -> None:
        self.namespaces = [f"ns-{i:04d}" for i in range(namespaces)]
        f = PodFactory(seed, ["proto"])
        self.protos: List[Tuple[bytes, bytes]] = []  # (running, succeeded) with placeholders
        for _ in range(prototypes):
            p = f.running(f.scheduled(f.new_pod()))
            done = f.terminated(p)
            pair = []
            for obj in (p, done):
                md = obj["metadata"]
                md.update(namespace="@@NS@@", name="@@NAME@@", uid="@@UID@@", resourceVersion="@@RV@@")
                pair.append(json.dumps(obj, separators=(",", ":")).encode())
            self.protos.append((pair[0], pair[1]))
        self.rv = 1000
        self.compacted = 0
        # (ns, name) -> [uid, proto, state(0 running / 1 succeeded), rv, bytes]
        self.pods: Dict[Tuple[str, str], list] = {}
        self.order: Dict[str, List[str]] = {}  # scope -> sorted names (rebuilt when dirty)
        self.dirty = True
        self.serial = 0
        for i in range(pods):
            ns = self.namespaces[i % namespaces]
            self._put(ns, f"pod-{i:07d}", f"{seed:04x}0000-0000-4000-8000-{i:012x}", i % prototypes, 0)

    def _render(self, ns: str, name: str, ent: list) -> bytes:
        raw = self.protos[ent[1]][ent[2]]
        return (raw.replace(_NS, ns.encode()).replace(_NAME, name.encode()).replace(_UID, ent[0].encode())
                .replace(_RV, str(ent[3]).encode()))

    def _put(self, ns: str, name: str, uid: str, proto: int, state: int) -> bytes:
        self.rv += 1
        ent = [uid, proto, state, self.rv, b""]
        ent[4] = self._render(ns, name, ent)
        self.pods[(ns, name)] = ent
        self.dirty = True
        return ent[4]

    def keys(self, scope: str) -> List[Tuple[str, str]]:
        if self.dirty:
            by_ns: Dict[str, List[Tuple[str, str]]] = {}
            for k in sorted(self.pods):
                by_ns.setdefault(k[0], []).append(k)
            self.order = {"*": sorted(self.pods)}
            self.order.update(by_ns)
            self.dirty = False
        return self.order.get(scope, [])

    def churn(self, n: int, seed: int) -> List[str]:
        """n pods finish, n are deleted, n are created — no watch events. The
        keys a watcher must notify for them (staging profile: every event)."""
        rng = random.Random(seed)
        live = sorted(self.pods)
        picks = rng.sample(live, min(len(live), 2 * n))
        out = []
        for ns, name in picks[:n]:
            ent = self.pods[(ns, name)]
            if ent[2] == 1:
                continue
            self._put(ns, name, ent[0], ent[1], 1)
            out.append(f"{ent[0]}|MODIFIED|Succeeded")
        for ns, name in picks[n:]:
            ent = self.pods.pop((ns, name))
            self.rv += 1
            self.dirty = True
            out.append(f"{ent[0]}|DELETED|{'Running' if ent[2] == 0 else 'Succeeded'}")
        for _ in range(n):
            self.serial += 1
            ns = self.namespaces[rng.randrange(len(self.namespaces))]
            uid = f"{seed:04x}ffff-0000-4000-8000-{self.serial:012x}"
            self._put(ns, f"new-{seed}-{self.serial:06d}", uid, rng.randrange(len(self.protos)), 0)
            out.append(f"{uid}|ADDED|Running")
        return out


class StormServer:
    def __init__(self, cluster: Cluster) -> None:
        self.c = cluster
        self.pod_watches: List[Tuple[str, asyncio.StreamWriter]] = []
        self.ns_watches: List[asyncio.StreamWriter] = []
        self.lists = 0
        self.list_bytes = 0
        self.watch_lists = 0

    def list_page(self, scope: str, limit: Optional[int], cont: Optional[str]) -> Tuple[int, bytes]:
        keys = self.c.keys(scope)
        start = 0
        if cont:
            rv_s, off = cont.split(":")
            if int(rv_s) < self.c.compacted:  # the snapshot the token points into is compacted
                body = json.dumps({"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 410,
                                   "reason": "Expired", "message": "continue token expired"}).encode()
                return 410, body
            start = int(off)
        end = len(keys) if not limit else min(len(keys), start + limit)
        items = b",".join(self.c.pods[k][4] for k in keys[start:end])
        md = b'{"resourceVersion":"%d"' % self.c.rv
        if end < len(keys):  # as kube-apiserver: the token and how many items are left
            md += b',"continue":"%d:%d","remainingItemCount":%d' % (self.c.rv, end, len(keys) - end)
        self.lists += 1
        body = b'{"kind":"PodList","apiVersion":"v1","metadata":%s},"items":[%s]}' % (md, items)
        self.list_bytes += len(body)
        return 200, body

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
                u = urlsplit(line.split()[1].decode())
                q = {k: v[-1] for k, v in parse_qs(u.query).items()}
                watch = q.get("watch", "").lower() in ("true", "1")
                path = u.path
                status = 200
                if path == "/version":
                    body = b'{"major":"1","minor":"33","gitVersion":"v1.33.1-storm"}'
                elif path == "/api/v1/namespaces":
                    if watch:  # the namespace set stays: a quiet watch
                        writer.write(_HDR)
                        self.ns_watches.append(writer)
                        await reader.read()
                        return
                    body = json.dumps({"kind": "NamespaceList", "apiVersion": "v1",
                                       "metadata": {"resourceVersion": str(self.c.rv)},
                                       "items": [{"metadata": {"name": n}} for n in self.c.namespaces]}).encode()
                elif path == "/api/v1/pods" or (path.startswith("/api/v1/namespaces/") and path.endswith("/pods")):
                    scope = "*" if path == "/api/v1/pods" else path.split("/")[4]
                    if watch:
                        rv = q.get("resourceVersion")
                        writer.write(_HDR)
                        if q.get("sendInitialEvents", "").lower() == "true":
                            # WatchList (KEP-3157): the scope's pods as ADDED, then the
                            # initial-events-end bookmark, then the live watch
                            await self.initial_events(scope, writer)
                            self.watch_lists += 1
                            self.pod_watches.append((scope, writer))
                            await reader.read()
                            return
                        if rv and rv != "0" and int(rv) < self.c.compacted:
                            err = json.dumps({"type": "ERROR", "object": {
                                "kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 410,
                                "reason": "Expired", "message": f"too old resource version: {rv}"}}).encode()
                            writer.write(_chunk(err + b"\n") + b"0\r\n\r\n")
                            await writer.drain()
                            return
                        self.pod_watches.append((scope, writer))
                        await reader.read()
                        return
                    limit = int(q["limit"]) if q.get("limit") else None
                    status, body = self.list_page(scope, limit, q.get("continue"))
                else:
                    status, body = 404, b"{}"
                reason = {200: b"OK", 404: b"Not Found", 410: b"Gone"}[status]
                writer.write(b"HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
                             % (status, reason, len(body)) + body)
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError, ValueError):
            return
        finally:
            self.pod_watches = [(s, w) for s, w in self.pod_watches if w is not writer]
            self.ns_watches = [w for w in self.ns_watches if w is not writer]
            writer.close()

    async def initial_events(self, scope: str, writer: asyncio.StreamWriter) -> None:
        """ADDED for every pod of the scope (one chunk per event, as the API
        server writes them), sent in ~1 MiB slices, then the bookmark."""
        buf = []
        size = 0
        for k in list(self.c.keys(scope)):
            ent = self.c.pods.get(k)
            if ent is None:
                continue
            buf.append(_chunk(b'{"type":"ADDED","object":' + ent[4] + b"}\n"))
            size += len(buf[-1])
            if size >= (1 << 20):
                writer.write(b"".join(buf))
                buf, size = [], 0
                await writer.drain()
        bm = {"type": "BOOKMARK", "object": {"kind": "Pod", "apiVersion": "v1", "metadata": {
            "resourceVersion": str(self.c.rv), "annotations": {"k8s.io/initial-events-end": "true"}}}}
        buf.append(_chunk(json.dumps(bm, separators=(",", ":")).encode() + b"\n"))
        writer.write(b"".join(buf))
        await writer.drain()

    def expire(self) -> int:
        self.c.rv += 1  # the compaction's own revision: every watch is now behind it
        self.c.compacted = self.c.rv
        err = json.dumps({"type": "ERROR", "object": {
            "kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 410, "reason": "Expired",
            "message": "too old resource version"}}).encode() + b"\n"
        n = 0
        for _, w in self.pod_watches:
            try:
                w.write(_chunk(err) + b"0\r\n\r\n")
                w.close()
                n += 1
            except Exception:  # noqa: BLE001
                pass
        self.pod_watches = []
        return n


async def serve(args) -> None:
    cluster = Cluster(args.namespaces, args.pods, args.seed)
    srv = StormServer(cluster)
    server = await asyncio.start_server(srv.handle, "127.0.0.1", args.port, limit=1 << 20)
    port = server.sockets[0].getsockname()[1]
    loop = asyncio.get_running_loop()
    rd = asyncio.StreamReader()
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(rd), sys.stdin)
    print("READY " + json.dumps({"port": port, "pods": len(cluster.pods), "namespaces": len(cluster.namespaces)}),
          flush=True)
    while True:
        line = (await rd.readline()).decode().split()
        if not line or line[0] == "QUIT":
            break
        cmd = line[0].upper()
        if cmd == "CHURN":
            keys = cluster.churn(int(line[1]), int(line[2]))
            path = os.path.join(args.out_dir or "/tmp", f"storm-expected-{os.getpid()}-{line[2]}.json")
            with open(path, "w") as fh:
                json.dump(keys, fh)
            reply = {"expected": path, "keys": len(keys)}
        elif cmd == "EXPIRE":
            reply = {"expired": srv.expire()}
        elif cmd == "STATS":
            reply = {"lists": srv.lists, "list_bytes": srv.list_bytes, "watch_lists": srv.watch_lists,
                     "pod_watches": len(srv.pod_watches),
                     "rv": cluster.rv, "pods": len(cluster.pods)}
        else:
            reply = {"error": f"unknown command {cmd}"}
        print("OK " + json.dumps(reply), flush=True)
    server.close()


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--namespaces", type=int, default=1000)
    ap.add_argument("--pods", type=int, default=100000, help="pods in the whole cluster")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out-dir", default=None)
    asyncio.run(serve(ap.parse_args(argv)))


if __name__ == "__main__":
    main()
