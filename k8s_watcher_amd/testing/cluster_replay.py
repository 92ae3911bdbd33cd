"""One logical API server over many namespaces, served by several processes.

The N-rank benchmark (``bench.py --gpus N``) runs the product's sharded
scale-out: every rank is one watcher shard (``watcher.shard``) that opens pod
watches only for the namespaces it owns (``namespace_scope: discover``,
``engine/namespaces.py``). They must all watch the *same* cluster, or the
scaling curve measures nothing but independent copies. This fixture is that
cluster:

* a deterministic event history: ``--pods`` pod lifecycles per step (ADDED →
  3×MODIFIED → DELETED, ≈4 KB of real-shaped Pod JSON per event), spread
  round-robin over ``--namespaces`` namespaces and interleaved in one global
  order with one global resourceVersion sequence, as etcd would;
* served by ``--workers`` processes that each ``listen()`` on the same port
  with ``SO_REUSEPORT`` — the kernel spreads the watch connections, so the
  fixture is not one core feeding N watchers; ``--groups`` front-ends (one
  port each, like the replicas of an HA API server) serve the same cluster,
  each optionally pinned near the watcher that uses it (``--group-cpus``);
* any namespace watch (``/api/v1/namespaces/<ns>/pods``), the cluster-wide
  watch (``/api/v1/pods``), LISTs of both, ``/api/v1/namespaces`` (LIST and a
  quiet WATCH) and ``/version``.

Rendering is byte splicing, not JSON work. Each pod is stamped from one of
``--prototypes`` lifecycles (namespace, name and uid spliced in once per scope
when its first watch arrives); per step only the resourceVersion (always 9
digits) and the first 8 hex digits of each uid (the step number — pods are
re-created with fresh uids every step) change. So every scope keeps ONE
buffer of its events and a step overwrites those fixed-width fields in place
(vectorised with numpy, a few bytes per event) before the buffer is written
to each of the scope's watch connections: per event the fixture does one
copy into the kernel, as a real API server's watch cache would.

Control (stdin lines → one stdout line each), forwarded to every worker::

    READY {json: port, events_per_step, notifiable_per_step, namespaces}
    PREPARE <k0> <k1>          compile the open watches' scopes ahead of the first step -> OK
    STEP <k>                   stream step k to every watch       -> SENT k <events> <notifiable>
    STEPS <k0> <k1>            steps k0..k1-1 back to back, each worker on its own (no
                               controller round trip between steps) -> SENT k1-1 <events> <notifiable>
    PACE <k> <rate> <count>    first <count> events of step k at <rate>/s (0 = max) -> SENT k n m
    WATCHERS                   -> SENT - <open watch streams over all workers>
    ZCSTATS                    -> ZC [per worker: {scope: {bytes, waits}}] (zero-copy sends)
    QUIT

``notifiable`` counts the events the production profile notifies: critical
(DELETED or a terminal phase) and in one of ``--targets``.
"""

from __future__ import annotations

import argparse
import asyncio
import collections
import json
import os
import random
import socket
import sys
import time
from typing import Dict, List, Optional, Tuple
from urllib.parse import parse_qs, urlsplit

import numpy as np

from .podgen import PodFactory

try:  # the watcher's native module also re-stamps fixture buffers (optional here)
    from ..ops.native import load as _load_native
    _stamp = _load_native().stamp_fields
except Exception:  # noqa: BLE001 - fixtures must run without the extension too
    _stamp = None

RV0 = 1_000_000_000  # every resourceVersion has exactly 10 digits (room for 180k steps of 50k events)
RV_DIGITS = 10
STEP_HEX = 8  # uid prefix: the step number
_TYPES = (b'{"type":"ADDED","object":', b'{"type":"MODIFIED","object":', b'{"type":"MODIFIED","object":',
          b'{"type":"MODIFIED","object":', b'{"type":"DELETED","object":')
_HDR = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n"
_NS_PH, _NAME_PH, _UID_PH = b"@@NS@@", b"@@NAME@@", b"@@UID@@"
_RV_FIELD = b'"resourceVersion":"' + b"0" * RV_DIGITS + b'"'
TERMINAL = ("Succeeded", "Failed")


def namespace_names(n: int) -> List[str]:
    return [f"tenant-{i:03d}" for i in range(n)]


def pod_uid(step: int, pod: int) -> bytes:
    return b"%08x-0000-4000-8000-%012x" % (step & 0xFFFFFFFF, pod)


class ClusterModel:
    """The cluster's per-step event history (built once, before the workers fork)."""

    def __init__(self, namespaces: List[str], pods: int, seed: int = 0, prototypes: int = 256,
                 targets: Optional[List[str]] = None, interleave: int = 64, critical_only: bool = True) -> None:
        self.namespaces = list(namespaces)
        self.pods = pods
        f = PodFactory(seed, ["proto-ns"])
        self.protos: List[List[bytes]] = []  # [proto][stage] -> object JSON with placeholders
        self.proto_phase: List[List[str]] = []
        self.name_prefix: List[str] = []
        for _ in range(min(prototypes, max(1, pods))):
            lc = f.lifecycle()
            md0 = lc[0][1]["metadata"]
            name, uid = md0["name"], md0["uid"]
            self.name_prefix.append(name[:-5])
            stages, phases = [], []
            for _et, obj in lc:
                obj["metadata"]["resourceVersion"] = "0" * RV_DIGITS
                obj["metadata"]["namespace"] = "@@NS@@"
                obj["metadata"]["name"] = "@@NAME@@"
                raw = json.dumps(obj, separators=(",", ":"), ensure_ascii=False).encode("utf-8")
                stages.append(raw.replace(uid.encode(), _UID_PH))
                phases.append((obj.get("status") or {}).get("phase") or "")
            self.protos.append(stages)
            self.proto_phase.append(phases)
        # global order: `interleave` lifecycles in flight, a seeded random pick each time
        rng = random.Random(seed + 1)
        order_pod, order_stage = [], []
        active: List[List[int]] = []  # [pod, next stage]
        made = 0
        while made < pods or active:
            while made < pods and len(active) < interleave:
                active.append([made, 0])
                made += 1
            i = rng.randrange(len(active))
            p = active[i]
            order_pod.append(p[0])
            order_stage.append(p[1])
            p[1] += 1
            if p[1] == 5:
                active.pop(i)
        self.ev_pod = np.array(order_pod, dtype=np.int64)
        self.ev_stage = np.array(order_stage, dtype=np.int8)
        self.E = len(order_pod)
        n_ns = len(self.namespaces)
        self.ev_ns = (self.ev_pod % n_ns).astype(np.int32)
        proto = self.ev_pod % len(self.protos)
        phase_terminal = np.array([[ph in TERMINAL for ph in stages] for stages in self.proto_phase])
        critical = (self.ev_stage == 4) | phase_terminal[proto, self.ev_stage]
        tset = set(targets if targets is not None else self.namespaces)
        is_target = np.array([ns in tset for ns in self.namespaces])
        # what the watchers notify: the production profile's critical-events
        # filter (critical_only), then the namespace filter; other profiles notify
        # every event in a target namespace
        self.notifiable = (critical if critical_only else np.ones(self.E, dtype=bool)) & is_target[self.ev_ns]
        self.ns_index = {ns: i for i, ns in enumerate(self.namespaces)}

    def events_in(self, ns: str) -> int:
        return int(np.count_nonzero(self.ev_ns == self.ns_index[ns]))

    def notifiable_upto(self, count: int) -> int:
        return int(np.count_nonzero(self.notifiable[:count]))

    def event_obj(self, g: int) -> bytes:
        """Object JSON of global event ``g`` with step 0 / RV placeholders (list & backlog paths)."""
        pod = int(self.ev_pod[g])
        ns = self.namespaces[int(self.ev_ns[g])].encode()
        p = pod % len(self.protos)
        name = f"{self.name_prefix[p]}{pod:05x}".encode()
        raw = self.protos[p][int(self.ev_stage[g])]
        return raw.replace(_NS_PH, ns).replace(_NAME_PH, name).replace(_UID_PH, pod_uid(0, pod))

    def compile(self, scope: str) -> "ScopeStream":
        gidx = (np.arange(self.E, dtype=np.int64) if scope == "*"
                else np.flatnonzero(self.ev_ns == self.ns_index[scope]).astype(np.int64))
        parts: List[bytes] = []
        ev_off = np.zeros(len(gidx) + 1, dtype=np.int64)
        rv_off = np.zeros(len(gidx), dtype=np.int64)
        uid_off: List[int] = []
        pos = 0
        for j, g in enumerate(gidx.tolist()):
            body = _TYPES[int(self.ev_stage[g])] + self.event_obj(g) + b"}\n"
            head = b"%x\r\n" % len(body)
            chunk = head + body + b"\r\n"
            base = pos + len(head)
            k = body.find(_RV_FIELD)
            rv_off[j] = base + k + len(_RV_FIELD) - 1 - RV_DIGITS
            uid = pod_uid(0, int(self.ev_pod[g]))
            k = body.find(uid)
            while k >= 0:
                uid_off.append(base + k)
                k = body.find(uid, k + 1)
            parts.append(chunk)
            pos += len(chunk)
            ev_off[j + 1] = pos
        base_buf = np.frombuffer(b"".join(parts), dtype=np.uint8)
        sc = ScopeStream(scope, base_buf, ev_off, rv_off, np.array(uid_off, dtype=np.int64), gidx, self.E)
        sc.pod = self.ev_pod[gidx]
        sc.stage = self.ev_stage[gidx]
        return sc


class ScopeStream:
    """The events of one watch scope (a namespace or ``*``) as patchable bytes."""

    def __init__(self, scope: str, base: np.ndarray, ev_off: np.ndarray, rv_off: np.ndarray,
                 uid_off: np.ndarray, gidx: np.ndarray, E: int) -> None:
        self.scope, self.base, self.ev_off, self.rv_off = scope, base, ev_off, rv_off
        self.uid_off, self.gidx, self.E = uid_off, gidx, E
        self.buf: Optional[np.ndarray] = None  # patched in place per step (render / ensure)
        self.buf_step = -1
        self._rv_done = 0  # fields of buf_step patched so far (indices into rv_off / uid_off)
        self._uid_done = 0
        self.pod: np.ndarray = np.zeros(0, dtype=np.int64)   # per local event: pod index (ClusterModel.compile)
        self.stage: np.ndarray = np.zeros(0, dtype=np.int8)  # ... and lifecycle stage (4 = DELETED)
        self._live: Dict[int, np.ndarray] = {}  # local prefix length -> live pods' last events

    _POW10 = 10 ** np.arange(RV_DIGITS - 1, -1, -1, dtype=np.int64)
    _RV_COLS = np.arange(RV_DIGITS, dtype=np.int64)
    _UID_COLS = np.arange(STEP_HEX, dtype=np.int64)

    @classmethod
    def _patch(cls, buf: np.ndarray, rv_off: np.ndarray, rvs: np.ndarray, uid_off: np.ndarray, step: int) -> None:
        uid = b"%08x" % (step & 0xFFFFFFFF)
        if _stamp is not None:  # native: ~1 ns per digit
            _stamp(buf, np.ascontiguousarray(rv_off, dtype=np.int64), np.ascontiguousarray(rvs, dtype=np.int64),
                   RV_DIGITS, np.ascontiguousarray(uid_off, dtype=np.int64), uid)
            return
        # two scatters per call (every digit of every field at once), not one per digit
        buf[rv_off[:, None] + cls._RV_COLS] = (rvs[:, None] // cls._POW10 % 10 + 48).astype(np.uint8)
        buf[uid_off[:, None] + cls._UID_COLS] = np.frombuffer(uid, dtype=np.uint8)

    def render(self, step: int) -> memoryview:
        """The whole step: the scope's one buffer, its fixed-width fields set for ``step``."""
        self.ensure(step, len(self.base))
        return memoryview(self.buf)

    def ensure(self, step: int, end: int) -> memoryview:
        """Set ``step``'s fields in the bytes before ``end`` (a field that starts
        there is set whole). Sending a step patches each slice just before it
        is written, so the first bytes leave at once instead of after a pass
        over the whole buffer, and patching overlaps the kernel's copies."""
        if self.buf is None:
            self.buf = self.base.copy()
        if self.buf_step != step:
            self.buf_step, self._rv_done, self._uid_done = step, 0, 0
        j1 = int(np.searchsorted(self.rv_off, end))
        u1 = int(np.searchsorted(self.uid_off, end))
        if j1 > self._rv_done or u1 > self._uid_done:
            j0, u0 = self._rv_done, self._uid_done
            self._patch(self.buf, self.rv_off[j0:j1], RV0 + step * self.E + self.gidx[j0:j1],
                        self.uid_off[u0:u1], step)
            self._rv_done, self._uid_done = j1, u1
        return memoryview(self.buf)

    def event_bytes(self, step: int, j: int) -> bytes:
        return self.range_bytes(step, j, j + 1)

    def range_bytes(self, step: int, j0: int, j1: int) -> bytes:
        """Local events [j0, j1) of ``step`` as chunk-framed bytes: one copy of
        the base slice with its fields stamped (the shared buffer untouched)."""
        a, b = int(self.ev_off[j0]), int(self.ev_off[j1])
        buf = self.base[a:b].copy()
        lo, hi = np.searchsorted(self.uid_off, [a, b])
        self._patch(buf, self.rv_off[j0:j1] - a, RV0 + step * self.E + self.gidx[j0:j1],
                    self.uid_off[lo:hi] - a, step)
        return buf.tobytes()

    def object_bytes(self, step: int, j: int) -> bytes:
        """The pod object JSON of local event ``j`` of ``step`` (a LIST item)."""
        ev = self.event_bytes(step, j)
        body = ev[ev.index(b"\r\n") + 2:-2]
        return body[body.index(b'"object":') + 9:-2]

    def live_events(self, j1: int) -> np.ndarray:
        """Local indices of the last event of every pod still alive after this
        scope's events [0, j1) of one step (its ADDED sent, its DELETED not),
        ascending. A step is always sent as a prefix, and every lifecycle
        ends inside its step, so this is all a partly sent step leaves live.
        Vectorised and cached per prefix: no per-event Python loop."""
        got = self._live.get(j1)
        if got is None:
            if j1 <= 0:
                got = np.zeros(0, dtype=np.int64)
            else:
                rev = self.pod[:j1][::-1]
                _, first = np.unique(rev, return_index=True)
                last = (j1 - 1 - first).astype(np.int64)  # each pod's last event in the prefix
                got = np.sort(last[self.stage[last] != 4])
            if len(self._live) > 64:
                self._live.clear()
            self._live[j1] = got
        return got

    def locate(self, g0: int, g1: int) -> Tuple[int, int]:
        """Local event range of global events [g0, g1)."""
        return int(np.searchsorted(self.gidx, g0)), int(np.searchsorted(self.gidx, g1))


def _sysctl_int(path: str, field: int = 0, default: int = 0) -> int:
    try:
        with open(path) as fh:
            return int(fh.read().split()[field])
    except (OSError, ValueError, IndexError):
        return default


def receive_queue_bound() -> int:
    """The most data a peer socket on this host can hold unread: its receive
    buffer — autotuned up to ``tcp_rmem[2]``, or set with SO_RCVBUF (doubled
    by the kernel, capped at ``rmem_max``) — and no advertised window beyond it."""
    return max(_sysctl_int("/proc/sys/net/ipv4/tcp_rmem", 2, 6 << 20),
               2 * _sysctl_int("/proc/sys/net/core/rmem_max", 0, 4 << 20))


def _tcp_written(sock: socket.socket) -> Optional[int]:
    """Bytes this connection has handed to the kernel so far (acknowledged +
    still queued), in the coordinate of ``tcpi_bytes_acked``; None if gone."""
    import fcntl
    import struct
    import termios
    try:
        info = sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_INFO, 256)
        outq = struct.unpack("i", fcntl.ioctl(sock.fileno(), termios.TIOCOUTQ, b"\0\0\0\0"))[0]
    except OSError:
        return None
    return struct.unpack_from("Q", info, 120)[0] + outq  # tcp_info.tcpi_bytes_acked


def _tcp_acked(sock: socket.socket) -> Optional[int]:
    import struct
    try:
        return struct.unpack_from("Q", sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_INFO, 256), 120)[0]
    except OSError:
        return None


RING_MAX_SLOTS = 64
def ring_slots(step_bytes: int, bound: int) -> int:
    """Slots for a scope whose step is ``step_bytes``: the two steps after a
    slot's cover the peer's unread bound (3 for a step above it), else enough
    that the steps sent between two uses of a slot exceed twice the bound;
    0 when that takes more than RING_MAX_SLOTS (tiny scopes keep copying)."""
    if step_bytes <= 0:
        return 0
    if step_bytes >= bound:
        return 3
    k = -(-2 * bound // step_bytes) + 2
    return k if k <= RING_MAX_SLOTS else 0


class ZeroCopyRing:
    """``slots`` stamped copies of one scope's step bytes in a memfd, sent with
    ``sendfile``: the kernel references the pages instead of copying them
    into the socket (``write`` copied every byte: at ~10 GB/s of watch
    stream that one copy held the fixture's core).

    A slot's pages stay referenced by socket buffers until the watcher has
    read them (on loopback the receiver's queue holds the sender's pages), so
    a slot is re-stamped for a new step only once every connection that was
    sent from it has had its data acknowledged past that point by more than
    the most the peer can hold unread (:func:`receive_queue_bound`):
    ``acked - bound >= end``. The cluster-wide watch's step is larger than
    that bound: three slots, a slot is reused two whole steps later and never
    waits. A namespace scope's step is smaller: it gets enough slots that the
    steps sent after a slot's exceed twice the bound (:func:`ring_slots`), so
    it does not wait either."""

    def __init__(self, base: np.ndarray, slots: int, bound: int) -> None:
        import mmap
        self.n, self.slots, self.bound = len(base), slots, bound
        self.fd = os.memfd_create("cluster-replay", getattr(os, "MFD_CLOEXEC", 0))
        os.ftruncate(self.fd, self.n * slots)
        self.mm = mmap.mmap(self.fd, self.n * slots)
        arr = np.frombuffer(self.mm, dtype=np.uint8)
        self.views = [arr[i * self.n:(i + 1) * self.n] for i in range(slots)]
        for v in self.views:
            v[:] = base
        self.file = os.fdopen(os.dup(self.fd), "rb", buffering=0)
        self.step = [-1] * slots
        self.sent: List[List[Tuple[socket.socket, int]]] = [[] for _ in range(slots)]
        self.next = 0
        self.lock = asyncio.Lock()
        self.waits = 0  # times a slot was not yet safe to re-stamp (stats)
        self.bytes = 0

    def _safe(self, i: int) -> bool:
        for sock, end in self.sent[i]:
            acked = _tcp_acked(sock)
            if acked is not None and sock.fileno() >= 0 and acked - self.bound < end:
                return False
        return True

    async def slot_for(self, sc: "ScopeStream", step: int) -> int:
        async with self.lock:
            if step in self.step:
                return self.step.index(step)
            i = self.next
            while not self._safe(i):
                self.waits += 1
                await asyncio.sleep(0.0005)
            self.next = (i + 1) % self.slots
            self.sent[i] = []
            self.step[i] = -1
            v = self.views[i]
            sc._patch(v, sc.rv_off, RV0 + step * sc.E + sc.gidx, sc.uid_off, step)
            self.step[i] = step
            return i

    def note_sent(self, i: int, sock: socket.socket) -> None:
        end = _tcp_written(sock)
        if end is not None:
            self.sent[i].append((sock, end))

    def close(self) -> None:
        self.file.close()
        self.views = []
        try:
            self.mm.close()
        except BufferError:
            pass
        os.close(self.fd)


class Worker:
    """One serving process: its share of the watch connections, every command."""

    def __init__(self, model: ClusterModel, sock: socket.socket, slice_bytes: int = 1 << 20,
                 zero_copy: bool = True, zc_budget: int = 3 << 30) -> None:
        self.m = model
        self.sock = sock
        self.slice = slice_bytes
        self.zero_copy = zero_copy
        self.rq_bound = receive_queue_bound() + (1 << 20)
        self.rings: Dict[str, ZeroCopyRing] = {}
        self.zc_budget = zc_budget  # memfd bytes this worker may give rings (slots x step, all scopes)
        self.zc_used = 0
        self.no_ring: set = set()  # scopes left on the copy path (too small, or over the budget)
        self.scopes: Dict[str, ScopeStream] = {}
        self.watchers: List[Tuple[str, asyncio.StreamWriter]] = []
        self.sent: List[List[int]] = []  # [step, g0, g1) ranges of the global history sent so far
        self.sent_end: List[int] = []    # ... the resourceVersion of each range's last event (bisect)
        self.partial: Dict[int, int] = {}  # step -> g1 for steps sent only in part (they leave live pods)
        self.rv = RV0 - 1
        self.tls_conns: set = set()  # live native TLS connections (TLSSTATS)

    # ------------------------------------------------------------------ state
    def scope(self, name: str) -> ScopeStream:
        s = self.scopes.get(name)
        if s is None:
            s = self.scopes[name] = self.m.compile(name)
        return s

    def _advance(self, step: int, g0: int, g1: int) -> None:
        E = self.m.E
        if self.sent and self.sent[-1][0] == step and self.sent[-1][2] == g0:
            self.sent[-1][2] = g1
            self.sent_end[-1] = RV0 + step * E + g1 - 1
        else:
            self.sent.append([step, g0, g1])
            self.sent_end.append(RV0 + step * E + g1 - 1)
        if g1 < E:
            self.partial[step] = max(g1, self.partial.get(step, 0))
        else:
            self.partial.pop(step, None)
        self.rv = RV0 + step * E + g1 - 1

    def backlog(self, scope: ScopeStream, since: int) -> List[bytes]:
        """This scope's events sent with resourceVersion > ``since`` (a watch
        resuming there), as a few framed byte ranges: the first range that
        ends past ``since`` is found by bisection, and each range is one
        vectorised copy — no per-event Python loop over the history."""
        import bisect
        E = self.m.E
        out = []
        for i in range(bisect.bisect_right(self.sent_end, since), len(self.sent)):
            step, g0, g1 = self.sent[i]
            g0 = max(g0, since - (RV0 + step * E) + 1)
            lo, hi = scope.locate(g0, g1)
            if hi > lo:
                out.append(scope.range_bytes(step, lo, hi))
        return out

    def live_objects(self, scope: ScopeStream) -> List[bytes]:
        """Object JSON of every pod alive now in this scope: O(live pods) —
        only partly sent steps leave pods alive (``ScopeStream.live_events``)."""
        items = []
        for step in sorted(self.partial):
            _, j1 = scope.locate(0, self.partial[step])
            for j in scope.live_events(j1).tolist():
                items.append(scope.object_bytes(step, j))
        return items

    def list_body(self, name: str) -> bytes:
        items = self.live_objects(self.scope(name))
        return (b'{"kind":"PodList","apiVersion":"v1","metadata":{"resourceVersion":"%d"},"items":[%s]}'
                % (self.rv, b",".join(items)))

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
                u = urlsplit(line.split()[1].decode())
                q = {k: v[-1] for k, v in parse_qs(u.query).items()}
                watch = q.get("watch", "").lower() in ("true", "1")
                path = u.path
                if path == "/version":
                    body = b'{"major":"1","minor":"33","gitVersion":"v1.33.1-cluster-replay"}'
                elif path == "/api/v1/namespaces":
                    if watch:  # the namespace set never changes here: a quiet watch
                        writer.write(_HDR)
                        await reader.read()
                        return
                    body = json.dumps({"kind": "NamespaceList", "apiVersion": "v1",
                                       "metadata": {"resourceVersion": str(RV0 - 1)},
                                       "items": [{"metadata": {"name": n}} for n in self.m.namespaces]}).encode()
                elif path == "/api/v1/pods" or (path.startswith("/api/v1/namespaces/") and path.endswith("/pods")):
                    name = "*" if path == "/api/v1/pods" else path.split("/")[4]
                    if name != "*" and name not in self.m.ns_index:
                        body = b'{"kind":"PodList","apiVersion":"v1","metadata":{"resourceVersion":"%d"},' \
                               b'"items":[]}' % self.rv
                    elif watch:
                        self.start_watch(name, writer, q.get("resourceVersion"))
                        await reader.read()  # hold until the client goes away
                        return
                    else:
                        body = self.list_body(name)
                else:
                    writer.write(b"HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\n\r\n")
                    await writer.drain()
                    continue
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n"
                             % len(body) + body)
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            self.watchers = [(s, w) for s, w in self.watchers if w is not writer]
            writer.close()

    def start_watch(self, name: str, writer: asyncio.StreamWriter, rv_param: Optional[str]) -> None:
        """Synchronous: backlog and registration happen between two sends."""
        writer.write(_HDR)
        if name in self.m.ns_index or name == "*":
            sc = self.scope(name)
            since = int(rv_param) if rv_param not in (None, "", "0") else -1
            if since < 0:
                # no resourceVersion: synthetic ADDED for the live pods (as kube-apiserver)
                for obj in self.live_objects(sc):
                    ev = _TYPES[0] + obj + b"}\n"
                    writer.write(b"%x\r\n%s\r\n" % (len(ev), ev))
            else:
                for data in self.backlog(sc, since):
                    writer.write(data)
        self.watchers.append((name, writer))

    # ------------------------------------------------------------------ streaming
    def _targets(self) -> List[Tuple[str, asyncio.StreamWriter]]:
        return [(s, w) for s, w in self.watchers if not w.is_closing()]

    async def prepare(self, k0: int, k1: int) -> None:
        for n in sorted({s for s, _ in self._targets()}):
            self.scope(n).render(k0)

    async def _send(self, w: asyncio.StreamWriter, sc: ScopeStream, k: int) -> None:
        """Write step ``k`` of ``sc`` in slices, each patched just before it
        goes out, waiting for the socket between them: the transport copies at
        most one slice, and the scope's buffer is free to be patched again once
        every connection's send has returned."""
        try:
            n = len(sc.base)
            if isinstance(w, _TlsWriter):
                # native TLS: the slices are queued as they are patched (the
                # next slice's patch touches none of the earlier ones' bytes)
                # and sealed on the TLS pool meanwhile; one drain per step,
                # before the buffer may be patched for the next step
                sl = self.slice * 4
                for i in range(0, n, sl):
                    w.write(sc.ensure(k, min(n, i + sl))[i:i + sl])
                await w.drain()
                return
            for i in range(0, n, self.slice):
                view = sc.ensure(k, min(n, i + self.slice))
                w.write(view[i:i + self.slice])
                await w.drain()
        except (ConnectionError, RuntimeError):
            pass

    def ring(self, name: str, w: asyncio.StreamWriter) -> Optional[ZeroCopyRing]:
        """The scope's zero-copy ring, when this connection can use one: plain
        TCP (sendfile cannot go through TLS), a step large enough for
        :func:`ring_slots` and room in the worker's memfd budget."""
        if not self.zero_copy or name in self.no_ring or w.get_extra_info("sslcontext") is not None:
            return None
        r = self.rings.get(name)
        if r is None:
            sc = self.scope(name)
            slots = ring_slots(len(sc.base), self.rq_bound)
            if not slots or self.zc_used + slots * len(sc.base) > self.zc_budget:
                self.no_ring.add(name)
                return None
            self.zc_used += slots * len(sc.base)
            r = self.rings[name] = ZeroCopyRing(sc.base, slots, self.rq_bound)
        return r

    async def _send_zc(self, w: asyncio.StreamWriter, sc: ScopeStream, ring: ZeroCopyRing, k: int) -> None:
        """sendfile the step from its ring slot: straight from here while the
        transport has nothing buffered (a small scope's step fits the socket
        buffer: one syscall, no asyncio sendfile machinery per namespace),
        the rest through the loop's sendfile, which waits for the socket."""
        loop = asyncio.get_running_loop()
        try:
            i = await ring.slot_for(sc, k)
            sock = w.get_extra_info("socket")
            raw = getattr(sock, "_sock", sock)  # asyncio's TransportSocket wraps the socket
            base = i * ring.n
            sent = 0
            if w.transport.get_write_buffer_size() == 0:
                try:
                    sent = os.sendfile(raw.fileno(), ring.file.fileno(), base, ring.n)
                except (BlockingIOError, InterruptedError):
                    sent = 0
            if sent < ring.n:
                await loop.sendfile(w.transport, ring.file, base + sent, ring.n - sent, fallback=False)
            ring.bytes += ring.n
            ring.note_sent(i, raw)
        except (ConnectionError, RuntimeError, OSError):
            pass

    async def step(self, k: int) -> None:
        targets = self._targets()
        self._advance(k, 0, self.m.E)  # before the first await: a watch joining now gets it as backlog
        sends = []
        for n, w in targets:
            r = self.ring(n, w)
            sends.append(self._send_zc(w, self.scope(n), r, k) if r is not None else self._send(w, self.scope(n), k))
        await asyncio.gather(*sends)

    async def pace(self, k: int, rate: float, count: int, tick: float = 0.0005) -> None:
        """The first ``count`` events of step ``k`` at ``rate`` ev/s over the whole
        cluster (0 = as fast as the sockets take them). Every ``tick`` seconds
        each watch gets, as one write, the contiguous slice of its scope's
        buffer covering the global events due by then — so the offered load
        can reach hundreds of thousands of events/s, and at low rates each
        event still leaves within ``tick`` of its schedule."""
        targets = self._targets()
        views = {n: self.scope(n).render(k) for n in {s for s, _ in targets}}
        pos = {id(w): self.scope(n).locate(0, 0)[0] for n, w in targets}
        t0 = time.monotonic()
        g0 = 0
        while g0 < count:
            if rate:
                due = min(count, int((time.monotonic() - t0) * rate) + 1)
            else:
                due = min(count, g0 + 4096)
            if due > g0:
                self._advance(k, g0, due)
                for n, w in targets:
                    sc = self.scopes[n]
                    j0 = pos[id(w)]
                    j1 = int(np.searchsorted(sc.gidx, due))
                    if j1 > j0:
                        w.write(views[n][int(sc.ev_off[j0]):int(sc.ev_off[j1])])
                        pos[id(w)] = j1
                g0 = due
            if g0 >= count:
                break
            if rate:
                await asyncio.sleep(max(0.0, min(tick, t0 + (g0 + 1) / rate - time.monotonic())))
            else:
                for _, w in targets:
                    try:
                        await w.drain()
                    except ConnectionError:
                        pass
        for _, w in self._targets():
            try:
                await w.drain()
            except ConnectionError:
                pass

    async def _accept_tls(self, tls) -> None:
        """https with the native TLS server: accept, hand the socket to
        OpenSSL for the handshake (on an executor thread), then serve the
        connection through _TlsReader / _TlsWriter."""
        import concurrent.futures
        loop = asyncio.get_running_loop()
        ex = concurrent.futures.ThreadPoolExecutor(max_workers=16, thread_name_prefix="tls")
        self.sock.setblocking(False)

        async def one(fd: int) -> None:
            try:
                conn = await loop.run_in_executor(ex, tls.accept, fd)
            except OSError:
                return
            self.tls_conns.add(conn)
            try:
                await self.handle(_TlsReader(conn), _TlsWriter(conn, ex))
            finally:
                self.tls_conns.discard(conn)

        while True:
            c, _ = await loop.sock_accept(self.sock)
            c.setblocking(False)
            asyncio.ensure_future(one(c.detach()))

    async def serve(self, ctrl_in: int, ctrl_out: int, ssl_ctx=None) -> None:
        loop = asyncio.get_running_loop()
        if ssl_ctx is not None and not isinstance(ssl_ctx, __import__("ssl").SSLContext):
            server = None  # native TLS (a _kwcore.TlsServerContext)
            acceptor = asyncio.ensure_future(self._accept_tls(ssl_ctx))
        else:
            server = await asyncio.start_server(self.handle, sock=self.sock, limit=1 << 20, ssl=ssl_ctx)
            acceptor = None
        reader = asyncio.StreamReader()
        await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), os.fdopen(ctrl_in, "rb"))
        out = os.fdopen(ctrl_out, "wb", buffering=0)
        out.write(b"READY\n")
        while True:
            line = await reader.readline()
            if not line:
                break
            parts = line.decode().split()
            cmd = parts[0].upper() if parts else ""
            reply = "OK"
            if cmd == "QUIT":
                break
            if cmd == "PREPARE":
                await self.prepare(int(parts[1]), int(parts[2]))
            elif cmd == "STEP":
                await self.step(int(parts[1]))
            elif cmd == "STEPS":  # back to back, no round trip to the controller between steps
                for k in range(int(parts[1]), int(parts[2])):
                    await self.step(k)
            elif cmd == "PACE":
                await self.pace(int(parts[1]), float(parts[2]), min(int(parts[3]), self.m.E))
            elif cmd == "WATCHERS":
                reply = str(len(self._targets()))
            elif cmd == "ZCSTATS":  # zero-copy sends: bytes, slot waits
                reply = json.dumps({n: {"bytes": r.bytes, "waits": r.waits} for n, r in self.rings.items()},
                                   separators=(",", ":"))
            elif cmd == "TLSSTATS":  # native TLS sends: bytes and where the senders' time went (summed)
                tot: Dict[str, int] = {"connections": 0}
                for conn in list(self.tls_conns):
                    tot["connections"] += 1
                    for key, v in conn.stats().items():
                        tot[key] = tot.get(key, 0) + v
                reply = json.dumps(tot, separators=(",", ":"))
            out.write(reply.encode() + b"\n")
        if server is not None:
            server.close()
        if acceptor is not None:
            acceptor.cancel()
        for r in self.rings.values():
            r.close()


class _TlsReader:
    """StreamReader's ``readline``/``read`` over a native TLS connection
    (``_kwcore.TlsConn``): requests are decrypted by OpenSSL on the event
    loop's thread when the socket is readable (non-blocking)."""

    def __init__(self, conn) -> None:
        self.conn = conn
        self.buf = bytearray()
        self.eof = False

    async def _fill(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            data = self.conn.recv(65536)
            if data is None:  # nothing yet: wait for the socket
                fd = self.conn.fileno()
                if fd < 0:
                    self.eof = True
                    return
                fut = loop.create_future()
                loop.add_reader(fd, lambda: fut.done() or fut.set_result(None))
                try:
                    await fut
                finally:
                    loop.remove_reader(fd)
                continue
            if not data:
                self.eof = True
            self.buf += data
            return

    async def readline(self) -> bytes:
        while True:
            i = self.buf.find(b"\n")
            if i >= 0:
                line = bytes(self.buf[:i + 1])
                del self.buf[:i + 1]
                return line
            if self.eof:
                line = bytes(self.buf)
                self.buf.clear()
                return line
            await self._fill()

    async def read(self) -> bytes:
        while not self.eof:
            await self._fill()
        data = bytes(self.buf)
        self.buf.clear()
        return data


class _TlsWriter:
    """StreamWriter's ``write``/``drain`` over a native TLS connection: writes
    queue in order and go out on an executor thread, sealed into TLS 1.3
    records on the context's thread pool (``_kwcore.TlsServerContext``) —
    the event loop never encrypts. A queued view must stay unchanged until
    ``drain()`` returns, as with the plain path's slices."""

    def __init__(self, conn, executor) -> None:
        self.conn = conn
        self.ex = executor
        self.q: "collections.deque" = collections.deque()
        self.task = None
        self.idle = asyncio.Event()
        self.idle.set()
        self.closed = False
        self.failed = False

    def write(self, data) -> None:
        if self.closed:
            return
        self.q.append(data)
        self.idle.clear()
        if self.task is None:
            self.task = asyncio.ensure_future(self._pump())

    def _send_parts(self, parts) -> None:
        conn = self.conn
        if conn is None:
            raise BrokenPipeError("closed")
        small = []
        for p in parts:  # small pieces (a watch's backlog, event by event) are sealed together
            if len(p) < (64 << 10):
                small.append(p)
                continue
            if small:
                conn.send(b"".join(small))
                small = []
            conn.send(p)
        if small:
            conn.send(b"".join(small))

    async def _pump(self) -> None:
        loop = asyncio.get_running_loop()
        try:
            while self.q:
                parts = list(self.q)  # everything queued so far: one executor hop
                self.q.clear()
                await loop.run_in_executor(self.ex, self._send_parts, parts)
        except OSError:
            self.failed = self.closed = True
            self.q.clear()
        finally:
            self.task = None
            self.idle.set()

    async def drain(self) -> None:
        await self.idle.wait()
        if self.failed:
            raise ConnectionResetError("TLS connection closed")

    def is_closing(self) -> bool:
        return self.closed

    def get_extra_info(self, name: str, default=None):
        return True if name == "sslcontext" else default

    def close(self) -> None:
        if self.conn is None:
            return
        self.closed = True
        conn, self.conn = self.conn, None

        async def later() -> None:
            await self.idle.wait()
            conn.close()
        asyncio.ensure_future(later())


def _cpu_list(text: str) -> set:
    out = set()
    for part in text.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part.strip():
            out.add(int(part))
    return out


def _reuseport_socket(port: int, listen: bool) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind(("127.0.0.1", port))
    if listen:
        s.listen(1024)
        s.setblocking(False)
    return s


def run(args) -> None:
    namespaces = (args.namespace_list.split(",") if args.namespace_list
                  else namespace_names(args.namespaces))
    targets = args.targets.split(",") if args.targets else None
    model = ClusterModel(namespaces, args.pods, args.seed, args.prototypes, targets,
                         critical_only=args.notify == "critical")
    # front-ends: like the replicas of an HA API server, each group of workers
    # listens on its own port and serves the same cluster (every worker holds
    # the whole history); a client picks one. --group-cpus pins each group.
    cpus = [_cpu_list(x) for x in args.group_cpus.split(";")] if args.group_cpus else []
    groups = max(1, args.groups)
    reserves = [_reuseport_socket(args.port if g == 0 else 0, listen=False) for g in range(groups)]
    ports = [r.getsockname()[1] for r in reserves]  # held; the workers listen on them
    workers = []  # (pid, ctrl_w, reply_r)
    for g in range(groups):
        for _ in range(max(1, args.workers)):
            c_r, c_w = os.pipe()
            r_r, r_w = os.pipe()
            pid = os.fork()
            if pid == 0:
                os.close(c_w)
                os.close(r_r)
                for r in reserves:
                    r.close()
                try:
                    if g < len(cpus) and cpus[g]:
                        os.sched_setaffinity(0, cpus[g])
                    ssl_ctx = None
                    if args.tls_cert:  # https API server (the watcher's TLS path)
                        if args.tls_engine == "native":  # records sealed on a thread pool (ops/csrc/tls13.inc)
                            ssl_ctx = _load_native().TlsServerContext(args.tls_cert, args.tls_key,
                                                                      threads=args.tls_threads)
                        else:
                            import ssl
                            ssl_ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
                            ssl_ctx.load_cert_chain(args.tls_cert, args.tls_key)
                    asyncio.run(Worker(model, _reuseport_socket(ports[g], listen=True),
                                       zero_copy=args.zero_copy != "off",
                                       zc_budget=int(args.zero_copy_budget_mb) << 20).serve(c_r, r_w, ssl_ctx))
                finally:
                    os._exit(0)
            os.close(c_r)
            os.close(r_w)
            workers.append((pid, os.fdopen(c_w, "wb", buffering=0), os.fdopen(r_r, "rb", buffering=0)))
    for _, _, rd in workers:
        assert rd.readline().strip() == b"READY"
    port = ports[0]
    info = {"port": port, "ports": ports, "events_per_step": model.E,
            "notifiable_per_step": model.notifiable_upto(model.E),
            "namespaces": {ns: model.events_in(ns) for ns in namespaces}, "workers": len(workers)}
    print("READY " + json.dumps(info, separators=(",", ":")), flush=True)
    for line in sys.stdin:
        parts = line.split()
        if not parts:
            continue
        cmd = parts[0].upper()
        for _, wr, _ in workers:
            wr.write(line.encode() if line.endswith("\n") else (line + "\n").encode())
        if cmd == "QUIT":
            break
        replies = [rd.readline().decode().strip() for _, _, rd in workers]
        if cmd == "STEP":
            print(f"SENT {parts[1]} {model.E} {model.notifiable_upto(model.E)}", flush=True)
        elif cmd == "STEPS":
            k = int(parts[2]) - int(parts[1])
            print(f"SENT {int(parts[2]) - 1} {model.E * k} {model.notifiable_upto(model.E) * k}", flush=True)
        elif cmd == "PACE":
            n = min(int(parts[3]), model.E)
            print(f"SENT {parts[1]} {n} {model.notifiable_upto(n)}", flush=True)
        elif cmd == "WATCHERS":
            print(f"SENT - {sum(int(r) for r in replies)}", flush=True)
        elif cmd == "ZCSTATS":
            print("ZC " + json.dumps([json.loads(r) for r in replies], separators=(",", ":")), flush=True)
        elif cmd == "TLSSTATS":
            print("TLS " + json.dumps([json.loads(r) for r in replies], separators=(",", ":")), flush=True)
        else:
            print("OK", flush=True)
    for pid, wr, _ in workers:
        try:
            wr.write(b"QUIT\n")
        except BrokenPipeError:
            pass
    for pid, _, _ in workers:
        try:
            os.waitpid(pid, 0)
        except ChildProcessError:
            pass


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--pods", type=int, default=10000, help="pod lifecycles per step, whole cluster")
    ap.add_argument("--namespaces", type=int, default=64)
    ap.add_argument("--namespace-list", default=None, help="comma-separated names instead of tenant-NNN")
    ap.add_argument("--targets", default=None, help="namespaces the watchers notify for (notifiable counts)")
    ap.add_argument("--workers", type=int, default=2, help="worker processes per front-end")
    ap.add_argument("--groups", type=int, default=1, help="front-ends (ports) serving the same cluster")
    ap.add_argument("--tls-cert", default=None, help="serve https with this certificate (and --tls-key)")
    ap.add_argument("--tls-key", default=None)
    ap.add_argument("--tls-engine", default="native", choices=["native", "python"],
                    help="native: OpenSSL handshake + TLS 1.3 records sealed on --tls-threads threads "
                         "(_kwcore.TlsServerContext); python: asyncio's ssl transport")
    ap.add_argument("--tls-threads", type=int, default=3, help="sealing threads per worker (native TLS)")
    ap.add_argument("--group-cpus", default=None, help="';'-separated CPU lists, one per front-end")
    ap.add_argument("--notify", default="critical", choices=["critical", "all"],
                    help="which events of the target namespaces count as notifiable: the production "
                         "profile's critical-events filter, or every one (development/staging)")
    ap.add_argument("--zero-copy", default="auto", choices=["auto", "off"],
                    help="auto: scopes whose step outgrows a peer's receive buffer are sent with sendfile "
                         "from a memfd ring (ZeroCopyRing); off: every scope is written (copied)")
    ap.add_argument("--zero-copy-budget-mb", type=int, default=3072,
                    help="memfd memory per worker for zero-copy rings (scopes past it copy)")
    ap.add_argument("--prototypes", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    run(ap.parse_args(argv))


if __name__ == "__main__":
    main()
