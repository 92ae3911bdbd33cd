"""Sharding the pod space across watcher processes.

The reference is one process watching the whole cluster (SURVEY §5.7,
``/root/reference/watcher/pod_watcher.py:264``, client-side namespace filter
``:226-229``). For clusters whose event rate exceeds one core,
``watcher.shard.count`` watcher processes split the work.

Two ways to decide which shard owns what:

* **per event** (``namespace_scope: client``, or ``shard.key: uid``): every
  process watches the whole cluster and keeps the pods with
  ``crc32(key) % count == index`` — ``key`` is the namespace or the uid.
  Simple, but every process still receives every event.
* **per watch** (``namespace_scope: server`` with a namespace list, or
  ``namespace_scope: discover``): each process opens watches only for the
  namespaces it owns, so the API server sends each event to exactly one
  shard and the work really divides by ``count``. Which namespaces a shard
  owns is computed by every shard from the same namespace set:

  - ``shard.assignment: hash`` (default) — ``crc32(namespace) % count``:
    each namespace's owner depends on nothing else, so namespaces created or
    deleted later never move the others. Balance is statistical;
  - ``shard.assignment: balanced`` — consistent hashing with bounded loads
    (Mirrokni, Thorup & Zadimoghaddam, SODA 2018): namespaces, in hash
    order, take the first shard clockwise on a ring of virtual nodes that
    still has room under ``ceil(n / count)``, so every shard owns ``floor``
    or ``ceil`` of ``n / count`` namespaces. Meant for a fixed namespace
    set: when ``ceil(n / count)`` changes, a few namespaces move to another
    shard.

A namespace that moves is handed over when ``shard.handover_dir`` names a
directory all shards share (a ReadWriteMany volume,
``deploy/k8s/statefulset-sharded.yaml``). It moves in two ways:

* **live** — ``balanced`` on a namespace-set change: the old owner stops its
  watch, waits until clusterapi has acknowledged (or given up) every
  notification it still owes for the namespace (``pending_in``: a retried
  MODIFIED cannot land after the new owner's notifications for the same
  pod), then writes its cached pods there (:func:`write_handover`, one JSON
  file, atomically renamed);
* **across a restart** — a new shard count (``replicas`` and
  ``K8S_WATCHER_SHARD_COUNT`` changed together restart every shard): each
  shard notes the layout in the directory's history (:func:`record_layout`),
  so every shard, new ones included, knows the previous layout and which
  namespaces it gains from whom. An old owner, starting with a checkpoint
  that holds namespaces it no longer owns, writes their record — pods and the
  checkpoint's owed notifications for them — before it starts any watch.

The new owner waits for that record (``shard.handover_wait_seconds``; while
the old owner has not restarted yet it still watches the namespace, so the
wait loses nothing), sends the record's owed notifications first, loads the
pods into its cache and only then LISTs — so pods that stayed are not
re-announced and a pod deleted while neither shard watched is reported
``DELETED`` by the new owner's reconcile, exactly once. Without the directory
(or if the old owner is gone and the wait runs out) the new owner's LIST
re-announces the pods as ``ADDED`` (at-least-once) and a deletion inside that
window is not reported; a record that comes after such a timeout is stale and
is discarded, not taken by a later move.

crc32 is stable across processes and Python versions, unlike ``hash()``.
"""

from __future__ import annotations

import base64
import bisect
import json
import os
import tempfile
import time
import zlib
from typing import Dict, Iterable, List, NamedTuple, Optional, Sequence, Tuple

from ..utils.config import ShardSettings

VNODES = 64  # ring points per shard


def shard_of(key: Optional[str], count: int) -> int:
    if count <= 1:
        return 0
    return zlib.crc32((key or "").encode("utf-8")) % count


def _h(s: str) -> int:
    return zlib.crc32(s.encode("utf-8"))


def balanced_assignment(names: Iterable[str], count: int) -> Dict[str, int]:
    """Namespace → shard for ``count`` shards, with at most ``ceil(n / count)``
    namespaces per shard (bounded-load consistent hashing, see module doc).
    Deterministic: every shard computes the same map from the same set."""
    uniq = sorted(set(names))
    if count <= 1:
        return {n: 0 for n in uniq}
    ring = sorted((_h(f"shard-{s}#{v}"), s) for s in range(count) for v in range(VNODES))
    points = [p for p, _ in ring]
    cap = -(-len(uniq) // count)
    load = [0] * count
    out: Dict[str, int] = {}
    for name in sorted(uniq, key=lambda n: (_h(n), n)):
        i = bisect.bisect_left(points, _h(name))
        for step in range(len(ring)):
            s = ring[(i + step) % len(ring)][1]
            if load[s] < cap:
                break
        load[s] += 1
        out[name] = s
    return out


def owner_of(namespace: str, names: Iterable[str], count: int, assignment: str) -> int:
    """The shard owning ``namespace`` when the namespace set is ``names``."""
    if count <= 1:
        return 0
    if assignment == "hash":
        return shard_of(namespace, count)
    return balanced_assignment(list(names) + [namespace], count).get(namespace, 0)


# ---------------------------------------------------------------- hand-over
HANDOVER_VERSION = 2


def _handover_path(directory: str, namespace: str) -> str:
    return os.path.join(directory, f"{namespace}.handover.json")


Pod = Tuple[str, Optional[str], Optional[str], Optional[str], Optional[bytes]]
Owed = Tuple[str, str, Optional[str], Optional[str], bytes]


class HandOver(NamedTuple):
    """A namespace's state from its old owner: its cached pods and the
    notifications for them that clusterapi had not acknowledged (the new
    owner sends those first, before anything of its own)."""
    pods: List[Pod]
    owed: List[Owed]
    src: int
    written_at: float


def write_handover(directory: str, namespace: str, src: int, dst: int, pods: List[Pod],
                   owed: Optional[List[Owed]] = None, layout: Optional[dict] = None) -> str:
    """The old owner's cached pods of ``namespace`` — ``(uid, rv, phase, name,
    core)`` — and its owed notifications ``(uid, etype, ns, name, body)`` for
    shard ``dst``, stamped with the time and the shard layout it was written
    under; written to a temporary name and renamed, so a reader sees the whole
    record or none."""
    os.makedirs(directory, exist_ok=True)
    doc = {"version": HANDOVER_VERSION, "namespace": namespace, "from": src, "to": dst,
           "written_at": time.time(), "layout": layout,
           "pods": [[u, rv, ph, nm, core.decode("utf-8", "replace") if core is not None else None]
                    for u, rv, ph, nm, core in pods],
           "owed": [[u, et, ns, nm, base64.b64encode(body).decode("ascii")] for u, et, ns, nm, body in owed or ()]}
    path = _handover_path(directory, namespace)
    fd, tmp = tempfile.mkstemp(prefix=f".{namespace}.", dir=directory)
    try:
        with os.fdopen(fd, "w") as f:
            json.dump(doc, f, separators=(",", ":"))
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    return path


def take_handover(directory: str, namespace: str, dst: int, not_before: float = 0.0,
                  layout: Optional[dict] = None) -> Optional[HandOver]:
    """The record for shard ``dst`` if one is there (consumed: the file is
    removed), else None. Records addressed to another shard are left alone; a
    record for ``dst`` that is stale — written before ``not_before`` (an old
    move whose new owner timed out), or under another shard layout than
    ``layout`` — is removed and not taken (round-5 advisor: a late record
    must not prime a later move)."""
    path = _handover_path(directory, namespace)
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None
    if doc.get("version") != HANDOVER_VERSION or doc.get("namespace") != namespace or doc.get("to") != dst:
        return None
    stale = doc.get("written_at", 0.0) < not_before or (layout is not None and doc.get("layout") != layout)
    try:
        os.unlink(path)
    except OSError:
        pass
    if stale:
        return None
    return HandOver([(u, rv, ph, nm, core.encode("utf-8") if core is not None else None)
                     for u, rv, ph, nm, core in doc.get("pods", [])],
                    [(u, et, ns, nm, base64.b64decode(body)) for u, et, ns, nm, body in doc.get("owed", [])],
                    int(doc.get("from", -1)), float(doc.get("written_at", 0.0)))


# ---------------------------------------------------------------- layout history
def layout_of(s: ShardSettings) -> dict:
    """What decides namespace ownership: the shard count and the assignment."""
    return {"count": s.count, "assignment": s.assignment, "key": s.key}


def record_layout(directory: str, layout: dict) -> Tuple[Optional[dict], float]:
    """Note ``layout`` in the shared directory's history and return the layout
    before it and when this one began: ``(previous, since)``. Every shard of a
    resharded deployment (count 2 -> 3, say) sees the same previous layout,
    whichever starts first — the first to start under the new layout moves
    ``current`` to ``previous``; the others find ``current`` already theirs.
    ``(None, now)`` for a first deployment."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, "layout.json")
    try:
        with open(path) as f:
            hist = json.load(f)
    except (OSError, ValueError):
        hist = {}
    if hist.get("current") == layout:
        return hist.get("previous"), float(hist.get("since", 0.0))
    new = {"current": layout, "previous": hist.get("current"), "since": time.time()}
    fd, tmp = tempfile.mkstemp(prefix=".layout.", dir=directory)
    try:
        with os.fdopen(fd, "w") as f:
            json.dump(new, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    return new["previous"], new["since"]


class ShardFilter:
    __slots__ = ("count", "index", "by_uid", "active", "assignment")

    def __init__(self, s: ShardSettings) -> None:
        self.count = s.count
        self.index = s.index
        self.by_uid = s.key == "uid"
        self.active = s.count > 1
        self.assignment = getattr(s, "assignment", "hash")

    def owns(self, uid: Optional[str], namespace: Optional[str]) -> bool:
        """Per-event ownership (cluster-wide watches)."""
        if not self.active:
            return True
        return shard_of(uid if self.by_uid else namespace, self.count) == self.index

    def namespaces(self, namespaces: Sequence[str]) -> List[str]:
        """The subset of ``namespaces`` this shard watches server-side, in the given order."""
        ns = list(dict.fromkeys(namespaces))
        if not self.active or self.by_uid:
            return ns
        if self.assignment == "hash":
            return [n for n in ns if shard_of(n, self.count) == self.index]
        owner = balanced_assignment(ns, self.count)
        return [n for n in ns if owner[n] == self.index]
