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
    shard, whose first LIST re-announces their pods as ``ADDED``
    (at-least-once for pods that exist across that hand-over). Deletions
    are not covered: the losing shard forgets the namespace's cached pods
    without notifying, and the gaining shard's LIST only sees pods that
    still exist, so a pod deleted between the two shards' views of the
    namespace set is never reported ``DELETED``. Use ``hash`` (namespaces
    never move) where every deletion must be reported.

crc32 is stable across processes and Python versions, unlike ``hash()``.
"""

from __future__ import annotations

import bisect
import zlib
from typing import Dict, Iterable, List, Optional, Sequence

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
