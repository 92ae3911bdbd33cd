"""Sharding the pod space across watcher processes.

The reference is one process watching the whole cluster. For
clusters whose event rate exceeds one core, ``watcher.shard.count`` watcher
processes split the work: a pod belongs to shard
``crc32(key) % count`` where ``key`` is its namespace (default — a namespace
stays whole, and with ``namespace_scope: server`` each process only opens
watches for its own namespaces) or its uid (even spread, one cluster-wide
watch per process). crc32 is stable across processes and Python versions,
unlike ``hash()``.
"""

from __future__ import annotations

import zlib
from typing import Iterable, List, Optional

from ..utils.config import ShardSettings


def shard_of(key: Optional[str], count: int) -> int:
    if count <= 1:
        return 0
    return zlib.crc32((key or "").encode("utf-8")) % count


class ShardFilter:
    __slots__ = ("count", "index", "by_uid", "active")

    def __init__(self, s: ShardSettings) -> None:
        self.count = s.count
        self.index = s.index
        self.by_uid = s.key == "uid"
        self.active = s.count > 1

    def owns(self, uid: Optional[str], namespace: Optional[str]) -> bool:
        if not self.active:
            return True
        return shard_of(uid if self.by_uid else namespace, self.count) == self.index

    def namespaces(self, namespaces: Iterable[str]) -> List[str]:
        """The subset of target namespaces this shard watches server-side."""
        ns = list(namespaces)
        if not self.active or self.by_uid:
            return ns
        return [n for n in ns if shard_of(n, self.count) == self.index]
