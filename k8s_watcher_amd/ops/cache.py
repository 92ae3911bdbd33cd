"""In-memory pod cache: phase-change diffing and relist reconciliation.

The reference README promises "Trigger an API call on phase changes"
(``/root/reference/README.md:7``) but ``handle_pod_event`` notifies on every
event (``pod_watcher.py:214-241``). This cache provides both modes
(``watcher.notify_on: all | phase_change``) and is also what lets the
reflector turn a post-410 relist into exact ADDED/MODIFIED/DELETED diffs
 and survive restarts through the checkpoint.

One entry per live pod: ``uid -> [resourceVersion, phase, namespace, name, core]``
where ``core`` is the last serialized payload core (or ``None`` if the pod
was never notified).

Two implementations share this interface: :class:`PodCache` (a dict of
lists, used by the Python engine) and ``_kwcore.PodCache`` (C++,
``ops/csrc/podcache.inc``), which the fused native pipeline updates without
creating Python objects. Callers other than the two pipelines use only the
methods below; ``get``/``items``/``pop`` of the native cache return copies.
"""

from __future__ import annotations

from typing import Dict, Iterator, List, Optional, Tuple

RV, PHASE, NS, NAME, CORE = range(5)
MISSING = object()


class PodCache:
    __slots__ = ("entries",)

    def __init__(self) -> None:
        self.entries: Dict[str, list] = {}

    def __len__(self) -> int:
        return len(self.entries)

    def __contains__(self, uid: str) -> bool:
        return uid in self.entries

    def get(self, uid: str) -> Optional[list]:
        return self.entries.get(uid)

    def observe(self, etype: str, uid: str, rv: Optional[str], phase: Optional[str],
                ns: Optional[str], name: Optional[str]):
        """Apply one event; return the previous phase or :data:`MISSING`."""
        ent = self.entries.get(uid)
        prev = MISSING if ent is None else ent[PHASE]
        if etype == "DELETED":
            if ent is not None:
                del self.entries[uid]
        elif ent is None:
            self.entries[uid] = [rv, phase, ns, name, None]
        else:
            ent[RV] = rv
            ent[PHASE] = phase
        return prev

    def set_core(self, uid: str, core: bytes) -> None:
        ent = self.entries.get(uid)
        if ent is not None:
            ent[CORE] = core

    def put(self, uid: str, rv: Optional[str], phase: Optional[str], ns: Optional[str],
            name: Optional[str], core: Optional[bytes] = None) -> None:
        self.entries[uid] = [rv, phase, ns, name, core]

    def pop(self, uid: str, default=None):
        return self.entries.pop(uid, default)

    def clear(self) -> None:
        self.entries.clear()

    def items(self) -> List[Tuple[str, list]]:
        return list(self.entries.items())

    def count_namespace(self, ns: Optional[str]) -> int:
        return sum(1 for ent in self.entries.values() if ent[NS] == ns)

    def namespaces(self) -> Dict[Optional[str], int]:
        out: Dict[Optional[str], int] = {}
        for ent in self.entries.values():
            out[ent[NS]] = out.get(ent[NS], 0) + 1
        return out

    def drop_namespaces(self, names) -> int:
        """Forget every pod of these namespaces; returns how many."""
        names = set(names)
        gone = [uid for uid, ent in self.entries.items() if ent[NS] in names]
        for uid in gone:
            del self.entries[uid]
        return len(gone)

    def drop_namespaces_except(self, names) -> int:
        keep = set(names)
        gone = [uid for uid, ent in self.entries.items() if ent[NS] not in keep]
        for uid in gone:
            del self.entries[uid]
        return len(gone)

    def to_records(self) -> List[list]:
        return [[uid] + ent[:4] + [ent[CORE].decode("utf-8") if ent[CORE] else None]
                for uid, ent in self.entries.items()]

    def load_records(self, records: List[list]) -> None:
        for r in records:
            uid, rv, phase, ns, name, core = r
            self.entries[uid] = [rv, phase, ns, name, core.encode("utf-8") if core else None]

    @classmethod
    def from_records(cls, records: List[list]) -> "PodCache":
        c = cls()
        c.load_records(records)
        return c


def make_pod_cache(native: bool, records: Optional[List[list]] = None):
    """A :class:`PodCache` or, for the native pipeline, a ``_kwcore.PodCache``."""
    if native:
        from .native import load
        cache = load().PodCache(MISSING)
    else:
        cache = PodCache()
    if records:
        cache.load_records(records)
    return cache


def phase_changed(etype: str, prev, phase: Optional[str]) -> bool:
    """``notify_on: phase_change`` decision given the cache's previous phase."""
    if etype == "DELETED" or prev is MISSING:
        return True
    return prev != phase
