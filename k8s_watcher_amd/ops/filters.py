"""Event filters.

* :func:`is_critical` — the production ``critical_events_only`` predicate
  (``/root/reference/watcher/pod_watcher.py:204-212``): an event is *kept* when
  it is ``DELETED``, when the pod has no ``status``, or when the phase is
  terminal (``Failed``/``Succeeded``). "Has no status" means the field is
  absent/null — a present-but-empty ``status: {}`` is a (truthy) library model
  in the reference, so such a pod is dropped unless terminal.
* :class:`NamespaceFilter` — the client-side target-namespace check
  (``:225-229``) as an O(1) set lookup; an empty list means every namespace.
"""

from __future__ import annotations

from typing import Iterable, Optional

from ..models.pod import TERMINAL_PHASES


def is_critical(event_type: str, has_status: bool, phase: Optional[str]) -> bool:
    return event_type == "DELETED" or not has_status or phase in TERMINAL_PHASES


class NamespaceFilter:
    __slots__ = ("namespaces", "allow_all")

    def __init__(self, namespaces: Iterable[str]) -> None:
        self.namespaces = frozenset(namespaces or ())
        self.allow_all = not self.namespaces

    def __call__(self, namespace: Optional[str]) -> bool:
        return self.allow_all or namespace in self.namespaces


class CriticalFilter:
    """Active only in production with ``watcher.alerts.critical_events_only`` (``:207-208``)."""

    __slots__ = ("active",)

    def __init__(self, environment: str, critical_events_only: bool) -> None:
        self.active = environment == "production" and bool(critical_events_only)

    def __call__(self, event_type: str, has_status: bool, phase: Optional[str]) -> bool:
        return (not self.active) or is_critical(event_type, has_status, phase)
