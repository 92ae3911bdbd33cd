"""Durable resume point: resourceVersion(s) + pod cache (BASELINE config #5).

The reference keeps its resume point only inside the library's ``Watch``
object (``pod_watcher.py:16``), so every restart replays every pod as
``ADDED``. Here the reflector's resourceVersion per watch scope and the pod
cache are written atomically (temp file + fsync + rename). On restart the
watcher resumes the watch from the saved resourceVersion without a LIST; if
that version has been compacted (410) the relist is diffed against the saved
cache, so unchanged pods are not re-notified.

Two formats:

* **2 (native engine and notifier core)** — ``_kwcore.PodCache.snapshot``
  (``ops/csrc/checkpoint.inc``) takes a *consistent cut* between two
  event-loop callbacks: the cache entries (payload cores by reference, not
  copied) plus every notification clusterapi has not acknowledged yet. No
  watch is paused and the notifier is not drained; the snapshot is serialised
  and fsynced on an executor thread while the watch goes on. A restart first
  re-submits the owed notifications, then resumes the watches — so nothing
  acknowledged is sent again except those, and nothing unacknowledged is lost.
* **1 (Python engine / asyncio pool)** — one JSON document written at a
  *quiescent* point (watches paused, notifier drained), as before.
"""

from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, List, Optional, Tuple

from ..ops.cache import PodCache, make_pod_cache

FORMAT_VERSION = 1
NATIVE_FORMAT_VERSION = 2
NATIVE_MAGIC = b"KWCKPT02"


def save_checkpoint(path: str, scopes: Dict[str, Optional[str]], cache: PodCache,
                    meta: Optional[dict] = None) -> None:
    doc = {"version": FORMAT_VERSION, "scopes": scopes, "meta": meta or {},
           "cache": cache.to_records()}
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".ckpt-", dir=d)
    try:
        with os.fdopen(fd, "w", encoding="utf-8") as fh:
            json.dump(doc, fh, separators=(",", ":"))
            fh.flush()
            os.fsync(fh.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


def native_header(scopes: Dict[str, Optional[str]], meta: Optional[dict] = None) -> bytes:
    return json.dumps({"version": NATIVE_FORMAT_VERSION, "scopes": scopes, "meta": meta or {}},
                      separators=(",", ":")).encode("utf-8")


def native_snapshot(cache, notifier_core=None):
    """The consistent cut (call on the event-loop thread); write it with
    ``snap.write(path, native_header(...))`` on an executor."""
    return cache.snapshot(notifier_core)


def write_native(snap, path: str, scopes: Dict[str, Optional[str]], meta: Optional[dict] = None) -> Tuple[int, float]:
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    return snap.write(path, native_header(scopes, meta))


def load_checkpoint(path: str, native_cache: bool = False
                    ) -> Optional[Tuple[Dict[str, Optional[str]], PodCache, dict, List[tuple]]]:
    """``(scopes, cache, meta, owed)`` or None when absent/unreadable/incompatible.

    ``native_cache`` loads into a ``_kwcore.PodCache`` (native pipeline);
    ``owed`` lists the notifications a format-2 checkpoint still owed, as
    ``(uid, type, ns, name, body)`` to re-submit before watching."""
    try:
        with open(path, "rb") as fh:
            head = fh.read(8)
    except OSError:
        return None
    if head == NATIVE_MAGIC:
        if not native_cache:
            return None  # written by the native engine; the Python engine relists
        cache = make_pod_cache(True)
        try:
            header, owed = cache.load_checkpoint(path)
            doc = json.loads(header)
        except (OSError, ValueError):
            return None
        if doc.get("version") != NATIVE_FORMAT_VERSION:
            return None
        return doc.get("scopes") or {}, cache, doc.get("meta") or {}, owed
    try:
        with open(path, "r", encoding="utf-8") as fh:
            doc = json.load(fh)
    except (OSError, ValueError):
        return None
    if not isinstance(doc, dict) or doc.get("version") != FORMAT_VERSION:
        return None
    return (doc.get("scopes") or {}, make_pod_cache(native_cache, doc.get("cache") or []),
            doc.get("meta") or {}, [])
