"""Durable resume point: resourceVersion(s) + pod cache (BASELINE config #5).

The reference keeps its resume point only inside the library's ``Watch``
object (``pod_watcher.py:16``), so every restart replays every pod as
``ADDED``. Here the reflector's resourceVersion per watch scope and the pod
cache are written atomically (temp file + fsync + rename) at a *quiescent*
point — the watch readers are paused and the notifier drained first — so the
saved cache never runs ahead of what clusterapi has acknowledged. On restart
the watcher resumes the watch from the saved resourceVersion without a LIST;
if that version has been compacted (410) the relist is diffed against the
saved cache, so unchanged pods are not re-notified.
"""

from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, Optional, Tuple

from ..ops.cache import PodCache, make_pod_cache

FORMAT_VERSION = 1


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


def load_checkpoint(path: str, native_cache: bool = False) -> Optional[Tuple[Dict[str, Optional[str]], PodCache, dict]]:
    """``(scopes, cache, meta)`` or None when absent/unreadable/incompatible.
    ``native_cache`` loads into a ``_kwcore.PodCache`` (native pipeline)."""
    try:
        with open(path, "r", encoding="utf-8") as fh:
            doc = json.load(fh)
    except FileNotFoundError:
        return None
    except (OSError, ValueError):
        return None
    if not isinstance(doc, dict) or doc.get("version") != FORMAT_VERSION:
        return None
    return doc.get("scopes") or {}, make_pod_cache(native_cache, doc.get("cache") or []), doc.get("meta") or {}
