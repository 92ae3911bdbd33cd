"""Watch-stream decoding: NDJSON bytes → compact event tuples.

This is the per-event hot path the reference pays inside the ``kubernetes``
library (line iteration, ``json.loads``, reflective ``V1Pod`` deserialisation;
SURVEY §3.2 "Hot loop"). Two engines share one interface:

* :class:`PyDecoder` — stdlib ``json`` + :mod:`..models.payload`; the
  semantic reference for the native engine.
* ``NativeDecoder`` (:mod:`.native`) — C++ single-pass extractor
  (``ops/csrc/kwcore.cpp``) that never builds Python objects for the pod body
  and emits the payload core bytes directly.

Event tuple layout (index constants below)::

    (type, uid, namespace, name, resourceVersion, phase, has_status, obj, extra)

``obj`` is the pod dict (Python engine) or the payload core bytes (native);
call ``decoder.core(ev)`` to get core bytes either way. ``extra`` carries the
``Status`` dict of an ``ERROR`` event, the error text of an ``INVALID`` line,
or — on a ``BOOKMARK`` — whether it ends a WatchList's initial events.
"""

from __future__ import annotations

import json
from typing import Any, Dict, List, Optional, Tuple

from ..models.payload import build_core
from ..net.http import json_input

E_TYPE, E_UID, E_NS, E_NAME, E_RV, E_PHASE, E_HAS_STATUS, E_OBJ, E_EXTRA = range(9)

ADDED, MODIFIED, DELETED, BOOKMARK, ERROR, INVALID = (
    "ADDED", "MODIFIED", "DELETED", "BOOKMARK", "ERROR", "INVALID")

# WatchList (``sendInitialEvents=true``): annotation on the BOOKMARK that ends the initial state
INITIAL_EVENTS_END = "k8s.io/initial-events-end"


def _s(v: Any) -> Optional[str]:
    """Identity fields are strings; anything else (null, numbers) reads as None."""
    return v if isinstance(v, str) else None


def event_from_object(etype: str, obj: Dict[str, Any]) -> tuple:
    if etype == ERROR:
        return (ERROR, None, None, None, None, None, False, None, obj)
    md = obj.get("metadata")
    if not isinstance(md, dict):  # not an object: absent (as the native engine reads it)
        md = {}
    st = obj.get("status")
    if st is not None and not isinstance(st, dict):
        st = None
    extra = None
    if etype == BOOKMARK:  # True on the WatchList end-of-initial-events marker
        ann = md.get("annotations")
        extra = isinstance(ann, dict) and ann.get(INITIAL_EVENTS_END) == "true"
    return (etype, _s(md.get("uid")), _s(md.get("namespace")), _s(md.get("name")),
            _s(md.get("resourceVersion")), _s(st.get("phase")) if st is not None else None,
            st is not None, obj, extra)


class PyDecoder:
    name = "python"

    def __init__(self, environment: str, state_format: str = "structured", extra: int = 0) -> None:
        self.environment = environment
        self.state_format = state_format
        self.extra = extra
        self._partial = b""
        self._cbuf = b""
        self._cremain = 0
        self._cstate = 0  # 0 size line, 1 data, 2 data CRLF, 3 trailers, 4 done

    def reset(self) -> None:
        self._partial = b""
        self._cbuf = b""
        self._cremain = 0
        self._cstate = 0

    def body_done(self) -> bool:
        return self._cstate == 4

    def feed_chunked(self, data: bytes) -> List[tuple]:
        """Like :meth:`feed` for input that still carries HTTP chunked framing."""
        buf = self._cbuf + data if self._cbuf else data
        self._cbuf = b""
        out: List[tuple] = []
        i, n = 0, len(buf)
        while i < n and self._cstate != 4:
            st = self._cstate
            if st == 1:
                take = min(self._cremain, n - i)
                out.extend(self.feed(buf[i:i + take]))
                i += take
                self._cremain -= take
                if self._cremain == 0:
                    self._cstate = 2
                continue
            nl = buf.find(b"\n", i)
            if nl < 0:
                if st != 2:
                    self._cbuf = buf[i:]
                break
            line = buf[i:nl].rstrip(b"\r")
            i = nl + 1
            if st == 0:
                size = int(line.split(b";", 1)[0].strip(), 16)
                if size == 0:
                    self._cstate = 3
                else:
                    self._cremain = size
                    self._cstate = 1
            elif st == 2:
                self._cstate = 0
            elif st == 3 and not line:
                self._cstate = 4
        return out

    def feed(self, data: bytes) -> List[tuple]:
        buf = self._partial + data if self._partial else data
        lines = buf.split(b"\n")
        self._partial = lines.pop()
        out = []
        for line in lines:
            if not line.strip():
                continue
            out.append(self.decode_line(line))
        return out

    def decode_line(self, line: bytes) -> tuple:
        try:
            doc = json.loads(line)
            etype = doc["type"]
            obj = doc["object"]
            if not isinstance(obj, dict):
                raise ValueError("object is not a JSON object")
        except (ValueError, KeyError, TypeError) as exc:
            return (INVALID, None, None, None, None, None, False, None, f"{exc}: {line[:200]!r}")
        return event_from_object(etype, obj)

    def decode_list(self, body: bytes) -> Tuple[Optional[str], Optional[str], List[tuple]]:
        doc = json.loads(json_input(body))  # a LIST page over 4 MiB arrives as an mmap
        md = doc.get("metadata") or {}
        items = doc.get("items") or []
        return (md.get("resourceVersion"), md.get("continue") or None,
                [event_from_object(ADDED, it) for it in items])

    def core(self, ev: tuple) -> bytes:
        return build_core(ev[E_OBJ], self.environment, self.state_format, self.extra)

    def core_from_summary(self, uid: str, ns: Optional[str], name: Optional[str],
                          phase: Optional[str]) -> bytes:
        pod = {"metadata": {"uid": uid, "namespace": ns, "name": name}}
        if phase is not None:
            pod["status"] = {"phase": phase}
        return build_core(pod, self.environment, self.state_format, self.extra)


VALIDATE_MODES = {"off": 0, "payload": 1, "full": 2}


def make_decoder(engine: str, environment: str, state_format: str = "structured", extra: int = 0,
                 validate: str = "payload"):
    """``engine="native"`` requires the C++ extension and raises if it is missing.
    ``extra`` is a :func:`..models.payload.extra_mask`; ``validate`` is
    ``watcher.validate`` (the Python engine always has json.loads' verdict)."""
    if engine == "python":
        return PyDecoder(environment, state_format, extra)
    from .native import NativeDecoder
    return NativeDecoder(environment, state_format, extra, validate)
