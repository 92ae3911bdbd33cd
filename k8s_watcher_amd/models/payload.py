"""The clusterapi pod payload (schema §2.3) — Python engine.

Field-for-field the dictionary the reference builds in
``/root/reference/watcher/pod_watcher.py:159-202`` (+ ``event_type`` at ``:233``),
computed from raw API JSON instead of library models:

* ``status: null`` → ``phase: "Unknown"``, empty ``conditions`` /
  ``container_statuses`` (``:167,175,183``);
* ``creation_timestamp`` → ``datetime.isoformat()`` text (``:197``);
* ``event_timestamp`` → ``datetime.now().isoformat()`` (``:199``);
* ``container_statuses[].state`` → by default the structured JSON object from
  the API. ``state_format="python_repr"`` reproduces the reference's
  ``str(V1ContainerState)`` pprint text exactly (``:181``).

The wire body is produced in two parts so the hot path never re-serialises:
a *core* (everything up to ``metadata``, closed) computed once per event and
cached per pod, and a per-delivery *tail* with ``event_timestamp`` and
``event_type``. The native engine (``ops/csrc/kwcore.cpp``) emits the same
core bytes; ``tests/test_native_parity.py`` holds both to the same output.
"""

from __future__ import annotations

import json
import pprint
from typing import Any, Dict, List, Optional

from ..utils.timefmt import event_timestamp, k8s_time_to_isoformat

_STATE_SCHEMA = {
    # V1ContainerState* attribute sets (kubernetes==33.1.0 openapi_types)
    "running": ("started_at",),
    "terminated": ("container_id", "exit_code", "finished_at", "message", "reason", "signal", "started_at"),
    "waiting": ("message", "reason"),
}
_STATE_TIME = {"started_at", "finished_at"}

# watcher.payload_extra_fields: opt-in fields the reference does not send
# (SURVEY §2.3 lists them as missing), emitted as an "extra" object after
# "metadata", in this order, each as the raw API value or null. Bit i of the
# mask = EXTRA_FIELDS[i] (the native engine uses the same bits).
EXTRA_FIELDS = ("pod_ip", "host_ip", "start_time", "qos_class", "resource_version", "owner_references")


def extra_mask(names) -> int:
    mask = 0
    for n in names or ():
        if n not in EXTRA_FIELDS:
            raise ValueError(f"unknown payload extra field {n!r} (choose from {list(EXTRA_FIELDS)})")
        mask |= 1 << EXTRA_FIELDS.index(n)
    return mask


def _extra(md: Dict[str, Any], st: Optional[Dict[str, Any]], mask: int) -> Dict[str, Any]:
    st = st if isinstance(st, dict) else {}
    src = (st.get("podIP"), st.get("hostIP"), st.get("startTime"), st.get("qosClass"),
           md.get("resourceVersion"), md.get("ownerReferences"))
    return {name: src[i] for i, name in enumerate(EXTRA_FIELDS) if mask >> i & 1}


def _lib_datetime(value: Optional[str]):
    """Parse like the library does (``dateutil.parser.parse``) so reprs match."""
    if value is None:
        return None
    try:
        from dateutil import parser as du_parser
        return du_parser.parse(value)
    except Exception:  # noqa: BLE001
        return value


def container_state_repr(state: Dict[str, Any]) -> str:
    """``str(V1ContainerState(...))`` as the reference sends it.

    A state (or sub-state) that is not a JSON object is something the
    library's deserialiser would refuse: ``ValueError`` (the line is INVALID)."""
    from .objects import snake_to_camel
    if not isinstance(state, dict):
        raise ValueError("container state is not an object")
    out: Dict[str, Any] = {}
    for sub, attrs in _STATE_SCHEMA.items():
        src = state.get(sub)
        if src is None:
            out[sub] = None
            continue
        if not isinstance(src, dict):
            raise ValueError(f"container state {sub!r} is not an object")
        d: Dict[str, Any] = {}
        for a in attrs:
            v = src.get(snake_to_camel(a))
            d[a] = _lib_datetime(v) if a in _STATE_TIME else v
        out[sub] = d
    return pprint.pformat(out)


def utc_tzinfo_repr() -> str:
    """How ``str(V1ContainerState)`` spells a zero UTC offset in this process:
    ``tzutc()``, or ``tzlocal()`` when the process runs in UTC (dateutil's
    rule); "" without dateutil (times then stay strings). The native
    python_repr renderer (``ops/csrc/pyrepr.inc``) is given this."""
    try:
        from dateutil import parser as du_parser
        return repr(du_parser.parse("2025-01-01T00:00:00Z").tzinfo)
    except Exception:  # noqa: BLE001
        return ""


def repr_fallback(environment: str, extra: int = 0):
    """object JSON bytes -> python_repr core bytes: what the native engine
    calls for the (rare) container states it leaves to this module."""
    def core(obj: bytes) -> bytes:
        return build_core(json.loads(obj), environment, "python_repr", extra)
    return core


def build_payload_dict(pod: Dict[str, Any], environment: str, state_format: str = "structured",
                       event_type: Optional[str] = None, ts_mode: Optional[str] = "local",
                       extra: int = 0) -> Dict[str, Any]:
    """The reference payload as a dict (``ts_mode=None`` omits ``event_timestamp``)."""
    md = pod.get("metadata") or {}
    st = pod.get("status")
    sp = pod.get("spec")
    if st is not None:
        conds: List[Dict[str, Any]] = [
            {"type": c.get("type"), "status": c.get("status"),
             "reason": c.get("reason"), "message": c.get("message")}
            for c in (st.get("conditions") or [])]
        css: List[Dict[str, Any]] = []
        for cs in st.get("containerStatuses") or []:
            state = cs.get("state")
            if state is None:
                sval: Any = None
            elif state_format == "python_repr":
                sval = container_state_repr(state)
            else:
                sval = state
            css.append({"name": cs.get("name"), "ready": cs.get("ready"),
                        "restart_count": cs.get("restartCount"), "state": sval})
        status = {"phase": st.get("phase"), "conditions": conds, "container_statuses": css}
    else:
        status = {"phase": "Unknown", "conditions": [], "container_statuses": []}
    if sp is not None:
        spec = {"node_name": sp.get("nodeName"),
                "containers": [{"name": c.get("name"), "image": c.get("image")}
                               for c in (sp.get("containers") or [])]}
    else:
        spec = {"node_name": None, "containers": []}
    out = {
        "name": md.get("name"),
        "namespace": md.get("namespace"),
        "uid": md.get("uid"),
        "environment": environment,
        "status": status,
        "spec": spec,
        "metadata": {
            "labels": md.get("labels") or {},
            "annotations": md.get("annotations") or {},
            "creation_timestamp": k8s_time_to_isoformat(md.get("creationTimestamp")),
        },
    }
    if extra:
        out["extra"] = _extra(md, st, extra)
    if ts_mode is not None:
        out["event_timestamp"] = event_timestamp(ts_mode)
    if event_type is not None:
        out["event_type"] = event_type
    return out


def build_core(pod: Dict[str, Any], environment: str, state_format: str = "structured", extra: int = 0) -> bytes:
    """Serialized payload *without* ``event_timestamp``/``event_type`` (ends with ``}``)."""
    d = build_payload_dict(pod, environment, state_format, None, None, extra)
    return json.dumps(d, ensure_ascii=False, separators=(",", ":")).encode("utf-8")


def finish_body(core: bytes, event_type: str, ts: str) -> bytes:
    """Append the per-delivery tail to a core: ``{...,"event_timestamp":..,"event_type":..}``."""
    return b"".join((core[:-1], b',"event_timestamp":"', ts.encode("ascii"),
                     b'","event_type":"', event_type.encode("ascii"), b'"}'))
