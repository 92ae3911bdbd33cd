"""Pod field accessors shared by the Python engine, the filters and the cache."""

from __future__ import annotations

import datetime as _dt
from typing import Any, Dict, Optional

from .objects import camel_to_snake, snake_to_camel  # noqa: F401  (re-export)

TERMINAL_PHASES = frozenset({"Failed", "Succeeded"})


def meta(pod: Dict[str, Any]) -> Dict[str, Any]:
    return pod.get("metadata") or {}


def pod_uid(pod: Dict[str, Any]) -> Optional[str]:
    return meta(pod).get("uid")


def pod_key(pod: Dict[str, Any]) -> str:
    m = meta(pod)
    return f"{m.get('namespace')}/{m.get('name')}"


def pod_phase(pod: Dict[str, Any]) -> Optional[str]:
    st = pod.get("status")
    if st is None:
        return None
    return st.get("phase")


def pod_rv(pod: Dict[str, Any]) -> Optional[str]:
    return meta(pod).get("resourceVersion")


def snake_dict_to_api(d: Any) -> Any:
    """Library ``to_dict()`` output (snake_case, datetimes) → API JSON shape."""
    from .objects import _MAP_FIELDS

    def conv(key: str, v: Any) -> Any:
        if isinstance(v, dict):
            if key in _MAP_FIELDS:
                return dict(v)
            return {snake_to_camel(k): conv(snake_to_camel(k), x) for k, x in v.items() if x is not None}
        if isinstance(v, list):
            return [conv(key, x) for x in v]
        if isinstance(v, _dt.datetime):
            iso = v.isoformat()
            return iso[:-6] + "Z" if iso.endswith("+00:00") else iso
        return v

    return conv("", d)
