"""Timestamp formatting with the reference's exact textual shapes.

* ``creation_timestamp`` — the reference serialises the library's tz-aware
  ``datetime`` with ``.isoformat()`` (``pod_watcher.py:197``), so the API's
  ``2025-07-09T01:51:28Z`` becomes ``2025-07-09T01:51:28+00:00``;
  fractional seconds become exactly six digits, and disappear when zero.
* ``event_timestamp`` — ``datetime.now().isoformat()`` (``pod_watcher.py:199``):
  local, naive, microseconds omitted when zero. ``utc`` mode is an opt-in fix
  that emits ``...+00:00``.
"""

from __future__ import annotations

import datetime as _dt
import re

_RFC3339 = re.compile(
    r"^(\d{4}-\d{2}-\d{2})[Tt ](\d{2}:\d{2}:\d{2})(?:\.(\d+))?(Z|z|[+-]\d{2}:?\d{2})?$")


def k8s_time_to_isoformat(value):
    """RFC3339 string from the API → ``datetime.isoformat()`` text; None passes through.

    Unparseable input is returned unchanged rather than raising: the payload
    must still be delivered.
    """
    if value is None:
        return None
    if not isinstance(value, str):
        return value
    m = _RFC3339.match(value)
    if not m:
        return value
    date, clock, frac, tz = m.groups()
    out = f"{date}T{clock}"
    if frac:
        micro = int((frac + "000000")[:6])
        if micro:
            out += f".{micro:06d}"
    if tz is None:
        return out
    if tz in ("Z", "z"):
        return out + "+00:00"
    if ":" not in tz:
        tz = tz[:3] + ":" + tz[3:]
    if tz == "-00:00":
        tz = "+00:00"
    return out + tz


def parse_k8s_time(value):
    """RFC3339 → tz-aware ``datetime`` (None / unparseable → None)."""
    if not value or not isinstance(value, str):
        return None
    iso = k8s_time_to_isoformat(value)
    try:
        return _dt.datetime.fromisoformat(iso)
    except ValueError:
        return None


def event_timestamp(mode: str = "local") -> str:
    if mode == "utc":
        return _dt.datetime.now(_dt.timezone.utc).isoformat()
    return _dt.datetime.now().isoformat()
