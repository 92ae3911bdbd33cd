"""``kubernetes.watch.Watch`` equivalent.

Behaviour reproduced from the library as used by the reference
(``/root/reference/watcher/pod_watcher.py:16,264,276``;
``test_k8s_mock.py:64-80``):

* ``stream(func, **kw)`` calls ``func(watch=True, _preload_content=False, ...)``
  and yields ``{"type", "object", "raw_object"}`` per line, ``object`` being an
  attribute view of the pod;
* it remembers the last ``metadata.resourceVersion``; when the server ends the
  stream and no ``timeout_seconds`` was given, it re-issues the watch from that
  version (no relist); with no version seen it stops;
* an ``ERROR`` event with code 410 is retried once from the same version; a
  second one raises :class:`~.client.ApiException` (status 410);
* ``stop()`` ends the generator after the current event.

For production use prefer :class:`k8s_watcher_amd.engine.reflector.Reflector`,
which relists and diffs on 410 instead of failing.
"""

from __future__ import annotations

import http.client
import json
from typing import Any, Callable, Dict, Iterator, Optional

from ...models.objects import ObjectView
from .client import ApiException


def iter_resp_lines(resp) -> Iterator[bytes]:
    """Lines of a streaming response. A connection cut mid-stream ends the
    iteration like a server close (the library raises ``ProtocolError``
    instead); the watch then resumes from the last resourceVersion."""
    buf = b""
    while True:
        try:
            chunk = resp.read1(65536) if hasattr(resp, "read1") else resp.read(65536)
        except (http.client.IncompleteRead, ConnectionError, OSError):
            chunk = b""
        if not chunk:
            break
        buf += chunk
        lines = buf.split(b"\n")
        buf = lines.pop()
        for line in lines:
            if line.strip():
                yield line
    if buf.strip():
        yield buf


class Watch:
    def __init__(self, return_type: Any = None) -> None:
        self._stop = False
        self.resource_version: Optional[str] = None
        self._raw_return_type = return_type

    def stop(self) -> None:
        self._stop = True

    def unmarshal_event(self, line: bytes) -> Dict[str, Any]:
        js = json.loads(line)
        obj = js.get("object")
        js["raw_object"] = obj
        if js.get("type") != "ERROR" and isinstance(obj, dict):
            js["object"] = ObjectView(obj)
            rv = (obj.get("metadata") or {}).get("resourceVersion")
            if rv:
                self.resource_version = rv
        return js

    def stream(self, func: Callable, *args: Any, **kwargs: Any) -> Iterator[Dict[str, Any]]:
        self._stop = False
        kwargs["watch"] = True
        kwargs["_preload_content"] = False
        if "resource_version" in kwargs:
            self.resource_version = kwargs["resource_version"]
        timeouts = "timeout_seconds" in kwargs
        retried_410 = False
        while True:
            resp = func(*args, **kwargs)
            try:
                for line in iter_resp_lines(resp):
                    event = self.unmarshal_event(line)
                    if event.get("type") == "ERROR":
                        obj = event.get("raw_object") or {}
                        code = obj.get("code")
                        if code == 410 and not retried_410:
                            retried_410 = True
                            break  # re-issue once from the same resourceVersion
                        raise ApiException(status=code, reason=obj.get("reason"), body=obj.get("message"))
                    retried_410 = False
                    yield event
                    if self._stop:
                        break
            finally:
                try:
                    resp.close()
                    conn = getattr(resp, "_k8s_conn", None)
                    if conn is not None:
                        conn.close()
                except Exception:  # noqa: BLE001
                    pass
            if self._stop or (timeouts and not retried_410):
                break
            if self.resource_version is None:
                break
            kwargs["resource_version"] = self.resource_version
