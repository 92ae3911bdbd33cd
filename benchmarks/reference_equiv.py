"""Reference-equivalent pipeline: the per-event work of highreso-gpu/k8s-watcher.

The reference cannot run here (``kubernetes`` is not installed, and as shipped
it fails setup at ``pod_watcher.py:140``), and it publishes no
numbers. BASELINE.md therefore prescribes measuring a
pipeline that does the reference's per-event work on the same replay:

1. read the chunked watch stream line by line on one thread
   (``kubernetes.watch.Watch.stream`` → ``iter_resp_lines``);
2. ``json.loads`` the line and deserialize the object into attribute-style
   models with datetimes parsed by ``dateutil`` (``ApiClient.deserialize``);
3. ``should_process_event`` → INFO log → namespace filter
   (``pod_watcher.py:204-229``);
4. ``_extract_pod_data`` including ``str(cs.state)`` (pprint of the model,
   ``pod_watcher.py:159-202``);
5. ``requests.Session.post(url, json=pod_data)`` — synchronous, no timeout,
   success iff 200 (``clusterapi_client.py:36-38``).

Step 2 is an *under*-estimate of the library (which also instantiates every
absent field as ``None`` and validates enums), so the comparison is generous
to the reference.
"""

from __future__ import annotations

import datetime as _dt
import http.client
import json
import logging
import time
from typing import Any, Dict, Optional
from urllib.parse import urlsplit

import requests
from dateutil import parser as du_parser

from k8s_watcher_amd.models.objects import _MAP_FIELDS, _TIME_FIELDS, camel_to_snake
from k8s_watcher_amd.models.payload import container_state_repr


class _Model:
    """Eagerly-built attribute object (stand-in for ``kubernetes.client.V1*``)."""

    def __init__(self, raw: Dict[str, Any]) -> None:
        self._raw = raw
        for k, v in raw.items():
            setattr(self, camel_to_snake(k), _convert(k, v))

    def __getattr__(self, name: str) -> Any:  # absent attributes read as None, like the library
        if name.startswith("__"):
            raise AttributeError(name)
        return None


def _convert(key: str, v: Any) -> Any:
    if isinstance(v, dict):
        return dict(v) if key in _MAP_FIELDS else _Model(v)
    if isinstance(v, list):
        return [_convert(key, x) for x in v]
    if key in _TIME_FIELDS and isinstance(v, str):
        return du_parser.parse(v)
    return v


class RefEquivWatcher:
    def __init__(self, environment: str, namespaces, critical_events_only: bool, sink_url: str,
                 logger: Optional[logging.Logger] = None, ca_file: Optional[str] = None) -> None:
        self.environment = environment
        self.namespaces = list(namespaces or [])
        self.critical = environment == "production" and critical_events_only
        self.session = requests.Session()
        # https clusterapi (bench --tls): verify against the test CA (per request:
        # a session-level verify loses to $REQUESTS_CA_BUNDLE in requests)
        self.post_kw = {"verify": ca_file} if ca_file else {}
        self.endpoint = sink_url.rstrip("/") + "/api/pods/update"
        self.logger = logger or logging.getLogger("watcher.pod_watcher")
        self.processed = 0
        self.backlog = 0  # handled before the first counted event (run(count_from_rv=...))
        self.first_event_after_s = None  # connect -> the read that brought the first counted event
        self.cpu_seconds = None  # this thread's CPU time over the counted events
        self.notified = 0
        self.latencies_ns = []

    # -- pod_watcher.py:204-212
    def should_process_event(self, event_type: str, pod) -> bool:
        if self.critical and event_type not in ["DELETED"] and pod.status and \
                pod.status.phase not in ["Failed", "Succeeded"]:
            return False
        return True

    # -- pod_watcher.py:159-202
    def extract_pod_data(self, pod) -> Dict[str, Any]:
        st = pod.status
        sp = pod.spec
        md = pod.metadata
        return {
            "name": md.name,
            "namespace": md.namespace,
            "uid": md.uid,
            "environment": self.environment,
            "status": {
                "phase": st.phase if st else "Unknown",
                "conditions": [{"type": c.type, "status": c.status, "reason": c.reason, "message": c.message}
                               for c in (st.conditions or [])] if st else [],
                "container_statuses": [
                    {"name": cs.name, "ready": cs.ready, "restart_count": cs.restart_count,
                     "state": container_state_repr(cs.state._raw) if cs.state else None}
                    for cs in (st.container_statuses or [])] if st else [],
            },
            "spec": {
                "node_name": sp.node_name if sp else None,
                "containers": [{"name": c.name, "image": c.image} for c in (sp.containers or [])] if sp else [],
            },
            "metadata": {
                "labels": md.labels or {},
                "annotations": md.annotations or {},
                "creation_timestamp": md.creation_timestamp.isoformat() if md.creation_timestamp else None,
            },
            "event_timestamp": _dt.datetime.now().isoformat(),
        }

    # -- pod_watcher.py:214-241 with the notify call enabled (clusterapi_client.py:20-53)
    def handle_pod_event(self, event_type: str, pod, read_ns: int) -> None:
        if not self.should_process_event(event_type, pod):
            return
        self.logger.info(f"Pod event detected: {event_type} - {pod.metadata.namespace}/{pod.metadata.name}")
        if self.namespaces and pod.metadata.namespace not in self.namespaces:
            self.logger.debug(f"Skipping pod {pod.metadata.namespace}/{pod.metadata.name} - not in target namespaces")
            return
        data = self.extract_pod_data(pod)
        data["event_type"] = event_type
        resp = self.session.post(self.endpoint, json=data, **self.post_kw)
        if resp.status_code == 200:
            self.notified += 1
            self.latencies_ns.append(time.monotonic_ns() - read_ns)

    def run(self, api_url: str, n_events: int, on_connected=None, warm_events: int = 0,
            on_warm=None, count_from_rv: Optional[int] = None) -> float:
        """Watch until ``n_events`` pod events were handled; returns elapsed seconds
        measured from ``on_connected()`` (which should trigger the replay) or, with
        ``warm_events``, from the moment that many events were handled (then
        ``on_warm()`` is called).

        ``count_from_rv``: events with a lower resourceVersion (what the API
        server sends a new watch before the replay: ADDED for the pods alive
        now) are handled but not counted, and the clock starts at the socket
        read that brought the first event at or past it — the first paced
        event — not at ``on_connected()``: the time the fixture takes to
        start the replay is not the reference's."""
        u = urlsplit(api_url)
        conn = http.client.HTTPConnection(u.hostname, u.port)
        conn.request("GET", "/api/v1/pods?watch=true")
        resp = conn.getresponse()
        t0 = time.perf_counter()
        if on_connected is not None:
            on_connected()
            t0 = time.perf_counter()
        t_conn = t0
        cpu0 = time.thread_time()
        counting = count_from_rv is None
        warm = warm_events <= 0
        buf = b""
        while self.processed < n_events:
            chunk = resp.read1(65536)
            if not chunk:
                break
            t_read = time.perf_counter()
            read_ns = time.monotonic_ns()
            buf += chunk
            lines = buf.split(b"\n")
            buf = lines.pop()
            for line in lines:
                if not line.strip():
                    continue
                ev = json.loads(line)
                obj = _Model(ev["object"])
                if not counting:
                    rv = (ev["object"].get("metadata") or {}).get("resourceVersion")
                    if rv is not None and int(rv) >= count_from_rv:
                        counting = True
                        t0 = t_read
                        cpu0 = time.thread_time()
                        self.first_event_after_s = t_read - t_conn
                        self.latencies_ns.clear()
                        self.backlog = self.processed
                        self.processed = self.notified = 0
                self.handle_pod_event(ev["type"], obj, read_ns)
                self.processed += 1
                if not warm and self.processed >= warm_events:
                    warm = True
                    self.latencies_ns.clear()
                    if on_warm is not None:
                        on_warm()
                    t0 = time.perf_counter()
        elapsed = time.perf_counter() - t0
        self.cpu_seconds = time.thread_time() - cpu0
        conn.close()
        return elapsed
