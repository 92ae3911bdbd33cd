"""Scriptable fake kube-apiserver (replaces the external mock at ``localhost:9988``).

The reference's only end-to-end path talks to a mock API server that is not
in the repository (``/root/reference/assets/config:5``,
``test_k8s_mock.py:37-80``). This module is that server, built to
be faithful where the watcher's correctness depends on it:

* ``GET /version``, ``GET /api/v1/namespaces`` (``limit``/``continue``);
* ``GET /api/v1/pods`` and ``/api/v1/namespaces/{ns}/pods`` — paginated LIST
  (``limit``/``continue``, ``labelSelector`` equality terms, ``fieldSelector``
  on ``metadata.namespace|name``, ``status.phase``, ``spec.nodeName``);
* WATCH on the same paths (``watch=true``): no/"0" resourceVersion → synthetic
  ``ADDED`` for current pods then live events; a resourceVersion → replay of
  the retained history after it; a compacted version → ``ERROR`` 410 event (or
  HTTP 410 with ``expired_as_http_status``); ``timeoutSeconds``;
  ``allowWatchBookmarks`` bookmarks on demand or periodically;
* WatchList (``sendInitialEvents=true``): initial state as ``ADDED`` events
  closed by a bookmark annotated ``k8s.io/initial-events-end``;
* ``coordination.k8s.io/v1`` Leases (GET/POST/PUT/DELETE, compare-and-swap on
  ``resourceVersion``) for leader election;
* one HTTP chunk per event, as the real server flushes;
* fault injection: drop every connection, expire every watch, fail the next
  N requests with a status, compact history, bearer-token auth (401).

Runs inside the caller's event loop (``await srv.start()``), in a background
thread (:class:`ServerThread`), or as a process
(``python -m k8s_watcher_amd.testing.fake_apiserver --port 9988``).
"""

from __future__ import annotations

import argparse
import asyncio
import base64
import collections
import copy
import gzip
import json
import threading
import time
import uuid
from typing import Any, Deque, Dict, List, Optional, Set, Tuple
from urllib.parse import parse_qs, urlsplit
from ..utils.aio import with_timeout

JSON = "application/json"


GZIP_THRESHOLD = 128 * 1024  # kube-apiserver compresses responses larger than this
LEASES_PREFIX = "/apis/coordination.k8s.io/v1/namespaces/"
_REASONS = {200: "OK", 201: "Created", 400: "Bad Request", 404: "Not Found", 405: "Method Not Allowed",
            409: "Conflict", 500: "Internal Server Error", 503: "Service Unavailable"}


def _chunk(data: bytes) -> bytes:
    return b"%x\r\n%s\r\n" % (len(data), data)


def _status(code: int, reason: str, message: str) -> Dict[str, Any]:
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
            "message": message, "reason": reason, "code": code}


def _match_labels(pod: Dict[str, Any], selector: Optional[str]) -> bool:
    if not selector:
        return True
    labels = (pod.get("metadata") or {}).get("labels") or {}
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k.strip()) == v.strip():
                return False
        elif "=" in term:
            k, v = term.replace("==", "=").split("=", 1)
            if labels.get(k.strip()) != v.strip():
                return False
        elif term.startswith("!"):
            if term[1:] in labels:
                return False
        elif term not in labels:
            return False
    return True


_FIELD_PATHS = {
    "metadata.namespace": lambda p: (p.get("metadata") or {}).get("namespace"),
    "metadata.name": lambda p: (p.get("metadata") or {}).get("name"),
    "status.phase": lambda p: (p.get("status") or {}).get("phase"),
    "spec.nodeName": lambda p: (p.get("spec") or {}).get("nodeName"),
}


def _match_fields(pod: Dict[str, Any], selector: Optional[str]) -> bool:
    if not selector:
        return True
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        neg = "!=" in term
        k, v = term.split("!=" if neg else "=", 1)
        k = k.strip().rstrip("=")
        get = _FIELD_PATHS.get(k)
        if get is None:
            continue
        val = get(pod) or ""
        if (val == v.strip()) == neg:
            return False
    return True


class _Watch:
    __slots__ = ("writer", "namespace", "labels", "fields", "bookmarks", "closed")

    def __init__(self, writer, namespace, labels, fields, bookmarks):
        self.writer = writer
        self.namespace = namespace
        self.labels = labels
        self.fields = fields
        self.bookmarks = bookmarks
        self.closed = asyncio.Event()

    def wants(self, pod: Dict[str, Any]) -> bool:
        md = pod.get("metadata") or {}
        if self.namespace and md.get("namespace") != self.namespace:
            return False
        return _match_labels(pod, self.labels) and _match_fields(pod, self.fields)


class FakeApiServer:
    def __init__(self, token: Optional[str] = None, history_limit: int = 1_000_000,
                 namespaces: Optional[List[str]] = None, expired_as_http_status: bool = False,
                 bookmark_interval: Optional[float] = None, start_rv: int = 1000,
                 watch_list: bool = True) -> None:
        self.token = token
        self.watch_list = watch_list  # serve sendInitialEvents=true (WatchList)
        # test hook: raw events a WatchList's initial stream carries after its
        # ADDED set (a server interleaving live events before the end bookmark)
        self.watch_list_inject: List[Dict[str, Any]] = []
        self.history_limit = history_limit
        self.extra_namespaces = list(namespaces or ["default", "kube-system"])
        self.expired_as_http_status = expired_as_http_status
        self.bookmark_interval = bookmark_interval
        self.rv = start_rv
        self.pods: Dict[Tuple[str, str], Dict[str, Any]] = {}
        # (rv, namespace, pod-for-filtering, encoded line)
        self.history: Deque[Tuple[int, str, Dict[str, Any], bytes]] = collections.deque()
        self.compacted_rv = start_rv
        self.watches: Set[_Watch] = set()
        self.writers: Set[asyncio.StreamWriter] = set()
        self.fail_next: List[Tuple[int, str, Optional[float]]] = []
        self.empty_watches = 0
        self.expire_continues = 0  # the next N paginated LIST continuations answer 410
        self.requests: List[Tuple[str, str]] = []
        self.server: Optional[asyncio.AbstractServer] = None
        self.port = 0
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self._bm_task: Optional[asyncio.Task] = None
        self.gzipped_responses = 0
        self.denied: Set[Tuple[str, str]] = set()  # (verb, resource) the fake RBAC refuses
        self.leases: Dict[Tuple[str, str], Dict[str, Any]] = {}
        self.lease_writes: List[Tuple[Tuple[str, str], Dict[str, Any]]] = []
        self.lease_fault: Optional[int] = None  # answer every lease request with this status
        self.lease_stall = 0.0  # seconds every lease request waits before it is answered
        self.expire_every_watch = False
        self.deleted_namespaces: Set[str] = set()
        self.ns_watches: Set[asyncio.StreamWriter] = set()
        self._known_ns: Set[str] = set(self.extra_namespaces)  # a lagging watch cache: every watch with an RV gets 410

    # ------------------------------------------------------------------ lifecycle
    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context=None) -> int:
        self.loop = asyncio.get_running_loop()
        self.scheme = "https" if ssl_context is not None else "http"
        self.server = await asyncio.start_server(self._handle, host, port, limit=1 << 20, ssl=ssl_context)
        self.port = self.server.sockets[0].getsockname()[1]
        if self.bookmark_interval:
            self._bm_task = asyncio.ensure_future(self._bookmark_loop())
        return self.port

    @property
    def url(self) -> str:
        return f"{getattr(self, 'scheme', 'http')}://127.0.0.1:{self.port}"

    async def stop(self) -> None:
        if self._bm_task:
            self._bm_task.cancel()
        if self.server is not None:
            self.server.close()
        self.drop_connections()
        if self.server is not None:
            try:
                await with_timeout(self.server.wait_closed(), 2)
            except asyncio.TimeoutError:
                pass

    async def _bookmark_loop(self) -> None:
        while True:
            await asyncio.sleep(self.bookmark_interval or 1.0)
            self.emit_bookmark()

    # ------------------------------------------------------------------ state mutation
    def _next_rv(self) -> int:
        self.rv += 1
        return self.rv

    def _record(self, etype: str, pod: Dict[str, Any]) -> None:
        rv = int(pod["metadata"]["resourceVersion"])
        line = json.dumps({"type": etype, "object": pod}, separators=(",", ":"),
                          ensure_ascii=False).encode("utf-8") + b"\n"
        ns = pod["metadata"].get("namespace", "")
        self.history.append((rv, ns, pod, line))
        while len(self.history) > self.history_limit:
            old = self.history.popleft()
            self.compacted_rv = old[0]
        data = _chunk(line)
        for w in list(self.watches):
            if w.wants(pod):
                try:
                    w.writer.write(data)
                except Exception:  # noqa: BLE001
                    self.watches.discard(w)

    # ------------------------------------------------------------------ namespaces
    def namespace_names(self) -> List[str]:
        return sorted(({ns for ns, _ in self.pods} | set(self.extra_namespaces)) - self.deleted_namespaces)

    def _ns_event(self, etype: str, name: str) -> None:
        obj = {"kind": "Namespace", "apiVersion": "v1",
               "metadata": {"name": name, "uid": str(uuid.uuid5(uuid.NAMESPACE_DNS, name)),
                            "resourceVersion": str(self._next_rv())},
               "status": {"phase": "Active"}}
        data = _chunk(json.dumps({"type": etype, "object": obj}, separators=(",", ":")).encode() + b"\n")
        for w in list(self.ns_watches):
            try:
                w.write(data)
            except Exception:  # noqa: BLE001
                self.ns_watches.discard(w)

    def _touch_namespace(self, name: str) -> None:
        if name not in self._known_ns or name in self.deleted_namespaces:
            self._known_ns.add(name)
            self.deleted_namespaces.discard(name)
            self._ns_event("ADDED", name)

    def add_namespace(self, name: str) -> None:
        if name not in self.extra_namespaces:
            self.extra_namespaces.append(name)
        self._touch_namespace(name)

    def delete_namespace(self, name: str) -> None:
        """Delete every pod in ``name`` (DELETED events), then the namespace itself."""
        for (ns, pname) in [k for k in self.pods if k[0] == name]:
            self.delete(ns, pname)
        if name in self.extra_namespaces:
            self.extra_namespaces.remove(name)
        self.deleted_namespaces.add(name)
        self._known_ns.discard(name)
        self._ns_event("DELETED", name)

    def create(self, pod: Dict[str, Any]) -> Dict[str, Any]:
        pod = copy.deepcopy(pod)
        md = pod.setdefault("metadata", {})
        md.setdefault("namespace", "default")
        self._touch_namespace(md["namespace"])
        md.setdefault("uid", str(uuid.uuid4()))
        md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
        md["resourceVersion"] = str(self._next_rv())
        self.pods[(md["namespace"], md["name"])] = pod
        self._record("ADDED", pod)
        return pod

    def update(self, pod: Dict[str, Any]) -> Dict[str, Any]:
        pod = copy.deepcopy(pod)
        md = pod["metadata"]
        key = (md.get("namespace", "default"), md["name"])
        if key not in self.pods:
            return self.create(pod)
        md["uid"] = self.pods[key]["metadata"]["uid"]
        md["resourceVersion"] = str(self._next_rv())
        self.pods[key] = pod
        self._record("MODIFIED", pod)
        return pod

    def delete(self, namespace: str, name: str, final: Optional[Dict[str, Any]] = None) -> Optional[Dict]:
        pod = self.pods.pop((namespace, name), None)
        if pod is None:
            return None
        pod = copy.deepcopy(final if final is not None else pod)
        pod["metadata"]["uid"] = pod["metadata"].get("uid") or str(uuid.uuid4())
        pod["metadata"]["resourceVersion"] = str(self._next_rv())
        self._record("DELETED", pod)
        return pod

    def apply(self, etype: str, pod: Dict[str, Any]) -> Dict[str, Any]:
        """Apply a generated ``(type, object)`` event (see :mod:`.podgen`)."""
        md = pod["metadata"]
        if etype == "ADDED":
            return self.create(pod)
        if etype == "MODIFIED":
            return self.update(pod)
        if etype == "DELETED":
            return self.delete(md.get("namespace", "default"), md["name"], final=pod) or pod
        raise ValueError(etype)

    def emit_bookmark(self) -> None:
        for w in list(self.watches):
            if w.bookmarks:
                line = json.dumps({"type": "BOOKMARK", "object": {
                    "kind": "Pod", "apiVersion": "v1",
                    "metadata": {"resourceVersion": str(self.rv),
                                 "annotations": {"k8s.io/initial-events-end": "true"}}}},
                    separators=(",", ":")).encode() + b"\n"
                w.writer.write(_chunk(line))

    def expire_watches(self) -> None:
        """Send ``ERROR 410`` to every open watch and end it (etcd compaction)."""
        line = json.dumps({"type": "ERROR", "object": _status(
            410, "Expired", "too old resource version")}).encode() + b"\n"
        for w in list(self.watches):
            try:
                w.writer.write(_chunk(line) + b"0\r\n\r\n")
                w.writer.close()
            except Exception:  # noqa: BLE001
                pass
            w.closed.set()
        self.watches.clear()

    def compact(self, keep_last: int = 0) -> None:
        """Forget history so resuming from an older resourceVersion yields 410."""
        while len(self.history) > keep_last:
            old = self.history.popleft()
            self.compacted_rv = old[0]
        if keep_last == 0:
            self.compacted_rv = self.rv

    def drop_connections(self) -> None:
        """Abort every client connection (simulated API-server restart)."""
        for w in list(self.watches):
            w.closed.set()
        self.watches.clear()
        for wr in list(self.writers):
            try:
                wr.transport.abort()
            except Exception:  # noqa: BLE001
                pass
        self.writers.clear()

    def fail_requests(self, n: int, status: int = 500, path_prefix: str = "",
                      retry_after: Optional[float] = None) -> None:
        """Answer the next ``n`` requests under ``path_prefix`` with ``status``
        (and a ``Retry-After`` header when given, as APF's 429 carries)."""
        for _ in range(n):
            self.fail_next.append((status, path_prefix, retry_after))

    def hang_up_watches(self, n: int) -> None:
        """The next ``n`` watches get a 200 with an empty body that ends at once
        (a proxy that closes every watch); backlog events are not sent."""
        self.empty_watches += n

    # ------------------------------------------------------------------ HTTP
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.writers.add(writer)
        try:
            while True:
                try:
                    line = await reader.readline()
                except (ConnectionError, asyncio.LimitOverrunError):
                    return
                if not line:
                    return
                headers: Dict[str, str] = {}
                while True:
                    h = await reader.readline()
                    if h in (b"\r\n", b"\n", b""):
                        break
                    k, _, v = h.decode("latin-1").partition(":")
                    headers[k.strip().lower()] = v.strip()
                n = int(headers.get("content-length", "0") or 0)
                body = await reader.readexactly(n) if n else b""
                parts = line.decode("latin-1").split()
                if len(parts) < 2:
                    return
                method, target = parts[0], parts[1]
                self.requests.append((method, target))
                keep = await self._route(method, target, headers, writer, body, reader)
                if not keep:
                    return
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            self.writers.discard(writer)
            try:
                writer.close()
            except Exception:  # noqa: BLE001
                pass

    def _send_json(self, writer, code: int, doc: Any, reason: str = "OK", gzip_ok: bool = False,
                   extra_headers: Optional[Dict[str, str]] = None) -> None:
        body = json.dumps(doc, separators=(",", ":"), ensure_ascii=False).encode("utf-8")
        extra = b"".join(f"{k}: {v}\r\n".encode("latin-1") for k, v in (extra_headers or {}).items())
        if gzip_ok and len(body) > GZIP_THRESHOLD:  # as the API server: only large responses
            body = gzip.compress(body, compresslevel=1)
            extra += b"Content-Encoding: gzip\r\n"
            self.gzipped_responses += 1
        writer.write(b"HTTP/1.1 %d %s\r\nContent-Type: application/json\r\n%sContent-Length: %d\r\n\r\n"
                     % (code, reason.encode(), extra, len(body)) + body)

    async def _route(self, method: str, target: str, headers: Dict[str, str], writer,
                     body: bytes = b"", reader: Optional[asyncio.StreamReader] = None) -> bool:
        u = urlsplit(target)
        q = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
        path = u.path
        if self.token is not None and headers.get("authorization") != f"Bearer {self.token}":
            self._send_json(writer, 401, _status(401, "Unauthorized", "Unauthorized"), "Unauthorized")
            return True
        if self.fail_next:
            st, prefix, retry_after = self.fail_next[0]
            if path.startswith(prefix):
                self.fail_next.pop(0)
                reason = "TooManyRequests" if st == 429 else "InternalError"
                self._send_json(writer, st, _status(st, reason, "injected failure"), "Injected",
                                extra_headers=None if retry_after is None
                                else {"Retry-After": f"{retry_after:g}"})
                return True
        if path == "/apis/authorization.k8s.io/v1/selfsubjectaccessreviews" and method == "POST":
            try:
                attrs = (json.loads(body).get("spec") or {}).get("resourceAttributes") or {}
            except ValueError:
                attrs = {}
            key = (attrs.get("verb"), attrs.get("resource"))
            allowed = key not in self.denied
            doc = {"apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview",
                   "spec": {"resourceAttributes": attrs},
                   "status": {"allowed": allowed, **({} if allowed else {"reason": "denied by the fake RBAC"})}}
            self._send_json(writer, 201, doc, "Created")
            return True
        if path.startswith(LEASES_PREFIX):
            if self.lease_stall:
                await asyncio.sleep(self.lease_stall)
            code, doc = self._lease(method, path[len(LEASES_PREFIX):], body)
            self._send_json(writer, code, doc, _REASONS.get(code, "OK"))
            return True
        if method != "GET":
            self._send_json(writer, 405, _status(405, "MethodNotAllowed", method), "Method Not Allowed")
            return True
        if path == "/version":
            self._send_json(writer, 200, {"major": "1", "minor": "33", "gitVersion": "v1.33.1-fake",
                                          "platform": "linux/amd64"})
            return True
        if path == "/api/v1/namespaces" and q.get("watch") in ("true", "1"):
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                         b"Transfer-Encoding: chunked\r\n\r\n")
            self.ns_watches.add(writer)
            try:
                await writer.drain()
                timeout = float(q.get("timeoutSeconds") or 3600)
                try:  # until the client goes away or the server-side timeout
                    await with_timeout(reader.read() if reader is not None else writer.wait_closed(), timeout)
                except (asyncio.TimeoutError, ConnectionError):
                    pass
                try:
                    writer.write(b"0\r\n\r\n")
                except Exception:  # noqa: BLE001
                    pass
            finally:
                self.ns_watches.discard(writer)
            return False
        if path == "/api/v1/namespaces":
            names = self.namespace_names()
            items = [{"kind": "Namespace", "apiVersion": "v1",
                      "metadata": {"name": n, "uid": str(uuid.uuid5(uuid.NAMESPACE_DNS, n))},
                      "status": {"phase": "Active"}} for n in names]
            self._send_json(writer, 200, self._paginate("NamespaceList", items, q))
            return True
        ns = None
        if path.startswith("/api/v1/namespaces/") and path.endswith("/pods"):
            ns = path[len("/api/v1/namespaces/"):-len("/pods")]
        elif path != "/api/v1/pods":
            self._send_json(writer, 404, _status(404, "NotFound", f"{path} not found"), "Not Found")
            return True
        if q.get("watch") in ("true", "1"):
            await self._watch(writer, ns, q)
            return False
        pods = [p for (pns, _), p in sorted(self.pods.items())
                if (ns is None or pns == ns) and _match_labels(p, q.get("labelSelector"))
                and _match_fields(p, q.get("fieldSelector"))]
        if q.get("continue") and self._continue_expired(q["continue"]):
            # as the API server once etcd compacted past the token's revision
            self._send_json(writer, 410, _status(
                410, "Expired", "The provided continue parameter is too old to display a consistent "
                "list result. You can start a new list without the continue parameter."), "Gone")
            return True
        self._send_json(writer, 200, self._paginate("PodList", pods, q),
                        gzip_ok="gzip" in headers.get("accept-encoding", ""))
        return True

    # ------------------------------------------------------------------ leases
    def _lease(self, method: str, rest: str, body: bytes) -> Tuple[int, Dict[str, Any]]:
        """coordination.k8s.io/v1 Leases: GET/PUT/DELETE one, POST to the
        collection; PUT with a stale ``metadata.resourceVersion`` → 409."""
        ns, _, tail = rest.partition("/")
        if not tail.startswith("leases"):
            return 404, _status(404, "NotFound", rest)
        name = tail[len("leases/"):] if tail.startswith("leases/") else ""
        try:
            doc = json.loads(body) if body else {}
        except ValueError:
            return 400, _status(400, "BadRequest", "invalid JSON body")
        if self.lease_fault is not None:
            code = self.lease_fault
            return code, _status(code, "InternalError", "injected lease failure")
        key = (ns, name or (doc.get("metadata") or {}).get("name", ""))
        cur = self.leases.get(key)
        if method == "GET" and name:
            if cur is None:
                return 404, _status(404, "NotFound", f'leases.coordination.k8s.io "{name}" not found')
            return 200, copy.deepcopy(cur)
        if method == "POST" and not name:
            if cur is not None:
                return 409, _status(409, "AlreadyExists", f'leases.coordination.k8s.io "{key[1]}" already exists')
            return 201, self._store_lease(key, doc)
        if method == "PUT" and name:
            if cur is None:
                return 404, _status(404, "NotFound", f'leases.coordination.k8s.io "{name}" not found')
            want = (doc.get("metadata") or {}).get("resourceVersion")
            if want and want != cur["metadata"]["resourceVersion"]:
                return 409, _status(409, "Conflict", "the object has been modified; please apply your "
                                                     "changes to the latest version and try again")
            return 200, self._store_lease(key, doc)
        if method == "DELETE" and name:
            if self.leases.pop(key, None) is None:
                return 404, _status(404, "NotFound", f'leases.coordination.k8s.io "{name}" not found')
            return 200, _status(200, "", "deleted") | {"status": "Success"}
        return 405, _status(405, "MethodNotAllowed", method)

    def _store_lease(self, key: Tuple[str, str], doc: Dict[str, Any]) -> Dict[str, Any]:
        obj = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
               "metadata": dict(doc.get("metadata") or {}), "spec": dict(doc.get("spec") or {})}
        md = obj["metadata"]
        md["namespace"], md["name"] = key
        old = self.leases.get(key)
        md["uid"] = old["metadata"]["uid"] if old else str(uuid.uuid4())
        md["resourceVersion"] = str(self._next_rv())
        self.leases[key] = obj
        self.lease_writes.append((key, copy.deepcopy(obj["spec"])))
        return copy.deepcopy(obj)

    def _continue_expired(self, token: str) -> bool:
        if self.expire_continues > 0:
            self.expire_continues -= 1
            return True
        try:
            return int(json.loads(base64.urlsafe_b64decode(token.encode()))["rv"]) < self.compacted_rv
        except (ValueError, KeyError, TypeError):
            return False

    def _paginate(self, kind: str, items: List[Dict[str, Any]], q: Dict[str, str]) -> Dict[str, Any]:
        start = 0
        rv = str(self.rv)
        if q.get("continue"):
            try:
                tok = json.loads(base64.urlsafe_b64decode(q["continue"].encode()))
                start, rv = int(tok["o"]), tok["rv"]
            except (ValueError, KeyError):
                start = 0
        limit = int(q.get("limit") or 0)
        end = len(items) if not limit else min(len(items), start + limit)
        meta: Dict[str, Any] = {"resourceVersion": rv}
        if end < len(items):
            meta["continue"] = base64.urlsafe_b64encode(
                json.dumps({"o": end, "rv": rv}).encode()).decode()
            meta["remainingItemCount"] = len(items) - end
        return {"kind": kind, "apiVersion": "v1", "metadata": meta, "items": items[start:end]}

    async def _watch(self, writer, ns: Optional[str], q: Dict[str, str]) -> None:
        w = _Watch(writer, ns, q.get("labelSelector"), q.get("fieldSelector"),
                   q.get("allowWatchBookmarks") in ("true", "1"))
        rv_param = q.get("resourceVersion")
        if self.empty_watches > 0:
            self.empty_watches -= 1
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                         b"Transfer-Encoding: chunked\r\n\r\n0\r\n\r\n")
            await writer.drain()
            return
        if q.get("sendInitialEvents") in ("true", "1"):
            await self._watch_list(writer, w, q)
            return
        if rv_param not in (None, "", "0"):
            try:
                since = int(rv_param)
            except ValueError:
                since = -1
            if since < self.compacted_rv or self.expire_every_watch:
                if self.expired_as_http_status:
                    self._send_json(writer, 410, _status(410, "Expired", "too old resource version"), "Gone")
                    await writer.drain()
                    return
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                             b"Transfer-Encoding: chunked\r\n\r\n")
                line = json.dumps({"type": "ERROR", "object": _status(
                    410, "Expired", f"too old resource version: {since} ({self.compacted_rv})")}).encode()
                writer.write(_chunk(line + b"\n") + b"0\r\n\r\n")
                await writer.drain()
                return
            backlog = [line for (rv, _, pod, line) in self.history if rv > since and w.wants(pod)]
        else:
            backlog = [json.dumps({"type": "ADDED", "object": p}, separators=(",", ":"),
                                  ensure_ascii=False).encode() + b"\n"
                       for _, p in sorted(self.pods.items()) if w.wants(p)]
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                     b"Transfer-Encoding: chunked\r\n\r\n")
        for line in backlog:
            writer.write(_chunk(line))
        await self._serve_watch(writer, w, q)

    async def _watch_list(self, writer, w: "_Watch", q: Dict[str, str]) -> None:
        """WatchList: ADDED for the current state, a bookmark annotated
        ``k8s.io/initial-events-end``, then live events. Like the real server it
        requires ``resourceVersionMatch=NotOlderThan`` and bookmarks, and is
        refused (422) when ``watch_list`` support is off."""
        if not self.watch_list:
            self._send_json(writer, 422, _status(422, "Invalid", "sendInitialEvents is forbidden for watch "
                                                               "unless the WatchList feature gate is enabled"),
                            "Unprocessable Entity")
            await writer.drain()
            return
        if q.get("resourceVersionMatch") != "NotOlderThan" or not w.bookmarks:
            self._send_json(writer, 422, _status(422, "Invalid", "sendInitialEvents requires "
                                                               "resourceVersionMatch=NotOlderThan and "
                                                               "allowWatchBookmarks=true"), "Unprocessable Entity")
            await writer.drain()
            return
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                     b"Transfer-Encoding: chunked\r\n\r\n")
        for _, p in sorted(self.pods.items()):
            if w.wants(p):
                writer.write(_chunk(json.dumps({"type": "ADDED", "object": p}, separators=(",", ":"),
                                               ensure_ascii=False).encode() + b"\n"))
        for ev in self.watch_list_inject:
            writer.write(_chunk(json.dumps(ev, separators=(",", ":"), ensure_ascii=False).encode() + b"\n"))
        end = {"type": "BOOKMARK", "object": {"kind": "Pod", "apiVersion": "v1", "metadata": {
            "resourceVersion": str(self.rv), "annotations": {"k8s.io/initial-events-end": "true"}}}}
        writer.write(_chunk(json.dumps(end, separators=(",", ":")).encode() + b"\n"))
        await self._serve_watch(writer, w, q)

    async def _serve_watch(self, writer, w: "_Watch", q: Dict[str, str]) -> None:
        self.watches.add(w)
        timeout = q.get("timeoutSeconds")
        try:
            await writer.drain()
            if timeout:
                try:
                    await with_timeout(w.closed.wait(), float(timeout))
                except asyncio.TimeoutError:
                    pass
            else:
                await w.closed.wait()
        except ConnectionError:
            pass
        finally:
            if w in self.watches:
                self.watches.discard(w)
                try:
                    writer.write(b"0\r\n\r\n")
                except Exception:  # noqa: BLE001
                    pass


class ServerThread:
    """Run a :class:`FakeApiServer` on its own event loop in a daemon thread."""

    def __init__(self, server: FakeApiServer, host: str = "127.0.0.1", port: int = 0,
                 ssl_context=None) -> None:
        self.server = server
        self.loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._host = host
        self._port = port
        self._ssl = ssl_context
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self) -> None:
        asyncio.set_event_loop(self.loop)
        self.loop.run_until_complete(self.server.start(self._host, self._port, self._ssl))
        self._ready.set()
        self.loop.run_forever()

    def start(self) -> "ServerThread":
        self.thread.start()
        self._ready.wait(10)
        return self

    def call(self, fn, *args, **kwargs):
        """Run ``fn`` on the server loop and return its result."""
        fut = asyncio.run_coroutine_threadsafe(self._wrap(fn, *args, **kwargs), self.loop)
        return fut.result(10)

    @staticmethod
    async def _wrap(fn, *args, **kwargs):
        res = fn(*args, **kwargs)
        if asyncio.iscoroutine(res):
            res = await res
        return res

    def stop(self) -> None:
        try:
            asyncio.run_coroutine_threadsafe(self.server.stop(), self.loop).result(5)
        except Exception:  # noqa: BLE001
            pass
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.thread.join(5)


async def replay_capture(srv: FakeApiServer, events: List[dict], speed: float = 1.0) -> int:
    """Apply captured watch events (``tools/capture.py``) at ``speed`` x the recorded pace
    (0 = as fast as possible). Each event is re-stamped with this server's resourceVersions."""
    loop = asyncio.get_running_loop()
    t0 = loop.time()
    n = 0
    for r in events:
        if speed > 0:
            delay = t0 + r["t"] / speed - loop.time()
            if delay > 0:
                await asyncio.sleep(delay)
        obj = r["object"]
        md = obj.get("metadata") or {}
        key = (md.get("namespace", "default"), md.get("name"))
        et = r["type"]
        if et == "ADDED" and key in srv.pods:
            et = "MODIFIED"  # a capture that starts mid-watch may repeat an ADDED
        elif et == "MODIFIED" and key not in srv.pods:
            et = "ADDED"
        elif et == "DELETED" and key not in srv.pods:
            continue
        srv.apply(et, obj)
        n += 1
        if speed <= 0 and n % 512 == 0:
            await asyncio.sleep(0)
    return n


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description="fake kube-apiserver for k8s-watcher")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9988)
    ap.add_argument("--token", default=None)
    ap.add_argument("--pods", type=int, default=10, help="pods to pre-create")
    ap.add_argument("--churn-rate", type=float, default=0.0, help="lifecycle events/s after start")
    ap.add_argument("--replay", default=None, help="serve a capture (k8s_watcher_amd.tools.capture)")
    ap.add_argument("--speed", type=float, default=1.0, help="replay pace: 1 = as recorded, 0 = flat out")
    args = ap.parse_args(argv)

    from .podgen import PodFactory, churn_events

    async def run() -> None:
        srv = FakeApiServer(token=args.token, bookmark_interval=30)
        if args.replay:
            from ..tools.capture import load_capture
            records = load_capture(args.replay)
            for r in records:
                if r["type"] == "LIST":
                    srv.create(r["object"])
            port = await srv.start(args.host, args.port)
            print(f"fake kube-apiserver listening on http://{args.host}:{port} (replaying {args.replay})",
                  flush=True)
            await replay_capture(srv, [r for r in records if r["type"] != "LIST"], args.speed)
            await asyncio.Event().wait()
        f = PodFactory(seed=1, namespaces=["default", "kube-system", "production", "monitoring"])
        for _ in range(args.pods):
            srv.create(f.running(f.new_pod()))
        port = await srv.start(args.host, args.port)
        print(f"fake kube-apiserver listening on http://{args.host}:{port}", flush=True)
        if args.churn_rate > 0:
            for et, obj in churn_events(10 ** 9, seed=2):
                srv.apply(et, obj)
                await asyncio.sleep(1.0 / args.churn_rate)
        else:
            await asyncio.Event().wait()

    try:
        asyncio.run(run())
    except KeyboardInterrupt:
        pass


if __name__ == "__main__":
    main()
