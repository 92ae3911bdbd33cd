"""Async subset of the Kubernetes core/v1 REST API that a pod watcher needs.

Replaces the ``kubernetes`` library calls the reference makes
(``/root/reference/watcher/pod_watcher.py:137-146,264``;
``test_k8s_connection.py:32-48``): ``GET /version``, ``GET /api/v1/namespaces``,
paginated ``GET /api/v1/pods`` (or ``/api/v1/namespaces/{ns}/pods``) and the
streaming watch on the same paths. Bodies are returned as raw bytes so the
event decoder (native or Python) is the only place JSON is parsed.
"""

from __future__ import annotations

import json
from typing import Callable, Dict, Optional, Tuple

from ..net.http import HttpClient, HttpError, Response, StreamResponse, json_input, parse_retry_after  # noqa: F401
from .kubeconfig import KubeEndpoint

USER_AGENT = "k8s-watcher-amd/1.0"


class ApiError(Exception):
    """Non-2xx answer from the API server (``status`` = HTTP code)."""

    def __init__(self, status: int, reason: str, body: bytes,
                 headers: Optional[Dict[str, str]] = None) -> None:
        self.status = status
        self.reason = reason
        self.body = body
        # seconds the server asked us to wait (429 from API Priority and
        # Fairness, 503 while starting); None when absent or not delta-seconds
        self.retry_after = parse_retry_after((headers or {}).get("retry-after"))
        msg = reason
        try:
            doc = json.loads(json_input(body))
            msg = doc.get("message") or reason
            self.k8s_reason = doc.get("reason")
        except (ValueError, AttributeError):
            self.k8s_reason = None
        super().__init__(f"({status}) {msg}")


def pods_path(namespace: Optional[str] = None) -> str:
    return f"/api/v1/namespaces/{namespace}/pods" if namespace else "/api/v1/pods"


class KubeApi:
    def __init__(self, endpoint: KubeEndpoint, timeout: float = 30.0, compression: bool = True,
                 keepalive: float = 30.0) -> None:
        self.endpoint = endpoint
        # LIST bodies of a large cluster shrink ~10x with gzip (the API server
        # compresses responses over 128 KiB when asked); watches stay uncompressed
        self.list_headers = {"Accept-Encoding": "gzip"} if compression else None
        headers = {"Accept": "application/json", "User-Agent": USER_AGENT}
        headers.update(endpoint.static_headers)
        self.http = HttpClient(endpoint.server, endpoint.ssl_context, headers=headers,
                               timeout=timeout, header_provider=endpoint.header_provider,
                               server_name=endpoint.tls_server_name, keepalive=keepalive)

    async def _get(self, path: str, query: Optional[Dict[str, object]] = None,
                   timeout: Optional[float] = None, headers: Optional[Dict[str, str]] = None) -> Response:
        resp = await self.http.request("GET", path, query=query, timeout=timeout, headers=headers)
        if not resp.ok:
            raise ApiError(resp.status, resp.reason, resp.body, resp.headers)
        return resp

    async def get_version(self) -> Dict[str, object]:
        """``GET /version`` — the connectivity probe the reference meant to run."""
        return (await self._get("/version")).json()

    async def list_namespaces(self, limit: Optional[int] = None, continue_token: Optional[str] = None) -> Dict:
        q: Dict[str, object] = {}
        if limit:
            q["limit"] = limit
        if continue_token:
            q["continue"] = continue_token
        return (await self._get("/api/v1/namespaces", q)).json()

    async def list_pods_raw(self, namespace: Optional[str] = None, limit: Optional[int] = None,
                            continue_token: Optional[str] = None, label_selector: Optional[str] = None,
                            field_selector: Optional[str] = None,
                            resource_version: Optional[str] = None,
                            timeout: Optional[float] = None) -> bytes:
        q: Dict[str, object] = {}
        if limit:
            q["limit"] = limit
        if continue_token:
            q["continue"] = continue_token
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        if resource_version is not None:
            q["resourceVersion"] = resource_version
        return (await self._get(pods_path(namespace), q, timeout, self.list_headers)).body

    async def watch_pods(self, sink: Callable[[bytes, int], None], namespace: Optional[str] = None,
                         resource_version: Optional[str] = None, timeout_seconds: Optional[int] = None,
                         allow_bookmarks: bool = True, label_selector: Optional[str] = None,
                         field_selector: Optional[str] = None,
                         connect_timeout: Optional[float] = None, raw_chunked: bool = False,
                         on_mode: Optional[Callable[[bool], None]] = None,
                         send_initial_events: bool = False, read_size: int = 0,
                         zero_copy: bool = False) -> StreamResponse:
        """Open ``?watch=true``; body bytes go to ``sink(data, read_ns)``.

        With ``raw_chunked`` the HTTP chunk framing is left in place for the
        decoder to strip natively; ``on_mode(framed)`` reports which it got.
        ``send_initial_events`` makes it a WatchList request (streamed initial
        state ending in a bookmark annotated ``k8s.io/initial-events-end``).
        """
        q: Dict[str, object] = {"watch": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        if send_initial_events:
            q["sendInitialEvents"] = "true"
            q["resourceVersionMatch"] = "NotOlderThan"
            allow_bookmarks = True  # required by the API server for WatchList
        if allow_bookmarks:
            q["allowWatchBookmarks"] = "true"
        if timeout_seconds:
            q["timeoutSeconds"] = int(timeout_seconds)
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        stream, err = await self.http.stream("GET", pods_path(namespace), sink, query=q,
                                             timeout=connect_timeout, raw_chunked=raw_chunked,
                                             on_mode=on_mode, read_size=read_size, zero_copy=zero_copy)
        if err is not None:
            raise ApiError(stream.status, stream.reason, err, stream.headers)
        return stream

    async def watch_namespaces(self, sink: Callable[[bytes, int], None],
                               resource_version: Optional[str] = None,
                               timeout_seconds: Optional[int] = None,
                               connect_timeout: Optional[float] = None) -> StreamResponse:
        """``GET /api/v1/namespaces?watch=true`` (namespace discovery for
        ``watcher.namespace_scope: discover``); de-chunked NDJSON to ``sink``."""
        q: Dict[str, object] = {"watch": "true", "allowWatchBookmarks": "true"}
        if resource_version:
            q["resourceVersion"] = resource_version
        if timeout_seconds:
            q["timeoutSeconds"] = int(timeout_seconds)
        stream, err = await self.http.stream("GET", "/api/v1/namespaces", sink, query=q,
                                             timeout=connect_timeout)
        if err is not None:
            raise ApiError(stream.status, stream.reason, err, stream.headers)
        return stream

    # ------------------------------------------------------------------ coordination.k8s.io/v1
    # Lease objects back leader election (engine/leader.py); the reference runs
    # a single replica and has no equivalent.
    async def _json(self, method: str, path: str, doc: Optional[Dict] = None,
                    timeout: Optional[float] = None) -> Dict:
        body = None if doc is None else json.dumps(doc, separators=(",", ":")).encode()
        hdrs = None if body is None else {"Content-Type": "application/json"}
        resp = await self.http.request(method, path, headers=hdrs, body=body, timeout=timeout)
        if not resp.ok:
            raise ApiError(resp.status, resp.reason, resp.body, resp.headers)
        return resp.json() if resp.body else {}

    async def get_lease(self, namespace: str, name: str, timeout: Optional[float] = None) -> Optional[Dict]:
        """The Lease, or ``None`` when it does not exist."""
        try:
            return await self._json("GET", lease_path(namespace, name), timeout=timeout)
        except ApiError as exc:
            if exc.status == 404:
                return None
            raise

    async def create_lease(self, namespace: str, lease: Dict, timeout: Optional[float] = None) -> Dict:
        return await self._json("POST", lease_path(namespace), lease, timeout)

    async def replace_lease(self, namespace: str, name: str, lease: Dict,
                            timeout: Optional[float] = None) -> Dict:
        """PUT; ``metadata.resourceVersion`` in ``lease`` makes it a compare-and-swap (409 on conflict)."""
        return await self._json("PUT", lease_path(namespace, name), lease, timeout)

    # ------------------------------------------------------------------ authorization.k8s.io/v1
    async def can_i(self, verb: str, resource: str, group: str = "", namespace: Optional[str] = None,
                    name: Optional[str] = None, timeout: Optional[float] = None) -> Tuple[bool, str]:
        """SelfSubjectAccessReview: may this identity ``verb`` the ``resource``? -> (allowed, reason)."""
        attrs: Dict[str, object] = {"verb": verb, "resource": resource, "group": group}
        if namespace:
            attrs["namespace"] = namespace
        if name:
            attrs["name"] = name
        doc = await self._json("POST", "/apis/authorization.k8s.io/v1/selfsubjectaccessreviews",
                               {"apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview",
                                "spec": {"resourceAttributes": attrs}}, timeout)
        st = doc.get("status") or {}
        return bool(st.get("allowed")), str(st.get("reason") or "")

    async def close(self) -> None:
        await self.http.close()


def lease_path(namespace: str, name: Optional[str] = None) -> str:
    base = f"/apis/coordination.k8s.io/v1/namespaces/{namespace}/leases"
    return f"{base}/{name}" if name else base


def split_list_body(body: bytes) -> Tuple[Dict, list]:
    """Parse a ``*List`` body into ``(metadata, items)`` with the stdlib decoder."""
    doc = json.loads(json_input(body))
    return doc.get("metadata") or {}, doc.get("items") or []


__all__ = ["ApiError", "HttpError", "KubeApi", "lease_path", "pods_path", "split_list_body"]
