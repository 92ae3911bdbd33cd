"""Synchronous subset of ``kubernetes.client``.

Covers every call the reference and its smoke scripts make
(``/root/reference/watcher/pod_watcher.py:137,146,264``,
``test_k8s_mock.py:21-80``, ``test_k8s_connection.py:21-48``) plus the
obvious neighbours: ``CoreV1Api.list_pod_for_all_namespaces``,
``list_namespaced_pod``, ``read_namespaced_pod``, ``list_namespace``,
``get_api_resources`` and ``VersionApi.get_code``. Responses are
:class:`~k8s_watcher_amd.models.objects.ObjectView` objects, so
``pods.items[0].metadata.name`` and ``version.git_version`` work as with the
library. ``watch=True`` + ``_preload_content=False`` returns the raw streaming
response consumed by :class:`..watch.Watch`.

Transport is stdlib ``http.client`` (TLS through the endpoint's SSLContext).
"""

from __future__ import annotations

import http.client
import json
from typing import Any, Dict, Optional
from urllib.parse import urlencode, urlsplit

from ...kube.kubeconfig import KubeEndpoint
from ...models.objects import ObjectView


class ApiException(Exception):
    """``kubernetes.client.exceptions.ApiException`` equivalent."""

    def __init__(self, status: Optional[int] = None, reason: Optional[str] = None,
                 body: Optional[str] = None, headers: Optional[Dict[str, str]] = None) -> None:
        self.status = status
        self.reason = reason
        self.body = body
        self.headers = headers
        super().__init__(f"({status})\nReason: {reason}\nHTTP response body: {body}")


class Configuration:
    """Holds the endpoint selected by ``config.load_*``; ``get_default_copy()`` like the library."""

    _default: Optional["Configuration"] = None

    def __init__(self, endpoint: Optional[KubeEndpoint] = None, timeout: float = 60.0) -> None:
        self.endpoint = endpoint
        self.timeout = timeout

    @property
    def host(self) -> Optional[str]:
        return self.endpoint.server if self.endpoint else None

    @classmethod
    def set_default(cls, conf: "Configuration") -> None:
        cls._default = conf

    @classmethod
    def get_default_copy(cls) -> "Configuration":
        if cls._default is None:
            return Configuration(KubeEndpoint(server="http://localhost"))
        return Configuration(cls._default.endpoint, cls._default.timeout)


class ApiClient:
    def __init__(self, configuration: Optional[Configuration] = None) -> None:
        self.configuration = configuration or Configuration.get_default_copy()
        ep = self.configuration.endpoint
        if ep is None:
            raise ApiException(reason="no cluster configured: call config.load_kube_config() first")
        self.endpoint = ep
        u = urlsplit(ep.server)
        self.scheme = u.scheme
        self.host = u.hostname or "localhost"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.base_path = u.path.rstrip("/")

    def _conn(self, timeout: Optional[float]) -> http.client.HTTPConnection:
        t = timeout if timeout is not None else self.configuration.timeout
        if self.scheme == "https":
            return http.client.HTTPSConnection(self.host, self.port, timeout=t,
                                               context=self.endpoint.ssl_context)
        return http.client.HTTPConnection(self.host, self.port, timeout=t)

    def call_api(self, path: str, query: Optional[Dict[str, Any]] = None, preload: bool = True,
                 timeout: Optional[float] = None):
        q = {k: ("true" if v is True else "false" if v is False else v)
             for k, v in (query or {}).items() if v is not None}
        target = self.base_path + path + (("?" + urlencode(q)) if q else "")
        headers = {"Accept": "application/json", "User-Agent": "k8s-watcher-amd-compat/1.0"}
        headers.update(self.endpoint.auth_headers())
        conn = self._conn(timeout)
        try:
            conn.request("GET", target, headers=headers)
            resp = conn.getresponse()
        except OSError as exc:
            conn.close()
            raise ApiException(reason=f"connection failed: {exc}") from None
        if not (200 <= resp.status < 300):
            body = resp.read().decode("utf-8", "replace")
            conn.close()
            raise ApiException(resp.status, resp.reason, body, dict(resp.getheaders()))
        if not preload:
            resp._k8s_conn = conn  # keep the connection alive with the response
            return resp
        data = resp.read()
        conn.close()
        return json.loads(data) if data else {}


def _list_query(kwargs: Dict[str, Any]) -> Dict[str, Any]:
    mapping = {"limit": "limit", "_continue": "continue", "label_selector": "labelSelector",
               "field_selector": "fieldSelector", "resource_version": "resourceVersion",
               "timeout_seconds": "timeoutSeconds", "watch": "watch",
               "allow_watch_bookmarks": "allowWatchBookmarks",
               "resource_version_match": "resourceVersionMatch"}
    return {mapping[k]: v for k, v in kwargs.items() if k in mapping}


class CoreV1Api:
    def __init__(self, api_client: Optional[ApiClient] = None) -> None:
        self.api_client = api_client or ApiClient()

    def _list(self, path: str, kwargs: Dict[str, Any]):
        preload = kwargs.pop("_preload_content", True)
        timeout = kwargs.pop("_request_timeout", None)
        if kwargs.get("watch"):
            preload = False
        res = self.api_client.call_api(path, _list_query(kwargs), preload=preload, timeout=timeout)
        return ObjectView(res) if preload else res

    def list_pod_for_all_namespaces(self, **kwargs):
        return self._list("/api/v1/pods", kwargs)

    def list_namespaced_pod(self, namespace: str, **kwargs):
        return self._list(f"/api/v1/namespaces/{namespace}/pods", kwargs)

    def read_namespaced_pod(self, name: str, namespace: str, **kwargs):
        return ObjectView(self.api_client.call_api(f"/api/v1/namespaces/{namespace}/pods/{name}"))

    def list_namespace(self, **kwargs):
        return self._list("/api/v1/namespaces", kwargs)

    def get_api_resources(self, **kwargs):
        return ObjectView(self.api_client.call_api("/api/v1"))


class VersionApi:
    def __init__(self, api_client: Optional[ApiClient] = None) -> None:
        self.api_client = api_client or ApiClient()

    def get_code(self, **kwargs):
        return ObjectView(self.api_client.call_api("/version"))
