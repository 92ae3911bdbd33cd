"""Single-request clusterapi clients.

Reference: ``ClusterApiClient`` (``/root/reference/watcher/clusterapi_client.py:6-61``)
— a ``requests.Session`` POSTing ``{base}/api/pods/update``. The same public
surface is kept (``update_pod_status(pod_data) -> bool``,
``health_check() -> bool``, bearer-key header, the same log lines) with the
reference's defects fixed: the ``timeout`` is honoured, the
endpoint paths come from ``clusterapi.endpoints``, any 2xx is success and
``clusterapi.retry`` is applied with exponential backoff. The constructor
accepts the three positional arguments the reference's factory passes
(``pod_watcher.py:108``), which its own ``__init__`` rejected.

:class:`ClusterApiClient` is synchronous (``requests``);
:class:`AsyncClusterApiClient` runs on the framework's asyncio HTTP client.
For high event rates use :class:`k8s_watcher_amd.parallel.notifier.NotifierPool`.
"""

from __future__ import annotations

import json
import logging
import time
from typing import Any, Dict, Optional

from ..net.http import HttpClient, HttpError, parse_retry_after
from ..utils.config import RetryPolicy
from ..utils.logsetup import NOTIFIER_LOGGER

RETRYABLE = frozenset({408, 425, 429, 500, 502, 503, 504})


class _Common:
    def __init__(self, base_url: str, api_key: Optional[str] = None, timeout: float = 30.0,
                 pod_update: str = "/api/pods/update", health: str = "/health",
                 retry: Optional[RetryPolicy] = None, verify_tls: bool = True, ca_file: Optional[str] = None,
                 cert_file: Optional[str] = None, key_file: Optional[str] = None) -> None:
        self.base_url = base_url.rstrip("/")
        self.verify_tls, self.ca_file, self.cert_file, self.key_file = verify_tls, ca_file, cert_file, key_file
        self.api_key = api_key
        self.timeout = timeout
        self.pod_update = pod_update
        self.health = health
        self.retry = retry or RetryPolicy(max_attempts=1, delay_seconds=0.0)
        self.logger = logging.getLogger(NOTIFIER_LOGGER)
        self.headers = {"Content-Type": "application/json"}
        if api_key:
            self.headers["Authorization"] = f"Bearer {api_key}"

    @property
    def endpoint(self) -> str:
        return f"{self.base_url}{self.pod_update}"

    @classmethod
    def from_settings(cls, c) -> "_Common":
        return cls(c.base_url, c.api_key or None, c.timeout, c.pod_update, c.health, c.retry,
                   verify_tls=c.verify_tls, ca_file=c.ca_file, cert_file=c.cert_file, key_file=c.key_file)


class ClusterApiClient(_Common):
    """Synchronous client (``requests``), API-compatible with the reference."""

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        import requests
        self._requests = requests
        self.session = requests.Session()
        self.session.headers.update(self.headers)
        # per request: a session-level ``verify`` loses to $REQUESTS_CA_BUNDLE in requests
        self._tls_kw: Dict[str, Any] = {"verify": self.ca_file or self.verify_tls}
        if self.cert_file:
            self._tls_kw["cert"] = (self.cert_file, self.key_file) if self.key_file else self.cert_file

    def update_pod_status(self, pod_data: Dict[str, Any]) -> bool:
        ep = self.endpoint
        self.logger.info(f"Calling clusterapi: {ep}")
        if self.logger.isEnabledFor(logging.DEBUG):
            self.logger.debug(f"Pod data: {json.dumps(pod_data, indent=2)}")
        body = json.dumps(pod_data).encode("utf-8")
        for attempt in range(1, max(1, self.retry.max_attempts) + 1):
            status = None
            retry_after = None
            try:
                resp = self.session.post(ep, data=body, timeout=self.timeout, **self._tls_kw)
                status = resp.status_code
                retry_after = parse_retry_after(resp.headers.get("Retry-After"))
                if 200 <= status < 300:
                    self.logger.info(f"Successfully updated pod data for {pod_data.get('name', 'unknown')}")
                    return True
                self.logger.error(f"Failed to update pod data. Status: {status}, Response: {resp.text}")
            except self._requests.exceptions.ConnectionError:
                self.logger.error(f"Connection error: Unable to connect to clusterapi at {ep}")
            except self._requests.exceptions.Timeout:
                self.logger.error(f"Timeout error: Request to {ep} timed out")
            except Exception as exc:  # noqa: BLE001 - parity
                self.logger.error(f"Unexpected error calling clusterapi: {exc}")
                return False
            if status is not None and status not in RETRYABLE:
                return False
            if attempt < self.retry.max_attempts:
                time.sleep(max(self.retry.delay(attempt), retry_after or 0.0))
        return False

    def health_check(self) -> bool:
        try:
            resp = self.session.get(f"{self.base_url}{self.health}", timeout=min(5.0, self.timeout), **self._tls_kw)
            return 200 <= resp.status_code < 300
        except Exception:  # noqa: BLE001 - parity: any failure -> False
            return False


class AsyncClusterApiClient(_Common):
    """Same API, ``async``, over the framework's keep-alive HTTP client."""

    def __init__(self, *args: Any, ssl_context=None, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        if ssl_context is None and self.base_url.startswith("https://"):
            import ssl
            ssl_context = ssl.create_default_context(cafile=self.ca_file)
            if self.cert_file:
                ssl_context.load_cert_chain(self.cert_file, self.key_file)
            if not self.verify_tls:
                ssl_context.check_hostname = False
                ssl_context.verify_mode = ssl.CERT_NONE
        self.http = HttpClient(self.base_url, ssl_context, headers=self.headers, timeout=self.timeout)

    async def update_pod_status(self, pod_data: Dict[str, Any]) -> bool:
        import asyncio
        ep = self.endpoint
        body = json.dumps(pod_data).encode("utf-8")
        for attempt in range(1, max(1, self.retry.max_attempts) + 1):
            status = None
            retry_after = None
            try:
                resp = await self.http.request("POST", self.pod_update, body=body)
                status = resp.status
                retry_after = parse_retry_after(resp.headers.get("retry-after"))
                if resp.ok:
                    return True
                self.logger.error(f"Failed to update pod data. Status: {status}, Response: {resp.text()}")
            except HttpError as exc:
                self.logger.error(f"Connection error: Unable to connect to clusterapi at {ep} ({exc})")
            if status is not None and status not in RETRYABLE:
                return False
            if attempt < self.retry.max_attempts:
                await asyncio.sleep(max(self.retry.delay(attempt), retry_after or 0.0))
        return False

    async def health_check(self) -> bool:
        try:
            resp = await self.http.request("GET", self.health, timeout=min(5.0, self.timeout))
            return resp.ok
        except Exception:  # noqa: BLE001
            return False

    async def close(self) -> None:
        await self.http.close()
