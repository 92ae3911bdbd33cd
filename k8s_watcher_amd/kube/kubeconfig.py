"""Kubeconfig and in-cluster credential loading.

The reference calls ``kubernetes.config.load_incluster_config()`` /
``load_kube_config(config_file=...)`` / ``load_kube_config()``
(``/root/reference/watcher/pod_watcher.py:115-134``). That library is not
available, so this module implements the subset of its behaviour a pod
watcher needs, returning a :class:`KubeEndpoint` (server URL, TLS context,
auth-header provider) instead of mutating a global ``Configuration``.

Kubeconfig support: ``current-context`` or an explicit context; ``$KUBECONFIG``
(``:``-separated, first definition of a name wins) then ``~/.kube/config``;
``server``, ``certificate-authority[-data]``, ``insecure-skip-tls-verify``,
``tls-server-name``; user ``token`` / ``tokenFile`` / basic auth /
``client-certificate[-data]`` + ``client-key[-data]`` / ``exec`` credential
plugins. Relative file paths resolve against the kubeconfig's directory.

In-cluster: ``$KUBERNETES_SERVICE_HOST``/``$KUBERNETES_SERVICE_PORT`` and the
service-account token + CA; the token file is re-read periodically so bound
(rotating) tokens keep working — something the reference's one-shot load
does not do.
"""

from __future__ import annotations

import base64
import json
import os
import ssl
import subprocess
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml

from ..net.http import HttpError

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ConfigException(Exception):
    """Same role as ``kubernetes.config.ConfigException`` (``pod_watcher.py:2,152``)."""


class CredentialError(ConfigException, HttpError):
    """The exec credential plugin failed while serving a request. A
    :class:`ConfigException` at setup time; at run time an :class:`HttpError`,
    so the reflector backs off and retries instead of ending the watch."""


@dataclass
class KubeEndpoint:
    server: str
    ssl_context: Optional[ssl.SSLContext] = None
    static_headers: Dict[str, str] = field(default_factory=dict)
    header_provider: Optional[Callable[[], Dict[str, str]]] = None
    namespace: Optional[str] = None
    source: str = ""
    context_name: Optional[str] = None
    tls_server_name: Optional[str] = None  # verify the server certificate against this name

    def auth_headers(self) -> Dict[str, str]:
        h = dict(self.static_headers)
        if self.header_provider is not None:
            h.update(self.header_provider())
        return h

    def invalidate_credentials(self) -> bool:
        """After a ``401``: drop the cached token so the next request re-reads
        the token file / re-runs the exec plugin (client-go does the same).
        An exec plugin is re-run on a background thread, keeping the old token
        until the new one arrives: the event loop never waits for the plugin.
        Returns False when the credentials are static (nothing to refresh)."""
        owner = getattr(self.header_provider, "__self__", None)
        inval = getattr(owner, "invalidate", None)
        if inval is None:
            return False
        inval()
        return True

    async def refresh_credentials(self) -> bool:
        """:meth:`invalidate_credentials`, then wait (off the event loop) until
        the fresh token is in place. False when there is nothing to refresh."""
        if not self.invalidate_credentials():
            return False
        owner = getattr(self.header_provider, "__self__", None)
        wait = getattr(owner, "wait_refreshed", None)
        if wait is not None:
            import asyncio
            await asyncio.get_running_loop().run_in_executor(None, wait)
        return True


# --------------------------------------------------------------------------- helpers


def _read_yaml(path: str) -> Dict[str, Any]:
    try:
        with open(path, "r", encoding="utf-8") as fh:
            data = yaml.safe_load(fh) or {}
    except FileNotFoundError:
        raise ConfigException(f"Invalid kube-config file. No configuration found: {path}") from None
    except yaml.YAMLError as exc:
        raise ConfigException(f"Invalid kube-config file {path}: {exc}") from None
    if not isinstance(data, dict):
        raise ConfigException(f"Invalid kube-config file {path}: not a mapping")
    return data


def kubeconfig_paths(config_file: Optional[str] = None) -> List[str]:
    if config_file:
        return [os.path.expanduser(config_file)]
    env = os.environ.get("KUBECONFIG")
    if env:
        return [os.path.expanduser(p) for p in env.split(os.pathsep) if p]
    return [os.path.expanduser("~/.kube/config")]


def _named(items: Optional[List[Dict[str, Any]]], key: str) -> Dict[str, Tuple[Dict[str, Any], str]]:
    out: Dict[str, Tuple[Dict[str, Any], str]] = {}
    for it in items or []:
        if isinstance(it, dict) and "name" in it:
            out[it["name"]] = (it.get(key) or {}, "")
    return out


class KubeConfigDocument:
    """The merged view of one or more kubeconfig files."""

    def __init__(self, paths: List[str]) -> None:
        self.paths = paths
        self.clusters: Dict[str, Tuple[Dict[str, Any], str]] = {}
        self.users: Dict[str, Tuple[Dict[str, Any], str]] = {}
        self.contexts: Dict[str, Tuple[Dict[str, Any], str]] = {}
        self.context_order: List[str] = []
        self.current_context: Optional[str] = None
        found = False
        for p in paths:
            if not os.path.exists(p):
                continue
            found = True
            doc = _read_yaml(p)
            base = os.path.dirname(os.path.abspath(p))
            for section, key, store in (("clusters", "cluster", self.clusters),
                                        ("users", "user", self.users),
                                        ("contexts", "context", self.contexts)):
                for name, (body, _) in _named(doc.get(section), key).items():
                    if name not in store:
                        store[name] = (body, base)
                        if section == "contexts":
                            self.context_order.append(name)
            if self.current_context is None and doc.get("current-context"):
                self.current_context = doc["current-context"]
        if not found:
            raise ConfigException(f"Invalid kube-config file. No configuration found: {':'.join(paths)}")

    def list_contexts(self) -> Tuple[List[Dict[str, Any]], Optional[Dict[str, Any]]]:
        ctxs = [{"name": n, "context": dict(self.contexts[n][0])} for n in self.context_order]
        active = next((c for c in ctxs if c["name"] == self.current_context), None)
        return ctxs, active


def _resolve(base: str, path: Optional[str]) -> Optional[str]:
    if not path:
        return None
    path = os.path.expanduser(path)
    return path if os.path.isabs(path) else os.path.join(base, path)


def _b64(data: str) -> bytes:
    return base64.b64decode(data.encode("ascii") if isinstance(data, str) else data)


def _load_cert_chain(ctx: ssl.SSLContext, cert_pem: bytes, key_pem: bytes) -> None:
    # ssl only loads client certs from files: stage them in private temp files.
    fds = []
    try:
        paths = []
        for blob in (cert_pem, key_pem):
            fd, p = tempfile.mkstemp(prefix="kw-", suffix=".pem")
            os.fchmod(fd, 0o600)
            with os.fdopen(fd, "wb") as fh:
                fh.write(blob)
            paths.append(p)
            fds.append(p)
        ctx.load_cert_chain(paths[0], paths[1])
    finally:
        for p in fds:
            try:
                os.unlink(p)
            except OSError:
                pass


def build_ssl_context(ca_file: Optional[str] = None, ca_data: Optional[bytes] = None,
                      insecure: bool = False, cert_pem: Optional[bytes] = None,
                      key_pem: Optional[bytes] = None) -> ssl.SSLContext:
    if insecure:
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif ca_file or ca_data:
        ctx = ssl.create_default_context(cafile=ca_file,
                                         cadata=ca_data.decode("ascii") if ca_data else None)
    else:
        ctx = ssl.create_default_context()
    if cert_pem and key_pem:
        _load_cert_chain(ctx, cert_pem, key_pem)
    # the same trust material for the native watch reader (net/reader.py),
    # which runs its own OpenSSL session on https watches
    ca_pem = ca_data
    if ca_file and not insecure:
        with open(ca_file, "rb") as fh:
            ca_pem = (fh.read() + b"\n" + ca_data) if ca_data else fh.read()
    ctx.kw_tls = {"ca_pem": None if insecure else ca_pem, "cert_pem": cert_pem if key_pem else None,
                  "key_pem": key_pem if cert_pem else None, "verify": not insecure}
    return ctx


class _ExecCredential:
    """Runs a client-go ``exec`` credential plugin and caches its token.

    Only the very first request waits for the plugin in the foreground
    (there is no token to send). Afterwards every refresh — ahead of the
    expiry, after a ``401`` (:meth:`invalidate`) or once the token expired —
    runs on one background thread while requests keep the last token; a
    failing plugin keeps the old token and surfaces as a retryable
    :class:`CredentialError`, never as a crash of the watch loop.
    """

    def __init__(self, spec: Dict[str, Any], base: str = "") -> None:
        self.spec = spec
        self.base = base  # a relative command path resolves against the kubeconfig's directory
        self._token: Optional[str] = None
        self._expiry: float = 0.0
        self._lock = threading.Lock()
        self._bg: Optional[threading.Thread] = None
        self.last_error: Optional[str] = None
        self.refreshes = 0

    def headers(self) -> Dict[str, str]:
        if self._token is None:
            try:
                self._refresh()  # nothing to send yet: this one request waits for the plugin
            except ConfigException as exc:
                raise CredentialError(str(exc)) from None
        elif self._expiry and time.time() >= self._expiry - 120:
            self._start_bg()  # refresh ahead of (or after) the expiry, off the event loop
        return {"Authorization": f"Bearer {self._token}"} if self._token else {}

    def invalidate(self) -> None:
        """A ``401``: re-run the plugin in the background, keep the old token meanwhile."""
        if self._token is None:
            return  # the next headers() runs it anyway
        self._start_bg()

    def wait_refreshed(self, timeout: float = 90.0) -> None:
        """Block (call from an executor thread) until a running refresh ends."""
        th = self._bg
        if th is not None:
            th.join(timeout)

    def _start_bg(self) -> None:
        with self._lock:
            if self._bg is not None:
                return
            self._bg = threading.Thread(target=self._refresh_bg, name="exec-credential", daemon=True)
            self._bg.start()

    def _refresh_bg(self) -> None:
        try:
            self._refresh()
        except ConfigException as exc:
            self.last_error = str(exc)  # keep the old token; the next 401 or expiry check retries
        finally:
            with self._lock:
                self._bg = None

    def _refresh(self) -> None:
        cmd = [self.spec.get("command")] + list(self.spec.get("args") or [])
        if not cmd[0]:
            raise ConfigException("exec credential plugin has no command")
        if self.base and os.sep in cmd[0] and not os.path.isabs(cmd[0]):
            cmd[0] = os.path.join(self.base, cmd[0])
        env = dict(os.environ)
        for item in self.spec.get("env") or []:
            if isinstance(item, dict) and item.get("name"):
                env[item["name"]] = str(item.get("value", ""))
        api_version = self.spec.get("apiVersion", "client.authentication.k8s.io/v1beta1")
        env["KUBERNETES_EXEC_INFO"] = json.dumps(
            {"apiVersion": api_version, "kind": "ExecCredential", "spec": {"interactive": False}})
        try:
            out = subprocess.run(cmd, env=env, capture_output=True, check=True, timeout=60).stdout
        except (OSError, subprocess.SubprocessError) as exc:
            raise ConfigException(f"exec credential plugin {cmd[0]!r} failed: {exc}") from None
        try:
            status = json.loads(out).get("status") or {}
        except ValueError:
            raise ConfigException("exec credential plugin returned invalid JSON") from None
        token = status.get("token")
        if not token:
            raise ConfigException("exec credential plugin returned no token")
        expiry = 0.0
        exp = status.get("expirationTimestamp")
        if exp:
            from ..utils.timefmt import parse_k8s_time
            dt = parse_k8s_time(exp)
            if dt is not None:
                expiry = dt.timestamp()
        self._token, self._expiry = token, expiry  # one assignment: a reader sees old or new, never half
        self.last_error = None
        self.refreshes += 1


class _TokenFile:
    """Bearer token read from a file and re-read every ``period`` seconds."""

    def __init__(self, path: str, period: float = 60.0) -> None:
        self.path = path
        self.period = period
        self._token = ""
        self._read_at = 0.0
        self._read()

    def _read(self) -> None:
        try:
            with open(self.path, "r", encoding="utf-8") as fh:
                self._token = fh.read().strip()
        except OSError as exc:
            if not self._token:
                raise ConfigException(f"cannot read token file {self.path}: {exc}") from None
        self._read_at = time.monotonic()

    def invalidate(self) -> None:
        self._read_at = float("-inf")  # re-read on the next request

    def headers(self) -> Dict[str, str]:
        if time.monotonic() - self._read_at > self.period:
            self._read()
        return {"Authorization": f"Bearer {self._token}"} if self._token else {}


# --------------------------------------------------------------------------- loaders


def list_kube_config_contexts(config_file: Optional[str] = None):
    """``(contexts, active_context)`` like ``kubernetes.config.list_kube_config_contexts``."""
    return KubeConfigDocument(kubeconfig_paths(config_file)).list_contexts()


def load_kube_config(config_file: Optional[str] = None, context: Optional[str] = None) -> KubeEndpoint:
    paths = kubeconfig_paths(config_file)
    doc = KubeConfigDocument(paths)
    ctx_name = context or doc.current_context
    if not ctx_name:
        raise ConfigException("Invalid kube-config file. Expected key current-context")
    if ctx_name not in doc.contexts:
        raise ConfigException(f"Invalid kube-config file. Expected object with name {ctx_name} in contexts list")
    ctx, _ = doc.contexts[ctx_name]
    cluster_name = ctx.get("cluster")
    if cluster_name not in doc.clusters:
        raise ConfigException(f"Invalid kube-config file. Expected object with name {cluster_name} in clusters list")
    cluster, cbase = doc.clusters[cluster_name]
    user, ubase = doc.users.get(ctx.get("user"), ({}, os.getcwd()))
    server = cluster.get("server")
    if not server:
        raise ConfigException(f"cluster {cluster_name!r} has no server")

    headers: Dict[str, str] = {}
    provider: Optional[Callable[[], Dict[str, str]]] = None
    if user.get("token"):
        headers["Authorization"] = f"Bearer {user['token']}"
    elif user.get("tokenFile"):
        provider = _TokenFile(_resolve(ubase, user["tokenFile"])).headers  # type: ignore[arg-type]
    elif user.get("exec"):
        provider = _ExecCredential(user["exec"], ubase).headers
    elif user.get("username") and user.get("password"):
        cred = base64.b64encode(f"{user['username']}:{user['password']}".encode()).decode()
        headers["Authorization"] = f"Basic {cred}"

    ssl_ctx = None
    if server.startswith("https://"):
        ca_data = _b64(cluster["certificate-authority-data"]) if cluster.get("certificate-authority-data") else None
        cert = key = None
        if user.get("client-certificate-data"):
            cert = _b64(user["client-certificate-data"])
        elif user.get("client-certificate"):
            with open(_resolve(ubase, user["client-certificate"]), "rb") as fh:  # type: ignore[arg-type]
                cert = fh.read()
        if user.get("client-key-data"):
            key = _b64(user["client-key-data"])
        elif user.get("client-key"):
            with open(_resolve(ubase, user["client-key"]), "rb") as fh:  # type: ignore[arg-type]
                key = fh.read()
        try:
            ssl_ctx = build_ssl_context(
                ca_file=_resolve(cbase, cluster.get("certificate-authority")),
                ca_data=ca_data,
                insecure=bool(cluster.get("insecure-skip-tls-verify")),
                cert_pem=cert, key_pem=key)
        except (ssl.SSLError, OSError, ValueError) as exc:
            raise ConfigException(f"TLS setup for cluster {cluster_name!r} failed: {exc}") from None
    return KubeEndpoint(server=server.rstrip("/"), ssl_context=ssl_ctx, static_headers=headers,
                        header_provider=provider, namespace=ctx.get("namespace"),
                        source=":".join(paths), context_name=ctx_name,
                        tls_server_name=cluster.get("tls-server-name") or None)


def load_incluster_config(sa_dir: str = SA_DIR, environ: Optional[Dict[str, str]] = None,
                          token_refresh_seconds: float = 60.0) -> KubeEndpoint:
    env = os.environ if environ is None else environ
    host = env.get("KUBERNETES_SERVICE_HOST")
    port = env.get("KUBERNETES_SERVICE_PORT")
    if not host or not port:
        raise ConfigException("Service host/port is not set.")
    token_path = os.path.join(sa_dir, "token")
    ca_path = os.path.join(sa_dir, "ca.crt")
    if not os.path.exists(token_path):
        raise ConfigException("Service token file does not exist.")
    if not os.path.exists(ca_path):
        raise ConfigException("Service certification file does not exist.")
    if ":" in host and not host.startswith("["):
        host = f"[{host}]"
    tok = _TokenFile(token_path, token_refresh_seconds)
    try:
        ctx = build_ssl_context(ca_file=ca_path)
    except (ssl.SSLError, OSError) as exc:
        raise ConfigException(f"in-cluster CA unusable: {exc}") from None
    ns = None
    ns_path = os.path.join(sa_dir, "namespace")
    if os.path.exists(ns_path):
        with open(ns_path, "r", encoding="utf-8") as fh:
            ns = fh.read().strip()
    return KubeEndpoint(server=f"https://{host}:{port}", ssl_context=ctx, header_provider=tok.headers,
                        namespace=ns, source="in-cluster")
