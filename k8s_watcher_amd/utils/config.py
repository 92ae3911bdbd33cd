"""Layered YAML configuration.

Reference behaviour being reproduced:

* ``config/base.yaml`` then ``config/<env>.yaml`` are read with ``yaml.safe_load``;
  an empty file counts as ``{}`` and a missing/broken file prints a message and
  counts as ``{}`` (``/root/reference/watcher/pod_watcher.py:19-45``).
* The environment file is deep-merged over the base: nested dicts merge
  recursively, every other value (lists included) is replaced wholesale
  (``pod_watcher.py:47-57``).
* After the merge, any string that is *entirely* ``${VAR}`` or
  ``${VAR:-default}`` is replaced by the environment variable (``""`` when
  unset and no default). No inline interpolation, no type coercion
  (``pod_watcher.py:59-75``).

Deliberate differences (documented in docs/DEVIATIONS.md):

* the config directory is CWD-relative like the reference, but can be
  overridden (``K8S_WATCHER_CONFIG_DIR`` / ``--config-dir``) and falls back to
  the directory that holds ``main.py`` when the CWD has no ``config/``;
* the merge deep-copies, so callers can mutate the result safely;
* :func:`settings_from_dict` turns the raw dict into a validated, typed
  :class:`Settings` object; unknown keys are kept in ``Settings.raw``.
"""

from __future__ import annotations

import copy
import logging
import os
import sys
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

SUPPORTED_ENVIRONMENTS = ("development", "staging", "production")

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class ConfigError(ValueError):
    """Raised for a configuration value that cannot be honoured."""


# --------------------------------------------------------------------------- raw layer


def resolve_config_dir(config_dir: Optional[str] = None) -> str:
    """Pick the directory that holds ``base.yaml`` and the per-env files.

    Precedence: explicit argument, ``$K8S_WATCHER_CONFIG_DIR``, ``./config``
    (the reference's CWD-relative lookup, ``pod_watcher.py:22``), then the
    ``config/`` directory next to this repository's ``main.py``.
    """
    if config_dir:
        return config_dir
    env_dir = os.environ.get("K8S_WATCHER_CONFIG_DIR")
    if env_dir:
        return env_dir
    if os.path.isdir("config"):
        return "config"
    return os.path.join(_REPO_ROOT, "config")


def load_config_file(path: str) -> Dict[str, Any]:
    """Read one YAML file; ``{}`` for a missing, empty or unreadable file.

    Messages are printed (not logged) because, as in the reference
    (``pod_watcher.py:39-45``), logging is configured *from* this config.
    """
    try:
        with open(path, "r", encoding="utf-8") as fh:
            data = yaml.safe_load(fh)
    except FileNotFoundError:
        print(f"Config file {path} not found")
        return {}
    except Exception as exc:  # noqa: BLE001 - parity: any error -> {}
        print(f"Error loading config {path}: {exc}")
        return {}
    if data is None:
        return {}
    if not isinstance(data, dict):
        print(f"Error loading config {path}: top level must be a mapping, got {type(data).__name__}")
        return {}
    return data


def deep_merge(base: Dict[str, Any], override: Dict[str, Any]) -> Dict[str, Any]:
    """Recursive merge, override wins; lists/scalars are replaced, not joined."""
    out = copy.deepcopy(base)
    for key, value in override.items():
        cur = out.get(key)
        if isinstance(cur, dict) and isinstance(value, dict):
            out[key] = deep_merge(cur, value)
        else:
            out[key] = copy.deepcopy(value)
    return out


def substitute_env(obj: Any, environ: Optional[Dict[str, str]] = None) -> Any:
    """Replace whole-string ``${VAR}`` / ``${VAR:-default}`` values recursively."""
    env = os.environ if environ is None else environ
    if isinstance(obj, dict):
        return {k: substitute_env(v, env) for k, v in obj.items()}
    if isinstance(obj, list):
        return [substitute_env(v, env) for v in obj]
    if isinstance(obj, str) and obj.startswith("${") and obj.endswith("}"):
        name = obj[2:-1]
        default = ""
        if ":-" in name:
            name, default = name.split(":-", 1)
        return env.get(name, default)
    return obj


def load_layered_config(environment: str, config_dir: Optional[str] = None,
                        environ: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    """base.yaml ⊕ <environment>.yaml, then env-var substitution."""
    cdir = resolve_config_dir(config_dir)
    base = load_config_file(os.path.join(cdir, "base.yaml"))
    env_cfg = load_config_file(os.path.join(cdir, f"{environment}.yaml"))
    return substitute_env(deep_merge(base, env_cfg), environ)


def get_path(cfg: Dict[str, Any], dotted: str, default: Any = None) -> Any:
    """``get_path(cfg, "watcher.alerts.critical_events_only")`` with a default."""
    cur: Any = cfg
    for part in dotted.split("."):
        if not isinstance(cur, dict) or part not in cur:
            return default
        cur = cur[part]
    return cur


# --------------------------------------------------------------------------- typed layer


def _as_bool(value: Any, key: str) -> bool:
    if isinstance(value, bool):
        return value
    if value is None:
        return False
    if isinstance(value, (int, float)):
        return bool(value)
    if isinstance(value, str):
        low = value.strip().lower()
        if low in ("1", "true", "yes", "on"):
            return True
        if low in ("", "0", "false", "no", "off"):
            return False
    raise ConfigError(f"{key}: expected a boolean, got {value!r}")


def _as_float(value: Any, key: str) -> float:
    try:
        return float(value)
    except (TypeError, ValueError):
        raise ConfigError(f"{key}: expected a number, got {value!r}") from None


def _bounded_float(value: Any, key: str, lo: float, hi: float) -> float:
    out = _as_float(value, key)
    if not lo <= out <= hi:
        raise ConfigError(f"{key}: expected a number in [{lo:g}, {hi:g}], got {value!r}")
    return out


def _as_int(value: Any, key: str) -> int:
    try:
        out = int(value)
    except (TypeError, ValueError):
        raise ConfigError(f"{key}: expected an integer, got {value!r}") from None
    return out


def _io_thread(value: Any) -> str:
    if value == "auto":
        return "auto"
    return "on" if _as_bool(value, "clusterapi.pool.io_thread") else "off"


def _bounded_int(value: Any, key: str, lo: int, hi: int) -> int:
    n = _as_int(value, key)
    if not lo <= n <= hi:
        raise ConfigError(f"{key}: {lo}..{hi}, got {n}")
    return n


# Keys that were settings once and are fixed now (their A/B measured, the
# winner kept: BENCHMARKS.md "Settings retired in round 6"). A config that
# still sets one loads; the value is ignored with a warning. watch_interval
# is the reference's key (a watch never polls): accepted silently.
RETIRED_KEYS = {
    "watcher": ("watch_list_idle_seconds", "watch_reader_depth", "hub_dispatch", "hub_framing",
                "partitioned_apply", "relist_slice_ms", "decode_affinity", "decode_l3_domain",
                "decode_spin_us", "malloc_trim_min_free_mb", "gc_freeze", "fd_table_reserve"),
    "clusterapi.pool": ("io_thread_on_rate", "io_thread_off_rate"),
    "clusterapi.spool": ("replay_batch",),
    "watcher.leader_election": ("release_on_shutdown",),
}


def retired_keys_in(cfg: Dict[str, Any]) -> List[str]:
    """The retired keys a merged config still sets (dotted paths)."""
    found = []
    for section, keys in RETIRED_KEYS.items():
        node: Any = cfg
        for part in section.split("."):
            node = node.get(part) if isinstance(node, dict) else None
        if isinstance(node, dict):
            found += [f"{section}.{k}" for k in keys if k in node]
    return found


def _choice(value: Any, key: str, choices: tuple) -> str:
    if value not in choices:
        raise ConfigError(f"{key}: expected one of {list(choices)}, got {value!r}")
    return value


@dataclass
class RetryPolicy:
    """Attempts/backoff for one retrying activity (``base.yaml`` ``retry:`` blocks).

    The reference declares these blocks but never reads them;
    here ``watcher.retry`` drives watch reconnects and ``clusterapi.retry``
    drives notify retries.
    """

    max_attempts: int = 3
    delay_seconds: float = 1.0
    multiplier: float = 2.0
    max_delay_seconds: float = 30.0
    jitter: float = 0.1

    def delay(self, attempt: int) -> float:
        """Backoff before retry number ``attempt`` (1-based), without jitter."""
        d = self.delay_seconds * (self.multiplier ** max(0, attempt - 1))
        return min(d, self.max_delay_seconds)


@dataclass
class KubernetesSettings:
    use_incluster_config: bool = False
    config_file: Optional[str] = None
    context: Optional[str] = None
    use_mock: bool = False
    request_timeout: float = 30.0
    compression: bool = True  # Accept-Encoding: gzip on LIST requests
    tcp_keepalive_seconds: float = 30.0  # dead-peer detection on API-server sockets (net/sockopt.py); 0 = off


@dataclass
class NotifierPoolSettings:
    connections: int = 16
    pipeline_depth: int = 32
    queue_size: int = 65536
    max_queued_bytes: int = 64 << 20  # backpressure also past this many owed body bytes
    coalesce: bool = False
    native: bool = True  # C++ notifier core (watcher.engine: native)
    # on: the native core serves its sockets on a dedicated thread
    # (profiles/notifier_io_thread_gpu_box.md); off: the event loop does;
    # auto: the thread while notifications run fast (parallel/native_notifier.py);
    # the config files' default is auto
    io_thread: str = "off"


@dataclass
class SpoolSettings:
    """``clusterapi.spool`` (parallel/spool.py): durable log of owed notifications."""

    path: Optional[str] = None  # None = off (reference: failed notifications are dropped)
    max_bytes: int = 1 << 30
    segment_bytes: int = 64 << 20
    fsync: bool = False
    replay_interval_seconds: float = 5.0


@dataclass
class ClusterApiSettings:
    enabled: bool = True
    base_url: str = "http://localhost:3000"
    api_key: str = ""
    pod_update: str = "/api/pods/update"
    health: str = "/health"
    timeout: float = 30.0
    retry: RetryPolicy = field(default_factory=lambda: RetryPolicy(3, 2.0))
    pool: NotifierPoolSettings = field(default_factory=NotifierPoolSettings)
    verify_tls: bool = True
    ca_file: Optional[str] = None
    cert_file: Optional[str] = None  # client certificate for mutual TLS (with key_file)
    key_file: Optional[str] = None
    health_check_on_start: bool = True
    spool: SpoolSettings = field(default_factory=SpoolSettings)
    rate_limit_qps: float = 0.0  # clusterapi.rate_limit.qps; 0 = unlimited
    rate_limit_burst: float = 100.0
    tcp_keepalive_seconds: float = 30.0  # dead-peer detection on clusterapi sockets (net/sockopt.py); 0 = off


@dataclass
class CheckpointSettings:
    path: Optional[str] = None
    interval_seconds: float = 5.0


@dataclass
class MetricsSettings:
    enabled: bool = False
    host: str = "0.0.0.0"
    port: int = 9090
    debug: bool = False  # also serve /debug/memory (Python object census, tracemalloc top sites)


@dataclass
class LeaderElectionSettings:
    """``watcher.leader_election`` (engine/leader.py): one active replica of several."""

    enabled: bool = False
    lease_name: str = "k8s-watcher-amd"
    lease_namespace: Optional[str] = None  # None = the pod's namespace, else "default"
    identity: Optional[str] = None  # None = $POD_NAME, else <hostname>_<random>
    lease_duration_seconds: float = 15.0
    renew_deadline_seconds: float = 10.0
    retry_period_seconds: float = 2.0
    exit_on_loss: bool = False


@dataclass
class WatcherSettings:
    log_level: str = "INFO"
    log_file: Optional[str] = None
    namespaces: List[str] = field(default_factory=list)
    namespace_scope: str = "client"  # client | server | discover
    namespace_drain_seconds: float = 5.0  # discover: a deleted namespace's pod watch runs until its pods are gone
    label_selector: Optional[str] = None
    field_selector: Optional[str] = None
    critical_events_only: bool = False
    notify_on: str = "all"  # all | phase_change
    initial_list: str = "notify"  # notify | skip
    initial_sync: str = "list"  # list | watch_list (sendInitialEvents, LIST fallback)
    payload_extra: int = 0  # watcher.payload_extra_fields as a models.payload.extra_mask
    watch_read_bytes: int = 4 << 20  # bytes per socket read on a plain-TCP watch (asyncio default 256 KiB)
    watch_reader: str = "native"  # native (ReaderHub thread, plain TCP + native engine) | asyncio
    watch_reader_buffers: int = 64  # ReaderHub pool: up to this many buffers of watch_read_bytes (allocated on use)
    watch_reader_max_bytes: int = 0  # ReaderHub read-ahead over all streams (0: the whole pool)
    # https watches: the reader hub reads and opens TLS 1.3 records itself
    # (native; openssl: SSL_read on the reader thread), on this many pool
    # threads besides the reader thread (-1: auto, utils/cpus.py)
    watch_tls_records: str = "native"
    watch_tls_threads: int = -1
    thread_pinning: str = "auto"  # auto: loop thread and reader thread on cores of their own in one L3 | loop | none
    retry: RetryPolicy = field(default_factory=lambda: RetryPolicy(3, 5.0))
    watch_timeout_seconds: int = 300
    list_page_size: int = 500
    relist_concurrency: int = 16  # scopes LISTing at once (a compaction 410s every namespace watch together); 0 = no cap
    engine: str = "native"  # native | python
    decode_threads: int = -1  # native engine: extra watch-decode threads, -1 = auto (utils/cpus.py)
    state_format: str = "structured"  # structured | python_repr
    # native engine: payload (every raw JSON token copied into a payload passes json.loads' rules) |
    # full (each whole watch line and LIST item must: INVALID exactly when the Python engine's json.loads
    # fails) | off (bracket matching only)
    validate: str = "payload"
    event_timestamp: str = "local"  # local | utc
    log_events: Optional[bool] = None  # None = follow log level (parity)
    checkpoint: CheckpointSettings = field(default_factory=CheckpointSettings)
    # native engine: every this many seconds the C heap's free pages go back to
    # the kernel (malloc_trim, off the event loop); 0 = never
    malloc_trim_seconds: float = 60.0
    shard: "ShardSettings" = field(default_factory=lambda: ShardSettings())
    leader_election: LeaderElectionSettings = field(default_factory=LeaderElectionSettings)


@dataclass
class ShardSettings:
    """Horizontal split of the pod space over ``count`` watcher processes."""

    count: int = 1
    index: int = 0
    key: str = "namespace"  # namespace | uid
    assignment: str = "hash"  # hash | balanced: namespace -> shard for per-namespace watches (parallel/shard.py)
    # a directory every shard can read and write (a shared volume): a shard
    # handing a namespace to another writes its cached pods there, and the new
    # owner's first LIST reconciles against them — no re-ADDED for pods that
    # stayed, DELETED for pods gone in between ("" = off: at-least-once ADDED,
    # deletions during a hand-over unreported; parallel/shard.py)
    handover_dir: str = ""
    handover_wait_seconds: float = 10.0  # the new owner waits this long for the old owner's record


@dataclass
class Settings:
    environment: str
    kubernetes: KubernetesSettings
    watcher: WatcherSettings
    clusterapi: ClusterApiSettings
    metrics: MetricsSettings
    raw: Dict[str, Any]

    @property
    def production(self) -> bool:
        return self.environment == "production"


def _retry(block: Any, key: str, default: RetryPolicy, min_attempts: int = 1) -> RetryPolicy:
    if not isinstance(block, dict):
        return copy.copy(default)
    return RetryPolicy(
        max_attempts=max(min_attempts, _as_int(block.get("max_attempts", default.max_attempts),
                                               f"{key}.max_attempts")),
        delay_seconds=max(0.0, _as_float(block.get("delay_seconds", default.delay_seconds), f"{key}.delay_seconds")),
        multiplier=max(1.0, _as_float(block.get("backoff_multiplier", default.multiplier), f"{key}.backoff_multiplier")),
        max_delay_seconds=_as_float(block.get("max_delay_seconds", default.max_delay_seconds), f"{key}.max_delay_seconds"),
        jitter=_as_float(block.get("jitter", default.jitter), f"{key}.jitter"),
    )


def _shard(block: Dict[str, Any]) -> ShardSettings:
    """``watcher.shard`` with ``$K8S_WATCHER_SHARD_INDEX/_COUNT`` taking precedence
    (set per process by :mod:`k8s_watcher_amd.parallel.launch`)."""
    count = os.environ.get("K8S_WATCHER_SHARD_COUNT", block.get("count", 1))
    index = os.environ.get("K8S_WATCHER_SHARD_INDEX", block.get("index", 0))
    s = ShardSettings(count=_as_int(count, "watcher.shard.count"), index=_as_int(index, "watcher.shard.index"),
                      key=_choice(block.get("key", "namespace"), "watcher.shard.key", ("namespace", "uid")),
                      assignment=_choice(block.get("assignment", "hash"), "watcher.shard.assignment",
                                         ("balanced", "hash")),
                      handover_dir=str(block.get("handover_dir") or ""),
                      handover_wait_seconds=_bounded_float(block.get("handover_wait_seconds", 10.0),
                                                           "watcher.shard.handover_wait_seconds", 0.0, 3600.0))
    if s.count < 1 or not 0 <= s.index < s.count:
        raise ConfigError(f"watcher.shard: index {s.index} outside [0, {s.count})")
    return s


def _payload_extra(names: Any) -> int:
    from ..models.payload import extra_mask
    if not isinstance(names, list):
        raise ConfigError(f"watcher.payload_extra_fields: expected a list, got {names!r}")
    try:
        return extra_mask(names)
    except ValueError as exc:
        raise ConfigError(f"watcher.payload_extra_fields: {exc}") from None


def _spool(block: Dict[str, Any]) -> SpoolSettings:
    key = "clusterapi.spool"
    sp = SpoolSettings(
        path=block.get("path") or None,
        max_bytes=_as_int(block.get("max_bytes", 1 << 30), f"{key}.max_bytes"),
        segment_bytes=_as_int(block.get("segment_bytes", 64 << 20), f"{key}.segment_bytes"),
        fsync=_as_bool(block.get("fsync", False), f"{key}.fsync"),
        replay_interval_seconds=_as_float(block.get("replay_interval_seconds", 5), f"{key}.replay_interval_seconds"),
    )
    if sp.max_bytes <= 0 or sp.segment_bytes <= 0 or sp.replay_interval_seconds <= 0:
        raise ConfigError(f"{key}: sizes, batch and interval must be positive")
    return sp


def _leader_election(block: Dict[str, Any]) -> LeaderElectionSettings:
    key = "watcher.leader_election"
    le = LeaderElectionSettings(
        enabled=_as_bool(block.get("enabled", False), f"{key}.enabled"),
        lease_name=str(block.get("lease_name") or "k8s-watcher-amd"),
        lease_namespace=block.get("lease_namespace") or None,
        identity=block.get("identity") or None,
        lease_duration_seconds=_as_float(block.get("lease_duration_seconds", 15), f"{key}.lease_duration_seconds"),
        renew_deadline_seconds=_as_float(block.get("renew_deadline_seconds", 10), f"{key}.renew_deadline_seconds"),
        retry_period_seconds=_as_float(block.get("retry_period_seconds", 2), f"{key}.retry_period_seconds"),
        exit_on_loss=_as_bool(block.get("exit_on_loss", False), f"{key}.exit_on_loss"),
    )
    if not 0 < le.retry_period_seconds < le.renew_deadline_seconds < le.lease_duration_seconds:
        raise ConfigError(f"{key}: need 0 < retry_period_seconds < renew_deadline_seconds < "
                          f"lease_duration_seconds, got {le.retry_period_seconds} / "
                          f"{le.renew_deadline_seconds} / {le.lease_duration_seconds}")
    return le


def _decode_threads(v: Any) -> int:
    if v is None or (isinstance(v, str) and v.strip().lower() == "auto"):
        return -1
    n = _as_int(v, "watcher.decode_threads")
    if not 0 <= n <= 64:
        raise ConfigError(f"watcher.decode_threads must be 'auto' or 0..64, got {v!r}")
    return n


def settings_from_dict(environment: str, cfg: Dict[str, Any]) -> Settings:
    """Validate the merged dict into :class:`Settings` (raises :class:`ConfigError`)."""
    for key in retired_keys_in(cfg):
        logging.getLogger("k8s_watcher_amd.config").warning(
            f"Config key {key} is no longer a setting (fixed; see docs/OPERATIONS.md): ignored")
    k = cfg.get("kubernetes") or {}
    w = cfg.get("watcher") or {}
    c = cfg.get("clusterapi") or {}
    m = cfg.get("metrics") or {}

    kube = KubernetesSettings(
        use_incluster_config=_as_bool(k.get("use_incluster_config", False), "kubernetes.use_incluster_config"),
        config_file=k.get("config_file") or None,
        context=k.get("context") or None,
        use_mock=_as_bool(k.get("use_mock", False), "kubernetes.use_mock"),
        request_timeout=_as_float(k.get("request_timeout", 30.0), "kubernetes.request_timeout"),
        compression=_as_bool(k.get("compression", True), "kubernetes.compression"),
        tcp_keepalive_seconds=max(0.0, _as_float(k.get("tcp_keepalive_seconds", 30.0),
                                                 "kubernetes.tcp_keepalive_seconds")),
    )

    level = str(w.get("log_level", "INFO")).upper()
    if not isinstance(logging.getLevelName(level), int):
        raise ConfigError(f"watcher.log_level: unknown level {w.get('log_level')!r}")
    namespaces = w.get("namespaces") or []
    if not isinstance(namespaces, list) or not all(isinstance(n, str) for n in namespaces):
        raise ConfigError(f"watcher.namespaces: expected a list of names, got {namespaces!r}")
    alerts = w.get("alerts") or {}
    ck = w.get("checkpoint") or {}
    watcher = WatcherSettings(
        log_level=level,
        log_file=w.get("log_file") or None,
        namespaces=list(namespaces),
        namespace_scope=_choice(w.get("namespace_scope", "client"), "watcher.namespace_scope",
                                ("client", "server", "discover")),
        namespace_drain_seconds=_bounded_float(w.get("namespace_drain_seconds", 5), "watcher.namespace_drain_seconds",
                                               0.0, 3600.0),
        label_selector=w.get("label_selector") or None,
        field_selector=w.get("field_selector") or None,
        critical_events_only=_as_bool(alerts.get("critical_events_only", False), "watcher.alerts.critical_events_only"),
        notify_on=_choice(w.get("notify_on", "all"), "watcher.notify_on", ("all", "phase_change")),
        initial_list=_choice(w.get("initial_list", "notify"), "watcher.initial_list", ("notify", "skip")),
        initial_sync=_choice(w.get("initial_sync", "list"), "watcher.initial_sync", ("list", "watch_list")),
        payload_extra=_payload_extra(w.get("payload_extra_fields") or []),
        watch_read_bytes=max(0, _as_int(w.get("watch_read_bytes", 4 << 20), "watcher.watch_read_bytes")),
        watch_reader=_choice(w.get("watch_reader", "native"), "watcher.watch_reader", ("native", "asyncio")),
        watch_reader_buffers=max(2, _as_int(w.get("watch_reader_buffers", 64), "watcher.watch_reader_buffers")),
        watch_reader_max_bytes=max(0, _as_int(w.get("watch_reader_max_bytes", 0), "watcher.watch_reader_max_bytes")),
        watch_tls_records=_choice(w.get("watch_tls_records", "native"), "watcher.watch_tls_records",
                                  ("native", "openssl")),
        watch_tls_threads=_bounded_int(w.get("watch_tls_threads", -1), "watcher.watch_tls_threads", -1, 32),
        malloc_trim_seconds=_bounded_float(w.get("malloc_trim_seconds", 60.0), "watcher.malloc_trim_seconds",
                                           0.0, 86400.0),
        thread_pinning=_choice(w.get("thread_pinning", "auto"), "watcher.thread_pinning", ("auto", "loop", "none")),
        retry=_retry(w.get("retry"), "watcher.retry", RetryPolicy(3, 5.0), min_attempts=0),
        watch_timeout_seconds=_as_int(w.get("watch_timeout_seconds", 300), "watcher.watch_timeout_seconds"),
        list_page_size=max(1, _as_int(w.get("list_page_size", 500), "watcher.list_page_size")),
        relist_concurrency=max(0, _as_int(w.get("relist_concurrency", 16), "watcher.relist_concurrency")),
        engine=_choice(w.get("engine", "native"), "watcher.engine", ("native", "python")),
        decode_threads=_decode_threads(w.get("decode_threads", "auto")),
        state_format=_choice(w.get("state_format", "structured"), "watcher.state_format", ("structured", "python_repr")),
        validate=_choice(w.get("validate", "payload"), "watcher.validate", ("off", "payload", "full")),
        event_timestamp=_choice(w.get("event_timestamp", "local"), "watcher.event_timestamp", ("local", "utc")),
        log_events=None if w.get("log_events") is None else _as_bool(w.get("log_events"), "watcher.log_events"),
        checkpoint=CheckpointSettings(
            path=ck.get("path") or None,
            interval_seconds=_as_float(ck.get("interval_seconds", 5.0), "watcher.checkpoint.interval_seconds"),
        ),
        shard=_shard(w.get("shard") or {}),
        leader_election=_leader_election(w.get("leader_election") or {}),
    )

    endpoints = c.get("endpoints") or {}
    auth = c.get("auth") or {}
    pool = c.get("pool") or {}
    clusterapi = ClusterApiSettings(
        enabled=_as_bool(c.get("enabled", True), "clusterapi.enabled"),
        base_url=str(c.get("base_url") or "http://localhost:3000").rstrip("/"),
        api_key=str(auth.get("api_key") or ""),
        pod_update=str(endpoints.get("pod_update", "/api/pods/update")),
        health=str(endpoints.get("health", "/health")),
        timeout=_as_float(c.get("timeout", 30), "clusterapi.timeout"),
        retry=_retry(c.get("retry"), "clusterapi.retry", RetryPolicy(3, 2.0)),
        pool=NotifierPoolSettings(
            connections=max(1, _as_int(pool.get("connections", 16), "clusterapi.pool.connections")),
            pipeline_depth=max(1, _as_int(pool.get("pipeline_depth", 32), "clusterapi.pool.pipeline_depth")),
            queue_size=max(1, _as_int(pool.get("queue_size", 65536), "clusterapi.pool.queue_size")),
            max_queued_bytes=max(1 << 16, _as_int(pool.get("max_queued_bytes", 64 << 20),
                                                  "clusterapi.pool.max_queued_bytes")),
            coalesce=_as_bool(pool.get("coalesce", False), "clusterapi.pool.coalesce"),
            native=_as_bool(pool.get("native", True), "clusterapi.pool.native"),
            io_thread=_io_thread(pool.get("io_thread", "auto")),
        ),
        verify_tls=_as_bool(c.get("verify_tls", True), "clusterapi.verify_tls"),
        ca_file=c.get("ca_file") or None,
        cert_file=c.get("cert_file") or None,
        key_file=c.get("key_file") or None,
        health_check_on_start=_as_bool(c.get("health_check_on_start", True), "clusterapi.health_check_on_start"),
        spool=_spool(c.get("spool") or {}),
        rate_limit_qps=max(0.0, _as_float((c.get("rate_limit") or {}).get("qps", 0), "clusterapi.rate_limit.qps")),
        rate_limit_burst=max(1.0, _as_float((c.get("rate_limit") or {}).get("burst", 100),
                                            "clusterapi.rate_limit.burst")),
        tcp_keepalive_seconds=max(0.0, _as_float(c.get("tcp_keepalive_seconds", 30.0),
                                                 "clusterapi.tcp_keepalive_seconds")),
    )

    metrics = MetricsSettings(
        enabled=_as_bool(m.get("enabled", False), "metrics.enabled"),
        host=str(m.get("host", "0.0.0.0")),
        port=_as_int(m.get("port", 9090), "metrics.port"),
        debug=_as_bool(m.get("debug", False), "metrics.debug"),
    )
    return Settings(environment, kube, watcher, clusterapi, metrics, cfg)


def load_settings(environment: str, config_dir: Optional[str] = None,
                  overrides: Optional[Dict[str, Any]] = None,
                  environ: Optional[Dict[str, str]] = None) -> Settings:
    """Full path: layered YAML → env substitution → optional overrides → :class:`Settings`."""
    raw = load_layered_config(environment, config_dir, environ)
    if overrides:
        raw = deep_merge(raw, overrides)
    return settings_from_dict(environment, raw)


def parse_override(expr: str) -> Dict[str, Any]:
    """``"watcher.notify_on=phase_change"`` → nested dict (value parsed as YAML)."""
    if "=" not in expr:
        raise ConfigError(f"override {expr!r}: expected key.path=value")
    key, value = expr.split("=", 1)
    node: Dict[str, Any] = {}
    cur = node
    parts = key.strip().split(".")
    for part in parts[:-1]:
        cur[part] = {}
        cur = cur[part]
    cur[parts[-1]] = yaml.safe_load(value)
    return node


def dump_effective(settings: Settings, stream=None) -> None:
    """Print the merged raw config as YAML (``--print-config``)."""
    yaml.safe_dump(settings.raw, stream or sys.stdout, sort_keys=False)
