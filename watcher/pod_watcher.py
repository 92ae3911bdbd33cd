"""``from watcher.pod_watcher import PodWatcher`` — the reference's class API on the new engine.

Method-for-method surface of ``/root/reference/watcher/pod_watcher.py``
(``PodWatcher.__init__/setup_k8s_client/start_watching/should_process_event/
handle_pod_event/_extract_pod_data`` and the config helpers), implemented as
thin adapters:

* config/logging → :mod:`k8s_watcher_amd.utils.config` / ``utils.logsetup``;
* ``setup_k8s_client`` → the compat ``kubernetes`` client with a working
  ``GET /version`` probe (the reference's ``get_api_version`` does not exist);
* ``handle_pod_event`` accepts library-style objects, attribute views or raw
  dicts, and returns the payload it built (``None`` when filtered); when a
  ``clusterapi_client`` is attached it is notified synchronously;
* ``start_watching`` runs the asynchronous :class:`WatcherService`
  (reflector + pipeline + notifier pool).
"""

from __future__ import annotations

import asyncio
import logging
import os
import signal
from typing import Any, Dict, Optional

from k8s_watcher_amd.compat.kubernetes import client as k8s_client
from k8s_watcher_amd.compat.kubernetes import config as k8s_config
from k8s_watcher_amd.compat.kubernetes import watch as k8s_watch
from k8s_watcher_amd.kube.kubeconfig import ConfigException
from k8s_watcher_amd.models.objects import raw_of
from k8s_watcher_amd.models.payload import build_payload_dict
from k8s_watcher_amd.ops.filters import CriticalFilter, NamespaceFilter
from k8s_watcher_amd.utils import config as cfg
from k8s_watcher_amd.utils.logsetup import setup_logging
from k8s_watcher_amd.notify.clusterapi import ClusterApiClient


class PodWatcher:
    def __init__(self, environment: str = "development", config_dir: Optional[str] = None) -> None:
        self.environment = environment
        self.config_dir = config_dir
        self.config = self._load_environment_config()
        self.settings = cfg.settings_from_dict(environment, self.config)
        self.v1 = None
        self.watch = k8s_watch.Watch()
        self.clusterapi_client: Optional[ClusterApiClient] = None
        self._setup_logging()
        self._critical = CriticalFilter(environment, self.settings.watcher.critical_events_only)
        self._namespaces = NamespaceFilter(self.settings.watcher.namespaces)

    # ------------------------------------------------------------------ config
    def _load_environment_config(self) -> Dict[str, Any]:
        return cfg.load_layered_config(self.environment, self.config_dir)

    def _load_config_file(self, config_file: str) -> Dict[str, Any]:
        return cfg.load_config_file(config_file)

    def _merge_configs(self, base: Dict[str, Any], override: Dict[str, Any]) -> Dict[str, Any]:
        return cfg.deep_merge(base, override)

    def _substitute_env_vars(self, config: Dict[str, Any]) -> Dict[str, Any]:
        return cfg.substitute_env(config)

    def _setup_logging(self) -> None:
        w = self.settings.watcher
        self.logger = setup_logging(self.environment, w.log_level, log_file=w.log_file)
        self.logger.info(f"Starting k8s-watcher in {self.environment} environment")

    def _setup_clusterapi_client(self) -> ClusterApiClient:
        c = self.settings.clusterapi
        self.logger.info(f"Setting up ClusterAPI client: {c.base_url}")
        self.logger.debug("API key provided for authentication" if c.api_key else "No API key provided")
        return ClusterApiClient.from_settings(c)

    # ------------------------------------------------------------------ client
    def setup_k8s_client(self) -> bool:
        k = self.settings.kubernetes
        try:
            if k.use_incluster_config:
                self.logger.info("Using in-cluster configuration")
                k8s_config.load_incluster_config()
            elif k.config_file:
                self.logger.info(f"Loading kubeconfig from: {k.config_file}")
                if not os.path.exists(k.config_file):
                    self.logger.error(f"Kubeconfig file not found: {k.config_file}")
                    return False
                k8s_config.load_kube_config(config_file=k.config_file, context=k.context)
            else:
                self.logger.info("Using default kubeconfig")
                k8s_config.load_kube_config(context=k.context)
            self.v1 = k8s_client.CoreV1Api()
            version = k8s_client.VersionApi().get_code().git_version
            self.logger.info(f"Successfully connected to Kubernetes API version: {version}")
            namespaces = self.v1.list_namespace(limit=5)
            self.logger.info(f"Sample namespaces: {[ns.metadata.name for ns in namespaces.items[:5]]}")
            return True
        except ConfigException as exc:
            self.logger.error(f"Kubernetes config error: {exc}")
            return False
        except Exception as exc:  # noqa: BLE001 - parity with pod_watcher.py:155-157
            self.logger.error(f"Error setting up k8s client: {exc}")
            return False

    # ------------------------------------------------------------------ per event
    def _extract_pod_data(self, pod: Any) -> Dict[str, Any]:
        return build_payload_dict(raw_of(pod), self.environment, self.settings.watcher.state_format,
                                  extra=self.settings.watcher.payload_extra,
                                  ts_mode=self.settings.watcher.event_timestamp)

    def should_process_event(self, event_type: str, pod: Any) -> bool:
        raw = raw_of(pod)
        st = raw.get("status")
        return self._critical(event_type, st is not None, (st or {}).get("phase"))

    def handle_pod_event(self, event_type: str, pod: Any) -> Optional[Dict[str, Any]]:
        raw = raw_of(pod)
        md = raw.get("metadata") or {}
        ns, name = md.get("namespace"), md.get("name")
        if not self.should_process_event(event_type, pod):
            return None
        self.logger.info(f"Pod event detected: {event_type} - {ns}/{name}")
        if not self._namespaces(ns):
            self.logger.debug(f"Skipping pod {ns}/{name} - not in target namespaces")
            return None
        data = self._extract_pod_data(pod)
        data["event_type"] = event_type
        if self.clusterapi_client is not None:
            if self.clusterapi_client.update_pod_status(data):
                self.logger.info(f"Successfully notified clusterapi about {event_type} event for {ns}/{name}")
            else:
                self.logger.error(f"Failed to notify clusterapi about {event_type} event for {ns}/{name}")
        return data

    # ------------------------------------------------------------------ run
    def _customised(self) -> bool:
        """True when a subclass overrides a per-event hook of the reference API."""
        cls = type(self)
        return any(getattr(cls, m) is not getattr(PodWatcher, m)
                   for m in ("handle_pod_event", "should_process_event", "_extract_pod_data"))

    def start_watching(self) -> None:
        """Run until SIGINT/SIGTERM or a fatal watch error.

        The stock class runs the asynchronous engine (:class:`WatcherService`).
        A subclass that overrides ``handle_pod_event``, ``should_process_event``
        or ``_extract_pod_data`` gets the reference's own loop instead
        (``pod_watcher.py:243-277``): every watch event is handed to
        ``self.handle_pod_event(type, pod)``, so the overrides run exactly as
        they did on the reference.
        """
        if self._customised():
            self._start_watching_per_event()
            return
        from k8s_watcher_amd.engine.service import SetupError, WatcherService

        async def run() -> None:
            svc = WatcherService(self.settings)
            if self.settings.watcher.leader_election.enabled:  # one active replica of several
                from k8s_watcher_amd.engine.leader import LeaderElectedService
                svc = LeaderElectedService(self.settings)
            loop = asyncio.get_running_loop()
            for sig in (signal.SIGINT, signal.SIGTERM):
                try:
                    loop.add_signal_handler(sig, svc.stop)
                except (NotImplementedError, RuntimeError):
                    pass
            await svc.run()

        try:
            asyncio.run(run())
        except SetupError:
            raise
        except KeyboardInterrupt:
            logging.getLogger("watcher.pod_watcher").info("Stopping Pod watcher...")

    def _start_watching_per_event(self) -> None:
        """The reference's synchronous loop over the compat ``Watch`` (``pod_watcher.py:243-277``),
        with its fixes: setup failure raises (exit 1) and the notifier is attached when enabled."""
        from k8s_watcher_amd.engine.service import SetupError
        if not self.setup_k8s_client():
            self.logger.error("Failed to setup Kubernetes client")
            raise SetupError("Failed to setup Kubernetes client")
        if self.settings.clusterapi.enabled and self.clusterapi_client is None:
            self.clusterapi_client = self._setup_clusterapi_client()
        self.logger.info(f"Starting Pod watcher in {self.environment} environment...")
        if self.settings.watcher.namespaces:
            self.logger.info(f"Monitoring namespaces: {self.settings.watcher.namespaces}")
        else:
            self.logger.info("Monitoring all namespaces")
        try:
            for event in self.watch.stream(self.v1.list_pod_for_all_namespaces):
                self.handle_pod_event(event["type"], event["object"])
        except KeyboardInterrupt:
            self.logger.info("Stopping Pod watcher...")
        except Exception as exc:
            self.logger.error(f"Error in Pod watcher: {exc}")
            raise
        finally:
            self.watch.stop()
