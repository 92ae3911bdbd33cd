"""``kubernetes.config`` subset: load a kubeconfig / in-cluster config as the default.

``load_kube_config(config_file=...)``, ``load_incluster_config()``,
``list_kube_config_contexts(config_file=...)`` and ``ConfigException`` — the
calls at ``/root/reference/watcher/pod_watcher.py:115-134`` and
``test_k8s_mock.py:17,27``.
"""

from __future__ import annotations

from typing import Optional

from ...kube import kubeconfig as _kc
from ...kube.kubeconfig import ConfigException  # noqa: F401  (re-export)
from .client import Configuration


def load_kube_config(config_file: Optional[str] = None, context: Optional[str] = None,
                     client_configuration: Optional[Configuration] = None,
                     persist_config: bool = True) -> None:
    ep = _kc.load_kube_config(config_file=config_file, context=context)
    if client_configuration is not None:
        client_configuration.endpoint = ep
    else:
        Configuration.set_default(Configuration(ep))


def load_incluster_config(client_configuration: Optional[Configuration] = None) -> None:
    ep = _kc.load_incluster_config()
    if client_configuration is not None:
        client_configuration.endpoint = ep
    else:
        Configuration.set_default(Configuration(ep))


def list_kube_config_contexts(config_file: Optional[str] = None):
    return _kc.list_kube_config_contexts(config_file)
