"""``from watcher.clusterapi_client import ClusterApiClient`` — see
:mod:`k8s_watcher_amd.notify.clusterapi` (reference: ``watcher/clusterapi_client.py``)."""

from k8s_watcher_amd.notify.clusterapi import AsyncClusterApiClient, ClusterApiClient  # noqa: F401

__all__ = ["ClusterApiClient", "AsyncClusterApiClient"]
