"""Compatibility package: the reference's import paths (``watcher.pod_watcher``,
``watcher.clusterapi_client``) backed by :mod:`k8s_watcher_amd`."""
