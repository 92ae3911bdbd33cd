#!/usr/bin/env python3
"""Manual smoke check against a (fake) API server — the reference's test_k8s_mock.py.

    python -m k8s_watcher_amd.testing.fake_apiserver --port 9988 --pods 5 &
    python scripts/smoke_mock.py [./assets/config]

Lists pods (limit=5) and namespaces, then watches for up to 5 events / 5 s.
Unlike the reference script it exits non-zero when a check fails.
"""

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_watcher_amd.compat.kubernetes import client, config, watch  # noqa: E402


def main(kubeconfig: str = "./assets/config") -> int:
    if not os.path.exists(kubeconfig):
        print(f"FAIL kubeconfig not found: {kubeconfig}")
        return 1
    config.load_kube_config(config_file=kubeconfig)
    contexts, active = config.list_kube_config_contexts(config_file=kubeconfig)
    print(f"context {active['name'] if active else '-'} -> cluster {active['context'].get('cluster') if active else '-'}")
    v1 = client.CoreV1Api()
    try:
        pods = v1.list_pod_for_all_namespaces(limit=5)
    except client.ApiException as exc:
        print(f"FAIL pod list: {exc}")
        return 1
    print(f"OK pod list: {len(pods.items)} pod(s)")
    for i, pod in enumerate(pods.items, 1):
        print(f"   {i}: {pod.metadata.namespace}/{pod.metadata.name} - {pod.status.phase if pod.status else '?'}")
    try:
        nss = v1.list_namespace()
        print(f"OK namespace list: {[n.metadata.name for n in nss.items]}")
    except client.ApiException as exc:
        print(f"WARN namespace list failed: {exc}")
    w = watch.Watch()
    start, n = time.time(), 0
    for ev in w.stream(v1.list_pod_for_all_namespaces, timeout_seconds=5):
        n += 1
        print(f"   watch event {n}: {ev['type']} - {ev['object'].metadata.name}")
        if time.time() - start > 5 or n >= 5:
            break
    w.stop()
    print(f"OK watch: {n} event(s)")
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:2]))
