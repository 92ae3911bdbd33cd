#!/usr/bin/env python3
"""The smallest possible watcher — the reference's deleted v0 prototype
``watcher/watcher.py`` (recovered from its .pyc), on the compat client.

    python examples/minimal_watch.py [kubeconfig]
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_watcher_amd.compat.kubernetes import client, config, watch  # noqa: E402


def start_watching(kubeconfig=None) -> None:
    config.load_kube_config(config_file=kubeconfig)
    v1 = client.CoreV1Api()
    w = watch.Watch()
    print("Starting to watch for Pod events...")
    try:
        for event in w.stream(v1.list_pod_for_all_namespaces):
            print(f"Event: {event['type']} Pod: {event['object'].metadata.name}")
    except Exception as exc:  # noqa: BLE001
        print(f"Error occurred: {exc}")
    finally:
        w.stop()


if __name__ == "__main__":
    start_watching(sys.argv[1] if len(sys.argv) > 1 else None)
