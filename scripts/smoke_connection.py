#!/usr/bin/env python3
"""Manual connectivity check — the reference's test_k8s_connection.py.

    python scripts/smoke_connection.py [./assets/config]

Checks ``/version``, a one-item namespace list and a one-item pod list; exits
non-zero on the first hard failure.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_watcher_amd.compat.kubernetes import client, config  # noqa: E402


def main(kubeconfig: str = "./assets/config") -> int:
    if not os.path.exists(kubeconfig):
        print(f"FAIL kubeconfig not found: {kubeconfig}")
        return 1
    config.load_kube_config(config_file=kubeconfig)
    v1 = client.CoreV1Api()
    print("CoreV1Api methods:", ", ".join(m for m in dir(v1) if not m.startswith("_")))
    try:
        print(f"OK server version: {client.VersionApi().get_code().git_version}")
    except client.ApiException as exc:
        print(f"WARN version failed: {exc}")
    for what, call in (("namespace", lambda: v1.list_namespace(limit=1)),
                       ("pod", lambda: v1.list_pod_for_all_namespaces(limit=1))):
        try:
            print(f"OK {what} list: {len(call().items)} item(s)")
        except client.ApiException as exc:
            print(f"FAIL {what} list: {exc}")
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:2]))
