"""Run N sharded watcher processes as one unit.

    python -m k8s_watcher_amd.parallel.launch --shards 4 production [main.py options]

Each child is ``main.py`` with ``K8S_WATCHER_SHARD_INDEX=i`` and
``K8S_WATCHER_SHARD_COUNT=N`` (see :mod:`.shard`). SIGINT/SIGTERM are
forwarded; when any child exits non-zero the others are stopped and that exit
code is returned, so an orchestrator (Kubernetes, systemd) restarts the set.
"""

from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def launch(shards: int, args: List[str], python: str = sys.executable) -> int:
    children: List[subprocess.Popen] = []
    for i in range(shards):
        env = dict(os.environ, K8S_WATCHER_SHARD_INDEX=str(i), K8S_WATCHER_SHARD_COUNT=str(shards),
                   K8S_WATCHER_LOCAL_PROCS=str(shards))  # they share this host's CPUs (utils/cpus.py)
        children.append(subprocess.Popen([python, os.path.join(ROOT, "main.py"), *args], env=env))

    stopping = False

    def forward(signum, _frame) -> None:
        nonlocal stopping
        stopping = True
        for c in children:
            if c.poll() is None:
                c.send_signal(signum)

    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    rc = 0
    try:
        while True:
            alive = [c for c in children if c.poll() is None]
            failed = [c for c in children if c.poll() not in (None, 0)]
            if failed and not stopping:
                rc = failed[0].returncode
                forward(signal.SIGTERM, None)
            if not alive:
                break
            time.sleep(0.1)
        if rc == 0:
            rc = next((c.returncode for c in children if c.returncode), 0)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--shards", type=int, required=True)
    ap.add_argument("rest", nargs=argparse.REMAINDER, help="arguments for main.py")
    a = ap.parse_args(argv)
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    if a.shards < 1:
        ap.error("--shards must be >= 1")
    return launch(a.shards, rest)


if __name__ == "__main__":
    sys.exit(main())
