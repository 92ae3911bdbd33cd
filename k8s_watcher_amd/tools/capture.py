"""Record a cluster's pod list + watch stream to a file, for offline replay.

Debugging a watcher against production traffic should not need production:
``capture`` writes the current pods and then every watch event, with their
arrival times, as JSON lines; ``python -m k8s_watcher_amd.testing.fake_apiserver
--replay <file>`` serves them again (at the recorded pace, faster, or as fast as
possible) so the watcher — or a new version of it — can be run against the same
input. The reference has no equivalent (its only test path is an external mock,
SURVEY §4).

Format, one JSON object per line::

    {"t": 0.0,   "type": "LIST",     "object": {...pod...}}    # state at start
    {"t": 1.234, "type": "MODIFIED", "object": {...pod...}}    # watch events, t = seconds since start

``BOOKMARK`` and ``ERROR`` events are not recorded (a replay makes its own); bookmarks
only advance the resume point, an ``ERROR`` (e.g. 410) ends the capture.

    python -m k8s_watcher_amd.tools.capture production --out pods.ndjson --seconds 600
    python -m k8s_watcher_amd.tools.capture --kubeconfig ~/.kube/config --namespace default --max-events 10000
"""

from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time
from typing import List, Optional

from ..kube.api import KubeApi, split_list_body
from ..kube.kubeconfig import load_incluster_config, load_kube_config


async def capture(api: KubeApi, out, namespace: Optional[str] = None, seconds: float = 0.0,
                  max_events: int = 0, page: int = 500, stop: Optional[asyncio.Event] = None) -> int:
    """Write LIST then watch events to ``out`` (a text file); returns the number of watch events."""
    t0 = time.monotonic()
    cont, rv = None, None
    while True:
        md, items = split_list_body(await api.list_pods_raw(namespace=namespace, limit=page, continue_token=cont))
        rv = rv or md.get("resourceVersion")
        for it in items:
            out.write(json.dumps({"t": 0.0, "type": "LIST", "object": it}, separators=(",", ":")) + "\n")
        cont = md.get("continue")
        if not cont:
            break
    n = 0
    buf = bytearray()
    done = asyncio.Event()
    expired: List[str] = []

    def sink(data, _read_ns: int) -> None:
        nonlocal n, rv
        buf.extend(data)
        cut = buf.rfind(b"\n")
        if cut < 0:
            return
        lines = bytes(buf[:cut]).split(b"\n")
        del buf[:cut + 1]
        now = round(time.monotonic() - t0, 6)
        for line in lines:
            if not line.strip() or done.is_set():
                continue
            ev = json.loads(line)
            obj = ev.get("object") or {}
            etype = ev.get("type")
            if etype == "ERROR":
                expired.append(str(obj.get("message") or obj))
                done.set()
                continue
            rv = (obj.get("metadata") or {}).get("resourceVersion") or rv
            if etype not in ("ADDED", "MODIFIED", "DELETED"):
                continue
            out.write(json.dumps({"t": now, "type": etype, "object": obj}, separators=(",", ":")) + "\n")
            n += 1
            if max_events and n >= max_events:
                done.set()

    deadline = t0 + seconds if seconds else None
    waiters = [asyncio.ensure_future(done.wait())]
    if stop is not None:
        waiters.append(asyncio.ensure_future(stop.wait()))
    try:
        # until --seconds, --max-events, a stop request or an ERROR event; a
        # watch the server ends (its request timeout) resumes from the last
        # resourceVersion, so a long capture is not cut short
        while not any(w.done() for w in waiters):
            left = None if deadline is None else deadline - time.monotonic()
            if left is not None and left <= 0:
                break
            buf.clear()
            opened = time.monotonic()
            stream = await api.watch_pods(sink, namespace=namespace, resource_version=rv, allow_bookmarks=True)
            try:
                await asyncio.wait([stream.finished] + waiters, timeout=left,
                                   return_when=asyncio.FIRST_COMPLETED)
            finally:
                stream.close()
            if time.monotonic() - opened < 1.0 and not any(w.done() for w in waiters):
                await asyncio.wait(waiters, timeout=1.0)  # pace a server that hangs up at once
    finally:
        for w in waiters:
            w.cancel()
    if expired:
        print(f"watch ended with an ERROR event: {expired[0]}", file=sys.stderr)
    out.flush()
    return n


def load_capture(path: str) -> List[dict]:
    with open(path) as fh:
        return [json.loads(line) for line in fh if line.strip()]


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="record pods + watch events for offline replay")
    ap.add_argument("environment", nargs="?", default=None,
                    help="take the cluster connection from this profile's config (else --kubeconfig)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--context", default=None)
    ap.add_argument("--in-cluster", action="store_true")
    ap.add_argument("--namespace", default=None, help="one namespace (default: all)")
    ap.add_argument("--out", default="capture.ndjson")
    ap.add_argument("--seconds", type=float, default=60.0, help="0 = until --max-events or Ctrl-C")
    ap.add_argument("--max-events", type=int, default=0)
    a = ap.parse_args(argv)
    if a.environment:
        from ..utils.config import load_settings
        k = load_settings(a.environment).kubernetes
        ep = load_incluster_config() if k.use_incluster_config else load_kube_config(
            config_file=k.config_file, context=k.context)
    elif a.in_cluster:
        ep = load_incluster_config()
    else:
        ep = load_kube_config(config_file=a.kubeconfig, context=a.context)

    async def run() -> int:
        api = KubeApi(ep)
        try:
            with open(a.out, "w") as fh:
                return await capture(api, fh, a.namespace, a.seconds, a.max_events)
        finally:
            await api.close()

    try:
        n = asyncio.run(run())
    except KeyboardInterrupt:
        n = -1
    print(f"captured to {a.out}" + (f": {n} watch events" if n >= 0 else ""), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
