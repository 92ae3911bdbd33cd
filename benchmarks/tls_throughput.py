#!/usr/bin/env python3
"""TLS record-layer throughput, both ends native (ops/csrc/tls13.inc).

    python -m benchmarks.tls_throughput [--gb 4] [--server-threads 3] [--client-threads 3] [--records openssl]

A sender thread seals ``--gb`` of bytes in 4 MiB calls on a
``TlsServerContext`` (its pool + writer thread); the reader hub reads and
opens them (``ReaderHub.set_tls``) and the consumer only hands buffers back.
No JSON, no pipeline: what one https watch stream can carry on this host, and
where each side's time goes. Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from k8s_watcher_amd.ops.native import load  # noqa: E402
from k8s_watcher_amd.testing.certs import make_pki  # noqa: E402


def thread_cpu() -> dict:
    import psutil
    return {t.id: t.user_time + t.system_time for t in psutil.Process().threads()}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--server-threads", type=int, default=3)
    ap.add_argument("--client-threads", type=int, default=3)
    ap.add_argument("--records", default="native", choices=["native", "openssl"])
    ap.add_argument("--buf-mb", type=int, default=4)
    args = ap.parse_args(argv)
    mod = load()
    pki = make_pki(tempfile.mkdtemp(prefix="tls-tp-"))
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    chunk = os.urandom(4 << 20)
    total = int(args.gb * (1 << 30)) // len(chunk) * len(chunk)
    sent = {}

    def serve() -> None:
        tls = mod.TlsServerContext(pki.server_crt, pki.server_key, threads=args.server_threads)
        c, _ = srv.accept()
        conn = tls.accept(c.detach())
        req = b""
        while not req.endswith(b"\r\n\r\n"):
            d = conn.recv(65536)
            if d is None:
                time.sleep(0.0005)
                continue
            if not d:
                return
            req += d
        t0 = time.monotonic()
        for _ in range(total // len(chunk)):
            conn.send(chunk)
        conn.flush()
        sent["s"] = time.monotonic() - t0
        sent["pool"] = tls.pool_stats()
        conn.close()

    th = threading.Thread(target=serve, name="tls-sender")
    th.start()
    hub = mod.ReaderHub(args.buf_mb << 20, 8)
    hub.set_tls(args.records == "native", args.client_threads)
    ctx = mod.TlsContext(ca_pem=open(pki.ca_crt, "rb").read())
    c = socket.create_connection(("127.0.0.1", srv.getsockname()[1]))
    sid = hub.add_tls(c.detach(), ctx, "127.0.0.1", b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
    cpu0 = thread_cpu()
    got, end, t_first = 0, None, None
    t0 = time.monotonic()
    while end is None:
        for s, buf, view, _ns, err in hub.take():
            if view is None:
                end = err
                continue
            if t_first is None:
                t_first = time.monotonic()
            got += len(view)
            view.release()
            hub.release(buf)
        if end is None:
            time.sleep(0.0002)
    el = time.monotonic() - (t_first or t0)
    cpu1 = thread_cpu()
    th.join()
    st = hub.stats()
    busy = sorted((round((cpu1[k] - cpu0.get(k, 0)) / el, 2) for k in cpu1), reverse=True)
    print(json.dumps({
        "gb": round(got / (1 << 30), 3), "seconds": round(el, 3), "gb_per_s": round(got / el / 1e9, 2),
        "end": end, "records": args.records, "server_threads": args.server_threads,
        "client_threads": args.client_threads,
        "client": {"recv_frac": round(st["recv_ns"] / 1e9 / el, 3), "decrypt_frac": round(st["decrypt_ns"] / 1e9 / el, 3),
                   "pool_busy_frac": [round(a / 1e9 / el, 3) for a, _ in st["tls_pool"]]},
        "server_pool_busy_frac": [round(a / 1e9 / el, 3) for a, _ in sent.get("pool", [])],
        "threads_busy": busy[:12]}), flush=True)
    hub.close()


if __name__ == "__main__":
    main()
