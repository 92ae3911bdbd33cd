"""A TLS 1.3 front for a plain-HTTP fixture: the https API server of the soak.

    python -m k8s_watcher_amd.testing.tls_front --backend 127.0.0.1:PORT \\
        --cert server.crt --key server.key [--key-update-mib 64] [--ticket-every-mib 0]

``testing/replay_server.py`` speaks plain HTTP; production reads its watch
over TLS from kube-apiserver (``/root/reference/config/production.yaml:6``,
``watcher/pod_watcher.py:115-118``). This front terminates TLS for it, one
thread per connection, with the fixture's native TLS server
(``_kwcore.TlsServerContext``, ``ops/csrc/tls13.inc``): it reads the client's
requests through OpenSSL and forwards them, and seals the backend's response
bytes itself — so it can do what a long-lived Go ``crypto/tls`` server
connection does over hours and a Python ``ssl`` peer cannot be made to do:

* a **KeyUpdate** every ``--key-update-mib`` MiB sent on a connection
  (Go's ``crypto/tls`` rotates an AES-GCM key after 2^24-ish records; the
  soak compresses that), which the watcher's record layer must follow;
* a **NewSessionTicket** every ``--ticket-every-mib`` MiB (skipped by the
  watcher), optionally cut over two records.

The backend's connection ending is passed on as it happened: an orderly close
(the replay fixture's 410 / server timeout) as close_notify + FIN, an abort
(its ``drop``: a reset) as a reset of the client connection.

Control on stdin, replies on stdout: ``READY <port>`` once listening;
``STATS`` -> ``STATS {json}`` (connections, bytes, key updates, tickets);
``QUIT``.
"""

from __future__ import annotations

import argparse
import json
import os
import select
import socket
import sys
import threading
from typing import Dict, Optional, Tuple


class TlsFront:
    def __init__(self, backend: Tuple[str, int], cert: str, key: str, key_update_mib: float = 0.0,
                 ticket_every_mib: float = 0.0, threads: int = 2, port: int = 0) -> None:
        from k8s_watcher_amd.ops.native import load
        self.backend = backend
        self.tls = load().TlsServerContext(cert, key, threads=threads)
        self.key_update_bytes = int(key_update_mib * (1 << 20))
        self.ticket_bytes = int(ticket_every_mib * (1 << 20))
        self.srv = socket.socket()
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind(("127.0.0.1", port))
        self.srv.listen(128)
        self.port = self.srv.getsockname()[1]
        self.lock = threading.Lock()
        self.stats: Dict[str, int] = {"connections": 0, "open": 0, "bytes_up": 0, "bytes_down": 0,
                                      "key_updates": 0, "tickets": 0, "aborts": 0, "closes": 0, "errors": 0}
        self._stop = False

    def _count(self, **kw: int) -> None:
        with self.lock:
            for k, v in kw.items():
                self.stats[k] += v

    def serve_forever(self) -> None:
        while not self._stop:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._conn, args=(c,), daemon=True).start()

    def close(self) -> None:
        self._stop = True
        try:
            self.srv.close()
        except OSError:
            pass

    def _ticket(self) -> bytes:
        body = (3600).to_bytes(4, "big") + os.urandom(4) + b"\x08" + os.urandom(8) + (96).to_bytes(2, "big") \
            + os.urandom(96) + b"\x00\x00"
        return b"\x04" + len(body).to_bytes(3, "big") + body

    def _conn(self, c: socket.socket) -> None:
        self._count(connections=1, open=1)
        conn = None
        be: Optional[socket.socket] = None
        how = "close"
        try:
            conn = self.tls.accept(c.detach())
            be = socket.create_connection(self.backend)
            be.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            fd = conn.fileno()
            since_key = since_ticket = 0
            tickets_sent = 0
            while True:
                r, _, _ = select.select([fd, be], [], [], 5.0)
                if fd in r:  # the client's requests (OpenSSL reads them)
                    d = conn.recv(1 << 16)
                    if d == b"":
                        how = "client"
                        break
                    if d:
                        be.sendall(d)
                        self._count(bytes_up=len(d))
                if be in r:  # the backend's response bytes, sealed here
                    try:
                        d = be.recv(1 << 20)
                    except ConnectionResetError:
                        how = "abort"
                        break
                    if not d:
                        how = "close"
                        break
                    conn.send(d)
                    since_key += len(d)
                    since_ticket += len(d)
                    self._count(bytes_down=len(d))
                    if self.ticket_bytes and since_ticket >= self.ticket_bytes:
                        t = self._ticket()  # every other one cut over two records
                        conn.send_record(22, t, split=len(t) // 2 if tickets_sent % 2 else 0)
                        tickets_sent += 1
                        since_ticket = 0
                        self._count(tickets=1)
                    if self.key_update_bytes and since_key >= self.key_update_bytes:
                        conn.key_update(split=2 if self.stats["key_updates"] % 2 else 0)
                        since_key = 0
                        self._count(key_updates=1)
        except (OSError, ValueError):
            how = "error"
        finally:
            if be is not None:
                be.close()
            if conn is not None:
                try:
                    if how == "abort":  # the backend reset its side: so does the front
                        conn.abort()
                        self._count(aborts=1)
                    else:
                        conn.close()  # close_notify, then FIN
                except OSError:
                    pass
                if how == "close":
                    self._count(closes=1)
                elif how == "error":
                    self._count(errors=1)
            self._count(open=-1)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--backend", required=True, help="host:port of the plain-HTTP fixture")
    ap.add_argument("--cert", required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--key-update-mib", type=float, default=64.0, help="KeyUpdate every N MiB per connection (0: none)")
    ap.add_argument("--ticket-every-mib", type=float, default=0.0, help="NewSessionTicket every N MiB (0: none)")
    ap.add_argument("--threads", type=int, default=2, help="sealing threads (large sends)")
    a = ap.parse_args(argv)
    host, port = a.backend.rsplit(":", 1)
    front = TlsFront((host, int(port)), a.cert, a.key, a.key_update_mib, a.ticket_every_mib, a.threads, a.port)
    threading.Thread(target=front.serve_forever, daemon=True).start()
    print(f"READY {front.port}", flush=True)
    for line in sys.stdin:
        cmd = line.strip().upper()
        if cmd == "QUIT":
            break
        if cmd == "STATS":
            with front.lock:
                print("STATS " + json.dumps(front.stats), flush=True)
    front.close()


if __name__ == "__main__":
    main()
