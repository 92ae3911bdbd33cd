"""TCP options for long-lived connections (watch streams, notifier pools).

The reference's transport (urllib3 under ``kubernetes``, ``requests`` for
clusterapi) sets no socket options, so a watch whose peer vanished without a
FIN/RST — API-server node lost, NAT or load-balancer entry expired — blocks
on ``recv`` until something above notices. client-go dials with
a 30 s TCP keep-alive for the same reason. Here every connection gets:

* ``SO_KEEPALIVE`` with ``TCP_KEEPIDLE``/``TCP_KEEPINTVL``/``TCP_KEEPCNT`` so
  a silent peer is detected in about ``idle + intvl * cnt`` seconds;
* ``TCP_USER_TIMEOUT`` so data that is never acknowledged fails the socket
  instead of retransmitting for ~15 minutes;
* ``TCP_NODELAY`` (requests and pipelined POSTs are written whole).

``keepalive_seconds <= 0`` leaves the kernel defaults (no keep-alive).
"""

from __future__ import annotations

import socket
from typing import Optional

DEFAULT_KEEPALIVE_SECONDS = 30.0


def tune_socket(sock: Optional[socket.socket], keepalive_seconds: float = DEFAULT_KEEPALIVE_SECONDS) -> bool:
    """Apply the options above to a connected or connecting TCP socket.

    Returns False (and changes nothing further) for non-TCP sockets, e.g. a
    Unix socket or a transport without a socket. Unsupported options on the
    running kernel are skipped silently.
    """
    if sock is None or sock.family not in (socket.AF_INET, socket.AF_INET6):
        return False
    _try(sock, socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    if keepalive_seconds and keepalive_seconds > 0:
        idle = max(1, int(keepalive_seconds))
        intvl = max(1, idle // 3)
        cnt = 3
        _try(sock, socket.SOL_SOCKET, socket.SO_KEEPALIVE, 1)
        _try(sock, socket.IPPROTO_TCP, getattr(socket, "TCP_KEEPIDLE", None), idle)
        _try(sock, socket.IPPROTO_TCP, getattr(socket, "TCP_KEEPINTVL", None), intvl)
        _try(sock, socket.IPPROTO_TCP, getattr(socket, "TCP_KEEPCNT", None), cnt)
        # unacknowledged data fails the connection after the same budget (milliseconds)
        _try(sock, socket.IPPROTO_TCP, getattr(socket, "TCP_USER_TIMEOUT", None),
             (idle + intvl * cnt) * 1000)
    return True


def _try(sock: socket.socket, level: int, opt: Optional[int], value: int) -> None:
    if opt is None:
        return
    try:
        sock.setsockopt(level, opt, value)
    except OSError:
        pass
