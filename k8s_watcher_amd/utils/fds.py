"""File-descriptor table sizing (``watcher.fd_table_reserve``).

Linux grows a process's descriptor table by doubling it when a new fd does
not fit (``expand_fdtable``). When the table is shared by several threads —
this process runs a decode pool, a reader thread and the notifier's I/O
thread — each growth waits for an RCU grace period before it frees the old
table, and the thread that opened the descriptor blocks meanwhile. On the
MI355X host (256 CPUs) a grace period took 130-220 ms: a 1,000-namespace start,
which opens two descriptors per watch (the socket and the reader hub's dup),
held the event loop that long five times, once per doubling from 128 to 4,096
(``benchmarks/relist_storm.py`` ``slow_turns``: the loop thread blocked in
``socket()`` with ~0.2 ms of CPU over each stall).

:func:`reserve_fd_table` grows the table once, up front, to the size the
service will need: a duplicate at a high descriptor number (``F_DUPFD``),
closed again at once. The table keeps its size (it never shrinks), so later sockets fit
without a growth. Done while the process still has one thread, the growth does
not wait for a grace period at all. The soft ``RLIMIT_NOFILE`` is raised to the
reservation (within the hard limit) first, as a watch per namespace needs it.
"""

from __future__ import annotations

import fcntl
import os
import resource
from typing import Optional


def fd_table_size() -> Optional[int]:
    """The descriptor table's current size (``FDSize`` in /proc/self/status)."""
    try:
        with open("/proc/self/status") as fh:
            for line in fh:
                if line.startswith("FDSize:"):
                    return int(line.split()[1])
    except (OSError, ValueError):
        pass
    return None


def reserve_fd_table(n: int) -> int:
    """Make descriptors below ``n`` fit the table without a growth; returns the
    table size reached (0 when nothing was done)."""
    if n <= 0:
        return 0
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = n if hard == resource.RLIM_INFINITY else min(n, hard)
    if soft != resource.RLIM_INFINITY and soft < want:
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
            soft = want
        except (ValueError, OSError):
            pass
    top = min(want, soft if soft != resource.RLIM_INFINITY else want) - 1
    size = fd_table_size()
    if top < 3 or (size is not None and size > top):
        return size or 0
    fd = os.open(os.devnull, os.O_RDONLY | os.O_CLOEXEC)
    try:
        # F_DUPFD: the lowest free descriptor >= top (never one another thread
        # holds, as dup2 onto a fixed number could be); the table grows to fit it
        try:
            high = fcntl.fcntl(fd, fcntl.F_DUPFD_CLOEXEC, top)
        except OSError:  # EMFILE / EINVAL: at the limit already
            return fd_table_size() or 0
        os.close(high)
    finally:
        os.close(fd)
    return fd_table_size() or 0
