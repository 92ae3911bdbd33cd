"""watcher.fd_table_reserve: the descriptor table grown once, up front (utils/fds.py)."""

import os
import subprocess
import sys

from conftest import ROOT


def test_reserve_grows_the_table_once_and_keeps_low_fds():
    code = (
        "from k8s_watcher_amd.utils.fds import fd_table_size, reserve_fd_table\n"
        "import os, resource\n"
        "before = fd_table_size()\n"
        "got = reserve_fd_table(4096)\n"
        "fd = os.open(os.devnull, os.O_RDONLY)\n"
        "print(before, got, fd_table_size(), fd, resource.getrlimit(resource.RLIMIT_NOFILE)[0])\n"
    )
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert out.returncode == 0, out.stderr
    before, got, after, fd, soft = (int(x) for x in out.stdout.split())
    assert before < 4096 <= got == after  # one growth, kept
    assert fd < 64  # new descriptors still take the lowest free number
    assert soft >= 4096 or soft == got


def test_reserve_is_bounded_by_the_hard_limit_and_zero_is_off():
    from k8s_watcher_amd.utils.fds import fd_table_size, reserve_fd_table
    assert reserve_fd_table(0) == 0
    code = (
        "import resource\n"
        "resource.setrlimit(resource.RLIMIT_NOFILE, (256, 512))\n"
        "from k8s_watcher_amd.utils.fds import reserve_fd_table\n"
        "print(reserve_fd_table(100000), resource.getrlimit(resource.RLIMIT_NOFILE)[0])\n"
    )
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert out.returncode == 0, out.stderr
    size, soft = (int(x) for x in out.stdout.split())
    assert soft == 512 and 512 <= size <= 1024
    assert fd_table_size() is None or fd_table_size() > 0
