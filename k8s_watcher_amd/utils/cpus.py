"""How many CPUs this process may actually use.

``os.cpu_count()`` reports the host; a container is limited by its CPU
affinity mask and by its cgroup CPU quota (``resources.limits.cpu`` in the
Deployment, ``deploy/k8s/deployment.yaml``). Thread pools that spin — the
native decode pool keeps its workers hot for ~60 µs between reads — must be
sized from the smaller of the two, or a 1-CPU pod would burn its quota
spinning.
"""

from __future__ import annotations

import math
import os
from typing import Optional

_CGROUP_FILES = ("/sys/fs/cgroup/cpu.max",                      # cgroup v2
                 "/sys/fs/cgroup/cpu/cpu.cfs_quota_us")         # cgroup v1


def cgroup_cpu_limit(root: str = "") -> Optional[float]:
    """CPU quota in CPUs, or None when unlimited / not visible."""
    v2 = root + _CGROUP_FILES[0]
    try:
        with open(v2) as fh:
            quota, period = (fh.read().split() + ["100000"])[:2]
        if quota != "max":
            return int(quota) / int(period)
        return None
    except (OSError, ValueError):
        pass
    try:
        with open(root + _CGROUP_FILES[1]) as fh:
            quota = int(fh.read().strip())
        with open(root + "/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            period = int(fh.read().strip())
        return quota / period if quota > 0 and period > 0 else None
    except (OSError, ValueError):
        return None


def available_cpus(root: str = "") -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    limit = cgroup_cpu_limit(root)
    if limit is not None:
        n = min(n, max(1, math.floor(limit)))
    return max(1, n)


def auto_decode_threads(cpus: Optional[int] = None) -> int:
    """Extra decode workers for one watch stream: leave a CPU for the event
    loop thread and one for the notifier side, use at most 3 (the serial
    apply phase caps the gain beyond ~4-way decode)."""
    cpus = available_cpus() if cpus is None else cpus
    return max(0, min(3, cpus - 2))
