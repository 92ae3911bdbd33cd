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
from typing import List, Optional

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


def local_processes() -> int:
    """Watcher processes sharing this host's CPU allowance: the shard launcher
    (parallel/launch.py) sets K8S_WATCHER_LOCAL_PROCS, torchrun LOCAL_WORLD_SIZE."""
    for key in ("K8S_WATCHER_LOCAL_PROCS", "LOCAL_WORLD_SIZE"):
        try:
            n = int(os.environ.get(key, "") or 0)
        except ValueError:
            n = 0
        if n > 0:
            return n
    return 1


OWN_CPUS_ENV = "K8S_WATCHER_OWN_CPUS"


def mark_own_cpus() -> None:
    """Declare this process's affinity mask its own: whoever set it (the
    benchmark's per-rank L3 placement, a launcher pinning each shard) gave
    the other local shards disjoint masks. Threads and children started
    later see it through the environment."""
    os.environ[OWN_CPUS_ENV] = "1"


def process_cpu_share(root: str = "") -> int:
    """CPUs this process may count on when ``local_processes()`` watchers run
    on the host: that many-th of its affinity mask — a cpuset container
    (``--cpuset-cpus``, a Kubernetes static CPU policy) gives every shard in it
    the same mask — unless the mask was declared this shard's own
    (:func:`mark_own_cpus`: each shard pinned to its own L3 domain); and that
    many-th of a cgroup quota, which they all share."""
    procs = local_processes()
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    own = os.environ.get(OWN_CPUS_ENV, "") not in ("", "0")
    share = aff if own else aff // procs
    limit = cgroup_cpu_limit(root)
    if limit is not None:
        share = min(share, math.floor(limit / procs))
    return max(1, share)


def auto_decode_threads(cpus: Optional[int] = None) -> int:
    """Decode workers (which also take the partitioned apply's partitions):
    leave a CPU each for the event-loop thread, the reader thread and the
    notifier's I/O thread, use at most 6. With the apply phase partitioned
    over them (watcher.partitioned_apply) the serial stage no longer caps the
    gain: six workers ran the cluster watch at 2.94-2.99M events/s on the
    MI355X host's 16-CPU share (profiles/r4/io_thread); round 3's four had
    cut the loop's wait for decode by ~40% (profiles/hub_framing_gpu_box.md).

    Without an explicit count, the CPUs are this process's share of the
    allowance when several shards run on the host: four ranks under one
    16-CPU quota asked for ~25 CPUs with 4 workers each and were throttled in
    123 of 134 scheduler periods (profiles/hub_framing_gpu_box.md)."""
    cpus = process_cpu_share() if cpus is None else cpus
    return max(0, min(6, cpus - 3))


def auto_tls_threads(cpus: Optional[int] = None) -> int:
    """Record-opening threads of an https watch besides the reader thread
    (watcher.watch_tls_threads: auto): AES-GCM opens ~3-5 GB/s per core and
    the cluster watch carries 12-16 GB/s over plain TCP, so up to 3 helpers
    where this process's share leaves room for them next to the decode
    workers, none on a small share (the reader opens alone)."""
    cpus = process_cpu_share() if cpus is None else cpus
    return max(0, min(3, (cpus - 6) // 2))


def auto_reader_threads(multi: bool, cpus: Optional[int] = None) -> int:
    """Reader-hub threads (net/reader.py): one for a single cluster-wide
    watch (one TCP stream is one thread's recv at most); with several watch
    streams (namespace scopes) two where this process's share has room for
    them beside the loop and the decode workers. With the read-ahead kept
    small (engine/service.py HUB_MULTI_READ_AHEAD), 64 namespace watches ran
    3.05-3.13M with two against 2.59-2.94M with one (profiles/r6/readers/final)."""
    cpus = process_cpu_share() if cpus is None else cpus
    return 2 if multi and cpus >= 12 else 1


def auto_decode_spin_us(cpus: Optional[int] = None) -> float:
    """Idle spin of the decode workers before they sleep: 20 us when this
    process has CPUs to spare (a share of 8 or more), else 0. Workers still
    hot when the next batch starts took the cluster-watch headline from
    2.17-2.23M to 2.34M ev/s for ~0.35 CPU (profiles/decode_spin_r3_gpu_box.md);
    under a tight shared quota that CPU is worth more to the other shards
    (profiles/decode_spin_sink_gpu_box.md, round 2)."""
    cpus = process_cpu_share() if cpus is None else cpus
    return 20.0 if cpus >= 8 else 0.0


def _parse_cpu_list(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def current_cpu() -> Optional[int]:
    """CPU the calling thread last ran on (field 39 of /proc/thread-self/stat)."""
    try:
        with open("/proc/thread-self/stat") as fh:
            stat = fh.read()
        return int(stat[stat.rindex(")") + 2:].split()[36])
    except (OSError, ValueError, IndexError):
        return None


def l3_domain_cpus(cpu: Optional[int] = None, root: str = "") -> Optional[set]:
    """Allowed CPUs sharing the last-level cache with ``cpu`` (default: the
    CPU this thread runs on). On chiplet CPUs (one L3 per CCD) keeping the
    event-loop thread and its decode workers inside one L3 keeps the watch
    bytes and decoded spans from crossing the fabric twice per event."""
    if cpu is None:
        cpu = current_cpu()
        if cpu is None:
            return None
    try:
        with open(f"{root}/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list") as fh:
            dom = _parse_cpu_list(fh.read())
    except (OSError, ValueError):
        return None
    try:
        dom &= os.sched_getaffinity(0)
    except (AttributeError, OSError):
        pass
    return dom or None


def l3_domains(root: str = "") -> List[frozenset]:
    """The allowed CPUs grouped by shared L3, ordered by lowest CPU number."""
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        return []
    doms = set()
    todo = set(allowed)
    while todo:
        cpu = min(todo)
        try:
            with open(f"{root}/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list") as fh:
                dom = frozenset(_parse_cpu_list(fh.read()) & allowed) or frozenset([cpu])
        except (OSError, ValueError):
            dom = frozenset([cpu])
        doms.add(dom)
        todo -= dom | {cpu}
    return sorted(doms, key=min)


def pin_to_l3_domain(min_cpus: int = 1, only_if_split: bool = False, index: Optional[int] = None) -> Optional[set]:
    """Restrict the calling thread (and threads it starts later, which inherit
    the mask) to one L3 domain; returns the CPU set or None.

    ``index``: that domain of :func:`l3_domains` (modulo their number) instead
    of the one the thread runs on — a launcher gives each watcher process its
    own chiplet this way. ``min_cpus``: leave the mask alone if the domain has
    fewer usable CPUs. ``only_if_split``: only pin when the allowed CPUs span
    several L3 domains (on a single-L3 machine pinning buys nothing)."""
    if index is not None and index >= 0:
        doms = l3_domains()
        dom = set(doms[index % len(doms)]) if doms else None
    else:
        dom = l3_domains_current()
    if not dom or len(dom) < min_cpus:
        return None
    if only_if_split:
        try:
            if dom >= os.sched_getaffinity(0):
                return None
        except (AttributeError, OSError):
            return None
    try:
        os.sched_setaffinity(0, dom)
    except OSError:
        return None
    return dom


def l3_domains_current() -> Optional[set]:
    return l3_domain_cpus()


def _cpu_times() -> dict:
    """cpu -> (idle+iowait jiffies, total jiffies) from /proc/stat."""
    out = {}
    with open("/proc/stat") as fh:
        for line in fh:
            if not line.startswith("cpu") or line.startswith("cpu "):
                continue
            f = line.split()
            vals = [int(x) for x in f[1:]]
            out[int(f[0][3:])] = (vals[3] + (vals[4] if len(vals) > 4 else 0), sum(vals[:8]))
    return out


def l3_domains_by_idle(sample_s: float = 0.25) -> List[frozenset]:
    """:func:`l3_domains`, most idle first (idle CPU time summed over a short
    sample). On a shared host a fixed choice can land on a chiplet that other
    tenants or interrupt handling keep busy."""
    import time
    doms = l3_domains()
    try:
        a = _cpu_times()
        time.sleep(sample_s)
        b = _cpu_times()
    except (OSError, ValueError):
        return doms

    def idle(dom) -> float:
        tot = 0.0
        for c in dom:
            if c in a and c in b:
                di, dt = b[c][0] - a[c][0], b[c][1] - a[c][1]
                tot += di / dt if dt > 0 else 1.0
        return tot

    return sorted(doms, key=lambda d: (-idle(d), min(d)))


def package_of(cpu: int, root: str = "") -> int:
    try:
        with open(f"{root}/sys/devices/system/cpu/cpu{cpu}/topology/physical_package_id") as fh:
            return int(fh.read().strip())
    except (OSError, ValueError):
        return 0


def assign_domains(wanted: List[int], doms: List[frozenset]) -> List[int]:
    """Give every process (in rank order) its wanted L3 domain index unless a
    lower rank already holds it; then the first free domain on the same
    socket (memory stays NUMA-local), else any free one, else share."""
    taken: set = set()
    out = []
    for w in wanted:
        choice = w
        if w in taken:
            pkg = package_of(min(doms[w])) if 0 <= w < len(doms) else 0
            free = [i for i in range(len(doms)) if i not in taken]
            same = [i for i in free if package_of(min(doms[i])) == pkg]
            choice = (same or free or [w])[0]
        taken.add(choice)
        out.append(choice)
    return out


def core_siblings(cpu: int, root: str = "") -> set:
    """The hardware threads of ``cpu``'s physical core (itself without SMT)."""
    try:
        with open(f"{root}/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list") as fh:
            return _parse_cpu_list(fh.read()) or {cpu}
    except (OSError, ValueError):
        return {cpu}


def reader_core_split(rest: set, min_cores: int = 4, root: str = "") -> Optional[tuple]:
    """``(reader_cpus, worker_cpus)``: the lowest physical core of ``rest``
    (what :func:`loop_core_split` left) for the reader hub's thread, the rest
    for the decode workers. With the watch body's kernel copy on the reader
    thread, one TCP stream of ~10 GB/s keeps it ~0.9 busy at the N=1 rate
    (profiles/r4): an SMT sibling busy decoding slowed it down. None when
    fewer than ``min_cores`` physical cores would be left to the workers."""
    if not rest:
        return None
    cores, seen = [], set()
    for c in sorted(rest):
        if c in seen:
            continue
        sib = core_siblings(c, root) & rest
        seen |= sib | {c}
        cores.append(sib or {c})
    if len(cores) - 1 < min_cores:
        return None
    return set(cores[0]), set(rest) - cores[0]


def loop_core_split(cpus: set, min_cores: int = 4, root: str = "") -> Optional[tuple]:
    """``(loop_cpus, other_cpus)`` for ``watcher.thread_pinning``: the lowest
    physical core of ``cpus`` (both hardware threads) for the event-loop
    thread, the rest for the decode workers, the reader thread — and, in the
    benchmark, the fixtures. The loop thread applies every event in stream
    order and bounds the rate; sharing its core with a busy SMT sibling cost
    up to a third of its speed on the MI355X host (profiles/thread_pinning_gpu_box.md).
    None when ``cpus`` lies in several L3 domains or has fewer than
    ``min_cores`` physical cores (nothing to gain, or too little to spare)."""
    if not cpus:
        return None
    first = min(cpus)
    try:
        with open(f"{root}/sys/devices/system/cpu/cpu{first}/cache/index3/shared_cpu_list") as fh:
            if not cpus <= _parse_cpu_list(fh.read()):
                return None
    except (OSError, ValueError):
        return None
    cores, seen = [], set()
    for c in sorted(cpus):
        if c in seen:
            continue
        sib = core_siblings(c, root) & cpus
        seen |= sib | {c}
        cores.append(sib or {c})
    if len(cores) < min_cores:
        return None
    loop = cores[0]
    return set(loop), set(cpus) - loop
