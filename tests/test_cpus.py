"""CPU budget and L3-domain helpers (utils/cpus.py) on fake sysfs trees."""

import os

import pytest

from k8s_watcher_amd.utils import cpus


def write(root, rel, text):
    p = os.path.join(str(root), rel.lstrip("/"))
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as fh:
        fh.write(text)


def test_cgroup_limits(tmp_path):
    write(tmp_path, "/sys/fs/cgroup/cpu.max", "250000 100000\n")
    assert cpus.cgroup_cpu_limit(str(tmp_path)) == 2.5
    write(tmp_path, "/sys/fs/cgroup/cpu.max", "max 100000\n")
    assert cpus.cgroup_cpu_limit(str(tmp_path)) is None
    v1 = tmp_path / "v1"
    write(v1, "/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "150000")
    write(v1, "/sys/fs/cgroup/cpu/cpu.cfs_period_us", "100000")
    assert cpus.cgroup_cpu_limit(str(v1)) == 1.5
    assert cpus.cgroup_cpu_limit(str(tmp_path / "none")) is None


def test_auto_decode_threads():
    assert cpus.auto_decode_threads(1) == 0
    assert cpus.auto_decode_threads(3) == 0
    assert cpus.auto_decode_threads(4) == 1
    assert cpus.auto_decode_threads(8) == 5
    assert cpus.auto_decode_threads(16) == 6
    assert cpus.auto_decode_threads(64) == 6


def test_parse_cpu_list():
    assert cpus._parse_cpu_list("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}


def test_assign_domains_resolves_conflicts():
    doms = [frozenset({i}) for i in range(4)]
    assert cpus.assign_domains([2, 2, 0, 2], doms) == [2, 0, 1, 3]
    assert cpus.assign_domains([1], doms) == [1]
    # more ranks than domains: the surplus shares
    assert cpus.assign_domains([0, 0], doms[:1]) == [0, 0]


def test_current_domain_is_allowed():
    dom = cpus.l3_domain_cpus()
    if dom is not None:
        assert dom <= os.sched_getaffinity(0)
    assert all(d for d in cpus.l3_domains())


def test_loop_core_split(tmp_path):
    """8 cores x 2 threads in one L3 (CPUs n and n+8 are siblings): the loop
    thread gets core 0 (CPUs 0 and 8), everything else goes to the workers.
    Fewer than 4 cores, or CPUs from two L3 domains: no split."""
    from k8s_watcher_amd.utils.cpus import loop_core_split
    for c in range(16):
        write(tmp_path, f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", "0-15")
        write(tmp_path, f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list", f"{c % 8},{c % 8 + 8}")
    loop, rest = loop_core_split(set(range(16)), root=str(tmp_path))
    assert loop == {0, 8} and rest == set(range(1, 8)) | set(range(9, 16))
    assert loop_core_split({0, 1, 8, 9}, root=str(tmp_path)) is None  # 2 cores
    write(tmp_path, "/sys/devices/system/cpu/cpu16/cache/index3/shared_cpu_list", "16-31")
    assert loop_core_split(set(range(17)), root=str(tmp_path)) is None  # spans two L3 domains


def test_auto_decode_threads_per_local_process(monkeypatch):
    """Shards on one host split a shared CPU allowance (launcher / torchrun
    env): the cgroup quota always, the affinity mask only when it is the whole
    host (a shard pinned to its own L3 domain keeps those CPUs)."""
    monkeypatch.delenv("K8S_WATCHER_LOCAL_PROCS", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    monkeypatch.delenv(cpus.OWN_CPUS_ENV, raising=False)
    monkeypatch.setattr(cpus.os, "cpu_count", lambda: 256)
    # the 1-GPU box: pinned to a 16-CPU domain under a 16-CPU job quota
    monkeypatch.setattr(cpus.os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(cpus, "cgroup_cpu_limit", lambda root="": 16.0)
    assert cpus.auto_decode_threads() == 6
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert cpus.process_cpu_share() == 4 and cpus.auto_decode_threads() == 1
    # a whole node without a quota: a shard pinned to its own domain keeps it
    monkeypatch.setattr(cpus, "cgroup_cpu_limit", lambda root="": None)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv(cpus.OWN_CPUS_ENV, "1")
    assert cpus.process_cpu_share() == 16 and cpus.auto_decode_threads() == 6
    monkeypatch.delenv(cpus.OWN_CPUS_ENV)
    # ... an unpinned one shares the host's CPUs
    monkeypatch.setattr(cpus.os, "sched_getaffinity", lambda pid: set(range(256)))
    assert cpus.process_cpu_share() == 32
    monkeypatch.setenv("K8S_WATCHER_LOCAL_PROCS", "128")
    assert cpus.process_cpu_share() == 2 and cpus.auto_decode_threads() == 0


def test_auto_decode_spin_us(monkeypatch):
    monkeypatch.delenv("K8S_WATCHER_LOCAL_PROCS", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    monkeypatch.setattr(cpus.os, "cpu_count", lambda: 256)
    monkeypatch.setattr(cpus.os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(cpus, "cgroup_cpu_limit", lambda root="": 16.0)
    assert cpus.auto_decode_spin_us() == 20.0
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert cpus.auto_decode_spin_us() == 0.0
    assert cpus.auto_decode_spin_us(8) == 20.0


def test_cpuset_container_splits_the_mask_between_local_shards(monkeypatch):
    """A cpuset-limited container (mask smaller than the host, no CFS quota)
    running N shards: every shard sees the same mask, so each gets 1/N of it —
    not the whole mask (advisor round 3: 4 workers and a 20 us spin each)."""
    monkeypatch.delenv("K8S_WATCHER_LOCAL_PROCS", raising=False)
    monkeypatch.delenv(cpus.OWN_CPUS_ENV, raising=False)
    monkeypatch.setattr(cpus.os, "cpu_count", lambda: 256)
    monkeypatch.setattr(cpus.os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(cpus, "cgroup_cpu_limit", lambda root="": None)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert cpus.process_cpu_share() == 4
    assert cpus.auto_decode_threads() == 1 and cpus.auto_decode_spin_us() == 0.0
    monkeypatch.setenv(cpus.OWN_CPUS_ENV, "1")  # the launcher pinned each shard to its own 16
    assert cpus.process_cpu_share() == 16 and cpus.auto_decode_spin_us() == 20.0


@pytest.mark.parametrize("own", [False, True])
def test_eight_local_ranks_get_sane_shares(monkeypatch, own):
    """The driver's 8-GPU node runs bench.py with 8 local ranks. Whatever
    the node looks like, no rank may plan for more CPUs than its share, and
    the ranks together never plan more decode workers + loop threads than
    the CPUs they have."""
    monkeypatch.delenv("K8S_WATCHER_LOCAL_PROCS", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    if own:
        monkeypatch.setenv(cpus.OWN_CPUS_ENV, "1")
    else:
        monkeypatch.delenv(cpus.OWN_CPUS_ENV, raising=False)
    monkeypatch.setattr(cpus.os, "cpu_count", lambda: 256)
    shapes = [  # (mask, quota)
        (set(range(256)), None),    # whole node
        (set(range(128)), 128.0),   # half the node, quota to match
        (set(range(64)), 32.0),     # cpuset + tighter quota
        (set(range(16)), 16.0),     # the 1-GPU box's allowance
        (set(range(8)), None),      # a small cpuset
    ]
    for mask, quota in shapes:
        if own:  # placement: each rank pinned to a disjoint 1/8 of the mask
            mine = set(sorted(mask)[:max(1, len(mask) // 8)])
        else:
            mine = mask
        monkeypatch.setattr(cpus.os, "sched_getaffinity", lambda pid, m=mine: set(m))
        monkeypatch.setattr(cpus, "cgroup_cpu_limit", lambda root="", q=quota: q)
        share = cpus.process_cpu_share()
        total = quota if quota is not None else len(mask)
        assert 1 <= share <= max(1, total // 8), (mask, quota, share)
        workers = cpus.auto_decode_threads()
        assert 8 * (workers + 3) <= max(24, total), (mask, quota, workers)  # + loop, reader, notifier I/O
        # spinning only with CPUs to spare
        assert cpus.auto_decode_spin_us() == (20.0 if share >= 8 else 0.0)


def test_reader_core_split(tmp_path):
    """thread_pinning auto: after the loop's core, the reader thread gets the
    next physical core (both hardware threads), the decode workers the rest;
    no reader core when fewer than 4 cores would be left to the workers."""
    from k8s_watcher_amd.utils.cpus import loop_core_split, reader_core_split
    for c in range(16):
        write(tmp_path, f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list", "0-15")
        write(tmp_path, f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list", f"{c % 8},{c % 8 + 8}")
    _, rest = loop_core_split(set(range(16)), root=str(tmp_path))
    reader, workers = reader_core_split(rest, root=str(tmp_path))
    assert reader == {1, 9} and workers == set(range(2, 8)) | set(range(10, 16))
    assert reader_core_split({1, 2, 3, 4, 9, 10, 11, 12}, root=str(tmp_path)) is None  # 3 cores left


def test_auto_reader_threads():
    """Two reader threads for several watch scopes on a CPU share of 12+,
    one otherwise (a single watch stream is one thread's recv at most)."""
    assert cpus.auto_reader_threads(False, 64) == 1
    assert cpus.auto_reader_threads(True, 16) == 2
    assert cpus.auto_reader_threads(True, 12) == 2
    assert cpus.auto_reader_threads(True, 8) == 1
