"""CPU budget and L3-domain helpers (utils/cpus.py) on fake sysfs trees."""

import os

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
    assert cpus.auto_decode_threads(2) == 0
    assert cpus.auto_decode_threads(4) == 2
    assert cpus.auto_decode_threads(64) == 3


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
