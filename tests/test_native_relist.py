"""Native LIST reconcile (``_kwcore.Relist``, ``ops/csrc/relist.inc``) against
the Python ``EventPipeline.reconcile``: same notifications, same cache, same
counters, for every filter combination, a cluster-wide and a namespace scope,
any page split and any slice budget. Plus the per-namespace index of the
native cache (``drop_namespaces``, ``count_namespace``) and a relist driven
end to end by the reflector against the fake API server (410 → relist)."""

import copy
import json
import time

import pytest

from conftest import run
from k8s_watcher_amd.engine.pipeline import EventPipeline
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.ops.decode import PyDecoder
from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.testing.podgen import PodFactory, event_line
from k8s_watcher_amd.utils.config import load_settings

NAMESPACES = ["default", "kube-system", "production", "batch"]


class Recorder:
    def __init__(self):
        self.calls = []

    def submit(self, uid, et, ns, name, core, read_ns, ts):
        self.calls.append((uid, et, ns, name, json.loads(core)))

    def flush(self):
        pass


def with_rv(pod, rv):
    pod = copy.deepcopy(pod)
    pod["metadata"]["resourceVersion"] = str(rv)
    return pod


def scenario(seed=5, n=240):
    """(watch lines that build the cache, LIST items of the later state)."""
    f = PodFactory(seed, NAMESPACES)
    pods = [f.running(f.scheduled(f.new_pod())) for _ in range(n)]
    rv = 1000
    lines, listed = [], []
    for i, p in enumerate(pods[: n * 2 // 3]):
        rv += 1
        lines.append(event_line("ADDED", with_rv(p, rv)))
    lines.append(event_line("ADDED", {"metadata": {"name": "bare", "namespace": "default", "uid": "u-bare",
                                                   "resourceVersion": "5"}}))  # cached without a core
    for i, p in enumerate(pods):
        k = i % 6
        if i >= n * 2 // 3:
            listed.append(with_rv(p, 5000 + i))                       # new: ADDED
        elif k == 0:
            continue                                                  # gone: DELETED from the cache
        elif k == 1:
            listed.append(with_rv(f.terminated(p, failed=i % 4 == 1), 7000 + i))  # MODIFIED (terminal)
        elif k == 2:
            listed.append(with_rv(p, 1001 + i))                       # unchanged rv (no event)
        else:
            listed.append(with_rv(f.terminated(p), 8000 + i))
    listed.append({"metadata": {"name": "nouid", "namespace": "batch", "resourceVersion": "9"}})
    return b"".join(lines), listed


def list_pages(items, page, rv="99999"):
    out = []
    for i in range(0, max(1, len(items)), page):
        chunk = items[i:i + page]
        last = i + page >= len(items)
        md = {"resourceVersion": rv}
        if not last:
            md["continue"] = f"tok{i + page}"
        out.append(json.dumps({"kind": "PodList", "apiVersion": "v1", "metadata": md, "items": chunk},
                              separators=(",", ":"), ensure_ascii=False).encode())
    return out


def make(env, ov, native):
    s = load_settings(env, overrides=ov, environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder(env), rec, m)
    p.log_events_setting = False
    if native:
        p.attach_native()
    return p, rec, m


def python_relist(p, items, scope, notify=True):
    _, _, evs = PyDecoder(p.settings.environment).decode_list(list_pages(items, 10**6)[0])
    return p.reconcile(evs, 0, notify=notify, scope_ns=scope)


def native_relist(p, items, scope, page=37, budget_us=50.0, notify=True):
    rl = p.native.relist(scope, notify)
    ctrl = []
    for body in list_pages(items, page):
        rl.page(body)
        done = False
        while not done:
            done, c = p.native_slice(rl.step, budget_us, 0)
            ctrl += c
        rv, cont = rl.page_meta()
        assert rv == "99999"
    done = False
    while not done:
        done, c = p.native_slice(rl.sweep, budget_us, 0)
        ctrl += c
    return ctrl, rl.stats()


def norm_cache(cache):
    return {u: [e[0], e[1], e[2], e[3], json.loads(e[4]) if e[4] else None] for u, e in cache.items()}


def strip_ts(calls):
    return sorted(((u or "", et, ns or "", nm or "", json.dumps(core, sort_keys=True)) for u, et, ns, nm, core in calls))


PROFILES = [
    ("staging", {}),
    ("production", {}),
    ("development", {}),
    ("development", {"watcher": {"notify_on": "phase_change"}}),
    ("staging", {"watcher": {"shard": {"count": 3, "index": 1}}}),
    ("staging", {"watcher": {"shard": {"count": 2, "index": 0, "key": "uid"}}}),
]
COUNTERS = ("events_received", "events_filtered_critical", "events_filtered_namespace", "events_unchanged",
            "events_other_shard")


@pytest.mark.parametrize("env,ov", PROFILES)
@pytest.mark.parametrize("scope", [None, "default"])
def test_native_relist_matches_python(env, ov, scope):
    lines, items = scenario()
    if scope is not None:
        items = [it for it in items if it["metadata"].get("namespace") == scope]
    a, ra, ma = make(env, ov, native=False)
    b, rb, mb = make(env, ov, native=True)
    a.handle_batch(PyDecoder(env).feed(lines), 0)
    b.handle_raw(lines, 0, framed=False)
    assert norm_cache(a.cache) == norm_cache(b.cache)
    ra.calls.clear()
    rb.calls.clear()
    c0a = {k: ma.c[k] for k in COUNTERS}
    c0b = {k: mb.c[k] for k in COUNTERS}
    ctrl_a = python_relist(a, items, scope)
    ctrl_b, st = native_relist(b, items, scope)
    assert ctrl_a == [] and ctrl_b == []
    assert strip_ts(ra.calls) == strip_ts(rb.calls)
    assert len(rb.calls) > 0 or env == "production"
    assert norm_cache(a.cache) == norm_cache(b.cache)
    assert {k: ma.c[k] - c0a[k] for k in COUNTERS} == {k: mb.c[k] - c0b[k] for k in COUNTERS}
    assert st["listed"] == len(items)
    assert st["added"] + st["modified"] + st["unchanged"] == st["listed"]
    assert st["steps"] > 2  # the small budget really sliced it
    assert st["unchanged"] > 0 or scope is not None


def test_native_relist_silent_primes_cache():
    lines, items = scenario(seed=9)
    a, ra, _ = make("staging", {}, native=False)
    b, rb, _ = make("staging", {}, native=True)
    a.handle_batch(PyDecoder("staging").feed(lines), 0)
    b.handle_raw(lines, 0, framed=False)
    ra.calls.clear()
    rb.calls.clear()
    python_relist(a, items, None, notify=False)
    native_relist(b, items, None, notify=False)
    assert ra.calls == rb.calls == []
    ca, cb = norm_cache(a.cache), norm_cache(b.cache)
    assert set(ca) == set(cb)
    assert {u: e[:4] for u, e in ca.items()} == {u: e[:4] for u, e in cb.items()}


def test_native_relist_restart_forgets_earlier_pages():
    lines, items = scenario(seed=3)
    b, rb, _ = make("staging", {}, native=True)
    b.handle_raw(lines, 0, framed=False)
    rl = b.native.relist(None, True)
    rl.page(list_pages(items, 50)[0])
    done = False
    while not done:
        done, _ = b.native_slice(rl.step, 1e6, 0)
    rl.restart()  # continue token expired: the LIST starts over unpaginated
    rl.page(list_pages(items, 10**6)[0])
    while not b.native_slice(rl.step, 1e6, 0)[0]:
        pass
    while not b.native_slice(rl.sweep, 1e6, 0)[0]:
        pass
    listed = {it["metadata"].get("uid") for it in items}
    assert set(u for u, _ in b.cache.items()) == {u if u else None for u in listed}


def test_native_relist_invalid_item_and_body():
    b, rb, m = make("staging", {}, native=True)
    rl = b.native.relist(None, True)
    good = {"metadata": {"name": "a", "namespace": "default", "uid": "ua", "resourceVersion": "1"}}
    body = (b'{"kind":"PodList","metadata":{"resourceVersion":"7"},"items":[' + json.dumps(good).encode()
            + b',{"metadata":{"name":1 2}},5,"s"]}')
    rl.page(body)
    done, ctrl = b.native_slice(rl.step, 1e6, 0)
    assert done and [c[0] for c in ctrl] == ["INVALID"]
    assert [c[0] for c in rb.calls] == ["ua"]
    rl2 = b.native.relist(None, True)
    rl2.page(b'{"kind":"PodList","items":[{"metadata":{}}')
    with pytest.raises(ValueError, match="invalid list body"):
        b.native_slice(rl2.step, 1e6, 0)


def test_native_cache_namespace_index():
    kw = load()
    c = kw.PodCache(None)
    for i in range(300):
        ns = NAMESPACES[i % 4]
        c.put(f"u{i}", str(i), "Running", ns, f"p{i}")
    c.put("u-none", "1", None, None, "x")
    assert c.count_namespace("default") == 75 and c.count_namespace(None) == 1
    assert c.count_namespace("nope") == 0
    assert c.namespaces() == {"default": 75, "kube-system": 75, "production": 75, "batch": 75, None: 1}
    c.put("u0", "9", "Running", "batch", "moved")  # a re-put moves the entry between namespace lists
    assert c.count_namespace("default") == 74 and c.count_namespace("batch") == 76
    assert c.drop_namespaces(["default", "nope"]) == 74
    assert c.count_namespace("default") == 0 and len(c) == 227
    c.observe("DELETED", "u1", None, None, None, None)
    assert c.count_namespace("kube-system") == 74
    assert c.drop_namespaces_except(["batch"]) == 74 + 75 + 1
    assert set(c.namespaces()) == {"batch"} and len(c) == 76
    assert c.pop("u0")[3] == "moved" and c.count_namespace("batch") == 75
    c.clear()
    assert c.namespaces() == {} and c.count_namespace("batch") == 0


def test_python_cache_drop_namespaces():
    from k8s_watcher_amd.ops.cache import PodCache
    c = PodCache()
    for i in range(40):
        c.put(f"u{i}", "1", "Running", NAMESPACES[i % 4], f"p{i}")
    assert c.drop_namespaces({"default"}) == 10 and c.count_namespace("default") == 0
    assert c.drop_namespaces_except({"batch"}) == 20
    assert c.namespaces() == {"batch": 10}


def test_native_relist_scope_leaves_other_namespaces():
    lines, items = scenario(seed=21)
    b, rb, _ = make("staging", {}, native=True)
    b.handle_raw(lines, 0, framed=False)
    before = b.cache.namespaces()
    rb.calls.clear()
    ctrl = b.delete_scope("production", 0)
    assert ctrl == []
    after = b.cache.namespaces()
    assert "production" not in after
    assert {k: v for k, v in before.items() if k != "production"} == after
    assert len(rb.calls) == before["production"] and all(c[1] == "DELETED" for c in rb.calls)


def test_reflector_relist_after_410_is_native():
    """A 410 mid-watch: the reflector relists through the native Relist, the
    pods changed while the watch was down arrive once, unchanged ones not at all."""
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
    from k8s_watcher_amd.testing.stub_sink import StubSink

    async def body():
        srv = FakeApiServer()
        await srv.start()
        sink = StubSink()
        await sink.start()
        f = PodFactory(17, ["default"])
        pods = [srv.create(f.running(f.new_pod())) for _ in range(30)]
        s = load_settings("staging", overrides={"clusterapi": {"base_url": sink.url},
                                                "watcher": {"engine": "native", "list_page_size": 7}},
                          environ={})
        svc = WatcherService(s, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
        await svc.start()
        await sink.state.wait_for(30, timeout=20)
        r = svc.reflectors[0]
        assert r.last_relist is not None and r.last_relist["added"] == 30
        # while the watch is expired: change 5, delete 5, add 5
        srv.expire_watches()
        srv.compact()
        for p in pods[:5]:
            srv.update(f.terminated(p))
        for p in pods[5:10]:
            srv.delete(p["metadata"]["namespace"], p["metadata"]["name"])
        for _ in range(5):
            srv.create(f.running(f.new_pod()))
        srv.compact()
        await sink.state.wait_for(45, timeout=20)
        await svc.notifier.drain(5)
        got = sink.state.payloads()[30:]
        st = r.last_relist
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
        return got, st, svc.metrics.c

    got, st, c = run(body())
    kinds = sorted(p["event_type"] for p in got)
    assert kinds == ["ADDED"] * 5 + ["DELETED"] * 5 + ["MODIFIED"] * 5, kinds
    assert st["unchanged"] == 20 and st["deleted"] == 5 and st["pages"] >= 4
    assert c["relist_deleted"] >= 5 and c["relists"] >= 2
