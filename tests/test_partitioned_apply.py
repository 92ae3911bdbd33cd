"""The partitioned apply (ops/csrc/engine.inc, pl_apply_partitioned): a
batch's apply phase split by pod-cache shard over the decode pool's threads
and the loop thread must leave exactly what the serial apply leaves — the same
notifications (exactly once, per pod in stream order), the same cache, the
same counters, control events and resume point — for every filter profile,
with the lines only the serial path takes (undecodable lines, ERROR events,
bookmarks, escaped uids, namespaces and phases never seen before, pods
without a uid) mixed in. VERDICT round 3, next-round item 3."""

import collections
import copy
import json
import random

import pytest

from conftest import run
from k8s_watcher_amd.engine.pipeline import EventPipeline
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.ops.decode import PyDecoder
from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.parallel.native_notifier import NativeNotifierPool
from k8s_watcher_amd.testing.podgen import churn_events, event_line
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import load_settings

NAMESPACES = ["default", "kube-system", "batch", "production", "monitoring"]


def stream(n_pods=600, seed=41) -> bytes:
    lines = [event_line(t, o) for t, o in churn_events(n_pods, seed=seed, namespaces=NAMESPACES)]
    rng = random.Random(seed)
    extra = [
        b"this is not json\n",
        b'{"type":"BOOKMARK","object":{"kind":"Pod","metadata":{"resourceVersion":"424242"}}}\n',
        b'{"type":"ERROR","object":{"kind":"Status","code":500,"message":"boom"}}\n',
        b'{"type":"ADDED","object":{"metadata":{"name":"nouid","namespace":"default"},"status":{"phase":"Failed"}}}\n',
        b'{"type":"DELETED","object":{"metadata":{"name":"nouid","namespace":"default"}}}\n',
    ]
    for x in extra:
        lines.insert(rng.randrange(len(lines)), x)
    # a pod whose uid is written with an escape, and a namespace / phase first seen mid-stream
    late = json.loads(lines[len(lines) // 2].decode())
    for i, (et, ph) in enumerate([("ADDED", "Pending"), ("MODIFIED", "Weird"), ("DELETED", "Weird")]):
        o = copy.deepcopy(late["object"])
        o["metadata"].update(uid="esc\\u0041-uid", namespace="late-ns", name="late-pod", resourceVersion=str(900 + i))
        o.setdefault("status", {})["phase"] = ph
        raw = json.dumps({"type": et, "object": o}).replace("esc\\\\u0041", "esc\\u0041").encode() + b"\n"
        lines.insert(len(lines) * (i + 2) // 5, raw)
    for i, et in enumerate(["ADDED", "MODIFIED", "DELETED"]):  # plain uid, new namespace + phase
        o = copy.deepcopy(late["object"])
        o["metadata"].update(uid=f"new-ns-uid", namespace="brand-new", name="np", resourceVersion=str(950 + i))
        o.setdefault("status", {})["phase"] = "Mystery" if i else "Pending"
        lines.insert(len(lines) * (i + 1) // 4, event_line(et, o))
    return b"".join(lines)


PROFILES = [
    ("staging", {}),
    ("production", {}),
    ("development", {"watcher": {"notify_on": "phase_change"}}),
    ("production", {"watcher": {"namespaces": []}}),
    ("staging", {"watcher": {"shard": {"count": 3, "index": 1}}}),
    ("staging", {"watcher": {"shard": {"count": 2, "index": 0, "key": "uid"}, "namespaces": ["batch"]}}),
    ("staging", {"watcher": {"state_format": "python_repr"}}),
]


def feed(env, ov, data, partitioned, piece=96 * 1024):
    async def body():
        sink = StubSink()
        await sink.start()
        s = load_settings(env, overrides=dict(ov, clusterapi={"base_url": sink.url, "health_check_on_start": False}),
                          environ={})
        m = Metrics()
        pool = NativeNotifierPool(s.clusterapi, m)
        p = EventPipeline(s, PyDecoder(env), pool, m)
        p.log_events_setting = False
        kw = load()
        dpool = kw.DecodePool(3)
        p.attach_native(dpool)
        prev = kw.set_partitioned_apply(partitioned)
        kw.probe(True)
        ctrl = []
        try:
            for i in range(0, len(data), piece):
                ctrl += [c[0] for c in p.handle_raw(data[i:i + piece], 1, framed=False)]
        finally:
            probe = kw.probe(False)
            kw.set_partitioned_apply(prev)
        assert await pool.drain(20)
        got = [(x["uid"], x["event_type"], x["status"]["phase"]) for x in sink.state.payloads()]
        cache = {u: [e[0], e[1], e[2], e[3], json.loads(e[4]) if e[4] else None] for u, e in p.cache.items()}
        counters = {k: v for k, v in m.c.items() if k.startswith(("events_", "bookmarks"))}
        rv = p.native.last_rv()
        parts = sum(w["parts"] for w in dpool.stats())
        await pool.close()
        await sink.stop()
        dpool.close()
        return got, cache, counters, rv, ctrl, probe, parts

    return run(body(), timeout=120)


def per_uid(got):
    out = collections.defaultdict(list)
    for u, et, ph in got:
        out[u].append((et, ph))
    return dict(out)


@pytest.mark.parametrize("env,ov", PROFILES)
def test_partitioned_apply_matches_serial(env, ov):
    data = stream()
    s_got, s_cache, s_cnt, s_rv, s_ctrl, s_probe, _ = feed(env, ov, data, partitioned=False)
    p_got, p_cache, p_cnt, p_rv, p_ctrl, p_probe, parts = feed(env, ov, data, partitioned=True)
    assert s_probe.get("partitioned_batches", 0) == 0
    assert p_probe["partitioned_batches"] > 0 and parts > 0  # the partitions ran, on the workers too
    assert collections.Counter(p_got) == collections.Counter(s_got)  # the same notifications, exactly once
    assert per_uid(p_got) == per_uid(s_got)                          # per pod in stream order
    assert p_cache == s_cache
    assert p_cnt == s_cnt
    assert p_rv == s_rv
    assert sorted(p_ctrl) == sorted(s_ctrl) and "ERROR" in s_ctrl and "INVALID" in s_ctrl


def test_partitioned_apply_under_many_small_and_large_batches():
    """Batch sizes around the threshold and whole-stream batches."""
    data = stream(n_pods=300, seed=7)
    base = feed("staging", {}, data, partitioned=False, piece=len(data))
    for piece in (9000, 40 * 1024, len(data)):
        got = feed("staging", {}, data, partitioned=True, piece=piece)
        assert per_uid(got[0]) == per_uid(base[0]) and got[1] == base[1] and got[2] == base[2], piece


def feed_group(data_by_ns, partitioned):
    """Several namespace pipelines sharing one pod cache and native notifier
    (the discover shape), bound to one reader hub: take_dispatch runs their
    reads as group batches, partitioned or not."""
    import os
    import socket
    import threading
    import time
    from test_reader_hub import _chunked, _dispatch_until

    async def body():
        sink = StubSink()
        await sink.start()
        s = load_settings("staging", overrides={"clusterapi": {"base_url": sink.url, "health_check_on_start": False},
                                                "watcher": {"namespace_scope": "discover"}}, environ={})
        m = Metrics()
        pool = NativeNotifierPool(s.clusterapi, m)
        kw = load()
        dpool = kw.DecodePool(3)
        core = kw.ReaderHub(256 * 1024, 32)
        first = None
        pipes, socks, sids = {}, [], {}
        for ns in data_by_ns:
            p = EventPipeline(s, PyDecoder("staging"), pool, m, cache=first.cache if first else None)
            first = first or p
            p.log_events_setting = False
            p.attach_native(dpool)
            p.sync_native_log()
            a, b = socket.socketpair()
            sid = core.add(os.dup(b.fileno()))
            core.bind(sid, p.native, True)
            pipes[ns], sids[sid] = p, ns
            socks += [a, b]
        prev = kw.set_partitioned_apply(partitioned)
        kw.probe(True)
        senders = [threading.Thread(target=socks[2 * i].sendall, args=(_chunked(d, piece=5000),), daemon=True)
                   for i, d in enumerate(data_by_ns.values())]
        for t in senders:
            t.start()
        time.sleep(0.2)
        done = []

        def on_item(it):
            sid, buf, view, read_ns, err = it
            p = pipes[sids[sid]]
            if buf == -2:
                p.native_result(view, read_ns)
                if err:
                    done.append(sid)
                return
            if view is not None:
                p.native_result(p.native.feed_chunked(view, read_ns), read_ns)
                if p.native.body_done():
                    done.append(sid)
                view.release()
                core.release(buf)

        try:
            _dispatch_until(core, lambda: len(done) == len(pipes), on_item, timeout=60)
        finally:
            probe = kw.probe(False)
            kw.set_partitioned_apply(prev)
        for t in senders:
            t.join()
        assert await pool.drain(20)
        got = [(x["uid"], x["event_type"], x["status"]["phase"]) for x in sink.state.payloads()]
        rvs = {ns: p.native.last_rv() for ns, p in pipes.items()}
        cache = {u: [e[0], e[1], e[2], e[3]] for u, e in first.cache.items()}
        for sid in sids:
            core.unbind(sid)
        core.close()
        for x in socks:
            x.close()
        await pool.close()
        await sink.stop()
        dpool.close()
        return got, rvs, cache, probe

    return run(body(), timeout=120)


def test_partitioned_group_batches_keep_each_namespace_resume_point():
    """Group batches of many namespace watches (one pipeline each, one shared
    cache): the partitioned apply leaves every pipeline the resume point, the
    notifications and the cache the serial apply does — the resume walk stops
    once every pipeline of the batch has its own resourceVersion."""
    lines = [event_line(t, o) for t, o in churn_events(400, seed=5, namespaces=NAMESPACES)]
    by_ns = {ns: [] for ns in NAMESPACES}
    for ln in lines:
        by_ns[json.loads(ln)["object"]["metadata"]["namespace"]].append(ln)
    data = {ns: b"".join(v) for ns, v in by_ns.items() if v}
    s_got, s_rvs, s_cache, _ = feed_group(data, partitioned=False)
    p_got, p_rvs, p_cache, p_probe = feed_group(data, partitioned=True)
    assert p_probe["partitioned_batches"] > 0
    assert p_rvs == s_rvs and all(s_rvs.values())
    assert collections.Counter(p_got) == collections.Counter(s_got)
    assert per_uid(p_got) == per_uid(s_got)
    assert p_cache == s_cache
