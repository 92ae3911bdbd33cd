"""WatchList initial sync (``watcher.initial_sync: watch_list``, engine/reflector.py).

Not in the reference, whose library LISTs implicitly; the
streamed form (``sendInitialEvents=true``) must give exactly the LIST result —
same notifications, same reconcile against the cache — and fall back to LIST
on API servers without it.
"""

import asyncio
import os

import pytest

from conftest import run
from k8s_watcher_amd.testing.podgen import PodFactory
from test_e2e_slice import check_schema, start_stack

WL = {"watcher": {"initial_sync": "watch_list"}}


@pytest.fixture(autouse=True)
def _short_idle(monkeypatch):
    """A server that never ends the initial events falls back after 0.5 s."""
    from k8s_watcher_amd.engine import reflector
    monkeypatch.setattr(reflector, "WATCH_LIST_IDLE_SECONDS", 0.5)


@pytest.mark.parametrize("engine", ["native", "python"])
def test_watch_list_initial_state_then_live(engine):
    async def body():
        f = PodFactory(seed=21, namespaces=["default", "kube-system", "batch"])
        pods = [f.running(f.new_pod()) for _ in range(12)]
        srv, sink, svc = await start_stack("development", overrides=WL, engine=engine, pods=pods)
        await svc.start()
        want = [p for p in pods if p["metadata"]["namespace"] in ("default", "kube-system")]
        await sink.state.wait_for(len(want), timeout=10)
        assert svc.metrics.c["watch_list_syncs"] == 1
        await asyncio.wait_for(svc.reflectors[0].connected.wait(), 5)
        watch_reqs = [t for _, t in srv.requests if "watch=true" in t]
        assert "sendInitialEvents=true" in watch_reqs[0] and "resourceVersionMatch=NotOlderThan" in watch_reqs[0]
        assert not any("watch" not in t and "/pods" in t for _, t in srv.requests)  # no LIST
        # after the initial-events-end bookmark the regular watch resumes from its RV
        assert "sendInitialEvents" not in watch_reqs[-1] and "resourceVersion=" in watch_reqs[-1]
        p = f.running(f.new_pod("default"))
        srv.create(p)
        await sink.state.wait_for(len(want) + 1, timeout=10)
        got = sink.state.payloads()
        for g in got:
            check_schema(g, "development")
        assert sorted(g["uid"] for g in got) == sorted([x["metadata"]["uid"] for x in want] + [p["metadata"]["uid"]])
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


@pytest.mark.parametrize("support", ["refused", "ignored"])
def test_watch_list_falls_back_to_list(support, monkeypatch):
    async def body():
        f = PodFactory(seed=22, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(4)]
        srv, sink, svc = await start_stack("staging", overrides=WL, pods=pods,
                                           server_kwargs={"watch_list": support != "refused"})
        if support == "ignored":
            # an API server that predates WatchList: the parameter is silently ignored
            orig = srv._watch

            async def no_watch_list(writer, ns, q):
                q = {k: v for k, v in q.items() if k not in ("sendInitialEvents", "resourceVersionMatch")}
                await orig(writer, ns, q)
            monkeypatch.setattr(srv, "_watch", no_watch_list)
        await svc.start()
        await sink.state.wait_for(4, timeout=10)
        await asyncio.sleep(0.2)
        assert svc.metrics.c["watch_list_syncs"] == 0 and svc.metrics.c["relists"] == 1
        assert svc.reflectors[0].watch_list is False
        uids = [g["uid"] for g in sink.state.payloads()]
        assert sorted(set(uids)) == sorted(p["metadata"]["uid"] for p in pods)
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


def test_watch_list_after_410_reconciles_like_relist():
    async def body():
        f = PodFactory(seed=23, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(5)]
        srv, sink, svc = await start_stack("staging", overrides=WL, pods=pods)
        await svc.start()
        await sink.state.wait_for(5, timeout=10)
        # while the watch is down: one pod deleted, one modified, one added, then history compacted
        srv.drop_connections()
        srv.delete("default", pods[0]["metadata"]["name"])
        changed = dict(pods[1])
        changed["status"] = dict(changed["status"], phase="Succeeded")
        srv.update(changed)
        added = f.running(f.new_pod("default"))
        srv.create(added)
        srv.compact()
        await sink.state.wait_for(8, timeout=10)
        await asyncio.sleep(0.3)
        tail = [(g["event_type"], g["uid"]) for g in sink.state.payloads()[5:]]
        assert sorted(tail) == sorted([("DELETED", pods[0]["metadata"]["uid"]),
                                       ("MODIFIED", pods[1]["metadata"]["uid"]),
                                       ("ADDED", added["metadata"]["uid"])])
        assert svc.metrics.c["watch_list_syncs"] == 2 and svc.metrics.c["expired_410"] >= 1
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


@pytest.mark.parametrize("compression", [True, False])
def test_gzip_list(compression):
    """LIST asks for gzip (``kubernetes.compression``); the fake API server, like the
    real one, compresses bodies over 128 KiB; the watcher decodes them transparently."""
    async def body():
        f = PodFactory(seed=24, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(150)]
        ov = {"kubernetes": {"compression": compression}, "watcher": {"list_page_size": 1000}}
        srv, sink, svc = await start_stack("staging", overrides=ov, pods=pods)
        await svc.start()
        await sink.state.wait_for(150, timeout=10)
        assert srv.gzipped_responses == (1 if compression else 0)
        assert sorted(g["uid"] for g in sink.state.payloads()) == sorted(p["metadata"]["uid"] for p in pods)
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


@pytest.mark.parametrize("status", [429, 401, 503])
def test_watch_list_transient_errors_keep_watch_list(status):
    """A throttled (429), unauthorised (401) or unavailable (503) WatchList
    request is retried as a WatchList — only "feature missing" answers
    (400/422...) downgrade the reflector to LIST for the rest of the process."""
    async def body():
        f = PodFactory(seed=25, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(3)]
        ov = {"watcher": {**WL["watcher"], "retry": {"delay_seconds": 0.05, "max_attempts": 0}}}
        srv, sink, svc = await start_stack("staging", overrides=ov, pods=pods)
        srv.fail_requests(1, status, path_prefix="/api/v1/pods", retry_after=0.1 if status == 429 else None)
        await svc.start()
        await sink.state.wait_for(3, timeout=10)
        assert svc.reflectors[0].watch_list is True
        assert svc.metrics.c["watch_list_syncs"] == 1 and svc.metrics.c["relists"] == 1
        assert not any("watch" not in t and "/pods" in t for _, t in srv.requests)  # never a LIST
        if status == 429:
            assert svc.metrics.c["api_throttled"] == 1
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


def test_native_watch_list_large_sync_is_sliced_and_exactly_once():
    """A 20k-pod WatchList sync on the native engine: applied read by read in
    relist_slice_ms slices (no Python object per pod, no whole-state
    reconcile), every pod notified once, and after a 410 the WatchList resync
    notifies only what changed."""
    import json as _json
    import subprocess
    import sys as _sys
    import tempfile

    from conftest import ROOT
    out = os.path.join(tempfile.mkdtemp(), "storm.json")
    res = subprocess.run([_sys.executable, os.path.join(ROOT, "benchmarks", "relist_storm.py"), "--scope", "cluster",
                          "--namespaces", "16", "--pods", "20000", "--churn", "300", "--slice-ms", "4",
                          "--initial-sync", "watch_list", "--json-out", out],
                         capture_output=True, text=True, timeout=400)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    d = _json.loads(open(out).read())
    assert d["initial"]["exactly_once"] and d["initial"]["notified"] == 20000
    assert d["storm"]["exactly_once"] and d["storm"]["expected"] == 900
    assert d["server"]["lists"] == 0
    # bounded slices: each step of the Relist is budgeted (4 ms here; a 20k-pod
    # reconcile of the Python path ran as one loop slice of ~0.5 s)
    assert d["initial"]["relist"]["max_slice_ms"] < 200 and d["storm"]["relist"]["max_slice_ms"] < 200


@pytest.mark.parametrize("engine", ["native", "python"])
def test_watch_list_skip_initial_deleted_is_silent(engine):
    """``initial_list: skip`` on a WatchList sync whose initial events carry a
    DELETED (a server interleaving a live deletion before the end bookmark):
    the cache forgets the pod, and nothing is sent — on the native path the
    DELETED goes through the watch path with the pipeline's silent flag, as
    the Relist's pages do (round-4 advisor finding)."""
    async def body():
        f = PodFactory(seed=26, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(4)]
        ov = {"watcher": {**WL["watcher"], "initial_list": "skip"}}
        srv, sink, svc = await start_stack("development", overrides=ov, engine=engine, pods=pods)
        gone = pods[1]
        srv.watch_list_inject = [{"type": "DELETED", "object": gone}]
        await svc.start()
        await asyncio.wait_for(svc.reflectors[0].connected.wait(), 5)
        await asyncio.sleep(0.3)
        assert svc.metrics.c["watch_list_syncs"] == 1
        assert sink.state.payloads() == []  # the primed state and the DELETED are both silent
        p = f.running(f.new_pod("default"))
        srv.create(p)
        await sink.state.wait_for(1, timeout=10)
        await asyncio.sleep(0.2)
        assert [(g["event_type"], g["uid"]) for g in sink.state.payloads()] == [("ADDED", p["metadata"]["uid"])]
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


@pytest.mark.parametrize("engine", ["native", "python"])
def test_watch_list_uid_twice_in_initial_events(engine):
    """A pod whose ADDED and a later MODIFIED both arrive in the initial
    events (one read): never two ADDEDs. The native collector closes its Relist
    page at the repeated uid, so the MODIFIED is compared with the ADDED
    (ADDED, then MODIFIED); the Python path keeps one entry per uid (ADDED of
    the final state)."""
    async def body():
        f = PodFactory(seed=27, namespaces=["default"])
        pods = [f.running(f.new_pod()) for _ in range(3)]
        srv, sink, svc = await start_stack("development", overrides=WL, engine=engine, pods=pods)
        later = dict(pods[0])
        later["metadata"] = dict(later["metadata"], resourceVersion=str(10 ** 6))
        later["status"] = dict(later["status"], phase="Succeeded")
        srv.watch_list_inject = [{"type": "MODIFIED", "object": later}]
        await svc.start()
        await sink.state.wait_for(3, timeout=10)
        await asyncio.sleep(0.3)
        uid = pods[0]["metadata"]["uid"]
        types = [g["event_type"] for g in sink.state.payloads() if g["uid"] == uid]
        assert types == (["ADDED", "MODIFIED"] if engine == "native" else ["ADDED"])
        assert sorted({g["uid"] for g in sink.state.payloads()}) == sorted(p["metadata"]["uid"] for p in pods)
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())
