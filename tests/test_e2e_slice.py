"""BASELINE config #1 / SURVEY §7.2: fake API server → watcher → stub clusterapi.

Ten ADDED pods across namespaces; the development profile filters to
``[default, kube-system]`` and every surviving payload must reach the sink with
the §2.3 schema. With a one-connection notifier pool they arrive in exactly the
order the pods were created (the reference's single synchronous POST loop);
a wider pool keeps order per pod only (``crc32(uid)`` picks the connection),
so there the test checks identity, not global order.
"""

import pytest

from conftest import run
from k8s_watcher_amd.engine.service import WatcherService
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import load_settings

PAYLOAD_KEYS = ["name", "namespace", "uid", "environment", "status", "spec", "metadata",
                "event_timestamp", "event_type"]


def check_schema(p, environment):
    assert list(p.keys()) == PAYLOAD_KEYS
    assert p["environment"] == environment
    assert list(p["status"].keys()) == ["phase", "conditions", "container_statuses"]
    assert list(p["spec"].keys()) == ["node_name", "containers"]
    assert list(p["metadata"].keys()) == ["labels", "annotations", "creation_timestamp"]
    for c in p["status"]["conditions"]:
        assert list(c.keys()) == ["type", "status", "reason", "message"]
    for cs in p["status"]["container_statuses"]:
        assert list(cs.keys()) == ["name", "ready", "restart_count", "state"]
    for c in p["spec"]["containers"]:
        assert list(c.keys()) == ["name", "image"]
    assert p["event_type"] in ("ADDED", "MODIFIED", "DELETED")


async def start_stack(environment="development", overrides=None, engine="native", pods=None,
                      sink_kwargs=None, server_kwargs=None):
    srv = FakeApiServer(**(server_kwargs or {}))
    await srv.start()
    for p in pods or []:
        srv.create(p)
    sink = StubSink(**(sink_kwargs or {}))
    await sink.start()
    ov = {"clusterapi": {"base_url": sink.url, "retry": {"delay_seconds": 0.01}},
          "watcher": {"engine": engine, "retry": {"delay_seconds": 0.01, "max_attempts": 0}}}
    if overrides:
        from k8s_watcher_amd.utils.config import deep_merge
        ov = deep_merge(ov, overrides)
    settings = load_settings(environment, overrides=ov)
    svc = WatcherService(settings, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics(True))
    return srv, sink, svc


@pytest.mark.parametrize("connections", [1, None])
@pytest.mark.parametrize("engine", ["native", "python"])
def test_ten_added_pods_development(engine, connections):
    async def body():
        ov = {"clusterapi": {"pool": {"connections": connections}}} if connections else None
        srv, sink, svc = await start_stack(engine=engine, overrides=ov)
        await svc.start()
        f = PodFactory(seed=7, namespaces=["default", "kube-system", "production", "batch"])
        created = [srv.create(f.running(f.new_pod())) for _ in range(10)]
        expected = [p for p in created if p["metadata"]["namespace"] in ("default", "kube-system")]
        await sink.state.wait_for(len(expected), timeout=10)
        await svc.notifier.drain(5)
        got = sink.state.payloads()
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
        return expected, got, svc.metrics

    expected, got, metrics = run(body())
    assert len(got) == len(expected) == 5
    for p in got:
        check_schema(p, "development")
        assert p["event_type"] == "ADDED"
        assert p["status"]["phase"] == "Running"
        assert p["metadata"]["creation_timestamp"].endswith("+00:00")
    if connections == 1:
        # one connection, in-order HTTP/1.1: the creation order, exactly
        assert [p["uid"] for p in got] == [p["metadata"]["uid"] for p in expected]
    else:
        # identity: same uids as created, each exactly once (order is per pod only)
        assert sorted(p["uid"] for p in got) == sorted(p["metadata"]["uid"] for p in expected)
    assert metrics.c["events_filtered_namespace"] == 5
    assert metrics.c["notify_delivered"] == 5


def test_initial_list_replays_existing_pods_as_added():
    f = PodFactory(seed=1, namespaces=["default"])
    pods = [f.running(f.new_pod()) for _ in range(4)]

    async def body():
        srv, sink, svc = await start_stack(pods=pods)
        await svc.start()
        await sink.state.wait_for(4, timeout=10)
        got = sink.state.payloads()
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
        return got

    got = run(body())
    assert [p["event_type"] for p in got] == ["ADDED"] * 4
    assert {p["name"] for p in got} == {p["metadata"]["name"] for p in pods}


def test_lifecycle_order_per_pod():
    async def body():
        srv, sink, svc = await start_stack(environment="staging")
        await svc.start()
        f = PodFactory(seed=3)
        n_events = 0
        for _ in range(20):
            for et, obj in f.lifecycle():
                srv.apply(et, obj)
                n_events += 1
        await sink.state.wait_for(n_events, timeout=10)
        got = sink.state.payloads()
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
        return got, n_events

    got, n = run(body())
    assert len(got) == n == 100
    by_uid = {}
    for p in got:
        by_uid.setdefault(p["uid"], []).append(p["event_type"])
    for seq in by_uid.values():
        assert seq == ["ADDED", "MODIFIED", "MODIFIED", "MODIFIED", "DELETED"]


@pytest.mark.parametrize("freeze", [True, False])
def test_gc_freeze_after_sync_and_unfreeze_at_shutdown(freeze, monkeypatch):
    """service.GC_FREEZE: start-up's survivors are frozen once every scope has
    synced (full collections skip them), and unfrozen at shutdown so a retired
    service (a leader's last term) is collectable."""
    import gc

    async def body():
        from k8s_watcher_amd.engine import service
        monkeypatch.setattr(service, "GC_FREEZE", freeze)
        srv, sink, svc = await start_stack()
        base = gc.get_freeze_count()
        await svc.start()
        during = gc.get_freeze_count()
        svc.stop()
        await svc.shutdown()
        after = gc.get_freeze_count()
        await sink.stop()
        await srv.stop()
        return base, during, after

    base, during, after = run(body())
    assert base == 0 and after == 0
    assert (during > 0) == freeze


def test_gc_freeze_leaves_an_embedders_freeze_alone():
    """An application that froze its own objects before starting the service
    keeps them frozen: the service neither freezes on top (its shutdown would
    thaw everything) nor unfreezes at shutdown (round-4 advisor finding)."""
    import gc

    async def body():
        srv, sink, svc = await start_stack()
        gc.freeze()
        mine = gc.get_freeze_count()
        try:
            await svc.start()
            svc.stop()
            await svc.shutdown()
            return mine, gc.get_freeze_count()
        finally:
            gc.unfreeze()
            await sink.stop()
            await srv.stop()

    mine, after = run(body())
    # still frozen (a few frozen objects may have been freed by refcount meanwhile)
    assert mine > 0 and mine - 1000 < after <= mine


@pytest.mark.parametrize("scope,framing,want", [("client", "auto", False), ("discover", "auto", True),
                                                ("client", "on", True), ("discover", "off", False)])
def test_hub_framing_auto_follows_the_watch_shape(scope, framing, want, monkeypatch):
    """service.HUB_FRAMING: auto — the reader thread frames bodies when there
    are several watch scopes, and leaves the one cluster-wide watch's framing
    to the loop (that reader thread is the bound: profiles/r5/framing_ab)."""
    async def body():
        from k8s_watcher_amd.engine import service
        monkeypatch.setattr(service, "HUB_FRAMING", framing)
        srv, sink, svc = await start_stack(overrides={"watcher": {"namespace_scope": scope}})
        await svc.start()
        got = svc._reader_hub.frame
        # the read-ahead follows the shape too: 8 MiB over several scopes, the pool for one watch
        max_bytes = svc._reader_hub.core.stats()["max_bytes"]
        assert max_bytes == (service.HUB_MULTI_READ_AHEAD if scope == "discover"
                             else svc.settings.watcher.watch_reader_buffers * (svc.settings.watcher.watch_read_bytes
                                                                               or (4 << 20))), max_bytes
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
        return got

    assert run(body()) is want
