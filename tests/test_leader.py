"""Lease-based leader election (engine/leader.py) against the fake API server.

The reference runs one replica and has no election; these tests
pin the protocol (compare-and-swap on the Lease, local-clock expiry, renew
deadline, release) and the service behaviour: of two replicas only the leader
notifies, and the standby takes over when the leader releases or dies.
"""

import asyncio

import pytest

from conftest import run
from k8s_watcher_amd.engine.leader import LeaderElectedService, LeaderElector, LeaderRecord, micro_time
from k8s_watcher_amd.kube.api import ApiError, KubeApi
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import ConfigError, LeaderElectionSettings, load_settings

FAST = dict(lease_duration_seconds=2, renew_deadline_seconds=1.5, retry_period_seconds=0.1)


class FakeClock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def le_settings(identity, **kw):
    return LeaderElectionSettings(enabled=True, identity=identity, lease_namespace="kube-system",
                                  **{**FAST, **kw})


def test_lease_crud_and_conflict():
    async def body():
        srv = FakeApiServer()
        await srv.start()
        api = KubeApi(KubeEndpoint(server=srv.url))
        try:
            assert await api.get_lease("ns", "l") is None
            created = await api.create_lease("ns", {"metadata": {"name": "l"}, "spec": {"holderIdentity": "a"}})
            rv = created["metadata"]["resourceVersion"]
            with pytest.raises(ApiError) as ei:
                await api.create_lease("ns", {"metadata": {"name": "l"}, "spec": {}})
            assert ei.value.status == 409
            got = await api.get_lease("ns", "l")
            assert got["spec"]["holderIdentity"] == "a"
            got["spec"]["holderIdentity"] = "b"
            upd = await api.replace_lease("ns", "l", got)
            assert upd["metadata"]["resourceVersion"] != rv
            stale = dict(got, metadata=dict(got["metadata"], resourceVersion=rv))
            with pytest.raises(ApiError) as ei:
                await api.replace_lease("ns", "l", stale)
            assert ei.value.status == 409
        finally:
            await api.close()
            await srv.stop()
    run(body())


def test_acquire_renew_and_expiry_on_local_clock():
    async def body():
        srv = FakeApiServer()
        await srv.start()
        api = KubeApi(KubeEndpoint(server=srv.url))
        ca, cb = FakeClock(), FakeClock()
        a = LeaderElector(api, le_settings("a"), clock=ca)
        b = LeaderElector(api, le_settings("b"), clock=cb)
        try:
            assert await a.try_acquire_or_renew()
            assert not await b.try_acquire_or_renew()
            assert b.holder == "a"
            # a renews: b sees a changed record, so its expiry window restarts
            ca.t += 1.0
            assert await a.try_acquire_or_renew()
            cb.t += 1.9
            assert not await b.try_acquire_or_renew()
            # a stops renewing; b's clock passes lease duration since it last saw a change
            cb.t += 2.1
            assert await b.try_acquire_or_renew()
            lease = srv.leases[("kube-system", "k8s-watcher-amd")]["spec"]
            assert lease["holderIdentity"] == "b" and lease["leaseTransitions"] == 1
            assert lease["leaseDurationSeconds"] == 2
            # a comes back: it is no longer the holder and must not steal it
            assert not await a.try_acquire_or_renew()
            assert a.holder == "b"
        finally:
            await api.close()
            await srv.stop()
    run(body())


def test_concurrent_candidates_single_winner():
    async def body():
        srv = FakeApiServer()
        await srv.start()
        apis = [KubeApi(KubeEndpoint(server=srv.url)) for _ in range(6)]
        els = [LeaderElector(api, le_settings(f"c{i}")) for i, api in enumerate(apis)]
        try:
            for _ in range(5):
                res = await asyncio.gather(*(e.try_acquire_or_renew() for e in els))
                assert sum(res) == 1
            holder = srv.leases[("kube-system", "k8s-watcher-amd")]["spec"]["holderIdentity"]
            assert [e.identity for e, r in zip(els, res) if r] == [holder]
        finally:
            for api in apis:
                await api.close()
            await srv.stop()
    run(body())


def test_release_hands_over_immediately_and_renew_deadline_steps_down():
    async def body():
        srv = FakeApiServer()
        await srv.start()
        api = KubeApi(KubeEndpoint(server=srv.url))
        a = LeaderElector(api, le_settings("a", lease_duration_seconds=30, renew_deadline_seconds=1.0))
        b = LeaderElector(api, le_settings("b", lease_duration_seconds=30, renew_deadline_seconds=1.0))
        ta = asyncio.ensure_future(a.run())
        await asyncio.wait_for(a.became_leader.wait(), 5)
        tb = asyncio.ensure_future(b.run())
        await asyncio.sleep(0.3)
        assert a.is_leader and not b.is_leader
        a.stop()
        await ta
        assert not a.is_leader
        # released: b takes over well before the 30 s lease would expire
        await asyncio.wait_for(b.became_leader.wait(), 3)
        # the API server starts failing lease writes: b must step down after the renew deadline
        srv.lease_fault = 503
        await asyncio.wait_for(b.lost.wait(), 4)
        assert not b.is_leader and b.metrics.c["lease_update_errors"] > 0
        srv.lease_fault = None
        await asyncio.wait_for(b.became_leader.wait(), 3)  # its own record: it re-acquires
        b.stop()
        await tb
        await api.close()
        await srv.stop()
    run(body(), timeout=30)


def test_stalled_lease_requests_step_down_within_renew_deadline():
    """A renew round is bounded by ONE deadline (what is left of
    renew_deadline since the last renew), not by per-request timeouts: with
    every lease request stalled, the leader stops leading before its lease
    could expire for the others — even while its request is still in flight."""
    async def body():
        srv = FakeApiServer()
        await srv.start()
        api = KubeApi(KubeEndpoint(server=srv.url), timeout=30)
        a = LeaderElector(api, le_settings("a", lease_duration_seconds=3, renew_deadline_seconds=1.0,
                                           retry_period_seconds=0.2))
        ta = asyncio.ensure_future(a.run())
        await asyncio.wait_for(a.became_leader.wait(), 5)
        await asyncio.sleep(0.3)
        srv.lease_stall = 30.0  # the API server accepts the request and never answers in time
        t_stall = asyncio.get_running_loop().time()
        await asyncio.wait_for(a.lost.wait(), 3)
        lost_after = asyncio.get_running_loop().time() - t_stall
        # stepped down within renew_deadline of the last renew (+ scheduling slack),
        # well before lease_duration (3 s) after it
        assert lost_after < 1.3, lost_after
        assert a.metrics.c["lease_update_errors"] >= 1
        srv.lease_stall = 0.0
        a.stop()
        ta.cancel()
        try:
            await ta
        except asyncio.CancelledError:
            pass
        await api.close()
        await srv.stop()
    run(body(), timeout=30)


def test_standby_refreshes_credentials_on_401(tmp_path):
    """A standby runs no reflector; its elector must refresh a rotated token
    itself on a 401, or it could never take over."""
    from k8s_watcher_amd.kube.kubeconfig import load_kube_config

    async def body():
        srv = FakeApiServer(token="one")
        await srv.start()
        tok = tmp_path / "tok"
        tok.write_text("one\n")
        cfg = tmp_path / "cfg"
        cfg.write_text(f"""
current-context: x
clusters: [{{name: c, cluster: {{server: "{srv.url}"}}}}]
contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
users: [{{name: u, user: {{tokenFile: tok}}}}]
""")
        api = KubeApi(load_kube_config(str(cfg)))
        b = LeaderElector(api, le_settings("b"))
        try:
            assert await b.try_acquire_or_renew()
            srv.token = "two"
            tok.write_text("two\n")
            assert not await b.try_acquire_or_renew()  # 401: refreshes (token file re-read)
            assert b.metrics.c["auth_refreshes"] == 1
            assert await b.try_acquire_or_renew()
        finally:
            await api.close()
            await srv.stop()
    run(body())


def test_settings_validation():
    s = load_settings("development", overrides={"watcher": {"leader_election": {"enabled": True}}})
    le = s.watcher.leader_election
    assert le.enabled and le.lease_duration_seconds == 15 and le.renew_deadline_seconds == 10
    with pytest.raises(ConfigError):
        load_settings("development", overrides={"watcher": {"leader_election": {
            "lease_duration_seconds": 5, "renew_deadline_seconds": 6}}})


def test_micro_time_and_record_roundtrip():
    assert micro_time(0) == "1970-01-01T00:00:00.000000Z"
    rec = LeaderRecord("x", 15, micro_time(1), micro_time(2), 3)
    assert LeaderRecord.from_lease({"spec": rec.spec()}) == rec


async def _replica(srv, sink, identity):
    ov = {"clusterapi": {"base_url": sink.url, "retry": {"delay_seconds": 0.01}},
          "watcher": {"retry": {"delay_seconds": 0.01, "max_attempts": 0},
                      "leader_election": {"enabled": True, "identity": identity, **FAST}}}
    settings = load_settings("development", overrides=ov)
    r = LeaderElectedService(settings, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
    return r, asyncio.ensure_future(r.run())


@pytest.mark.parametrize("crash", [False, True])
def test_only_leader_notifies_and_standby_takes_over(crash):
    async def body():
        srv = FakeApiServer()
        await srv.start()
        sink = StubSink()
        await sink.start()
        f = PodFactory(seed=5, namespaces=["default"])
        a, ta = await _replica(srv, sink, "replica-a")
        await asyncio.wait_for(a.elector.became_leader.wait() if a.elector else asyncio.sleep(0), 5)
        while a.elector is None or not a.elector.is_leader:
            await asyncio.sleep(0.02)
        b, tb = await _replica(srv, sink, "replica-b")
        while b.elector is None:
            await asyncio.sleep(0.02)
        await asyncio.sleep(0.3)
        for _ in range(5):
            srv.create(f.running(f.new_pod()))
        await sink.state.wait_for(5, timeout=10)
        await asyncio.sleep(0.3)
        assert len(sink.state.payloads()) == 5  # b is standby: nothing doubled
        assert not b.elector.is_leader and b.service is None
        if crash:
            # leader dies without releasing: stop renewing, drop its term
            a.elector.release = lambda: asyncio.sleep(0)  # no hand-over write
            ta.cancel()
            try:
                await ta
            except asyncio.CancelledError:
                pass
        else:
            a.stop()
            await ta
        await asyncio.wait_for(b.elector.became_leader.wait(), 6)
        while b.service is None or not b.service.started.is_set():
            await asyncio.sleep(0.02)
        # the new leader lists the cluster: existing pods are re-sent once (at-least-once)
        await sink.state.wait_for(10, timeout=10)
        srv.create(f.running(f.new_pod()))
        await sink.state.wait_for(11, timeout=10)
        got = sink.state.payloads()
        assert len({p["uid"] for p in got}) == 6
        b.stop()
        await tb
        assert srv.leases[("default", "k8s-watcher-amd")]["spec"]["holderIdentity"] == ""
        await sink.stop()
        await srv.stop()
    run(body(), timeout=45)


def test_one_lease_per_shard():
    from k8s_watcher_amd.engine.leader import shard_lease
    s = load_settings("staging", overrides={"watcher": {"shard": {"count": 3, "index": 2},
                                                        "leader_election": {"enabled": True}}}, environ={})
    assert shard_lease(s).lease_name == "k8s-watcher-amd-shard-2"
    s1 = load_settings("staging", overrides={"watcher": {"leader_election": {"enabled": True}}}, environ={})
    assert shard_lease(s1).lease_name == "k8s-watcher-amd"


def _native_threads() -> int:
    """Kernel threads of this process that are not Python threads (the asyncio
    default executor grows lazily up to its bound; it is not what is counted)."""
    import os
    import threading
    return len(os.listdir("/proc/self/task")) - len(threading.enumerate())


def test_terms_do_not_leak_decode_pool_threads():
    """Every term builds a new WatcherService with its own native decode pool;
    a term that ends must take the pool's threads with it (shutdown closes the
    pool), not leave them until the garbage collector frees the old service —
    which the shared Metrics gauges keep reachable."""
    async def body():
        srv = FakeApiServer()
        await srv.start()
        sink = StubSink()
        await sink.start()
        ov = {"clusterapi": {"base_url": sink.url, "retry": {"delay_seconds": 0.01}},
              "watcher": {"engine": "native", "decode_threads": 3,
                          "retry": {"delay_seconds": 0.01, "max_attempts": 0},
                          "leader_election": {"enabled": True, "identity": "solo", "exit_on_loss": False,
                                              **FAST}}}
        settings = load_settings("development", overrides=ov)
        r = LeaderElectedService(settings, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
        t = asyncio.ensure_future(r.run())
        counts = []
        for term in range(3):
            while r.service is None or not r.service.started.is_set():
                await asyncio.sleep(0.02)
            assert r.terms == term + 1
            svc = r.service
            counts.append(_native_threads())
            # another candidate takes the lease: this term ends (lease lost) ...
            key = ("default", "k8s-watcher-amd")
            spec = dict(srv.leases[key]["spec"], holderIdentity="intruder")
            srv.leases[key] = dict(srv.leases[key], spec=spec)
            while r.service is svc:
                await asyncio.sleep(0.02)
            # ... and never renews it, so "solo" leads again once it expires
        r.stop()
        await t
        await asyncio.sleep(0.2)
        after = _native_threads()
        await sink.stop()
        await srv.stop()
        return counts, after

    counts, after = run(body(), timeout=60)
    # the same number of threads in every term: nothing left over from the earlier ones
    assert counts[0] == counts[1] == counts[2], counts
    assert after <= counts[0] - 3, (counts, after)  # and the last term's pool is gone too
