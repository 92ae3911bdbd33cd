"""HA soak in miniature: two leader-elected replicas sharing a checkpoint, pod
churn throughout, a graceful hand-over, API-server connection drops and a
compaction (410) — every pod's *final* state must reach clusterapi.

The reference has one replica, no resume and no relist; this
checks the combination of engine/leader.py, the checkpoint and the reflector.
With a graceful hand-over the outgoing leader drains, writes the checkpoint and
releases the lease, so the incoming one resumes from that resourceVersion with
the same pod cache — deletions made around the hand-over are not lost.
"""

import asyncio
import random

from conftest import run
from k8s_watcher_amd.engine.leader import LeaderElectedService
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import load_settings

LE = dict(lease_duration_seconds=2, renew_deadline_seconds=1.5, retry_period_seconds=0.1)


def replica(srv, sink, identity, ck):
    ov = {"clusterapi": {"base_url": sink.url, "retry": {"delay_seconds": 0.01, "max_attempts": 20}},
          "watcher": {"retry": {"delay_seconds": 0.01, "max_attempts": 0},
                      "checkpoint": {"path": ck, "interval_seconds": 0.2},
                      "leader_election": {"enabled": True, "identity": identity, **LE}}}
    r = LeaderElectedService(load_settings("staging", overrides=ov), endpoint=KubeEndpoint(server=srv.url),
                             metrics=Metrics())
    return r, asyncio.ensure_future(r.run())


def test_graceful_handover_under_churn_keeps_final_state(tmp_path):
    async def body():
        rng = random.Random(7)
        srv = FakeApiServer()
        await srv.start()
        sink = StubSink()
        await sink.start()
        ck = str(tmp_path / "ck.json")
        f = PodFactory(seed=8, namespaces=["default", "batch"])
        live = {}
        for _ in range(20):
            p = f.running(f.new_pod())
            srv.create(p)
            live[p["metadata"]["uid"]] = p
        a, ta = replica(srv, sink, "a", ck)
        while a.service is None or not a.service.started.is_set():
            await asyncio.sleep(0.02)
        b, tb = replica(srv, sink, "b", ck)
        deleted = set()

        async def churn(n):
            for _ in range(n):
                op = rng.random()
                if op < 0.3 or not live:
                    p = f.running(f.new_pod())
                    srv.create(p)
                    live[p["metadata"]["uid"]] = p
                elif op < 0.75:
                    uid = rng.choice(sorted(live))
                    p = live[uid]
                    p = f.terminated(p, failed=rng.random() < 0.5) if rng.random() < 0.5 else f.running(p)
                    srv.update(p)
                    live[uid] = p
                else:
                    uid = rng.choice(sorted(live))
                    p = live.pop(uid)
                    srv.delete(p["metadata"]["namespace"], p["metadata"]["name"])
                    deleted.add(uid)
                await asyncio.sleep(0.005)

        await churn(60)
        srv.drop_connections()          # API server restart: resume from the last resourceVersion
        await churn(40)
        a.stop()                        # graceful hand-over while pods keep changing
        await churn(40)
        await ta
        while b.service is None or not b.service.started.is_set():
            await asyncio.sleep(0.02)
        srv.expire_watches()            # 410 Gone on the open watch: relist and diff against the cache
        await churn(60)
        # quiescence: nothing new at the sink for a while
        last, stable = -1, 0
        while stable < 10:
            await asyncio.sleep(0.05)
            stable = stable + 1 if sink.state.count == last else 0
            last = sink.state.count
        final = {}
        for p in sink.state.payloads():
            final[p["uid"]] = p
        for uid, p in live.items():
            got = final.get(uid)
            assert got is not None, f"pod {uid} never notified"
            assert got["event_type"] != "DELETED" and got["status"]["phase"] == p["status"]["phase"], (uid, got)
        for uid in deleted:
            if uid in final:  # pods created and deleted while unobserved may never appear at all
                assert final[uid]["event_type"] == "DELETED", (uid, final[uid]["event_type"])
        assert b.elector.is_leader and b.metrics.c["expired_410"] >= 1
        b.stop()
        await tb
        await sink.stop()
        await srv.stop()
    run(body(), timeout=60)
