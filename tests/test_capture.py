"""Capture a watch stream to a file and replay it (tools/capture.py, fake_apiserver replay)."""

import asyncio
import io
import json

from conftest import run
from k8s_watcher_amd.kube.api import KubeApi
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer, replay_capture
from k8s_watcher_amd.testing.podgen import PodFactory, churn_events
from k8s_watcher_amd.tools.capture import capture, load_capture
from test_e2e_slice import start_stack


def test_capture_then_replay_gives_the_same_notifications(tmp_path):
    async def body():
        src = FakeApiServer()
        f = PodFactory(seed=51, namespaces=["default"])
        for _ in range(5):
            src.create(f.running(f.new_pod()))
        await src.start()
        api = KubeApi(KubeEndpoint(server=src.url))
        path = tmp_path / "cap.ndjson"
        stop = asyncio.Event()
        with open(path, "w") as fh:
            task = asyncio.ensure_future(capture(api, fh, max_events=30, stop=stop))
            await asyncio.sleep(0.2)
            for et, obj in churn_events(6, seed=52, namespaces=["default"]):
                src.apply(et, obj)
                await asyncio.sleep(0.002)
            n = await asyncio.wait_for(task, 10)
        await api.close()
        await src.stop()
        recs = load_capture(str(path))
        assert n == 30 and sum(r["type"] == "LIST" for r in recs) == 5
        assert all(recs[i]["t"] <= recs[i + 1]["t"] for i in range(len(recs) - 1))

        # replay into a fresh API server with a watcher attached
        srv, sink, svc = await start_stack("staging")
        for r in recs:
            if r["type"] == "LIST":
                srv.create(r["object"])
        await svc.start()
        await sink.state.wait_for(5, timeout=10)
        await replay_capture(srv, [r for r in recs if r["type"] != "LIST"], speed=0)
        await sink.state.wait_for(35, timeout=10)
        got = [(p["event_type"], p["uid"]) for p in sink.state.payloads()]
        want = [("ADDED", r["object"]["metadata"]["uid"]) for r in recs if r["type"] == "LIST"]
        want += [(r["type"], r["object"]["metadata"]["uid"]) for r in recs if r["type"] != "LIST"]
        def per_pod(seq):  # the notifier keeps each pod's order; pods interleave freely
            out = {}
            for et, uid in seq:
                out.setdefault(uid, []).append(et)
            return out
        assert per_pod(got) == per_pod(want)
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


def test_capture_resumes_when_the_server_ends_the_watch(tmp_path):
    async def body():
        src = FakeApiServer()
        f = PodFactory(seed=53, namespaces=["default"])
        await src.start()
        api = KubeApi(KubeEndpoint(server=src.url))
        out = io.StringIO()
        task = asyncio.ensure_future(capture(api, out, max_events=6))
        await asyncio.sleep(0.2)
        pods = [src.create(f.running(f.new_pod())) for _ in range(3)]
        await asyncio.sleep(0.2)
        src.drop_connections()  # API server restart: the capture re-watches from the last RV
        await asyncio.sleep(1.2)
        for p in pods:
            src.update(f.terminated(p))
        n = await asyncio.wait_for(task, 10)
        await api.close()
        await src.stop()
        recs = [json.loads(line) for line in out.getvalue().splitlines()]
        assert n == 6
        assert [r["type"] for r in recs] == ["ADDED"] * 3 + ["MODIFIED"] * 3  # nothing lost, nothing twice
    run(body())
