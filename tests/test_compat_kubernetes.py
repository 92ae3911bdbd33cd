"""The ``kubernetes``-client subset and the reference smoke flows (C14, C15)."""

import textwrap
import threading
import time

import pytest

from k8s_watcher_amd.compat.kubernetes import client, config, watch
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer, ServerThread
from k8s_watcher_amd.testing.podgen import PodFactory


@pytest.fixture
def api(tmp_path):
    srv = FakeApiServer(token="abc")
    st = ServerThread(srv).start()
    f = PodFactory(seed=3, namespaces=["default", "kube-system"])
    for _ in range(7):
        st.call(srv.create, f.running(f.new_pod()))
    kc = tmp_path / "kubeconfig"
    kc.write_text(textwrap.dedent(f"""
        current-context: m
        clusters: [{{name: m, cluster: {{server: "http://127.0.0.1:{srv.port}"}}}}]
        contexts: [{{name: m, context: {{cluster: m, user: u}}}}]
        users: [{{name: u, user: {{token: abc}}}}]
        """))
    config.load_kube_config(config_file=str(kc))
    yield st, srv, f, str(kc)
    st.stop()


def test_mock_smoke_flow(api):
    """test_k8s_mock.py:17-80 against the fake API server, with assertions."""
    st, srv, f, kc = api
    v1 = client.CoreV1Api()
    contexts, active = config.list_kube_config_contexts(config_file=kc)
    assert active["context"]["cluster"] == "m"
    pods = v1.list_pod_for_all_namespaces(limit=5)
    assert len(pods.items) == 5
    assert all(p.status.phase == "Running" for p in pods.items)
    assert pods.metadata._continue  # paginated
    rest = v1.list_pod_for_all_namespaces(limit=5, _continue=pods.metadata._continue)
    assert len(rest.items) == 2
    nss = v1.list_namespace()
    assert {n.metadata.name for n in nss.items} >= {"default", "kube-system"}
    w = watch.Watch()
    got = []
    for ev in w.stream(v1.list_pod_for_all_namespaces, timeout_seconds=5):
        got.append((ev["type"], ev["object"].metadata.name))
        if len(got) >= 5:
            break
    w.stop()
    assert len(got) == 5 and all(t == "ADDED" for t, _ in got)


def test_connection_smoke_flow(api):
    """test_k8s_connection.py:16-48."""
    v1 = client.CoreV1Api()
    assert client.VersionApi().get_code().git_version == "v1.33.1-fake"
    assert len(v1.list_namespace(limit=1).items) == 1
    assert len(v1.list_pod_for_all_namespaces(limit=1).items) == 1
    assert len(v1.list_namespaced_pod("default").items) >= 1


def test_bad_token_is_api_exception(api, tmp_path):
    st, srv, f, kc = api
    bad = tmp_path / "bad"
    bad.write_text(open(kc).read().replace("token: abc", "token: nope"))
    config.load_kube_config(config_file=str(bad))
    with pytest.raises(client.ApiException) as ei:
        client.CoreV1Api().list_namespace()
    assert ei.value.status == 401


def test_watch_resumes_from_last_resource_version(api):
    st, srv, f, kc = api
    v1 = client.CoreV1Api()
    w = watch.Watch()
    seen = []

    def produce():
        time.sleep(0.3)
        st.call(srv.drop_connections)  # server goes away mid-watch ...
        time.sleep(0.3)
        st.call(srv.create, f.new_pod(name="after-restart"))  # ... and comes back with new events

    threading.Thread(target=produce, daemon=True).start()
    for ev in w.stream(v1.list_pod_for_all_namespaces):
        seen.append(ev["object"].metadata.name)
        if ev["object"].metadata.name == "after-restart":
            w.stop()
    # initial 7 ADDED then exactly one new event: the resume did not replay history
    assert len(seen) == 8 and seen[-1] == "after-restart"


def test_watch_410_twice_raises(api):
    st, srv, f, kc = api
    v1 = client.CoreV1Api()
    st.call(srv.compact)
    w = watch.Watch()
    with pytest.raises(client.ApiException) as ei:
        for _ in w.stream(v1.list_pod_for_all_namespaces, resource_version="1"):
            pass
    assert ei.value.status == 410
