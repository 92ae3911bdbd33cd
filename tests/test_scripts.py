"""The manual smoke scripts and the v0 example (C16) run green
against the fake API server."""

import os
import signal
import subprocess
import sys
import textwrap
import time

import pytest

from conftest import ROOT
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer, ServerThread
from k8s_watcher_amd.testing.podgen import PodFactory


@pytest.fixture
def kubeconfig(tmp_path):
    srv = FakeApiServer(token="s")
    st = ServerThread(srv).start()
    f = PodFactory(seed=4, namespaces=["default", "kube-system"])
    for _ in range(6):
        st.call(srv.create, f.running(f.new_pod()))
    kc = tmp_path / "kc"
    kc.write_text(textwrap.dedent(f"""
        current-context: c
        clusters: [{{name: c, cluster: {{server: "http://127.0.0.1:{srv.port}"}}}}]
        contexts: [{{name: c, context: {{cluster: c, user: u}}}}]
        users: [{{name: u, user: {{token: s}}}}]
        """))
    yield str(kc)
    st.stop()


@pytest.mark.parametrize("script", ["smoke_mock.py", "smoke_connection.py"])
def test_smoke_scripts(kubeconfig, script):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", script), kubeconfig],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout
    if script == "smoke_mock.py":
        assert "OK pod list: 5 pod(s)" in r.stdout and "OK watch: 5 event(s)" in r.stdout


def test_smoke_script_fails_without_server(tmp_path):
    kc = tmp_path / "kc"
    kc.write_text("current-context: c\nclusters: [{name: c, cluster: {server: 'http://127.0.0.1:1'}}]\n"
                  "contexts: [{name: c, context: {cluster: c, user: u}}]\nusers: [{name: u, user: {}}]\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "smoke_connection.py"), str(kc)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1


def test_minimal_example_prints_events(kubeconfig):
    p = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "examples", "minimal_watch.py"), kubeconfig],
                         stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    lines = []
    deadline = time.time() + 20
    while len(lines) < 7 and time.time() < deadline:
        line = p.stdout.readline()
        if not line:
            break
        lines.append(line.strip())
    p.send_signal(signal.SIGINT)
    p.wait(10)
    assert lines[0] == "Starting to watch for Pod events..."
    assert sum(1 for ln in lines if ln.startswith("Event: ADDED Pod: ")) == 6
