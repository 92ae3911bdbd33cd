"""CLI contract (reference main.py:5-27) and the ``watcher`` compat API."""

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

MAIN = os.path.join(ROOT, "main.py")


def cli(*args, env=None, timeout=60, cwd=ROOT):
    e = dict(os.environ)
    e.pop("ENVIRONMENT", None)
    e.update(env or {})
    return subprocess.run([sys.executable, MAIN, *args], capture_output=True, text=True, env=e,
                          timeout=timeout, cwd=cwd)


def test_unsupported_environment():
    r = cli("local")
    assert r.returncode == 1
    assert r.stdout.splitlines() == ["Error: Unsupported environment 'local'",
                                     "Supported environments: ['development', 'staging', 'production']"]


def test_environment_precedence_argv_over_env():
    r = cli("staging", "--print-config", env={"ENVIRONMENT": "production"})
    assert r.returncode == 0
    assert "Starting k8s-watcher in 'staging' environment" in r.stdout
    r = cli("--print-config", env={"ENVIRONMENT": "production"})
    assert "Starting k8s-watcher in 'production' environment" in r.stdout
    assert "critical_events_only: true" in r.stdout
    r = cli("--print-config")
    assert "Starting k8s-watcher in 'development' environment" in r.stdout


def test_set_override_and_bad_config():
    r = cli("staging", "--print-config", "--set", "watcher.notify_on=phase_change")
    assert "notify_on: phase_change" in r.stdout
    r = cli("staging", "--set", "watcher.log_level=LOUD")
    assert r.returncode == 1 and "Error starting watcher:" in r.stdout


def test_setup_failure_exits_nonzero(tmp_path):
    (tmp_path / "base.yaml").write_text("kubernetes:\n  config_file: ./does-not-exist\n")
    (tmp_path / "staging.yaml").write_text("")
    r = cli("staging", "--config-dir", str(tmp_path))
    assert r.returncode == 1  # the reference exits 0 here
    assert "Kubeconfig file not found: ./does-not-exist" in r.stderr
    assert "Failed to setup Kubernetes client" in r.stderr


@pytest.fixture
def cluster(tmp_path):
    srv = FakeApiServer(token="cli")
    st = ServerThread(srv).start()
    f = PodFactory(seed=2, namespaces=["default"])
    for _ in range(3):
        st.call(srv.create, f.running(f.new_pod()))
    kc = tmp_path / "kubeconfig"
    kc.write_text(textwrap.dedent(f"""
        current-context: c
        clusters: [{{name: c, cluster: {{server: "http://127.0.0.1:{srv.port}"}}}}]
        contexts: [{{name: c, context: {{cluster: c, user: u}}}}]
        users: [{{name: u, user: {{token: cli}}}}]
        """))
    cfg = tmp_path / "config"
    cfg.mkdir()
    (cfg / "base.yaml").write_text(textwrap.dedent(f"""
        kubernetes:
          config_file: {kc}
        clusterapi:
          enabled: false
        watcher:
          log_level: INFO
        """))
    (cfg / "staging.yaml").write_text("")
    yield st, srv, str(cfg)
    st.stop()


def test_check_mode(cluster):
    st, srv, cfg = cluster
    r = cli("staging", "--config-dir", cfg, "--check")
    assert r.returncode == 0, r.stderr
    assert "Successfully connected to Kubernetes API version: v1.33.1-fake" in r.stderr
    assert "Sample namespaces: ['default', 'kube-system']" in r.stderr
    assert "Permission OK: watch pods (cluster-wide)" in r.stderr


def test_check_mode_reports_missing_rbac(cluster):
    st, srv, cfg = cluster
    srv.denied.add(("watch", "pods"))
    r = cli("staging", "--config-dir", cfg, "--check", "--set", "watcher.leader_election.enabled=true",
            "--set", "watcher.leader_election.lease_namespace=ops")
    assert r.returncode == 1, r.stderr
    assert "Permission missing: watch pods (cluster-wide) (denied by the fake RBAC)" in r.stderr
    assert "Permission OK: update coordination.k8s.io/leases in ops" in r.stderr


def test_sigterm_graceful_shutdown(cluster):
    st, srv, cfg = cluster
    e = dict(os.environ)
    e.pop("ENVIRONMENT", None)
    p = subprocess.Popen([sys.executable, MAIN, "staging", "--config-dir", cfg], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, env=e, cwd=ROOT)
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            if any("/api/v1/pods" in t and "watch=true" in t for _, t in srv.requests):
                break
            time.sleep(0.05)
        time.sleep(0.2)
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=20)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, err
    assert "Monitoring all namespaces" in err
    assert err.count("Pod event detected: ADDED - default/") == 3
    assert "Stopping Pod watcher..." in err


def test_podwatcher_compat_api(cluster, monkeypatch):
    st, srv, cfg = cluster
    from watcher.pod_watcher import PodWatcher
    w = PodWatcher("production", config_dir=cfg)
    assert w.settings.environment == "production"
    assert w._merge_configs({"a": {"b": 1}}, {"a": {"c": 2}}) == {"a": {"b": 1, "c": 2}}
    monkeypatch.setenv("X_TEST", "v")
    assert w._substitute_env_vars({"k": "${X_TEST}"}) == {"k": "v"}
    assert w.setup_k8s_client() is True
    pods = w.v1.list_pod_for_all_namespaces()
    pod = pods.items[0]
    data = w._extract_pod_data(pod)
    assert data["name"] == pod.metadata.name and data["environment"] == "production"
    # the temp config dir has no production.yaml, so critical_events_only is off here
    assert w.handle_pod_event("MODIFIED", pod)["event_type"] == "MODIFIED"
    assert w.handle_pod_event("ADDED", {"metadata": {"name": "x", "namespace": "default"}})["status"]["phase"] \
        == "Unknown"


def test_podwatcher_filters_like_reference(tmp_path):
    from watcher.pod_watcher import PodWatcher
    w = PodWatcher("production", config_dir=os.path.join(ROOT, "config"))
    running = {"metadata": {"name": "r", "namespace": "default"}, "status": {"phase": "Running"}}
    failed = {"metadata": {"name": "f", "namespace": "default"}, "status": {"phase": "Failed"}}
    other_ns = {"metadata": {"name": "o", "namespace": "batch"}, "status": {"phase": "Failed"}}
    assert w.should_process_event("MODIFIED", running) is False
    assert w.handle_pod_event("MODIFIED", running) is None
    assert w.handle_pod_event("DELETED", running)["event_type"] == "DELETED"
    assert w.handle_pod_event("MODIFIED", failed)["status"]["phase"] == "Failed"
    assert w.handle_pod_event("MODIFIED", other_ns) is None


def test_two_replicas_leader_election_cli(cluster):
    """Two ``main.py`` processes with leader election: one watches; SIGTERM on it
    releases the lease and the other takes over (lists and logs the pods)."""
    st, srv, cfg = cluster
    e = dict(os.environ)
    e.pop("ENVIRONMENT", None)
    sets = ["--set", "watcher.leader_election.enabled=true", "--set", "watcher.leader_election.lease_namespace=default",
            "--set", "watcher.leader_election.lease_duration_seconds=4",
            "--set", "watcher.leader_election.renew_deadline_seconds=3",
            "--set", "watcher.leader_election.retry_period_seconds=0.2"]

    def start(name):
        return subprocess.Popen([sys.executable, MAIN, "staging", "--config-dir", cfg, *sets,
                                 "--set", f"watcher.leader_election.identity={name}"],
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e, cwd=ROOT)

    def watches():
        return sum(1 for _, t in srv.requests if "/api/v1/pods" in t and "watch=true" in t)

    def wait_for(pred, limit=30):
        deadline = time.time() + limit
        while time.time() < deadline and not pred():
            time.sleep(0.05)
        assert pred()

    a = start("replica-a")
    b = None
    try:
        wait_for(lambda: watches() == 1)
        b = start("replica-b")
        wait_for(lambda: any(t.endswith("/leases/k8s-watcher-amd") and m == "GET" for m, t in srv.requests[-5:]))
        time.sleep(1.0)
        assert watches() == 1  # b is a standby
        a.send_signal(signal.SIGTERM)
        out_a, err_a = a.communicate(timeout=20)
        assert a.returncode == 0, err_a
        assert "Released lease default/k8s-watcher-amd" in err_a
        wait_for(lambda: watches() == 2)
        time.sleep(0.5)
        b.send_signal(signal.SIGTERM)
        out_b, err_b = b.communicate(timeout=20)
    finally:
        for p in (a, b):
            if p is not None and p.poll() is None:
                p.kill()
    assert b.returncode == 0, err_b
    assert "Acquired leadership of lease default/k8s-watcher-amd as replica-b" in err_b
    assert err_b.count("Pod event detected: ADDED - default/") == 3


def test_podwatcher_subclass_hooks_run_per_event(cluster):
    """A reference user's subclass overriding handle_pod_event keeps working:
    start_watching hands every event to the override (pod_watcher.py:266-269)."""
    import threading
    from watcher.pod_watcher import PodWatcher
    st, srv, cfg = cluster
    seen = []

    class Mine(PodWatcher):
        def handle_pod_event(self, event_type, pod):
            seen.append((event_type, pod.metadata.namespace, pod.metadata.name))
            if len(seen) == 4:
                self.watch.stop()  # ends the stream after this event
            return super().handle_pod_event(event_type, pod)

    w = Mine("staging", config_dir=cfg)
    assert w._customised() and not PodWatcher("staging", config_dir=cfg)._customised()
    t = threading.Thread(target=w.start_watching, daemon=True)
    t.start()
    deadline = time.time() + 20
    while len(seen) < 3 and time.time() < deadline:
        time.sleep(0.05)
    assert [s[0] for s in seen] == ["ADDED"] * 3
    f = PodFactory(seed=9, namespaces=["default"])
    st.call(srv.create, f.running(f.new_pod()))
    t.join(20)
    assert not t.is_alive() and len(seen) == 4 and seen[3][0] == "ADDED"
