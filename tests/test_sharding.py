"""Multi-process sharding (parallel/shard.py, parallel/launch.py) and the
multi-rank bench path (gloo, world_size 2)."""

import collections
import json
import os
import signal
import socket
import subprocess
import sys
import textwrap
import time

import pytest

from conftest import ROOT
from k8s_watcher_amd.parallel.shard import ShardFilter, shard_of
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer, ServerThread
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import ConfigError, ShardSettings, load_settings


def test_shard_partition_is_total_and_disjoint():
    keys = [f"ns-{i}" for i in range(200)]
    owners = collections.Counter()
    for k in keys:
        hits = [i for i in range(4) if ShardFilter(ShardSettings(4, i)).owns("uid", k)]
        assert len(hits) == 1
        owners[hits[0]] += 1
    assert all(v > 20 for v in owners.values())
    assert shard_of("x", 1) == 0


def test_shard_env_overrides(monkeypatch):
    monkeypatch.setenv("K8S_WATCHER_SHARD_COUNT", "3")
    monkeypatch.setenv("K8S_WATCHER_SHARD_INDEX", "2")
    s = load_settings("staging", environ={})
    assert (s.watcher.shard.count, s.watcher.shard.index) == (3, 2)
    monkeypatch.setenv("K8S_WATCHER_SHARD_INDEX", "3")
    with pytest.raises(ConfigError):
        load_settings("staging", environ={})


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_launcher_two_shards_exactly_once(tmp_path):
    import asyncio
    import threading

    srv = FakeApiServer()
    st = ServerThread(srv).start()
    sink = StubSink()
    sink_loop = asyncio.new_event_loop()
    sink_port = free_port()
    threading.Thread(target=lambda: (sink_loop.run_until_complete(sink.start(port=sink_port)),
                                     sink_loop.run_forever()), daemon=True).start()
    kc = tmp_path / "kc"
    kc.write_text(textwrap.dedent(f"""
        current-context: c
        clusters: [{{name: c, cluster: {{server: "http://127.0.0.1:{srv.port}"}}}}]
        contexts: [{{name: c, context: {{cluster: c, user: u}}}}]
        users: [{{name: u, user: {{token: x}}}}]
        """))
    cfg = tmp_path / "cfg"
    cfg.mkdir()
    (cfg / "base.yaml").write_text(textwrap.dedent(f"""
        kubernetes: {{config_file: {kc}}}
        clusterapi: {{base_url: "http://127.0.0.1:{sink_port}"}}
        watcher: {{log_level: INFO}}
        """))
    (cfg / "staging.yaml").write_text("")
    env = dict(os.environ)
    env.pop("ENVIRONMENT", None)
    p = subprocess.Popen([sys.executable, "-m", "k8s_watcher_amd.parallel.launch", "--shards", "2", "staging",
                          "--config-dir", str(cfg)], cwd=ROOT, env=env,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        deadline = time.time() + 30
        while time.time() < deadline and sum("watch=true" in t for _, t in srv.requests) < 2:
            time.sleep(0.05)
        f = PodFactory(seed=8, namespaces=[f"ns-{i}" for i in range(10)])
        expected = []
        for _ in range(20):
            pod = st.call(srv.create, f.new_pod())
            expected.append(pod["metadata"]["uid"])
        deadline = time.time() + 20
        while time.time() < deadline and sink.state.count < 20:
            time.sleep(0.05)
        time.sleep(0.3)
        p.send_signal(signal.SIGTERM)
        _, err = p.communicate(timeout=20)
    finally:
        if p.poll() is None:
            p.kill()
        st.stop()
        sink_loop.call_soon_threadsafe(sink_loop.stop)
    got = [json.loads(b)["uid"] for _, b in sink.state.received]
    assert sorted(got) == sorted(expected), err[-2000:]
    assert p.returncode == 0
    assert "Shard 0/2" in err and "Shard 1/2" in err


def test_bench_two_ranks_gloo():
    port = free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--pods-per-step", "300",
                        "--ref-events", "0", "--latency-seconds", "0.5", "--sink-workers", "1"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * 1500
    assert d["value"] > 0 and d["scaling"] == "weak"
