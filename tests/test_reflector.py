"""Watch robustness (BASELINE config #5): resume, 410 relist,
bookmarks, retries, checkpoint restart — each asserting exactly-once delivery."""

import asyncio
import collections
import math
import time

import pytest

from conftest import run
from k8s_watcher_amd.engine.reflector import WatchFailed
from k8s_watcher_amd.engine.service import WatcherService
from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import deep_merge, load_settings


class Stack:
    def __init__(self, environment="staging", overrides=None, server_kwargs=None, sink_kwargs=None):
        self.environment = environment
        self.overrides = overrides or {}
        self.server_kwargs = server_kwargs or {}
        self.sink_kwargs = sink_kwargs or {}
        self.factory = PodFactory(seed=21, namespaces=["default", "kube-system", "batch"])

    async def __aenter__(self):
        self.srv = FakeApiServer(**self.server_kwargs)
        await self.srv.start()
        self.sink = StubSink(**self.sink_kwargs)
        await self.sink.start()
        return self

    def service(self, extra=None):
        ov = {"clusterapi": {"base_url": self.sink.url, "retry": {"delay_seconds": 0.01, "max_attempts": 5},
                             "health_check_on_start": False},
              "watcher": {"retry": {"delay_seconds": 0.01, "max_attempts": 0}}}
        ov = deep_merge(deep_merge(ov, self.overrides), extra or {})
        self.settings = load_settings(self.environment, overrides=ov)
        self.svc = WatcherService(self.settings, endpoint=KubeEndpoint(server=self.srv.url), metrics=Metrics(True))
        return self.svc

    async def settle(self, n, timeout=10):
        await self.sink.state.wait_for(n, timeout)
        await asyncio.sleep(0.05)
        await self.svc.notifier.drain(5)

    def delivered(self):
        return [(p["uid"], p["event_type"], p["status"]["phase"]) for p in self.sink.state.payloads()]

    async def __aexit__(self, *exc):
        if getattr(self, "svc", None) is not None:
            self.svc.stop()
            await self.svc.shutdown()
        await self.sink.stop()
        await self.srv.stop()


def lifecycle_apply(st, n_pods):
    evs = []
    for _ in range(n_pods):
        for et, obj in st.factory.lifecycle():
            st.srv.apply(et, obj)
            evs.append((obj["metadata"]["uid"], et))
    return evs


def assert_exactly_once(delivered, expected):
    assert collections.Counter((u, t) for u, t, _ in delivered) == collections.Counter(expected)


def test_resume_after_connection_drop_no_loss_no_dup():
    async def body():
        async with Stack() as st:
            svc = st.service()
            await svc.start()
            first = lifecycle_apply(st, 5)
            await st.settle(len(first))
            st.srv.drop_connections()  # simulated API-server restart, history kept
            second = lifecycle_apply(st, 5)
            await st.settle(len(first) + len(second))
            assert_exactly_once(st.delivered(), first + second)
            assert svc.metrics.c["relists"] == 1  # only the initial list
            assert svc.metrics.c["expired_410"] == 0

    run(body())


@pytest.mark.parametrize("as_http_status", [False, True])
def test_410_relists_and_diffs_against_cache(as_http_status):
    async def body():
        async with Stack(server_kwargs={"expired_as_http_status": as_http_status}) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            keep = [st.srv.create(f.running(f.new_pod())) for _ in range(3)]
            doomed = st.srv.create(f.running(f.new_pod()))
            changing = st.srv.create(f.running(f.new_pod()))
            await st.settle(5)
            # while the watch is down: etcd compacts past our resourceVersion
            st.srv.drop_connections()
            st.srv.delete("default" if False else doomed["metadata"]["namespace"], doomed["metadata"]["name"])
            st.srv.update(f.terminated(changing))
            newcomer = st.srv.create(f.running(f.new_pod()))
            st.srv.compact()
            st.srv.expire_watches()
            await st.settle(8)
            got = st.delivered()
            assert len(got) == 8
            tail = {(u, t) for u, t, _ in got[5:]}
            assert tail == {(doomed["metadata"]["uid"], "DELETED"), (changing["metadata"]["uid"], "MODIFIED"),
                            (newcomer["metadata"]["uid"], "ADDED")}
            assert svc.metrics.c["expired_410"] >= 1 and svc.metrics.c["relists"] == 2
            # unchanged pods were not re-notified
            assert [u for u, _, _ in got].count(keep[0]["metadata"]["uid"]) == 1

    run(body())


@pytest.mark.parametrize("as_http_status", [False, True])
def test_repeated_410_relists_back_off(as_http_status):
    """An API server that answers every watch with 410 (a watch cache lagging
    behind etcd) must not be LIST-stormed: consecutive relists that make no
    progress wait exponentially longer (reflector.run, expired_backoff)."""
    async def body():
        async with Stack(server_kwargs={"expired_as_http_status": as_http_status}) as st:
            f = st.factory
            st.srv.create(f.running(f.new_pod()))
            svc = st.service({"watcher": {"retry": {"delay_seconds": 0.1, "multiplier": 2.0,
                                                    "max_delay_seconds": 30, "jitter": 0}}})
            st.srv.expire_every_watch = True
            await svc.start()
            t0 = time.monotonic()
            await asyncio.sleep(3.0)
            elapsed = time.monotonic() - t0
            lists = [t for m, t in st.srv.requests if t.startswith("/api/v1/pods") and "watch=" not in t]
            # delays 0.1, 0.2, 0.4, 0.8, 1.6 s: at most 1 + log2(elapsed / 0.1 + 1) relists
            assert 3 <= len(lists) <= 2 + math.log2(elapsed / 0.1 + 1), (len(lists), elapsed)
            assert svc.metrics.c["expired_relist_backoffs"] >= len(lists) - 2
            # the pod was notified exactly once: relists diff against the cache
            await svc.notifier.drain(5)
            assert len(st.sink.state.payloads()) == 1
            # progress resets the backoff: a healthy watch after the storm resumes at once
            st.srv.expire_every_watch = False
            await asyncio.sleep(2.0)
            st.srv.create(f.running(f.new_pod()))
            await st.settle(2, timeout=10)

    run(body())


def test_bookmark_advances_resume_point():
    async def body():
        async with Stack() as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            st.srv.create(f.new_pod())
            await st.settle(1)
            # traffic the watcher does not see (other scope) moves the RV on; a bookmark reports it
            st.srv.rv += 500
            st.srv.emit_bookmark()
            await asyncio.sleep(0.1)
            rv = svc.reflectors[0].rv
            assert rv == str(st.srv.rv)
            assert svc.metrics.c["bookmarks"] >= 1
            st.srv.compact()  # history before the bookmark is gone; resume must not 410
            st.srv.drop_connections()
            st.srv.create(f.new_pod())
            await st.settle(2)
            assert svc.metrics.c["expired_410"] == 0

    run(body())


def test_server_timeout_seconds_resumes():
    async def body():
        async with Stack(overrides={"watcher": {"watch_timeout_seconds": 1}}) as st:
            svc = st.service()
            await svc.start()
            await asyncio.sleep(1.4)  # first watch ends server-side
            evs = lifecycle_apply(st, 2)
            await st.settle(len(evs))
            assert_exactly_once(st.delivered(), evs)
            assert svc.metrics.c["watch_restarts"] >= 1

    run(body())


def test_transient_api_errors_retry():
    async def body():
        async with Stack() as st:
            st.srv.fail_requests(3, 500, "/api/v1/pods")
            svc = st.service()
            await svc.start()
            evs = lifecycle_apply(st, 1)
            await st.settle(len(evs))
            assert_exactly_once(st.delivered(), evs)

    run(body())


def test_retry_budget_exhausted_is_fatal():
    async def body():
        async with Stack(overrides={"watcher": {"retry": {"max_attempts": 2}}}) as st:
            svc = st.service()
            await svc.start()
            st.srv.fail_requests(50, 503, "/api/v1/pods")
            st.srv.drop_connections()
            with pytest.raises(WatchFailed):
                await asyncio.wait_for(svc.wait(), 10)

    run(body())


def test_parse_retry_after():
    from k8s_watcher_amd.kube.api import parse_retry_after
    assert parse_retry_after("1") == 1.0
    assert parse_retry_after(" 2.5 ") == 2.5
    assert parse_retry_after("9999") == 300.0  # capped
    for bad in (None, "", "-1", "nan", "Wed, 21 Oct 2015 07:28:00 GMT"):
        assert parse_retry_after(bad) is None


def test_429_honours_retry_after_without_spending_retry_budget():
    # API Priority and Fairness answers 429 + Retry-After: the watcher waits
    # as asked and does not exit after max_attempts throttled requests
    async def body():
        async with Stack() as st:
            svc = st.service({"watcher": {"retry": {"delay_seconds": 0.01, "max_attempts": 2}}})
            await svc.start()
            st.srv.fail_requests(4, 429, "/api/v1/pods", retry_after=0.15)
            t0 = time.monotonic()
            st.srv.drop_connections()
            evs = lifecycle_apply(st, 2)
            await st.settle(len(evs))
            assert_exactly_once(st.delivered(), evs)
            assert time.monotonic() - t0 >= 4 * 0.15 * 0.9  # waited Retry-After, not the 10 ms backoff
            assert svc.metrics.c["api_throttled"] == 4
            assert svc.metrics.c["retry_after_waits"] == 4
            assert not any(t.done() for t in svc._tasks)

    run(body())


def test_retry_after_on_5xx_counts_as_failure_but_waits():
    async def body():
        async with Stack() as st:
            svc = st.service({"watcher": {"retry": {"delay_seconds": 0.01, "max_attempts": 5}}})
            await svc.start()
            st.srv.fail_requests(2, 503, "/api/v1/pods", retry_after=0.2)
            t0 = time.monotonic()
            st.srv.drop_connections()
            evs = lifecycle_apply(st, 1)
            await st.settle(len(evs))
            assert time.monotonic() - t0 >= 2 * 0.2 * 0.9
            assert svc.metrics.c["retry_after_waits"] == 2
            assert svc.metrics.c["api_throttled"] == 0

    run(body())


def test_expired_list_continue_falls_back_to_one_unpaginated_list():
    # a continue token that outlived etcd compaction (410 mid-pagination):
    # the state is taken in one LIST without limit, each pod notified once
    async def body():
        async with Stack(overrides={"watcher": {"list_page_size": 2}}) as st:
            f = st.factory
            pods = [st.srv.create(f.running(f.new_pod())) for _ in range(7)]
            st.srv.expire_continues = 1
            svc = st.service()
            await svc.start()
            await st.settle(7)
            got = st.delivered()
            assert sorted(u for u, _, _ in got) == sorted(p["metadata"]["uid"] for p in pods)
            assert {t for _, t, _ in got} == {"ADDED"}
            assert svc.metrics.c["list_continue_expired"] == 1
            assert svc.metrics.c["relists"] == 1
            lists = [t for m, t in st.srv.requests if t.startswith("/api/v1/pods") and "watch=" not in t]
            assert "limit=2" in lists[0] and "continue=" in lists[1] and "limit=" not in lists[2]
            # and the watch resumes from the full list's resourceVersion
            evs = lifecycle_apply(st, 1)
            await st.settle(7 + len(evs))

    run(body())


def test_fake_apiserver_expires_continue_after_compaction():
    import json as _json
    import urllib.request

    async def body():
        srv = FakeApiServer()
        await srv.start()
        f = PodFactory(seed=3)
        for _ in range(3):
            srv.create(f.new_pod())
        loop = asyncio.get_running_loop()

        def get(url):
            try:
                with urllib.request.urlopen(url) as r:
                    return r.status, _json.loads(r.read())
            except urllib.error.HTTPError as e:
                return e.code, _json.loads(e.read())

        st1, page = await loop.run_in_executor(None, get, srv.url + "/api/v1/pods?limit=1")
        tok = page["metadata"]["continue"]
        st2, _ = await loop.run_in_executor(None, get, srv.url + "/api/v1/pods?limit=1&continue=" + tok)
        srv.create(f.new_pod())
        srv.compact()
        st3, err = await loop.run_in_executor(None, get, srv.url + "/api/v1/pods?limit=1&continue=" + tok)
        await srv.stop()
        return st1, st2, st3, err

    st1, st2, st3, err = run(body())
    assert (st1, st2, st3) == (200, 200, 410) and err["reason"] == "Expired"


def test_short_watches_back_off_without_failing():
    # a proxy that ends every watch at once: reconnects are paced by the
    # backoff (no hot loop) and do not spend the failure budget
    async def body():
        async with Stack() as st:
            st.srv.hang_up_watches(4)
            svc = st.service({"watcher": {"retry": {"delay_seconds": 0.05, "max_attempts": 2}}})
            t0 = time.monotonic()
            await svc.start()
            evs = lifecycle_apply(st, 2)
            await st.settle(len(evs))
            assert_exactly_once(st.delivered(), evs)
            assert svc.metrics.c["short_watches"] == 4
            assert time.monotonic() - t0 >= 0.05 * 4 * 0.5  # backed off between reconnects
            watches = [t for m, t in st.srv.requests if "watch=" in t]
            assert len(watches) == 5
            assert not any(t.done() for t in svc._tasks)  # the watch did not give up

    run(body())


def test_checkpoint_restart_exactly_once(tmp_path):
    ck = str(tmp_path / "ckpt.json")

    async def body():
        async with Stack(overrides={"watcher": {"checkpoint": {"path": ck, "interval_seconds": 0.2}}}) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            pods = [st.srv.create(f.running(f.new_pod())) for _ in range(4)]
            await st.settle(4)
            svc.stop()
            await svc.shutdown()
            # watcher down: changes happen
            st.srv.update(f.terminated(pods[0]))
            st.srv.delete(pods[1]["metadata"]["namespace"], pods[1]["metadata"]["name"])
            late = st.srv.create(f.running(f.new_pod()))
            svc2 = st.service()
            await svc2.start()
            await st.settle(7)
            got = st.delivered()
            assert len(got) == 7, got
            assert {(u, t) for u, t, _ in got[4:]} == {
                (pods[0]["metadata"]["uid"], "MODIFIED"), (pods[1]["metadata"]["uid"], "DELETED"),
                (late["metadata"]["uid"], "ADDED")}
            assert svc2.metrics.c["relists"] == 0  # resumed straight from the checkpointed RV

    run(body())


def test_native_checkpoint_carries_owed_notifications(tmp_path):
    """Format 2 (native engine + notifier core) is a consistent cut taken
    without pausing the watch or draining the notifier: notifications
    clusterapi has not acknowledged are stored in the checkpoint and re-sent
    first after a crash — none lost, none of the acknowledged ones repeated."""
    ck = str(tmp_path / "ckpt.bin")

    async def body():
        ov = {"watcher": {"checkpoint": {"path": ck, "interval_seconds": 3600}},
              "clusterapi": {"retry": {"delay_seconds": 30, "max_attempts": 5}}}
        async with Stack(overrides=ov) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            acked = [st.srv.create(f.running(f.new_pod())) for _ in range(3)]
            await st.settle(3)
            st.sink.state.down = True  # clusterapi answers 503: the next ones stay owed (retry in 30 s)
            owed = [st.srv.create(f.running(f.new_pod())) for _ in range(5)]
            for _ in range(200):
                if svc.metrics.c["notify_retried"] >= 5:
                    break
                await asyncio.sleep(0.01)
            assert svc.notifier.outstanding() == 5
            assert await svc.checkpoint_now()  # no drain: returns with 5 still owed
            assert svc.last_checkpoint["checkpoint_owed"] == 5
            assert svc.last_checkpoint["checkpoint_pods"] == 8
            with open(ck, "rb") as fh:
                assert fh.read(8) == b"KWCKPT02"
            # crash: no final checkpoint, the owed requests die with the process
            svc.stop()
            await svc.shutdown(drain_timeout=0, checkpoint=False)
            st.sink.state.down = False
            svc2 = st.service()
            await svc2.start()
            await st.settle(8)
            got = st.delivered()
            assert sorted(u for u, _, _ in got) == sorted(p["metadata"]["uid"] for p in acked + owed)
            assert svc2.metrics.c["checkpoint_owed_resent"] == 5
            assert svc2.metrics.c["relists"] == 0  # resumed from the checkpointed RV

    run(body())


def test_checkpoint_restart_after_compaction_diffs(tmp_path):
    ck = str(tmp_path / "ckpt.json")

    async def body():
        async with Stack(overrides={"watcher": {"checkpoint": {"path": ck}}}) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            pods = [st.srv.create(f.running(f.new_pod())) for _ in range(4)]
            await st.settle(4)
            svc.stop()
            await svc.shutdown()
            st.srv.update(f.terminated(pods[2]))
            st.srv.compact()
            svc2 = st.service()
            await svc2.start()
            await st.settle(5)
            got = st.delivered()
            assert len(got) == 5
            assert got[-1][:2] == (pods[2]["metadata"]["uid"], "MODIFIED")
            assert svc2.metrics.c["expired_410"] == 1

    run(body())


def test_notify_on_phase_change():
    async def body():
        async with Stack(overrides={"watcher": {"notify_on": "phase_change"}}) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            p = st.srv.create(f.new_pod())          # ADDED Pending        -> notify
            p = st.srv.update(f.scheduled(p))       # Pending -> Pending   -> suppressed
            p = st.srv.update(f.running(p))         # Running              -> notify
            p = st.srv.update(f.running(p))         # Running -> Running   -> suppressed
            st.srv.delete(p["metadata"]["namespace"], p["metadata"]["name"])  # DELETED -> notify
            await st.settle(3)
            assert [t for _, t, _ in st.delivered()] == ["ADDED", "MODIFIED", "DELETED"]
            assert svc.metrics.c["events_unchanged"] == 2

    run(body())


def test_initial_list_skip():
    async def body():
        async with Stack(overrides={"watcher": {"initial_list": "skip"}}) as st:
            f = st.factory
            for _ in range(3):
                st.srv.create(f.running(f.new_pod()))
            svc = st.service()
            await svc.start()
            new = st.srv.create(f.new_pod())
            await st.settle(1)
            assert [u for u, _, _ in st.delivered()] == [new["metadata"]["uid"]]
            assert len(svc.pipeline.cache) == 4

    run(body())


def test_server_side_namespace_scope():
    async def body():
        async with Stack(environment="development",
                         overrides={"watcher": {"namespace_scope": "server"}}) as st:
            f = st.factory
            svc = st.service()
            await svc.start()
            assert len(svc.reflectors) == 2
            pods = [st.srv.create(f.new_pod()) for _ in range(6)]  # default/kube-system/batch round-robin
            wanted = [p["metadata"]["uid"] for p in pods if p["metadata"]["namespace"] != "batch"]
            await st.settle(len(wanted))
            assert sorted(u for u, _, _ in st.delivered()) == sorted(wanted)
            # the API server itself never sent the batch pods
            assert svc.metrics.c["events_filtered_namespace"] == 0
            assert any("/namespaces/default/pods" in t for _, t in st.srv.requests)

    run(body())


def test_401_rereads_rotated_token_file(tmp_path):
    # a rotated service-account / kubeconfig tokenFile: the 401 makes the
    # watcher re-read the file at once instead of waiting for the 60 s period
    from k8s_watcher_amd.kube.kubeconfig import load_kube_config

    async def body():
        async with Stack(server_kwargs={"token": "one"}) as st:
            tok = tmp_path / "tok"
            tok.write_text("one\n")
            cfg = tmp_path / "cfg"
            cfg.write_text(f"""
current-context: x
clusters: [{{name: c, cluster: {{server: "{st.srv.url}"}}}}]
contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
users: [{{name: u, user: {{tokenFile: tok}}}}]
""")
            st.service()
            svc = WatcherService(st.settings, endpoint=load_kube_config(str(cfg)), metrics=Metrics(True))
            st.svc = svc
            await svc.start()
            first = lifecycle_apply(st, 1)
            await st.settle(len(first))
            st.srv.token = "two"
            tok.write_text("two\n")
            st.srv.drop_connections()
            second = lifecycle_apply(st, 1)
            await st.settle(len(first) + len(second))
            assert_exactly_once(st.delivered(), first + second)
            assert svc.metrics.c["auth_refreshes"] >= 1

    run(body())


def test_invalidate_credentials_static_and_exec(tmp_path):
    import sys

    from k8s_watcher_amd.kube.kubeconfig import load_kube_config
    counter = tmp_path / "n"
    counter.write_text("0")
    plugin = tmp_path / "plugin.py"
    plugin.write_text(
        "import json,pathlib\np=pathlib.Path(%r)\nn=int(p.read_text())+1\np.write_text(str(n))\n"
        "print(json.dumps({'apiVersion':'client.authentication.k8s.io/v1beta1','kind':'ExecCredential',"
        "'status':{'token':'t%%d' %% n}}))\n" % str(counter))
    cfg = tmp_path / "cfg"
    cfg.write_text(f"""
current-context: x
clusters: [{{name: c, cluster: {{server: "http://h"}}}}]
contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
users:
- name: u
  user:
    exec: {{apiVersion: client.authentication.k8s.io/v1beta1, command: "{sys.executable}", args: ["{plugin}"]}}
""")
    ep = load_kube_config(str(cfg))
    assert ep.auth_headers() == {"Authorization": "Bearer t1"}
    assert ep.auth_headers() == {"Authorization": "Bearer t1"}  # cached
    assert ep.invalidate_credentials()  # re-runs the plugin on a thread, old token meanwhile
    ep.header_provider.__self__.wait_refreshed()
    assert ep.auth_headers() == {"Authorization": "Bearer t2"}
    assert not KubeEndpoint(server="http://h", static_headers={"Authorization": "Bearer s"}).invalidate_credentials()


def _exec_kubeconfig(tmp_path, server_url, script):
    import sys
    plugin = tmp_path / "plugin.py"
    plugin.write_text(script)
    cfg = tmp_path / "cfg"
    cfg.write_text(f"""
current-context: x
clusters: [{{name: c, cluster: {{server: "{server_url}"}}}}]
contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
users:
- name: u
  user:
    exec: {{apiVersion: client.authentication.k8s.io/v1beta1, command: "{sys.executable}", args: ["{plugin}"]}}
""")
    return cfg


def test_401_reruns_exec_plugin_off_the_event_loop(tmp_path):
    """A 401 re-runs the exec credential plugin on a thread: the event loop
    keeps running while the (slow) plugin works, and a failing plugin is a
    retried watch failure, not the end of the watcher."""
    from k8s_watcher_amd.kube.kubeconfig import load_kube_config
    state = tmp_path / "state"
    state.write_text("0 ok")
    script = ("import json, pathlib, sys, time\n"
              "p = pathlib.Path(%r)\n"
              "n, mode = p.read_text().split()\n"
              "n = int(n) + 1\n"
              "p.write_text(f'{n} {mode}')\n"
              "if n > 1: time.sleep(0.6)\n"
              "if mode == 'fail': sys.exit(3)\n"
              "print(json.dumps({'apiVersion': 'client.authentication.k8s.io/v1beta1', 'kind': 'ExecCredential',"
              " 'status': {'token': 'tok-%%s' %% (1 if n == 1 else 2)}}))\n") % str(state)

    async def body():
        async with Stack(server_kwargs={"token": "tok-1"}) as st:
            cfg = _exec_kubeconfig(tmp_path, st.srv.url, script)
            st.service({"watcher": {"retry": {"delay_seconds": 0.05, "max_attempts": 0}}})
            svc = WatcherService(st.settings, endpoint=load_kube_config(str(cfg)), metrics=Metrics(True))
            st.svc = svc
            await svc.start()
            first = lifecycle_apply(st, 1)
            await st.settle(len(first))
            # the token is revoked and the plugin starts failing for a while
            state.write_text(state.read_text().split()[0] + " fail")
            st.srv.token = "tok-2"
            st.srv.drop_connections()
            gaps, last = [], time.monotonic()
            t_end = time.monotonic() + 2.0
            while time.monotonic() < t_end:
                await asyncio.sleep(0.01)
                now = time.monotonic()
                gaps.append(now - last)
                last = now
            # the plugin sleeps 0.6 s per run: none of it was spent on the loop
            assert max(gaps) < 0.3, max(gaps)
            assert not any(t.done() for t in svc._tasks)  # the reflector is still retrying
            state.write_text(state.read_text().split()[0] + " ok")
            second = lifecycle_apply(st, 1)
            await st.settle(len(first) + len(second), timeout=20)
            assert_exactly_once(st.delivered(), first + second)
            assert svc.metrics.c["auth_refreshes"] >= 2

    run(body(), timeout=60)


@pytest.mark.parametrize("engine", ["python", "native"])
def test_relist_page_over_4mib(engine):
    """A LIST page of 4 MiB or more is read into an anonymous mapping
    (net/http.py _body_buffer); the Python decoder's json.loads must take it
    (it only takes str/bytes/bytearray), or the scope never syncs."""
    async def body():
        async with Stack() as st:
            f = st.factory
            big = "x" * 20000
            uids = []
            for _ in range(240):  # 240 x ~24 KB: one ~5.5 MiB page
                pod = f.running(f.new_pod())
                pod["metadata"].setdefault("annotations", {})["blob"] = big
                uids.append(st.srv.create(pod)["metadata"]["uid"])
            svc = st.service({"watcher": {"engine": engine, "list_page_size": 500},
                              "kubernetes": {"compression": False}})  # identity: the body is the mapping
            await svc.start()
            await st.settle(len(uids))
            assert sorted(u for u, _, _ in st.delivered()) == sorted(uids)

    run(body())
