"""clusterapi notifier pool: success codes, retries,
timeouts, per-pod ordering, superseding, coalescing and backpressure."""

import asyncio
import random
import time

import pytest

from conftest import run
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.models.payload import build_core
from k8s_watcher_amd.parallel.native_notifier import NativeNotifierPool
from k8s_watcher_amd.parallel.notifier import NotifierPool
from k8s_watcher_amd.testing.stub_sink import StubSink
from k8s_watcher_amd.utils.config import ClusterApiSettings, NotifierPoolSettings, RetryPolicy

TS = "2025-01-01T00:00:00.000001"


def settings(url, **kw):
    pool = NotifierPoolSettings(connections=kw.pop("connections", 4), pipeline_depth=kw.pop("depth", 1),
                                queue_size=kw.pop("queue_size", 1000), coalesce=kw.pop("coalesce", False),
                                max_queued_bytes=kw.pop("max_bytes", 64 << 20))
    retry = RetryPolicy(kw.pop("attempts", 3), kw.pop("delay", 0.01), 2.0, 1.0, 0.0)
    return ClusterApiSettings(base_url=url, pool=pool, retry=retry, **kw)


def core(uid, phase="Running", name=None):
    pod = {"metadata": {"name": name or f"pod-{uid}", "namespace": "default", "uid": uid},
           "status": {"phase": phase}}
    return build_core(pod, "production")


def _threaded_native(s, metrics=None, **kw):
    """The native core serving its sockets on its own thread (``clusterapi.pool.io_thread``)."""
    import dataclasses
    return NativeNotifierPool(dataclasses.replace(s, pool=dataclasses.replace(s.pool, io_thread="on")),
                              metrics, **kw)


@pytest.fixture(params=["python", "native", "native-io-thread"])
def pool_cls(request):
    """Every test runs against the asyncio pool and the native-core pool, the
    latter driven from the event loop (default) and on its own I/O thread."""
    return {"python": NotifierPool, "native": NativeNotifierPool, "native-io-thread": _threaded_native}[request.param]


async def with_pool(cls, sink_kwargs=None, **kw):
    sink = StubSink(**(sink_kwargs or {}))
    await sink.start()
    m = Metrics(record_samples=True)
    pool = cls(settings(sink.url, **kw), m)
    return sink, pool, m


async def close(sink, pool):
    await pool.close()
    await sink.stop()


def test_delivers_with_headers_and_latency(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls, api_key="k3y")
        for i in range(20):
            pool.submit(f"u{i}", "ADDED", "default", f"p{i}", core(f"u{i}"), 0, TS)
        pool.flush()
        assert await pool.drain(5)
        heads = list(sink.state.heads)
        got = sink.state.payloads()
        await close(sink, pool)
        return heads, got, m

    heads, got, m = run(body())
    assert len(got) == 20 and m.c["notify_delivered"] == 20
    assert all(b"Authorization: Bearer k3y" in h for h in heads)
    assert all(h.startswith(b"POST /api/pods/update HTTP/1.1") for h in heads)
    assert got[0]["event_timestamp"] == TS and got[0]["event_type"] == "ADDED"
    assert m.latency.n == 20


@pytest.mark.parametrize("status", [201, 204])
def test_any_2xx_is_success(pool_cls, status):
    async def body():
        sink, pool, m = await with_pool(pool_cls, {"success_status": status})
        pool.submit("u", "ADDED", "default", "p", core("u"), 0, TS)
        pool.flush()
        await pool.drain(5)
        await close(sink, pool)
        return m

    m = run(body())
    assert m.c["notify_delivered"] == 1 and m.c["notify_failed"] == 0


def test_5xx_retried_4xx_not(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls)
        sink.state.fail_next = [500, 503]
        pool.submit("a", "ADDED", "default", "a", core("a"), 0, TS)
        pool.flush()
        await pool.drain(5)
        sink.state.fail_next = [400]
        pool.submit("b", "ADDED", "default", "b", core("b"), 0, TS)
        pool.flush()
        await pool.drain(5)
        names = [p["name"] for p in sink.state.payloads()]
        await close(sink, pool)
        return names, m

    names, m = run(body())
    assert names == ["pod-a"]
    assert m.c["notify_retried"] == 2 and m.c["notify_failed"] == 1 and m.c["notify_delivered"] == 1


def test_retry_after_delays_the_retry(pool_cls):
    # 429/503 with Retry-After: the retry waits what clusterapi asked for,
    # not the 10 ms policy delay
    async def body():
        sink, pool, m = await with_pool(pool_cls, attempts=4)
        sink.state.fail_next = [429, 503]
        sink.state.retry_after = 0.2
        t0 = time.monotonic()
        pool.submit("a", "ADDED", "default", "a", core("a"), 0, TS)
        pool.flush()
        assert await pool.drain(5)
        elapsed = time.monotonic() - t0
        names = [p["name"] for p in sink.state.payloads()]
        await close(sink, pool)
        return names, m, elapsed

    names, m, elapsed = run(body())
    assert names == ["pod-a"]
    assert elapsed >= 2 * 0.2 * 0.9
    assert m.c["notify_retried"] == 2 and m.c["notify_retry_after_waits"] == 2


@pytest.mark.parametrize("native", [False, True])
def test_scanner_reports_retry_after(native):
    from k8s_watcher_amd.net.http import response_scanner
    sc = response_scanner(native)
    out = sc.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n"
                  b"HTTP/1.1 429 Too Many Requests\r\nRetry-After: 3\r\nContent-Length: 2\r\n\r\n{}"
                  b"HTTP/1.1 503 Service Unavailable\r\nretry-after:  0.5 \r\nContent-Length: 0\r\n\r\n"
                  b"HTTP/1.1 503 Service Unavailable\r\nRetry-After: 9999\r\nContent-Length: 0\r\n\r\n"
                  b"HTTP/1.1 503 Service Unavailable\r\nRetry-After: Wed, 21 Oct 2015 07:28:00 GMT\r\n"
                  b"Content-Length: 0\r\n\r\n"
                  b"HTTP/1.1 500 Internal Server Error\r\nContent-Length: 0\r\n\r\n")
    assert out == [200, (429, True, b"{}", 3.0), (503, True, b"", 0.5), (503, True, b"", 300.0),
                   (503, True, b"", -1.0), (500, True, b"", -1.0)]


def test_gives_up_after_max_attempts(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls, {"fail_rate": 1.0}, attempts=3)
        pool.submit("a", "ADDED", "default", "a", core("a"), 0, TS)
        pool.flush()
        assert await pool.drain(5)
        await close(sink, pool)
        return m, sink.state.failed

    m, failed = run(body())
    assert failed == 3 and m.c["notify_failed"] == 1 and m.c["notify_retried"] == 2


def test_timeout_aborts_and_retries(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls, {"latency": 0.6}, timeout=0.2, attempts=2, delay=0.3)
        pool.submit("a", "ADDED", "default", "a", core("a"), 0, TS)
        pool.flush()
        await asyncio.sleep(0.35)
        sink.state.latency = 0.0  # clusterapi recovers
        assert await pool.drain(5)
        await close(sink, pool)
        return m

    m = run(body())
    assert m.c["notify_retried"] == 1 and m.c["notify_delivered"] == 1


def test_stale_retry_is_superseded(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls, connections=1, delay=0.2)
        sink.state.fail_next = [503]
        pool.submit("u", "MODIFIED", "default", "p", core("u", "Running"), 0, TS)
        pool.flush()
        await asyncio.sleep(0.05)  # first attempt failed, retry scheduled in 0.2 s
        pool.submit("u", "MODIFIED", "default", "p", core("u", "Succeeded"), 0, TS)
        pool.flush()
        await pool.drain(5)
        phases = [p["status"]["phase"] for p in sink.state.payloads()]
        await close(sink, pool)
        return phases, m

    phases, m = run(body())
    assert phases == ["Succeeded"]  # the stale Running body never reaches clusterapi
    assert m.c["notify_superseded"] == 1


def test_coalesce_replaces_unsent_body(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls, coalesce=True, connections=1)
        for ph in ("Pending", "Running", "Succeeded"):
            pool.submit("u", "MODIFIED", "default", "p", core("u", ph), 0, TS)
        pool.flush()
        await pool.drain(5)
        phases = [p["status"]["phase"] for p in sink.state.payloads()]
        await close(sink, pool)
        return phases, m

    phases, m = run(body())
    # the connection is not up at submit time, so all three coalesce into one request
    assert phases == ["Succeeded"] and m.c["notify_coalesced"] == 2


@pytest.mark.parametrize("depth", [1, 8])
def test_per_pod_order_under_random_failures(pool_cls, depth):
    rng = random.Random(3)
    order = ["Pending", "Running", "Succeeded"]

    async def body():
        sink, pool, m = await with_pool(pool_cls, {"fail_rate": 0.2, "fail_status": 503, "seed": 5},
                                        connections=4, depth=depth, attempts=8, delay=0.005)
        uids = [f"u{i}" for i in range(40)]
        steps = {u: 0 for u in uids}
        while any(s < 3 for s in steps.values()):
            u = rng.choice([u for u, s in steps.items() if s < 3])
            pool.submit(u, "MODIFIED", "default", u, core(u, order[steps[u]]), 0, TS)
            steps[u] += 1
            if rng.random() < 0.3:
                pool.flush()
                await asyncio.sleep(0)
        pool.flush()
        assert await pool.drain(10)
        got = sink.state.payloads()
        await close(sink, pool)
        return got, m

    got, m = run(body())
    seen = {}
    for p in got:
        idx = order.index(p["status"]["phase"])
        assert idx >= seen.get(p["uid"], -1), "an older state overwrote a newer one"
        seen[p["uid"]] = idx
    assert all(v == 2 for v in seen.values()) and len(seen) == 40  # final state always delivered
    assert m.c["notify_failed"] == 0


def test_backpressure_signals(pool_cls):
    flips = []

    async def body():
        sink = StubSink(latency=0.05)
        await sink.start()
        pool = pool_cls(settings(sink.url, queue_size=8, connections=2), Metrics(),
                            on_saturation=flips.append)
        for i in range(20):
            pool.submit(f"u{i}", "ADDED", "default", "p", core(f"u{i}"), 0, TS)
        pool.flush()
        assert pool.saturated
        await pool.drain(10)
        await close(sink, pool)

    run(body())
    assert flips == [True, False]


def test_backpressure_by_bytes(pool_cls):
    """clusterapi.pool.max_queued_bytes: few but large notifications (pods
    with big annotations) saturate the pool by bytes long before queue_size;
    it releases once both counts are back under half."""
    flips = []

    async def body():
        sink = StubSink(latency=0.05)
        await sink.start()
        pool = pool_cls(settings(sink.url, queue_size=10_000, connections=2, max_bytes=1 << 16), Metrics(),
                        on_saturation=flips.append)
        big = build_core({"metadata": {"name": "p", "namespace": "default", "uid": "u",
                                       "annotations": {"blob": "x" * 20_000}}, "status": {"phase": "Running"}},
                         "production")
        for i in range(5):  # 5 x ~20 KB > 64 KiB, 5 << queue_size
            pool.submit(f"u{i}", "ADDED", "default", "p", big, 0, TS)
        pool.flush()
        assert pool.saturated and pool.outstanding() == 5
        assert pool.outstanding_bytes() >= 5 * 20_000
        await pool.drain(10)
        assert pool.outstanding_bytes() == 0
        await close(sink, pool)

    run(body())
    assert flips == [True, False]


def test_unreachable_sink_then_recovery(pool_cls):
    async def body():
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        m = Metrics()
        pool = pool_cls(settings(f"http://127.0.0.1:{port}", attempts=2, delay=0.01), m)
        pool.submit("a", "ADDED", "default", "a", core("a"), 0, TS)
        pool.flush()
        assert await pool.drain(5)
        failed = m.c["notify_failed"]
        sink = StubSink()
        await sink.start(port=port)
        pool.submit("b", "ADDED", "default", "b", core("b"), 0, TS)
        pool.flush()
        assert await pool.drain(10)
        n = sink.state.count
        await close(sink, pool)
        return failed, n

    failed, n = run(body())
    assert failed == 1 and n == 1


def test_health_check(pool_cls):
    async def body():
        sink, pool, m = await with_pool(pool_cls)
        ok = await pool.health_check()
        await close(sink, pool)
        bad = pool_cls(settings("http://127.0.0.1:1"), Metrics())
        nok = await bad.health_check(timeout=1)
        await bad.close()
        return ok, nok

    assert run(body()) == (True, False)


def test_latency_and_rtt_histograms(pool_cls):
    """Both pools fill the event->ack latency and request->ack RTT histograms
    (the native core buckets them in C++; raw samples only with record_samples)."""
    async def body():
        sink, pool, m = await with_pool(pool_cls, sink_kwargs={"latency": 0.002})
        for i in range(20):
            pool.submit(f"u{i}", "ADDED", "default", f"p{i}", core(f"u{i}"), time.monotonic_ns(), TS)
        pool.flush()
        assert await pool.drain(5)
        assert m.latency.n == 20 and m.rtt.n == 20
        assert len(m.latency.samples) == 20
        assert m.rtt.percentile_ns(50) >= 2e6 and m.latency.total_ns >= m.rtt.total_ns
        text = m.prometheus_text()
        assert 'k8s_watcher_notify_rtt_seconds_count 20' in text
        assert 'k8s_watcher_notify_latency_seconds_count 20' in text
        await close(sink, pool)
    run(body())


def test_rate_limit_paces_requests(pool_cls):
    """clusterapi.rate_limit: a burst goes out at once, the rest at `qps`."""
    async def body():
        sink, pool, m = await with_pool(pool_cls, rate_limit_qps=200.0, rate_limit_burst=10.0, depth=4)
        t0 = time.monotonic()
        for i in range(50):
            pool.submit(f"u{i}", "ADDED", "default", f"p{i}", core(f"u{i}"), 0, TS)
        pool.flush()
        await asyncio.sleep(0.05)
        early = sink.state.count
        assert 10 <= early <= 22  # the burst plus ~10 refilled tokens
        assert await pool.drain(5)
        took = time.monotonic() - t0
        assert sink.state.count == 50 and 0.15 <= took <= 1.5  # 40 beyond the burst at 200/s ~ 0.2 s
        await close(sink, pool)
    run(body())


def test_compat_clients_honour_retry_after():
    """The reference-compatible clients (sync and async) wait the sink's Retry-After."""
    import threading

    from k8s_watcher_amd.notify.clusterapi import AsyncClusterApiClient, ClusterApiClient

    async def body():
        sink = StubSink()
        await sink.start()
        sink.state.retry_after = 0.2
        s = settings(sink.url, attempts=3)
        sink.state.fail_next = [429]
        ac = AsyncClusterApiClient.from_settings(s)
        t0 = time.monotonic()
        assert await ac.update_pod_status({"name": "a", "uid": "1"})
        t_async = time.monotonic() - t0
        sink.state.fail_next = [503]
        sc = ClusterApiClient.from_settings(s)
        out = {}

        def post():
            t1 = time.monotonic()
            out["ok"] = sc.update_pod_status({"name": "b", "uid": "2"})
            out["t"] = time.monotonic() - t1

        t = threading.Thread(target=post)
        t.start()
        while t.is_alive():
            await asyncio.sleep(0.01)
        assert out["ok"] and sink.state.count == 2
        await sink.stop()
        return t_async, out["t"]

    t_async, t_sync = run(body())
    assert t_async >= 0.18 and t_sync >= 0.18


def test_io_thread_auto_switches_both_ways_without_loss(monkeypatch):
    """``clusterapi.pool.io_thread: auto``: a burst above ``IO_THREAD_ON_RATE``
    hands the sockets to the I/O thread, a quiet spell hands them back; every
    notification is delivered exactly once across the switches, per pod in order."""
    import dataclasses
    monkeypatch.setattr(NativeNotifierPool, "IO_THREAD_ON_RATE", 500.0)
    monkeypatch.setattr(NativeNotifierPool, "IO_THREAD_OFF_RATE", 100.0)

    async def body():
        sink = StubSink(latency=0.002)  # responses lag: requests are in flight while switching
        await sink.start()
        m = Metrics(record_samples=True)
        s = settings(sink.url, depth=4)
        s = dataclasses.replace(s, pool=dataclasses.replace(s.pool, io_thread="auto"))
        pool = NativeNotifierPool(s, m)
        sent = []
        modes = []
        for burst in range(3):
            t_end = time.monotonic() + 0.6
            k = 0
            while time.monotonic() < t_end:  # >= 2,000/s for 0.6 s, even on a loaded machine (3 per turn)
                for _ in range(3):
                    uid = f"u{k % 50}"
                    pool.submit(uid, "MODIFIED", "default", f"b{burst}-{k}", core(uid, name=f"b{burst}-{k}"), 0, TS)
                    sent.append((uid, f"b{burst}-{k}"))
                    k += 1
                pool.flush()
                await asyncio.sleep(0.0005)
            modes.append(pool.threaded)
            assert await pool.drain(10)
            await asyncio.sleep(0.5)  # quiet: back to the loop
            modes.append(pool.threaded)
        got = [(p["uid"], p["name"]) for p in sink.state.payloads()]
        await close(sink, pool)
        return sent, got, modes, m

    sent, got, modes, m = run(body(), timeout=60)
    assert True in modes and modes[-1] is False
    assert m.c["notify_io_switches"] >= 2
    assert sorted(got) == sorted(sent) and len(got) == len(set(got))  # exactly once
    by_uid = {}
    for uid, name in got:
        by_uid.setdefault(uid, []).append(name)
    order = {name: i for i, (_u, name) in enumerate(sent)}
    assert all(seq == sorted(seq, key=order.get) for seq in by_uid.values())  # per pod in order


def test_io_thread_auto_hands_back_with_requests_in_flight(monkeypatch):
    """The hand-back to the loop does not wait for a quiet queue: requests the
    thread sent are answered on the loop after the switch, none lost."""
    import dataclasses
    monkeypatch.setattr(NativeNotifierPool, "IO_THREAD_ON_RATE", 500.0)
    monkeypatch.setattr(NativeNotifierPool, "IO_THREAD_OFF_RATE", 100.0)

    async def body():
        sink = StubSink(latency=0.3)  # every response arrives well after the burst ends
        await sink.start()
        m = Metrics(record_samples=True)
        s = settings(sink.url, depth=64, connections=2)
        s = dataclasses.replace(s, pool=dataclasses.replace(s.pool, io_thread="auto"))
        pool = NativeNotifierPool(s, m)
        n = 0
        t_end = time.monotonic() + 0.5
        while time.monotonic() < t_end:  # well above IO_THREAD_ON_RATE even on a loaded machine
            for _ in range(3):
                pool.submit(f"u{n}", "ADDED", "default", f"p{n}", core(f"u{n}"), 0, TS)
                n += 1
            pool.flush()
            await asyncio.sleep(0.001)
        was_threaded = pool.threaded
        for _ in range(100):  # quiet now: back to the loop while responses are still owed
            if not pool.threaded:
                break
            await asyncio.sleep(0.02)
        owed_at_switch = pool.outstanding()
        assert await pool.drain(10)
        got = len(sink.state.payloads())
        await close(sink, pool)
        return n, got, was_threaded, owed_at_switch, m

    n, got, was_threaded, owed, m = run(body(), timeout=60)
    assert was_threaded and m.c["notify_io_switches"] >= 2
    assert owed > 0  # the switch really happened with requests in flight
    assert got == n and m.c["notify_delivered"] == n
