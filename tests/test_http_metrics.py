"""HTTP/1.1 response parser edge cases and the metrics endpoint."""

import pytest

from conftest import run
from k8s_watcher_amd.metrics import LatencyHistogram, Metrics, start_metrics_server
from k8s_watcher_amd.net.http import HttpClient, HttpError, ResponseParser


def parse_all(data, step=None, **reset):
    p = ResponseParser()
    p.reset(**reset)
    done = []
    p.on_complete = lambda q: done.append((q.status, q.headers, q.body()))
    if step is None:
        rest = p.feed(data)
    else:
        rest = b""
        for i in range(0, len(data), step):
            rest = p.feed(data[i:i + step])
    return p, done, rest


def test_content_length_and_keepalive():
    p, done, rest = parse_all(b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\nX-A: 1\r\n\r\nhelloEXTRA")
    assert done[0][0] == 200 and done[0][2] == b"hello" and rest == b"EXTRA"
    assert done[0][1]["x-a"] == "1" and p.keep_alive


@pytest.mark.parametrize("step", [None, 1, 3, 7])
def test_chunked_with_extensions_and_trailers(step):
    data = (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n"
            b"5;ext=1\r\nhello\r\n6\r\n world\r\n0\r\nTrailer: x\r\n\r\n")
    p, done, _ = parse_all(data, step)
    assert done[0][2] == b"hello world"


def test_connection_close_and_http10():
    p, done, _ = parse_all(b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 0\r\n\r\n")
    assert not p.keep_alive and done
    p, done, _ = parse_all(b"HTTP/1.0 200 OK\r\nContent-Length: 0\r\n\r\n")
    assert not p.keep_alive


def test_until_close_body():
    p, done, _ = parse_all(b"HTTP/1.1 200 OK\r\n\r\nabc")
    assert not done
    p.feed(b"def")
    p.feed_eof()
    assert done[0][2] == b"abcdef"


def test_no_body_statuses_and_head():
    _, done, rest = parse_all(b"HTTP/1.1 204 No Content\r\n\r\nHTTP/1.1")
    assert done[0][0] == 204 and rest == b"HTTP/1.1"
    _, done, _ = parse_all(b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\n", no_body=True)
    assert done[0][2] == b""


def test_raw_chunked_passthrough():
    got = []
    p = ResponseParser()
    p.reset(raw_chunked=True)
    p.on_body = got.append
    p.feed(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n")
    p.feed(b"0\r\n\r\n")
    assert b"".join(got) == b"3\r\nabc\r\n0\r\n\r\n" and p.state == ResponseParser.RAW


def test_malformed_raises():
    with pytest.raises(HttpError):
        parse_all(b"NOTHTTP 200 OK\r\n\r\n")
    with pytest.raises(HttpError):
        parse_all(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n")
    p = ResponseParser()
    p.feed(b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\n\r\nabc")
    with pytest.raises(HttpError):
        p.feed_eof()


def test_latency_histogram_percentiles():
    h = LatencyHistogram(record_samples=True)
    for v in range(1, 101):
        h.observe_ns(v * 1000)
    assert h.percentile_ns(50) == 50_000 and h.percentile_ns(99) == 99_000
    h2 = LatencyHistogram()
    for v in range(1, 101):
        h2.observe_ns(v * 1000)
    assert 50_000 <= h2.percentile_ns(50) <= 60_000  # bucket upper bound


def test_metrics_server_endpoints():
    async def body():
        m = Metrics()
        m.inc("events_received", 7)
        m.latency.observe_ns(2_000_000)
        m.gauges["cached_pods"] = lambda: 3.0
        srv = await start_metrics_server(m, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = HttpClient(f"http://127.0.0.1:{port}")
        metrics = (await c.request("GET", "/metrics")).text()
        ready0 = (await c.request("GET", "/readyz")).status
        m.ready = True
        ready1 = (await c.request("GET", "/readyz")).status
        health = (await c.request("GET", "/healthz")).status
        missing = (await c.request("GET", "/nope")).status
        await c.close()
        srv.close()
        return metrics, ready0, ready1, health, missing

    metrics, r0, r1, h, nf = run(body())
    assert "k8s_watcher_events_received_total 7" in metrics
    assert "k8s_watcher_cached_pods 3.0" in metrics
    assert 'k8s_watcher_notify_latency_seconds_bucket{le="+Inf"} 1' in metrics
    assert (r0, r1, h, nf) == (503, 200, 200, 404)


def test_closed_streams_leave_the_client():
    """Every watch reconnect used to leave its protocol (and its read buffer,
    up to watcher.watch_read_bytes = 4 MiB) in HttpClient._all: a slow leak
    per reconnect that the long soak exposed. Closed connections, stream or
    pooled, must drop out of the client's books and free their buffer."""
    import asyncio

    async def body():
        async def handle(reader, writer):
            await reader.readuntil(b"\r\n\r\n")
            writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n")
            await writer.drain()
            await reader.read()  # until the client hangs up
            writer.close()

        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = HttpClient(f"http://127.0.0.1:{port}")
        got, protos = [], []
        for _ in range(5):
            stream, err = await c.stream("GET", "/watch", lambda d, _ns: got.append(bytes(d)),
                                         read_size=4 << 20, zero_copy=True)
            assert err is None
            protos.append(stream._proto)
            stream.close()
            await asyncio.wait_for(stream.finished, 5)
        await asyncio.sleep(0)
        left = len(c._all)
        await c.close()
        srv.close()
        return got, left, [p._rbuf for p in protos]

    got, left, bufs = run(body())
    assert len(got) == 5 and left == 0
    assert all(b is None for b in bufs)

def test_debug_memory_endpoint_only_when_enabled():
    import tracemalloc

    async def body():
        m = Metrics()
        plain = await start_metrics_server(m, "127.0.0.1", 0)
        dbg = await start_metrics_server(m, "127.0.0.1", 0, debug=True)
        out = []
        for srv in (plain, dbg):
            c = HttpClient(f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}")
            r = await c.request("GET", "/debug/memory")
            out.append((r.status, r.json() if r.status == 200 else None))
            await c.close()
            srv.close()
        return out

    tracemalloc.start()
    try:
        (s0, _), (s1, doc) = run(body())
    finally:
        tracemalloc.stop()
    assert s0 == 404 and s1 == 200
    assert doc["gc_objects"] > 1000 and "builtins.dict" in doc["types"]
    assert doc["garbage_collected"] >= 0  # counted after a collection: live objects only
    assert doc["tracemalloc"]["traced_bytes"] > 0 and doc["tracemalloc"]["top"]


def test_memory_census_counts_frozen_objects_and_keeps_them_frozen():
    """With watcher.gc_freeze the census thaws the frozen set to count it (and
    to collect any of it that became garbage), then freezes what is live again."""
    import gc
    from k8s_watcher_amd.metrics import memory_census

    class Marker:
        pass

    keep = [Marker() for _ in range(50)]
    gc.freeze()
    try:
        doc = memory_census(top=1000)
        assert doc["frozen_before"] > 0
        assert doc["types"].get(f"{Marker.__module__}.{Marker.__qualname__}", 0) >= 50
        assert gc.get_freeze_count() > 0
    finally:
        gc.unfreeze()
    del keep
