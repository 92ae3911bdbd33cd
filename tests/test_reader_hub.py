"""Native watch reader (``_kwcore.ReaderHub`` + ``net/reader.WatchReaderHub``).

The hub must deliver every byte of every adopted stream, in order per stream,
signal end of stream, stop reading a paused stream (TCP flow control does the
rest), and leave the asyncio transport in charge of the connection's life.
"""

import asyncio
import os
import socket
import time

import pytest

from conftest import run
from k8s_watcher_amd.net.http import HttpClient
from k8s_watcher_amd.net.reader import WatchReaderHub
from k8s_watcher_amd.ops.native import load


def _drain(core, want_bytes, timeout=5.0):
    got, ends = {}, []
    deadline = time.monotonic() + timeout
    while sum(len(v) for v in got.values()) < want_bytes or (want_bytes == 0 and not ends):
        if time.monotonic() > deadline:
            break
        for sid, buf, view, read_ns, err in core.take():
            if view is not None:
                assert read_ns > 0
                got.setdefault(sid, bytearray()).extend(view)
                view.release()
                core.release(buf)
            else:
                ends.append((sid, err))
        time.sleep(0.001)
    return got, ends


@pytest.mark.parametrize("readers", [1, 3])
def test_hub_reads_streams_in_order_and_signals_eof(readers):
    mod = load()
    core = mod.ReaderHub(64 * 1024, 4)
    assert core.set_readers(readers) and len(core.thread_ids()) == readers
    pairs = [socket.socketpair() for _ in range(3)]
    sids = [core.add(os.dup(b.fileno())) for a, b in pairs]
    payload = {sid: os.urandom(300_000) for sid in sids}  # several buffers each
    for (a, _b), sid in zip(pairs, sids):
        a.setblocking(True)
    import threading

    def send(a, data):
        a.sendall(data)
        a.shutdown(socket.SHUT_WR)

    ths = [threading.Thread(target=send, args=(a, payload[sid])) for (a, _b), sid in zip(pairs, sids)]
    for t in ths:
        t.start()
    got, ends = _drain(core, sum(len(v) for v in payload.values()))
    for t in ths:
        t.join()
    deadline = time.monotonic() + 5
    while len(ends) < 3 and time.monotonic() < deadline:
        ends += [(sid, err) for sid, buf, view, _ns, err in core.take() if view is None]
        time.sleep(0.001)
    assert {sid: bytes(v) for sid, v in got.items()} == payload
    assert sorted(ends) == sorted((sid, 0) for sid in sids)
    assert core.stats()["reads"] > 0
    core.close()
    for a, b in pairs:
        a.close()
        b.close()


def test_last_read_times_a_streams_reads():
    """last_read(sid): when the stream's last read with bytes ended, on
    time.monotonic()'s clock (the reflectors' idle checks of bound streams,
    which never pass through Python per read); 0.0 before any, and for an
    unknown stream."""
    core = load().ReaderHub(64 * 1024, 4)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    assert core.last_read(sid) == 0.0 and core.last_read(sid + 99) == 0.0
    t0 = time.monotonic()
    a.sendall(b"x" * 1000)
    got, _ = _drain(core, 1000)
    t1 = time.monotonic()
    assert len(got[sid]) == 1000
    assert t0 <= core.last_read(sid) <= t1
    core.close()
    a.close()
    b.close()


def test_hub_pause_stops_reading_and_remove_closes():
    mod = load()
    core = mod.ReaderHub(64 * 1024, 2)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    b.close()  # the hub's dup is the only reader now
    core.pause(sid, True)
    a.sendall(b"x" * 1000)
    time.sleep(0.1)
    assert core.take() == []  # paused: nothing read
    core.pause(sid, False)
    got, _ = _drain(core, 1000)
    assert bytes(got[sid]) == b"x" * 1000
    core.remove(sid)  # closes the hub's fd: the peer sees EOF
    a.settimeout(2)
    assert a.recv(10) == b""
    core.close()
    a.close()


def test_pool_exhaustion_is_backpressure_not_loss():
    """With every buffer held by the consumer the hub stops polling; data waits
    in the socket and arrives, complete and in order, once buffers return."""
    mod = load()
    core = mod.ReaderHub(4096, 2)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    data = os.urandom(200_000)
    import threading
    t = threading.Thread(target=a.sendall, args=(data,))
    t.start()
    time.sleep(0.1)
    held = []
    deadline = time.monotonic() + 2
    while len(held) < 2 and time.monotonic() < deadline:
        held += [(buf, bytes(view)) for _s, buf, view, _ns, _e in core.take() if view is not None]
        time.sleep(0.005)
    assert len(held) == 2
    time.sleep(0.1)
    assert core.take() == []  # pool empty: not reading
    assert core.stats()["starved"] >= 0
    out = bytearray(b"".join(x for _, x in held))
    for buf, _ in held:
        core.release(buf)
    got, _ = _drain(core, len(data) - len(out))
    t.join()
    out += got[sid]
    assert bytes(out) == data
    core.close()
    a.close()
    b.close()


def test_http_stream_adopted_by_hub_end_to_end():
    """HttpClient hands a zero-copy raw stream to the hub after its head; the
    sink gets the same bytes, the server's close ends `finished`, and a client
    close reaches the server."""

    async def body():
        closed_by_client = asyncio.get_running_loop().create_future()

        async def handle(reader, writer):
            req = await reader.readuntil(b"\r\n\r\n")
            writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
            if b"/short" in req:
                writer.write(b"5\r\nhello\r\n0\r\n\r\n")
                await writer.drain()
                writer.close()
                return
            for i in range(200):
                chunk = (b"%05d" % i) * 200
                writer.write(b"%x\r\n%s\r\n" % (len(chunk), chunk))
            await writer.drain()
            await reader.read()
            closed_by_client.set_result(True)
            writer.close()

        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        c = HttpClient(f"http://127.0.0.1:{port}")
        hub = WatchReaderHub(64 * 1024, 4)
        c.reader_hub = hub
        got = bytearray()
        stream, err = await c.stream("GET", "/long", lambda d, _ns: got.extend(d), raw_chunked=True,
                                     read_size=1 << 20, zero_copy=True)
        assert err is None and stream._proto.hub is hub
        want = sum(len(b"%x\r\n" % 1000) + 1000 + 2 for _ in range(200))
        for _ in range(500):
            if len(got) >= want:
                break
            await asyncio.sleep(0.01)
        long_ok = len(got) == want and b"00199" in got
        stream.close()
        by_client = await asyncio.wait_for(closed_by_client, 5)
        await asyncio.wait_for(stream.finished, 5)
        short = bytearray()
        s2, err2 = await c.stream("GET", "/short", lambda d, _ns: short.extend(d), raw_chunked=True,
                                  read_size=1 << 20, zero_copy=True)
        await asyncio.wait_for(s2.finished, 5)  # the server's close ends it
        stats = hub.stats()
        hub.close()
        await c.close()
        srv.close()
        return long_ok, by_client, bytes(short), stats

    long_ok, by_client, short, stats = run(body())
    assert long_ok and by_client
    assert short.endswith(b"0\r\n\r\n")
    assert stats["streams"] == 0  # both streams left the hub


def test_tls_streams_stay_on_asyncio():
    pytest.importorskip("ssl")
    from k8s_watcher_amd.net import reader as reader_mod

    class FakeTransport:
        def is_closing(self):
            return False

        def get_extra_info(self, name):
            return object() if name == "sslcontext" else None

    class P:
        transport = FakeTransport()

    async def body():
        hub = reader_mod.WatchReaderHub(64 * 1024, 2)
        ok = hub.adopt(P())
        hub.close()
        return ok

    assert run(body()) is False


@pytest.mark.parametrize("depth", [2, 4])
def test_read_ahead_is_capped_per_stream(depth):
    """However large the pool, one stream gets at most two buffers (or
    watcher.watch_reader_depth) ahead of the consumer: a slow event loop
    leaves the backlog in the socket (TCP flow control), not in user memory."""
    mod = load()
    core = mod.ReaderHub(4096, 16)
    core.set_depth(depth)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    data = os.urandom(400_000)
    import threading
    t = threading.Thread(target=a.sendall, args=(data,))
    t.start()
    time.sleep(0.2)
    held = []
    for _ in range(20):
        held += [(buf, bytes(view)) for _s, buf, view, _ns, _e in core.take() if view is not None]
        time.sleep(0.01)
    assert (1 if depth == 2 else 3) <= len(held) <= depth
    out = bytearray(b"".join(x for _, x in held))
    for buf, _ in held:
        core.release(buf)
    got, _ = _drain(core, len(data) - len(out))
    t.join()
    out += got[sid]
    assert bytes(out) == data
    core.close()
    a.close()
    b.close()


def test_read_ahead_is_capped_in_bytes_over_all_streams():
    """``max_bytes``: many streams together hold at most about that many bytes
    read but not handed back (what the loop reads next stays in cache); the
    rest waits in the sockets and arrives, complete and in order per stream."""
    import threading
    mod = load()
    core = mod.ReaderHub(64 * 1024, 64, max_bytes=96 * 1024)
    assert core.stats()["max_bytes"] == 96 * 1024
    pairs = [socket.socketpair() for _ in range(8)]
    sids = [core.add(os.dup(b.fileno())) for _a, b in pairs]
    payload = {sid: os.urandom(150_000) for sid in sids}
    ths = [threading.Thread(target=a.sendall, args=(payload[sid],)) for (a, _b), sid in zip(pairs, sids)]
    for t in ths:
        t.start()
    time.sleep(0.2)
    held = []
    for _ in range(20):
        held += [(sid, buf, bytes(view)) for sid, buf, view, _ns, _e in core.take() if view is not None]
        time.sleep(0.01)
    # one read may overshoot the budget by at most a buffer
    assert 0 < sum(len(x) for _s, _b, x in held) <= 96 * 1024 + 64 * 1024
    assert core.stats()["over_budget"] > 0
    got = {}
    for sid, buf, x in held:
        got.setdefault(sid, bytearray()).extend(x)
        core.release(buf)
    more, _ = _drain(core, sum(len(v) for v in payload.values()) - sum(len(x) for _s, _b, x in held))
    for t in ths:
        t.join()
    for sid, v in more.items():
        got.setdefault(sid, bytearray()).extend(v)
    assert {sid: bytes(v) for sid, v in got.items()} == payload
    core.close()
    for a, b in pairs:
        a.close()
        b.close()


@pytest.mark.parametrize("readers", [1, 3])
def test_take_and_remove_race_the_reader_thread(readers):
    """The hub thread recv()s outside its lock. Under a steady flood on many
    streams, takes that land while it is appending to an entry, releases, and
    removals of streams it is reading must keep every stream's bytes a gap-free,
    in-order prefix of what was sent (complete for the streams never removed)."""
    import random
    import threading
    mod = load()
    core = mod.ReaderHub(64 * 1024, 16)
    core.set_readers(readers)  # several threads: streams spread over them, each stays with one
    pairs = [socket.socketpair() for _ in range(12)]
    for a, _b in pairs:
        a.setblocking(True)
    sids = [core.add(os.dup(b.fileno())) for _a, b in pairs]
    payload = {sid: os.urandom(600_000) for sid in sids}
    stop = threading.Event()

    def send(a, data):
        try:
            for i in range(0, len(data), 8192):
                if stop.is_set():
                    return
                a.sendall(data[i:i + 8192])
        except OSError:  # the hub closed a removed stream
            pass

    ths = [threading.Thread(target=send, args=(a, payload[sid]), daemon=True) for (a, _b), sid in zip(pairs, sids)]
    for t in ths:
        t.start()
    rng = random.Random(3)
    to_remove = set(rng.sample(sids, 4))
    gone = set()
    got = {sid: bytearray() for sid in sids}
    deadline = time.monotonic() + 20
    want = sum(len(payload[s]) for s in sids if s not in to_remove)
    while time.monotonic() < deadline:
        for sid, buf, view, _ns, _err in core.take():
            if view is not None:
                got[sid].extend(view)
                view.release()
                core.release(buf)
        for sid in sorted(to_remove - gone):
            if len(got[sid]) > 100_000 and rng.random() < 0.2:
                core.remove(sid)  # usually while the thread is reading it
                gone.add(sid)
        if sum(len(got[s]) for s in sids if s not in to_remove) >= want and gone == to_remove:
            break
        time.sleep(0.0002)
    stop.set()
    assert gone == to_remove
    for sid in sids:
        assert bytes(got[sid]) == payload[sid][:len(got[sid])]  # in order, no gap
        if sid not in to_remove:
            assert len(got[sid]) == len(payload[sid])
    core.close()
    for _a, b in pairs:  # senders blocked on a removed stream now fail and exit
        b.close()
    for t in ths:
        t.join(10)
    for a, _b in pairs:
        a.close()


def _chunked(data: bytes, piece: int = 7000) -> bytes:
    out = bytearray()
    for i in range(0, len(data), piece):
        part = data[i:i + piece]
        out += b"%x\r\n" % len(part) + part + b"\r\n"
    return bytes(out + b"0\r\n\r\n")


def _dispatch_until(core, pred, on_item, timeout=10.0):
    deadline = time.monotonic() + timeout
    touched_all = set()
    while not pred() and time.monotonic() < deadline:
        items, touched = core.take_dispatch()
        touched_all.update(touched)
        for it in items:
            on_item(it)
        time.sleep(0.001)
    return touched_all


@pytest.mark.parametrize("ov", [{}, {"watcher": {"namespaces": ["none-of-these"]}}])
def test_take_dispatch_feeds_bound_pipeline_like_handle_raw(ov):
    """A stream bound to a native Pipeline is fed by take_dispatch itself: the
    submits, cache, resume RV and control events equal handle_raw's on the
    same bytes, only reads that need Python come back, an unbound stream on
    the same hub still gets its raw buffers, and the end of the body is
    reported once."""
    from test_native_pipeline import Recorder, run_native, stream
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.utils.config import load_settings

    data = stream()
    want_calls, want_cache, _, want_rv, want_ctrl = run_native("production", ov, data)
    s = load_settings("production", overrides=ov, environ={})
    rec = Recorder()
    p = EventPipeline(s, PyDecoder("production"), rec, Metrics())
    p.log_events_setting = False
    p.attach_native()
    p.sync_native_log()
    core = load().ReaderHub(16 * 1024, 8)  # small buffers: many reads, lines split across them
    (a, b), (c, d) = socket.socketpair(), socket.socketpair()
    bound, plain = core.add(os.dup(b.fileno())), core.add(os.dup(d.fileno()))
    core.bind(bound, p.native, True)
    raw = _chunked(data)
    import threading
    sender = threading.Thread(target=a.sendall, args=(raw,), daemon=True)  # the hub's small pool fills: send meanwhile
    sender.start()
    c.sendall(b"plain bytes")
    c.shutdown(socket.SHUT_WR)
    ctrl, plain_got, done, attention = [], bytearray(), [], [0]

    def on_item(it):
        sid, buf, view, read_ns, err = it
        if buf == -2:
            assert sid == bound and not isinstance(view, BaseException)
            attention[0] += 1
            ctrl.extend(e[0] for e in p.native_result(view, read_ns))
            if err:
                done.append(sid)
            return
        if view is None:
            return
        if sid == bound:  # after one that needed Python in the same batch: the sink's path
            ctrl.extend(e[0] for e in p.native_result(p.native.feed_chunked(view, read_ns), read_ns))
            if p.native.body_done():
                done.append(sid)
        else:
            plain_got.extend(view)
        view.release()
        core.release(buf)

    touched = _dispatch_until(core, lambda: done and plain_got == b"plain bytes", on_item)
    sender.join()
    assert done == [bound] and bytes(plain_got) == b"plain bytes"
    assert {bound, plain} <= touched
    assert rec.calls == want_calls
    assert {u: list(e) for u, e in p.cache.items()} == {u: list(e) for u, e in want_cache.items()}
    assert ctrl == want_ctrl and "ERROR" in ctrl
    assert p.native.last_rv() == want_rv
    stats = core.stats()
    if not want_calls:  # nothing to submit: only the control events and the end came back
        assert attention[0] <= len(want_ctrl) + 1 < stats["reads"]
    core.unbind(bound)
    core.close()
    for x in (a, b, c, d):
        x.close()


def test_buffers_grow_for_a_busy_stream_and_stay_small_for_quiet_ones():
    """Size classes: a stream whose buffers fill before they are taken moves
    up to buf_bytes reads; a trickling stream keeps the smallest class, so
    many quiet streams do not starve the pool (nbufs * buf_bytes of memory)."""
    import threading
    mod = load()
    core = mod.ReaderHub(1 << 20, 4)  # 4 MiB of memory: 4 big buffers, or 256 small ones
    (a, b), (c, d) = socket.socketpair(), socket.socketpair()
    busy, quiet = core.add(os.dup(b.fileno())), core.add(os.dup(d.fileno()))
    payload = os.urandom(12 << 20)
    t = threading.Thread(target=a.sendall, args=(payload,), daemon=True)
    t.start()
    c.sendall(b"x" * 100)
    sizes, got, qgot = [], bytearray(), bytearray()
    deadline = time.monotonic() + 20
    while (len(got) < len(payload) or len(qgot) < 100) and time.monotonic() < deadline:
        time.sleep(0.01)  # a slow consumer: buffers fill before they are taken
        for sid, buf, view, read_ns, err in core.take():
            if view is None:
                continue
            (got if sid == busy else qgot).extend(view)
            if sid == busy:
                sizes.append(len(view))
            view.release()
            core.release(buf)
    t.join()
    assert bytes(got) == payload and bytes(qgot) == b"x" * 100
    assert max(sizes) > 256 << 10  # grew past the 256 KiB class
    assert core.stats()["allocated_bytes"] <= 4 << 20
    core.close()
    for x in (a, b, c, d):
        x.close()


def test_take_dispatch_groups_many_bound_streams_like_serial_feeding():
    """Reads of many bound streams are decoded as one batch (pl_run_group):
    each stream's pipeline still sees exactly what serial feeding gives —
    submits, cache, resume RV, control events — with reads of several streams
    (and several reads of one stream) in one take."""
    import threading
    from test_native_pipeline import Recorder, run_native, stream
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.utils.config import load_settings

    data = stream()
    want_calls, want_cache, _, want_rv, want_ctrl = run_native("production", {}, data)
    s = load_settings("production", environ={})
    pool = load().DecodePool(2)
    core = load().ReaderHub(256 * 1024, 16)
    n = 12
    pipes, recs, socks, sids = [], [], [], []
    for _ in range(n):
        rec = Recorder()
        p = EventPipeline(s, PyDecoder("production"), rec, Metrics())
        p.log_events_setting = False
        p.attach_native(pool)
        p.sync_native_log()
        a, b = socket.socketpair()
        sid = core.add(os.dup(b.fileno()))
        core.bind(sid, p.native, True)
        pipes.append(p)
        recs.append(rec)
        socks += [a, b]
        sids.append(sid)
    by_sid = dict(zip(sids, pipes))
    raw = _chunked(data, piece=3000)
    # every stream's bytes arrive before the first take: one take holds reads of all of them
    senders = [threading.Thread(target=socks[2 * i].sendall, args=(raw,), daemon=True) for i in range(n)]
    for t in senders:
        t.start()
    time.sleep(0.2)
    ctrl = {sid: [] for sid in sids}
    done = []

    def on_item(it):
        sid, buf, view, read_ns, err = it
        p = by_sid[sid]
        if buf == -2:
            assert not isinstance(view, BaseException), view
            ctrl[sid].extend(e[0] for e in p.native_result(view, read_ns))
            if err:
                done.append(sid)
            return
        if view is None:
            return
        ctrl[sid].extend(e[0] for e in p.native_result(p.native.feed_chunked(view, read_ns), read_ns))
        if p.native.body_done():
            done.append(sid)
        view.release()
        core.release(buf)

    _dispatch_until(core, lambda: len(done) == n, on_item, timeout=30)
    for t in senders:
        t.join()
    assert sorted(done) == sorted(sids)
    for sid, p, rec in zip(sids, pipes, recs):
        assert rec.calls == want_calls
        assert {u: list(e) for u, e in p.cache.items()} == {u: list(e) for u, e in want_cache.items()}
        assert ctrl[sid] == want_ctrl
        assert p.native.last_rv() == want_rv
    for sid in sids:
        core.unbind(sid)
    core.close()
    for x in socks:
        x.close()


def test_busy_streams_grow_only_to_their_share_of_the_pool():
    """With many streams, a stream's buffer class stops at one buffer per
    stream fitting the pool: 16 streams on 4 MiB read at most 256 KiB at a
    time, so busy namespace watches do not starve each other."""
    import threading
    core = load().ReaderHub(1 << 20, 4)  # 4 MiB: 1 MiB, 256, 64, 16 KiB classes
    pairs = [socket.socketpair() for _ in range(16)]
    sids = [core.add(os.dup(b.fileno())) for _a, b in pairs]
    busy = sids[0]
    payload = os.urandom(8 << 20)
    t = threading.Thread(target=pairs[0][0].sendall, args=(payload,), daemon=True)
    t.start()
    sizes, got = [], bytearray()
    deadline = time.monotonic() + 20
    while len(got) < len(payload) and time.monotonic() < deadline:
        time.sleep(0.01)  # a slow consumer: buffers fill before they are taken
        for sid, buf, view, read_ns, err in core.take():
            if view is None:
                continue
            assert sid == busy
            got.extend(view)
            sizes.append(len(view))
            view.release()
            core.release(buf)
    t.join()
    assert bytes(got) == payload
    assert 64 << 10 < max(sizes) <= 256 << 10
    core.close()
    for a, b in pairs:
        a.close()
        b.close()


@pytest.mark.parametrize("buf_bytes", [16 * 1024, 64 * 1024])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_hub_framing_matches_pipeline_framing_on_random_chunking(seed, buf_bytes):
    """Once a chunked body is bound, the hub frames it (chunk de-framing and
    line splitting on its reader thread, HubFramer) and the pipeline walks
    line items: random chunk sizes, random send pieces and small buffers put
    chunk headers, line ends and buffer ends everywhere — the result is
    identical to the pipeline framing the same bytes itself."""
    import random
    import threading
    from test_native_pipeline import Recorder, run_native, stream
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.utils.config import load_settings

    rng = random.Random(seed)
    data = stream()
    want_calls, want_cache, _, want_rv, want_ctrl = run_native("production", {}, data)
    out, i = bytearray(), 0
    while i < len(data):
        n = rng.choice([1, 2, 7, 100, 1000, 4000, 9000, 30000])
        part = data[i:i + n]
        out += b"%x\r\n" % len(part) + part + b"\r\n"
        i += n
    raw = bytes(out + b"0\r\n\r\n")
    s = load_settings("production", environ={})
    rec = Recorder()
    p = EventPipeline(s, PyDecoder("production"), rec, Metrics())
    p.log_events_setting = False
    p.attach_native(load().DecodePool(2))
    p.sync_native_log()
    core = load().ReaderHub(buf_bytes, 16)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    core.bind(sid, p.native, True)

    def send():
        j = 0
        while j < len(raw):
            n = rng.choice([1, 5, 333, 4096, 20000, 70000])
            a.sendall(raw[j:j + n])
            j += n
            if rng.random() < 0.2:
                time.sleep(0.001)

    t = threading.Thread(target=send, daemon=True)
    t.start()
    ctrl, done = [], []

    def on_item(it):
        sid_, buf, view, read_ns, err = it
        assert sid_ == sid and buf == -2, it  # a bound body never comes back raw
        assert not isinstance(view, BaseException), view
        ctrl.extend(e[0] for e in p.native_result(view, read_ns))
        if err:
            done.append(sid_)

    _dispatch_until(core, lambda: done, on_item, timeout=30)
    t.join()
    assert done == [sid]
    assert rec.calls == want_calls
    assert {u: list(e) for u, e in p.cache.items()} == {u: list(e) for u, e in want_cache.items()}
    assert ctrl == want_ctrl
    assert p.native.last_rv() == want_rv and p.native.body_done()
    st = core.stats()
    assert st["framed_reads"] > 0 and st["frame_ns"] > 0  # the hub did frame (after the first take)
    assert st["recv_bytes"] == len(raw) and st["recv_ns"] > 0
    core.close()
    a.close()
    b.close()


def test_reader_depth_bounds():
    core = load().ReaderHub(16 * 1024, 4)
    with pytest.raises(ValueError):
        core.set_depth(9)
    core.set_depth(4)
    assert core.stats()["depth"] == 4
    core.close()


def test_hub_framing_reports_bad_chunk_size_like_the_pipeline():
    """A framing error found by the hub surfaces as the pipeline's ValueError
    for that read, after the lines before it were applied."""
    from test_native_pipeline import Recorder, stream
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.utils.config import load_settings

    lines = stream().split(b"\n")
    first, second = b"\n".join(lines[:3]) + b"\n", b"\n".join(lines[3:6]) + b"\n"
    s = load_settings("staging", environ={})
    rec = Recorder()
    p = EventPipeline(s, PyDecoder("staging"), rec, Metrics())
    p.log_events_setting = False
    p.attach_native()
    p.sync_native_log()
    core = load().ReaderHub(64 * 1024, 4)
    a, b = socket.socketpair()
    sid = core.add(os.dup(b.fileno()))
    core.bind(sid, p.native, True)
    a.sendall(b"%x\r\n" % len(first) + first + b"\r\n")
    results = []
    deadline = time.monotonic() + 5
    while core.stats()["reads"] < 1 and time.monotonic() < deadline:
        time.sleep(0.01)
    time.sleep(0.05)
    items, _ = core.take_dispatch()  # the first read goes through the pipeline; framing is handed to the hub
    for it in items:  # its submits (a Python notifier here)
        p.native_result(it[2], it[3])
    a.sendall(b"%x\r\n" % len(second) + second + b"\r\nzz\r\n")
    _dispatch_until(core, lambda: bool(results), lambda it: results.append(it), timeout=5)
    assert len(results) == 1
    sid_, buf, res, _read_ns, _done = results[0]
    assert buf == -2 and isinstance(res, ValueError) and "bad chunk size line zz" in str(res)
    assert core.stats()["framed_reads"] > 0
    # the lines before the error were applied (the cache has them), as when the
    # pipeline frames the same bytes itself
    ref = EventPipeline(s, PyDecoder("staging"), Recorder(), Metrics())
    ref.log_events_setting = False
    ref.attach_native()
    with pytest.raises(ValueError, match="bad chunk size line zz"):
        ref.native.feed_chunked(b"%x\r\n" % len(first) + first + b"\r\n" + b"%x\r\n" % len(second) + second
                                + b"\r\nzz\r\n", 1)
    assert {u: list(e) for u, e in p.cache.items()} == {u: list(e) for u, e in ref.cache.items()}
    assert len(p.cache.items()) > 0
    core.close()
    a.close()
    b.close()


def test_runtime_log_level_reaches_every_hub_dispatched_scope():
    """Several namespace scopes share one notifier and event log, so the hub
    flushes them once per dispatch; each bound scope's native pipeline must
    still pick up a runtime change of the log switches (advisor round 3: only
    the last-bound scope's pipeline did)."""
    import logging

    from conftest import run
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
    from k8s_watcher_amd.testing.podgen import PodFactory
    from k8s_watcher_amd.testing.stub_sink import StubSink
    from k8s_watcher_amd.utils.config import load_settings
    from k8s_watcher_amd.utils.logsetup import SERVICE_LOGGER

    names = ["ns-a", "ns-b", "ns-c"]

    async def body():
        srv = FakeApiServer(namespaces=names)
        await srv.start()
        sink = StubSink()
        await sink.start()
        s = load_settings("staging", overrides={
            "clusterapi": {"base_url": sink.url, "health_check_on_start": False},
            "watcher": {"engine": "native", "namespace_scope": "discover", "watch_reader": "native",
                        "retry": {"delay_seconds": 0.05, "max_attempts": 0}}})
        log = logging.getLogger(SERVICE_LOGGER)
        old = log.level
        log.setLevel(logging.WARNING)
        svc = WatcherService(s, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
        try:
            await svc.start()
            f = PodFactory(seed=3, namespaces=names)
            for ns in names:
                srv.create(f.new_pod(namespace=ns))
            await sink.state.wait_for(3, timeout=10)
            assert svc.metrics.c["watches_hub_dispatch"] == len(names)
            assert {r.pipeline._native_log for r in svc.reflectors} == {(False, False)}
            log.setLevel(logging.INFO)  # at run time: every scope's native pipeline must follow
            for ns in names:
                srv.create(f.new_pod(namespace=ns))
            await sink.state.wait_for(6, timeout=10)
            flags = sorted((r.namespace, r.pipeline._native_log) for r in svc.reflectors)
        finally:
            log.setLevel(old)
            svc.stop()
            await svc.shutdown()
            await sink.stop()
            await srv.stop()
        return flags

    flags = run(body(), timeout=60)
    assert flags == [(ns, (True, False)) for ns in names], flags


def test_take_dispatch_merges_queued_reads_of_one_stream():
    """Reads of one bound stream queued by the time the loop takes them go
    through its pipeline as one call (GroupRead::more, engine.inc) when its
    submits are native: the same notifications, per pod in stream order, the
    same cache and resume RV as feeding the bytes serially — with fewer calls
    than reads."""
    import asyncio
    import threading

    from conftest import run
    from test_native_pipeline import run_native
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.parallel.native_notifier import NativeNotifierPool
    from k8s_watcher_amd.testing.podgen import churn_events, event_line
    from k8s_watcher_amd.testing.stub_sink import StubSink
    from k8s_watcher_amd.utils.config import load_settings

    data = b"".join(event_line(t, o) for t, o in churn_events(200, seed=29))
    want_calls, want_cache, _, want_rv, _ = run_native("staging", {}, data)

    async def body():
        sink = StubSink()
        await sink.start()
        s = load_settings("staging", overrides={"clusterapi": {"base_url": sink.url, "health_check_on_start": False}},
                          environ={})
        m = Metrics()
        pool = NativeNotifierPool(s.clusterapi, m)
        p = EventPipeline(s, PyDecoder("staging"), pool, m)
        p.log_events_setting = False
        p.attach_native()
        p.sync_native_log()
        core = load().ReaderHub(16 * 1024, 256)
        a, b = socket.socketpair()
        sid = core.add(os.dup(b.fileno()))
        core.bind(sid, p.native, True)
        sender = threading.Thread(target=a.sendall, args=(_chunked(data),), daemon=True)
        sender.start()
        done = []
        deadline = time.monotonic() + 20
        while not done and time.monotonic() < deadline:
            await asyncio.sleep(0.02)  # let several reads queue up before each take
            items, _ = core.take_dispatch()
            for sid_, buf, view, read_ns, err in items:
                if buf == -2:
                    p.native_result(view, read_ns)
                    if err:
                        done.append(sid_)
                elif view is not None:  # after a read that needed Python: fed directly
                    p.native_result(p.native.feed_chunked(view, read_ns), read_ns)
                    view.release()
                    core.release(buf)
                    if p.native.body_done():
                        done.append(sid_)
            pool.flush()
        sender.join()
        assert await pool.drain(10)
        got = [(x["uid"], x["event_type"]) for x in sink.state.payloads()]
        stats = core.stats()
        cache = {u: list(e) for u, e in p.cache.items()}
        rv = p.native.last_rv()
        core.unbind(sid)
        core.close()
        await pool.close()
        await sink.stop()
        a.close()
        b.close()
        return got, stats, cache, rv

    got, stats, cache, rv = run(body(), timeout=60)
    want = [(c[0], c[1]) for c in want_calls]
    assert sorted(got) == sorted(want)  # exactly once
    by_uid = lambda seq: {u: [t for uu, t in seq if uu == u] for u, _ in seq}  # noqa: E731
    assert by_uid(got) == by_uid(want)  # per pod, in stream order
    assert cache == {u: list(e) for u, e in want_cache.items()} and rv == want_rv
    assert stats["merged_reads"] > 0 and stats["dispatch_batches"] < stats["reads"], stats


def test_dispatch_delivery_is_sliced_across_loop_turns_in_order():
    """A storm's dispatch (hundreds of reads needing Python at once) is delivered
    over several loop turns, at most DISPATCH_SLICE_S each, in arrival order; no
    new take_dispatch runs while a rest is pending (a bound stream's later reads
    must stay behind its attention read)."""

    class Core:
        def __init__(self, batches):
            self.batches, self.takes, self.released = list(batches), 0, []

        def take_dispatch(self):
            self.takes += 1
            return self.batches.pop(0) if self.batches else ([], [])

        def release(self, buf):
            self.released.append(buf)

    class Proto:
        def __init__(self, log, sid):
            self.log, self.sid, self.hub_sync = log, sid, None

        def hub_native(self, result, read_ns, done):
            time.sleep(0.0005)
            self.log.append((self.sid, result))

        def hub_data(self, view, read_ns):
            self.log.append((self.sid, bytes(view)))

    async def main():
        hub = object.__new__(WatchReaderHub)
        hub.loop = asyncio.get_running_loop()
        hub.DISPATCH_SLICE_S = 0.002
        log, turns = [], []
        first = [(sid, -2, ("r", sid), 1, 0) for sid in range(200)]
        first.append((7, 3, memoryview(b"later"), 1, 0))  # a plain read of stream 7 behind its attention read
        second = [(7, -2, ("r2", 7), 1, 0)]
        hub.core = Core([(first, list(range(200))), (second, [7])])
        hub.protos = {sid: Proto(log, sid) for sid in range(200)}
        hub._flush, hub._pending, hub._soon, hub.closed = {"k": lambda: turns.append(len(log))}, None, None, False
        hub._groups = {}
        hub._on_ready()
        assert hub._pending is not None and hub.core.takes == 1 and len(log) < 200
        n = len(log)
        hub._on_ready()  # an eventfd wake-up while a rest is pending: the scheduled turn delivers it
        assert len(log) == n and hub.core.takes == 1
        while hub._pending is not None:
            await asyncio.sleep(0)  # the scheduled turns deliver the rest, taking nothing new
            assert hub.core.takes == 1 or hub._pending is None
        hub._on_ready()  # now the next take
        assert hub.core.takes == 2
        assert log == [(sid, ("r", sid)) for sid in range(200)] + [(7, b"later"), (7, ("r2", 7))]
        assert hub.core.released == [3]
        assert len(turns) >= 3  # flushed after every turn

    run(main())


def test_set_readers_bounds_and_spread():
    """set_readers: 1..8 threads, never fewer than running; streams added
    after it go to the thread with the fewest (thread_ids names them all)."""
    core = load().ReaderHub(64 * 1024, 8)
    with pytest.raises(ValueError):
        core.set_readers(0)
    with pytest.raises(ValueError):
        core.set_readers(9)
    assert core.set_readers(2) and core.set_readers(2)
    assert not core.set_readers(1)  # threads never go away while the hub runs
    ids = core.thread_ids()
    assert len(ids) == 2 and len(set(ids)) == 2 and all(ids)
    core.close()


def test_service_spreads_namespace_watches_over_reader_threads(monkeypatch):
    """Several namespace scopes with two reader threads (engine/service.py
    HUB_READERS): every pod of every namespace is notified once, the hub
    runs two threads."""
    from conftest import run
    from k8s_watcher_amd.engine import service
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
    from k8s_watcher_amd.testing.podgen import PodFactory
    from k8s_watcher_amd.testing.stub_sink import StubSink
    from k8s_watcher_amd.utils.config import load_settings

    monkeypatch.setattr(service, "HUB_READERS", 2)
    names = [f"ns-{i}" for i in range(6)]

    async def body():
        srv = FakeApiServer(namespaces=names)
        await srv.start()
        sink = StubSink()
        await sink.start()
        s = load_settings("staging", overrides={
            "clusterapi": {"base_url": sink.url, "health_check_on_start": False},
            "watcher": {"engine": "native", "namespace_scope": "discover",
                        "retry": {"delay_seconds": 0.05, "max_attempts": 0}}}, environ={})
        svc = WatcherService(s, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
        try:
            await svc.start()
            f = PodFactory(seed=5, namespaces=names)
            for _ in range(5):
                for ns in names:
                    srv.create(f.new_pod(namespace=ns))
            await sink.state.wait_for(30, timeout=15)
            readers = len(svc._reader_hub.core.thread_ids())
            got = sink.state.payloads()
        finally:
            svc.stop()
            await svc.shutdown()
            await sink.stop()
            await srv.stop()
        return readers, got

    readers, got = run(body(), timeout=60)
    assert readers == 2
    keys = [(p["uid"], p["event_type"]) for p in got]
    assert len(keys) == 30 and len(set(keys)) == 30


@pytest.mark.parametrize("readers,seed", [(1, 0), (1, 1), (2, 0), (2, 1)])
def test_starved_streams_are_all_woken_when_bytes_wait(readers, seed):
    """Many streams over a one-buffer read-ahead budget, in rounds: a few
    streams send a lot, most send a few hundred bytes (and drain at once),
    the consumer takes everything before the next round. A stream disarmed
    over the budget is re-armed as buffers come back; a re-armed stream whose
    socket was drained gets no event, so it must not use up the wake-ups —
    before round 6's fix the streams still holding bytes stayed disarmed once
    every buffer was back (stalled in every one of these cases, one reader or
    two; a 64-namespace bench with an 8 MiB read-ahead hung on the box)."""
    import random
    import threading
    rng = random.Random(seed)
    n = 48
    core = load().ReaderHub(64 << 10, 64, 64 << 10)
    core.set_readers(readers)
    pairs = [socket.socketpair() for _ in range(n)]
    for a, _b in pairs:
        a.setblocking(True)
    sids = [core.add(os.dup(b.fileno())) for _a, b in pairs]
    idx = {sid: i for i, sid in enumerate(sids)}
    got = [0] * n
    try:
        for r in range(30):
            sizes = [rng.choice((0, 300, 300, 300, 300, 300, 150_000)) for _ in range(n)]
            want = [g + s for g, s in zip(got, sizes)]
            ths = [threading.Thread(target=a.sendall, args=(b"y" * s,)) for (a, _b), s in zip(pairs, sizes) if s]
            for t in ths:
                t.start()
            last = time.monotonic()
            while got != want:
                items = core.take()
                for sid, buf, view, _ns, _err in items:
                    if view is not None:
                        got[idx[sid]] += len(view)
                        view.release()
                        core.release(buf)
                if items:
                    last = time.monotonic()
                else:
                    stalled = [(i, want[i] - got[i], core.stream_state(sids[i])) for i in range(n) if got[i] != want[i]]
                    assert time.monotonic() - last < 3.0, f"round {r}: stalled {stalled[:4]}"
                time.sleep(0.0003)
            for t in ths:
                t.join()
    finally:
        core.close()
        for a, b in pairs:
            a.close()
            b.close()
