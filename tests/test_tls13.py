"""TLS 1.3 records outside OpenSSL's record layer (``ops/csrc/tls13.inc``).

The reader hub takes over an https watch's receive direction after the
request: it reads ciphertext itself, frames whole records and opens them —
on a thread pool when a read carries enough — each record's content landing
at its place in the read buffer. The replay fixture's ``TlsServerContext``
seals its sending direction the same way. Both must be byte-exact against
OpenSSL's own record layer on the other end, follow a KeyUpdate, skip session
tickets, end on close_notify, fail on a forged record, and leave TLS 1.2
sessions on ``SSL_read``.
"""

import os
import socket
import ssl
import threading
import time

import pytest

from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.testing.certs import make_pki

REQ = b"GET /watch HTTP/1.1\r\nHost: x\r\n\r\n"


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    return make_pki(str(tmp_path_factory.mktemp("pki")))


def _listener():
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(4)
    return srv


def _client(hub, pki, port, request=REQ):
    mod = load()
    ctx = mod.TlsContext(ca_pem=open(pki.ca_crt, "rb").read())
    c = socket.create_connection(("127.0.0.1", port))
    return hub.add_tls(c.detach(), ctx, "127.0.0.1", request)


def _drain(hub, sid, timeout=30.0):
    got, end = bytearray(), None
    t_end = time.monotonic() + timeout
    while end is None and time.monotonic() < t_end:
        for s, buf, view, ns, err in hub.take():
            assert s == sid
            if view is not None:
                assert ns > 0  # a batch received ahead (the overlap) still has its arrival time
            if view is None:
                end = err
            else:
                got += view
                view.release()
                hub.release(buf)
        time.sleep(0.001)
    return bytes(got), end


def _native_server(pki, srv, body_parts, threads=2, key_update_at=None, forge=False, result=None, **ctx_kw):
    """Serve one connection with the fixture's native TLS server: read the
    request, then send the parts (a KeyUpdate before part ``key_update_at``),
    then close_notify (or a forged record)."""
    tls = load().TlsServerContext(pki.server_crt, pki.server_key, threads=threads, **ctx_kw)
    c, _ = srv.accept()
    conn = tls.accept(c.detach())
    req = b""
    while not req.endswith(b"\r\n\r\n"):
        d = conn.recv(65536)
        if d is None:
            time.sleep(0.001)
            continue
        if not d:
            break
        req += d
    for i, part in enumerate(body_parts):
        if key_update_at is not None and i == key_update_at:
            conn.key_update()
        conn.send(part)
    if forge:  # a record no key opens: 0x17 0x0303, 40 bytes of noise (after the queued records)
        conn.flush()
        os.write(conn.fileno(), b"\x17\x03\x03\x00\x28" + os.urandom(40))
        time.sleep(0.2)
    if result is not None:
        result["req"] = req
        result["stats"] = conn.stats()
        result["pool"] = tls.pool_stats()
    conn.close()


@pytest.mark.parametrize("threads", [0, 3])
def test_large_body_opened_in_parallel_is_byte_exact_across_a_key_update(pki, threads):
    parts = [os.urandom(700_000) for _ in range(6)] + [b"tail" * 1000]
    want = b"".join(parts)
    srv = _listener()
    res = {}
    t = threading.Thread(target=_native_server, args=(pki, srv, parts), kwargs={"key_update_at": 3, "result": res})
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, threads)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid)
    t.join()
    assert end == 0 and got == want
    assert res["req"] == REQ
    st = hub.stats()
    assert st["tls_taken"] == 1 and st["tls_kept"] == 0
    assert st["tls_key_updates"] == 1
    assert st["tls_records"] >= len(want) // 16384
    if threads:  # big reads went to the pool, and its threads did open records
        assert st["tls_pooled_records"] > 0 and sum(n for _, n in st["tls_pool"][1:]) > 0
    assert sum(n for _, n in res["pool"]) > 0  # the server sealed on its pool too
    hub.close()
    srv.close()


@pytest.mark.parametrize("ring_budget", [2 << 30, 0])
def test_large_sends_through_the_sendfile_ring_wrap_byte_exact(pki, ring_budget):
    """The fixture's sender seals large sends into a memfd ring and sends them
    with sendfile; a region is sealed over only once the peer has read it.
    Many times the ring's size, with a key update and small (copied) sends
    interleaved, arrives byte-exact; with no ring budget every send is copied."""
    big = [os.urandom(4 << 20) for _ in range(3)]
    parts = []
    for i in range(30):  # 120 MiB in 4 MiB sends: several turns of the ring
        parts.append(big[i % 3])
        if i % 7 == 3:
            parts.append(b"small-%d;" % i)  # below RING_MIN_SEND: the copy path, in order
    want = b"".join(parts)
    srv = _listener()
    res = {}
    t = threading.Thread(target=_native_server, args=(pki, srv, parts),
                         kwargs={"key_update_at": 12, "result": res, "ring_budget": ring_budget})
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, 2)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid, timeout=120)
    t.join()
    assert end == 0 and len(got) == len(want) and got == want
    assert hub.stats()["tls_key_updates"] == 1
    st = res["stats"]
    if ring_budget:
        assert st["ring_bytes"] >= 29 * (4 << 20)  # every large send went through the ring
    else:
        assert st["ring_bytes"] == 0
    hub.close()
    srv.close()


def test_forged_record_fails_the_stream(pki):
    srv = _listener()
    t = threading.Thread(target=_native_server, args=(pki, srv, [b"x" * 100_000]), kwargs={"forge": True})
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, 2)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid)
    t.join()
    assert end is not None and end < 0
    assert got == b"x" * 100_000  # what came before the forged record was delivered
    assert "authentication" in hub.error_text(sid)
    hub.close()
    srv.close()


def _python_server(pki, srv, body, max_version=None):
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(pki.server_crt, pki.server_key)
    if max_version is not None:
        ctx.maximum_version = max_version
    c, _ = srv.accept()
    with ctx.wrap_socket(c, server_side=True) as s:
        req = b""
        while not req.endswith(b"\r\n\r\n"):
            req += s.recv(65536)
        s.sendall(body)
        try:
            s.unwrap()  # close_notify; the hub closes without one of its own once it has read the stream's end
        except (ssl.SSLError, OSError):
            pass


@pytest.mark.parametrize("version", ["tls1.3", "tls1.2"])
def test_openssl_peer_tickets_and_tls12_fallback(pki, version):
    """Against Python's ssl (OpenSSL's own record layer): TLS 1.3 is taken
    over — its NewSessionTicket records are skipped, close_notify ends the
    stream; TLS 1.2 stays on SSL_read. Same bytes either way."""
    body = os.urandom(3_000_000)
    srv = _listener()
    mv = ssl.TLSVersion.TLSv1_2 if version == "tls1.2" else None
    t = threading.Thread(target=_python_server, args=(pki, srv, body, mv))
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, 2)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid)
    t.join()
    assert end == 0 and got == body
    st = hub.stats()
    if version == "tls1.3":
        assert st["tls_taken"] == 1 and st["tls_tickets"] >= 1
    else:
        assert st["tls_taken"] == 0 and st["tls_kept"] == 1
    hub.close()
    srv.close()


def test_records_off_keeps_ssl_read(pki):
    body = os.urandom(500_000)
    srv = _listener()
    t = threading.Thread(target=_python_server, args=(pki, srv, body))
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(False, 0)  # watcher.watch_tls_records: openssl
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid)
    t.join()
    assert end == 0 and got == body
    assert hub.stats()["tls_taken"] == 0
    hub.close()
    srv.close()


def test_hkdf_traffic_keys_match_rfc8448():
    """The key schedule's last step against RFC 8448 §3 (simple 1-RTT
    handshake): HKDF-Expand-Label of the published
    server_application_traffic_secret_0 gives the published write key and iv
    (the records above also open against OpenSSL's own sealing)."""
    assert load().tls13_selftest()


def test_many_connections_share_the_sealing_pool(pki):
    """Several connections of one TlsServerContext send at once from their own
    threads (the fixture's executor): its CryptoPool runs one batch at a time
    and every stream arrives byte-exact (a shared-lock race here once aborted
    the fixture with 64 namespace watches)."""
    mod = load()
    tls = mod.TlsServerContext(pki.server_crt, pki.server_key, threads=3)
    srv = _listener()
    n = 6
    bodies = [os.urandom(1_500_000) for _ in range(n)]

    def serve_one():
        c, _ = srv.accept()
        conn = tls.accept(c.detach())
        req = b""
        while not req.endswith(b"\r\n\r\n"):
            d = conn.recv(65536)
            if d is None:
                time.sleep(0.001)
                continue
            req += d
        i = int(req.split(b"/")[1].split(b" ")[0])
        for off in range(0, len(bodies[i]), 300_000):
            conn.send(bodies[i][off:off + 300_000])
        conn.close()

    threads = [threading.Thread(target=serve_one) for _ in range(n)]
    for t in threads:
        t.start()
    hub = mod.ReaderHub(1 << 20, 32)
    hub.set_tls(True, 2)
    ctx = mod.TlsContext(ca_pem=open(pki.ca_crt, "rb").read())
    sids = {}
    for i in range(n):
        c = socket.create_connection(srv.getsockname())
        sids[hub.add_tls(c.detach(), ctx, "127.0.0.1", b"GET /%d HTTP/1.1\r\nHost: x\r\n\r\n" % i)] = i
    got = {sid: bytearray() for sid in sids}
    ends = {}
    t_end = time.monotonic() + 60
    while len(ends) < n and time.monotonic() < t_end:
        for s, buf, view, _ns, err in hub.take():
            if view is None:
                ends[s] = err
            else:
                got[s] += view
                view.release()
                hub.release(buf)
        time.sleep(0.001)
    for t in threads:
        t.join()
    assert all(e == 0 for e in ends.values()) and len(ends) == n
    for sid, i in sids.items():
        assert bytes(got[sid]) == bodies[i]
    hub.close()
    srv.close()


# ----------------------------------------------------------------------------
# round 6: the record layer's less travelled branches (VERDICT r5 "what's
# weak" #2) — padding, split post-handshake messages, alerts, every suite,
# a malformed header behind good records, truncation, ring memory


def _serve(pki, srv, script, suites=None, result=None, threads=2):
    """One connection on the native fixture server: read the request, then
    ``script(conn)`` does the sending; close_notify after it unless it
    returns False."""
    tls = load().TlsServerContext(pki.server_crt, pki.server_key, threads=threads, ciphersuites=suites)
    c, _ = srv.accept()
    conn = tls.accept(c.detach())
    req = b""
    t_end = time.monotonic() + 10
    while not req.endswith(b"\r\n\r\n") and time.monotonic() < t_end:
        d = conn.recv(65536)
        if d is None:
            time.sleep(0.001)
            continue
        if not d:
            break
        req += d
    if result is not None:
        result["cipher"] = conn.cipher()
    if script(conn) is not False:
        conn.close()
    else:
        conn.flush()


def _run(pki, script, suites=None, buf=1 << 20, nbufs=8, threads=2, result=None):
    srv = _listener()
    res = {} if result is None else result
    t = threading.Thread(target=_serve, args=(pki, srv, script), kwargs={"suites": suites, "result": res})
    t.start()
    hub = load().ReaderHub(buf, nbufs)
    hub.set_tls(True, threads)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = _drain(hub, sid)
    t.join()
    st = hub.stats()
    err = hub.error_text(sid)
    hub.close()
    srv.close()
    return got, end, st, err, res


@pytest.mark.parametrize("pad", [1, 300, 4096])
def test_padded_records_are_byte_exact(pki, pad):
    """RFC 8446 §5.4: zero padding after the content type, inside the
    encryption — the hub finds the type as the last non-zero byte."""
    big, small = os.urandom(2_000_000), os.urandom(777)

    def script(conn):
        conn.send(big, pad=pad)
        conn.send(small, pad=pad)

    got, end, st, _err, _ = _run(pki, script)
    assert end == 0 and got == big + small
    assert st["tls_taken"] == 1
    assert st["tls_records"] >= len(big) // (16384 - pad)


def _ticket(n):
    """A NewSessionTicket handshake message (RFC 8446 §4.6.1) with an n-byte ticket."""
    body = (7200).to_bytes(4, "big") + os.urandom(4) + b"\x08" + os.urandom(8) + n.to_bytes(2, "big") + os.urandom(n) \
        + b"\x00\x00"
    return b"\x04" + len(body).to_bytes(3, "big") + body


def test_post_handshake_messages_split_over_records(pki):
    """A NewSessionTicket cut over two records, then a KeyUpdate cut after
    its second byte: both are reassembled (§5.1), the ticket is skipped, and
    every record after the KeyUpdate opens with the next key."""
    a, b, c = os.urandom(300_000), os.urandom(5_000), os.urandom(900_000)

    def script(conn):
        conn.send(a)
        t = _ticket(3000)
        conn.send_record(22, t, split=1500)
        conn.send(b)
        conn.key_update(split=2)
        conn.send(c)

    got, end, st, err, _ = _run(pki, script)
    assert end == 0 and got == a + b + c, err
    assert st["tls_tickets"] == 1 and st["tls_key_updates"] == 1


def test_key_update_split_at_every_offset(pki):
    parts = [os.urandom(50_000) for _ in range(5)]

    def script(conn):
        for i, p in enumerate(parts):
            conn.send(p)
            if i < 4:
                conn.key_update(split=i + 1)  # cut after byte 1, 2, 3, 4 of the 5-byte message

    got, end, st, err, _ = _run(pki, script, threads=0)
    assert end == 0 and got == b"".join(parts), err
    assert st["tls_key_updates"] == 4


def test_record_interleaved_with_a_split_message_fails(pki):
    def script(conn):
        conn.send(b"a" * 1000)
        t = _ticket(100)
        conn.send_record(22, t[:50])  # half a message ...
        conn.send(b"b" * 10)          # ... then application data: not allowed (§5.1)

    got, end, _st, err, _ = _run(pki, script)
    assert end is not None and end < 0
    assert got == b"a" * 1000
    assert "interleaved" in err


def test_data_after_a_key_update_in_its_record_fails(pki):
    def script(conn):
        conn.send(b"x" * 100)
        conn.send_record(22, bytes([24, 0, 0, 1, 0]) + _ticket(10))  # KeyUpdate must end its record
        return False

    got, end, _st, err, _ = _run(pki, script)
    assert end is not None and end < 0 and got == b"x" * 100
    assert "key update" in err


@pytest.mark.parametrize("desc", [40, 80])
def test_fatal_alert_ends_the_stream_with_an_error(pki, desc):
    """A fatal alert (handshake_failure, internal_error) is an error with its
    code — unlike close_notify — and what came before it is delivered."""
    body = os.urandom(200_000)

    def script(conn):
        conn.send(body)
        conn.send_record(21, bytes([2, desc]))
        return False

    got, end, _st, err, _ = _run(pki, script)
    assert end is not None and end < 0
    assert got == body
    assert f"alert {desc}" in err


@pytest.mark.parametrize("suite,key_bits", [("TLS_AES_128_GCM_SHA256", 128), ("TLS_AES_256_GCM_SHA384", 256)])
def test_each_aes_gcm_suite_is_taken_over(pki, suite, key_bits):
    """Both AES-GCM suites, forced on the server (an OpenSSL client offers
    AES-256 first, so AES-128 needs the server to insist): HKDF over
    SHA-256 / SHA-384, 16- / 32-byte keys, across a KeyUpdate."""
    a, b = os.urandom(1_500_000), os.urandom(600_000)

    def script(conn):
        conn.send(a)
        conn.key_update()
        conn.send(b)

    got, end, st, err, res = _run(pki, script, suites=suite)
    assert res["cipher"] == (suite, True)
    assert end == 0 and got == a + b, err
    assert st["tls_taken"] == 1 and st["tls_kept"] == 0 and st["tls_key_updates"] == 1


def test_chacha20_peer_stays_on_ssl_read(pki):
    """A server that only speaks ChaCha20-Poly1305: the hub cannot open its
    records, so the stream stays on SSL_read (tls_kept) — and a KeyUpdate
    there is OpenSSL's business — with the same bytes delivered."""
    a, b = os.urandom(800_000), os.urandom(300_000)

    def script(conn):
        conn.send(a)
        conn.key_update()
        conn.send(b)

    got, end, st, err, res = _run(pki, script, suites="TLS_CHACHA20_POLY1305_SHA256")
    assert res["cipher"] == ("TLS_CHACHA20_POLY1305_SHA256", False)
    assert end == 0 and got == a + b, err
    assert st["tls_taken"] == 0 and st["tls_kept"] == 1


def _paused_run(pki, send):
    """The hub's stream is paused once the request is in, the server writes
    everything ``send(conn)`` makes, then the stream resumes: the hub meets
    it all in one receive."""
    srv = _listener()
    sent = threading.Event()

    def script(conn):
        ready.wait(10)
        send(conn)
        sent.set()
        time.sleep(0.3)
        return False

    ready = threading.Event()
    t = threading.Thread(target=_serve, args=(pki, srv, script))
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, 2)
    sid = _client(hub, pki, srv.getsockname()[1])
    t_end = time.monotonic() + 10
    while hub.stats()["tls_taken"] + hub.stats()["tls_kept"] == 0 and time.monotonic() < t_end:
        time.sleep(0.002)  # the handshake and the request are done
    hub.pause(sid, True)
    ready.set()
    sent.wait(10)
    time.sleep(0.1)
    hub.pause(sid, False)
    got, end = _drain(hub, sid)
    t.join()
    err = hub.error_text(sid)
    st = hub.stats()
    hub.close()
    srv.close()
    return got, end, err, st


def test_bad_header_after_good_records_in_one_read_delivers_them_all(pki):
    """Several good records and then a malformed header arrive in one
    receive: every good record is delivered, then the stream fails
    (round-5 advisor: the failure used to cut the batch after its first)."""
    parts = [bytes([65 + i]) * 3000 for i in range(4)]

    def send(conn):
        for p in parts:
            conn.send(p)
        conn.flush()
        os.write(conn.fileno(), b"\x16\x03\x03\x00\x20" + b"\x00" * 32)  # a plaintext handshake header

    got, end, err, st = _paused_run(pki, send)
    assert got == b"".join(parts)
    assert end is not None and end < 0 and "unexpected record" in err
    assert st["tls_records"] == 4


def test_truncated_inside_a_record_is_an_error(pki):
    """The peer closes TCP in the middle of a record without close_notify:
    a truncated stream, reported as an error (as OpenSSL's own read would),
    not as an orderly close."""
    body = os.urandom(40_000)

    def send(conn):
        conn.send(body)
        conn.flush()
        fd = conn.fileno()
        os.write(fd, b"\x17\x03\x03\x04\x00" + os.urandom(100))  # header of 1,024 bytes, 100 of them
        s = socket.socket(fileno=os.dup(fd))
        s.shutdown(socket.SHUT_WR)
        s.close()

    got, end, err, _st = _paused_run(pki, send)
    assert got == body
    assert end is not None and end < 0 and "truncated" in err


def test_ring_memory_is_counted_in_the_pool_and_shrinks_with_the_class(pki):
    """The ciphertext ring is hub memory: it shows in ``allocated_bytes``
    (``watch_reader_allocated_bytes``) and ``tls_ring_bytes``, grows with the
    stream's buffer class and shrinks back when a quiet stream's class
    drops (round-5 advisor) — after a second, not per read (a busy stream's
    class moves between reads; a resize per read halved https throughput)."""
    burst = os.urandom(12_000_000)
    seen = {"max_ring": 0, "max_alloc": 0}
    srv = _listener()
    go_quiet = threading.Event()

    def script(conn):
        conn.send(burst)
        conn.flush()
        go_quiet.wait(20)
        for _ in range(12):
            conn.send(b"q" * 500)
            conn.flush()
            time.sleep(0.15)  # quiet for 1.8 s: a ring shrinks after 1 s larger than needed

    t = threading.Thread(target=_serve, args=(pki, srv, script))
    t.start()
    hub = load().ReaderHub(1 << 20, 8)
    hub.set_tls(True, 2)
    sid = _client(hub, pki, srv.getsockname()[1])
    got, end = bytearray(), None
    t_end = time.monotonic() + 30
    while end is None and time.monotonic() < t_end:
        st = hub.stats()
        seen["max_ring"] = max(seen["max_ring"], st["tls_ring_bytes"])
        seen["max_alloc"] = max(seen["max_alloc"], st["allocated_bytes"])
        assert st["allocated_bytes"] >= st["tls_ring_bytes"]
        for _s, buf, view, _ns, err in hub.take():
            if view is None:
                end = err
                continue
            got += view
            view.release()
            hub.release(buf)
            if len(got) >= len(burst):
                go_quiet.set()
        if len(got) >= len(burst) + 8 * 500 and end is None:  # quiet for a while, stream still open
            seen["quiet_ring"] = hub.stats()["tls_ring_bytes"]
        time.sleep(0.004)  # a slow consumer: the stream's buffers fill and its class grows
    t.join()
    assert end == 0 and bytes(got) == burst + b"q" * 6000
    assert seen["max_ring"] > 1 << 20            # two 1 MiB batches' worth while busy
    assert 0 < seen["quiet_ring"] < 200 << 10    # back to the small class's ring once quiet
    assert seen["max_alloc"] <= (8 << 20) + (3 << 20)
    assert hub.stats()["tls_ring_bytes"] == 0    # released with the stream
    hub.close()
    srv.close()


@pytest.mark.parametrize("readers", [1, 2])
def test_many_tls_streams_share_the_pool_with_their_rings(pki, readers):
    """Sixteen https streams on a 1 MiB pool: rings and buffers together
    stay near the pool's memory, and every stream is delivered whole (a
    stream's first buffer never waits behind rings)."""
    mod = load()
    tls = mod.TlsServerContext(pki.server_crt, pki.server_key, threads=2)
    srv = _listener()
    n = 16
    bodies = [os.urandom(400_000) for _ in range(n)]

    def serve_one():
        c, _ = srv.accept()
        conn = tls.accept(c.detach())
        req = b""
        while not req.endswith(b"\r\n\r\n"):
            d = conn.recv(65536)
            if d is None:
                time.sleep(0.001)
                continue
            req += d
        i = int(req.split(b"/")[1].split(b" ")[0])
        conn.send(bodies[i])
        conn.close()

    threads = [threading.Thread(target=serve_one) for _ in range(n)]
    for t in threads:
        t.start()
    hub = mod.ReaderHub(256 << 10, 4)
    hub.set_tls(True, 2)
    hub.set_readers(readers)  # two reader threads share the one CryptoPool (one batch at a time)
    ctx = mod.TlsContext(ca_pem=open(pki.ca_crt, "rb").read())
    sids = {}
    for i in range(n):
        c = socket.create_connection(srv.getsockname())
        sids[hub.add_tls(c.detach(), ctx, "127.0.0.1", b"GET /%d HTTP/1.1\r\nHost: x\r\n\r\n" % i)] = i
    got = {sid: bytearray() for sid in sids}
    ends, peak = {}, 0
    t_end = time.monotonic() + 60
    while len(ends) < n and time.monotonic() < t_end:
        peak = max(peak, hub.stats()["allocated_bytes"])
        for s, buf, view, _ns, err in hub.take():
            if view is None:
                ends[s] = err
            else:
                got[s] += view
                view.release()
                hub.release(buf)
        time.sleep(0.001)
    for t in threads:
        t.join()
    assert len(ends) == n and all(e == 0 for e in ends.values())
    for sid, i in sids.items():
        assert bytes(got[sid]) == bodies[i]
    # the pool is 1 MiB; beyond it only first buffers (16 KiB) and minimal rings (~33 KiB) per stream
    assert peak <= (1 << 20) + n * (16 << 10) + n * (34 << 10)
    hub.close()
    srv.close()
