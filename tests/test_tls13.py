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
        for s, buf, view, _ns, err in hub.take():
            assert s == sid
            if view is None:
                end = err
            else:
                got += view
                view.release()
                hub.release(buf)
        time.sleep(0.001)
    return bytes(got), end


def _native_server(pki, srv, body_parts, threads=2, key_update_at=None, forge=False, result=None):
    """Serve one connection with the fixture's native TLS server: read the
    request, then send the parts (a KeyUpdate before part ``key_update_at``),
    then close_notify (or a forged record)."""
    tls = load().TlsServerContext(pki.server_crt, pki.server_key, threads=threads)
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
