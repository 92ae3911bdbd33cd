"""https clusterapi on both notifier pools: the native core runs TLS itself
(OpenSSL on its non-blocking sockets), the asyncio pool through asyncio's SSL
transports. Certificates are checked against ``clusterapi.ca_file`` and the
host (here an IP SAN), unless ``clusterapi.verify_tls`` is off."""

import asyncio
import ssl

import pytest

from conftest import run
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.parallel.native_notifier import NativeNotifierPool
from k8s_watcher_amd.parallel.notifier import NotifierPool
from k8s_watcher_amd.testing.certs import make_pki
from k8s_watcher_amd.testing.stub_sink import StubSink
from test_notifier import TS, _threaded_native, core, settings


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    return make_pki(str(tmp_path_factory.mktemp("pki")))


@pytest.fixture(params=["python", "native", "native-io-thread"])
def pool_cls(request):
    """The native core runs TLS from the event loop and, with
    ``pool.io_thread``, on its I/O thread (SSL_read / SSL_write outside the
    core lock)."""
    return {"python": NotifierPool, "native": NativeNotifierPool, "native-io-thread": _threaded_native}[request.param]


async def tls_sink(pki, **kw):
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(pki.server_crt, pki.server_key)
    sink = StubSink(**kw)
    await sink.start(ssl_context=ctx)
    assert sink.url.startswith("https://")
    return sink


def test_https_delivery_pipelined(pool_cls, pki):
    async def body():
        sink = await tls_sink(pki)
        m = Metrics()
        pool = pool_cls(settings(sink.url, ca_file=pki.ca_crt, connections=3, depth=4), m)
        assert await pool.health_check()
        if hasattr(pool, "warm_up"):
            await pool.warm_up()
        for i in range(200):
            pool.submit(f"u{i % 20}", "MODIFIED", "default", f"p{i % 20}", core(f"u{i % 20}", name=f"v{i}"), 0, TS)
            if i % 7 == 0:
                pool.flush()
                await asyncio.sleep(0)
        pool.flush()
        assert await pool.drain(10)
        assert m.c["notify_failed"] == 0 and m.c["notify_delivered"] + m.c["notify_superseded"] == 200
        last = {}
        for p in sink.state.payloads():
            last[p["uid"]] = p["name"]
        assert last == {f"u{k}": f"v{180 + k}" for k in range(20)}  # per-pod order held over TLS
        await pool.close()
        await sink.stop()
    run(body())


def test_https_large_bodies(pool_cls, pki):
    """Bodies larger than one TLS record (16 KiB) and than the socket buffer."""
    async def body():
        sink = await tls_sink(pki)
        m = Metrics()
        pool = pool_cls(settings(sink.url, ca_file=pki.ca_crt, connections=1, depth=8), m)
        big = core("big", name="x" * 300_000)
        for i in range(6):
            pool.submit(f"b{i}", "ADDED", "default", "p", big, 0, TS)
        pool.flush()
        assert await pool.drain(20)
        assert m.c["notify_delivered"] == 6 and len(sink.state.received[0][1]) > 300_000
        await pool.close()
        await sink.stop()
    run(body())


@pytest.mark.parametrize("verify", [True, False])
def test_untrusted_certificate(pool_cls, pki, verify):
    """Without the CA the server certificate is rejected (notification fails);
    with verify_tls off the same server is accepted."""
    async def body():
        sink = await tls_sink(pki)
        m = Metrics()
        pool = pool_cls(settings(sink.url, verify_tls=verify, attempts=1), m)
        pool.submit("u", "ADDED", "default", "p", core("u"), 0, TS)
        pool.flush()
        assert await pool.drain(10)
        if verify:
            assert m.c["notify_failed"] == 1 and sink.state.count == 0
        else:
            assert m.c["notify_delivered"] == 1 and sink.state.count == 1
        await pool.close()
        await sink.stop()
    run(body())


def test_service_uses_native_core_for_https(pki):
    from k8s_watcher_amd.testing.podgen import PodFactory
    from test_e2e_slice import start_stack

    async def body():
        srv, sink, svc = await start_stack("staging", overrides={"clusterapi": {"ca_file": pki.ca_crt}})
        await sink.stop()
        sink = await tls_sink(pki)
        svc.settings.clusterapi.base_url = sink.url
        await svc.start()
        assert isinstance(svc.notifier, NativeNotifierPool) and svc.notifier.tls
        f = PodFactory(seed=31, namespaces=["default"])
        for _ in range(5):
            srv.create(f.running(f.new_pod()))
        await sink.state.wait_for(5, timeout=10)
        svc.stop()
        await svc.shutdown()
        await sink.stop()
        await srv.stop()
    run(body())


@pytest.mark.parametrize("with_cert", [True, False])
def test_mutual_tls(pool_cls, pki, with_cert):
    """clusterapi.cert_file/key_file: a sink that requires a client certificate
    accepts the pool only when it presents one signed by the CA."""
    async def body():
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(pki.server_crt, pki.server_key)
        ctx.load_verify_locations(pki.ca_crt)
        ctx.verify_mode = ssl.CERT_REQUIRED
        sink = StubSink()
        await sink.start(ssl_context=ctx)
        m = Metrics()
        kw = {"cert_file": pki.client_crt, "key_file": pki.client_key} if with_cert else {}
        pool = pool_cls(settings(sink.url, ca_file=pki.ca_crt, attempts=1, **kw), m)
        pool.submit("u", "ADDED", "default", "p", core("u"), 0, TS)
        pool.flush()
        assert await pool.drain(10)
        if with_cert:
            assert m.c["notify_delivered"] == 1 and sink.state.count == 1
        else:
            assert m.c["notify_failed"] == 1 and sink.state.count == 0
        await pool.close()
        await sink.stop()
    run(body())


def test_compat_clients_over_mutual_tls(pki):
    """The reference-compatible clients (sync and async) honour the same TLS settings."""
    import threading
    from k8s_watcher_amd.notify.clusterapi import AsyncClusterApiClient, ClusterApiClient
    from k8s_watcher_amd.testing.stub_sink import StubSink as _Sink

    async def body():
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(pki.server_crt, pki.server_key)
        ctx.load_verify_locations(pki.ca_crt)
        ctx.verify_mode = ssl.CERT_REQUIRED
        sink = _Sink()
        await sink.start(ssl_context=ctx)
        s = settings(sink.url, ca_file=pki.ca_crt, cert_file=pki.client_crt, key_file=pki.client_key)
        ac = AsyncClusterApiClient.from_settings(s)
        assert await ac.update_pod_status({"name": "a", "uid": "1"})
        sc = ClusterApiClient.from_settings(s)
        out = {}
        t = threading.Thread(target=lambda: out.update(ok=sc.update_pod_status({"name": "b", "uid": "2"}),
                                                       health=sc.health_check()))
        t.start()
        while t.is_alive():
            await asyncio.sleep(0.01)
        assert out == {"ok": True, "health": True}
        assert sink.state.count == 2
        await sink.stop()
    run(body())
