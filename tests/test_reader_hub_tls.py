"""https watches through the native reader hub (``ReaderHub.add_tls``).

The hub owns an https watch from the TCP connect on: OpenSSL handshake with
the kubeconfig's trust material (CA data or file, client certificate for
mutual TLS, ``tls-server-name``), the request, then decrypted bytes into the
pooled buffers. Everything the asyncio TLS path guaranteed must still hold:
certificate and host-name verification, response heads and error statuses,
the server's close, the client's close.
"""

import asyncio
import base64
import ssl
import textwrap

import pytest

from conftest import run
from k8s_watcher_amd.kube.api import ApiError, KubeApi
from k8s_watcher_amd.kube.kubeconfig import load_kube_config
from k8s_watcher_amd.net.http import HttpError
from k8s_watcher_amd.net.reader import WatchReaderHub
from k8s_watcher_amd.testing.certs import make_pki
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
from k8s_watcher_amd.testing.podgen import PodFactory


def write(path, text):
    path.write_text(textwrap.dedent(text))
    return str(path)


def server_context(pki, mutual=False):
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(pki.server_crt, pki.server_key)
    if mutual:
        ctx.load_verify_locations(pki.ca_crt)
        ctx.verify_mode = ssl.CERT_REQUIRED
    return ctx


def kubeconfig(tmp_path, pki, port, name="cfg", server_name=None, mutual=True):
    b64 = lambda p: base64.b64encode(pki.read(p)).decode()  # noqa: E731
    extra = f", tls-server-name: {server_name}" if server_name else ""
    user = (f"{{token: t0k, client-certificate-data: {b64(pki.client_crt)}, client-key-data: {b64(pki.client_key)}}}"
            if mutual else "{token: t0k}")
    return write(tmp_path / name, f"""
        current-context: x
        clusters: [{{name: c, cluster: {{server: "https://127.0.0.1:{port}",
                                       certificate-authority-data: {b64(pki.ca_crt)}{extra}}}}}]
        contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
        users: [{{name: u, user: {user}}}]
        """)


def test_https_watch_decrypted_by_the_hub_with_mutual_tls(tmp_path):
    pki = make_pki(str(tmp_path / "pki"))

    async def body():
        srv = FakeApiServer(token="t0k")
        await srv.start(ssl_context=server_context(pki, mutual=True))
        api = KubeApi(load_kube_config(kubeconfig(tmp_path, pki, srv.port)))
        hub = WatchReaderHub(1 << 20, 8)
        api.http.reader_hub = hub
        got = bytearray()
        f = PodFactory(seed=3)
        for _ in range(20):
            srv.create(f.running(f.new_pod()))
        stream = await api.watch_pods(lambda d, _ns: got.extend(d), raw_chunked=True, zero_copy=True,
                                      read_size=1 << 20)
        adopted = stream._proto.hub is hub
        for _ in range(300):  # 20 synthetic ADDED for the live pods
            if got.count(b'"type":"ADDED"') >= 20:
                break
            await asyncio.sleep(0.01)
        for _ in range(30):
            srv.create(f.running(f.new_pod()))
        for _ in range(300):
            if got.count(b'"type":"ADDED"') >= 50:
                break
            await asyncio.sleep(0.01)
        stats = hub.stats()
        stream.close()
        await asyncio.wait_for(stream.finished, 5)
        left = hub.stats()["streams"]
        hub.close()
        await api.close()
        await srv.stop()
        return adopted, bytes(got), stats, left

    adopted, got, stats, left = run(body())
    assert adopted and stats["reads"] > 0 and left == 0
    assert got.count(b'"type":"ADDED"') == 50


def test_hub_tls_verifies_the_host_name(tmp_path):
    """tls-server-name that the certificate does not cover: the hub's
    handshake fails with the verification error, as the asyncio path does."""
    pki = make_pki(str(tmp_path / "pki"))

    async def body(name):
        srv = FakeApiServer(token="t0k")
        await srv.start(ssl_context=server_context(pki))
        api = KubeApi(load_kube_config(kubeconfig(tmp_path, pki, srv.port, f"cfg-{name}", name, mutual=False)))
        hub = WatchReaderHub(1 << 20, 4)
        api.http.reader_hub = hub
        try:
            stream = await api.watch_pods(lambda d, _ns: None, raw_chunked=True, zero_copy=True)
            ok = stream._proto.hub is hub
            stream.close()
            return ok
        finally:
            hub.close()
            await api.close()
            await srv.stop()

    assert run(body("localhost")) is True
    with pytest.raises(HttpError, match="certificate verify failed|hostname mismatch|handshake"):
        run(body("wrong.example"))


def test_hub_tls_error_status_and_server_close(tmp_path):
    """A 401 answer arrives as an ApiError with its body; a watch the server
    ends (timeoutSeconds) resolves `finished`."""
    pki = make_pki(str(tmp_path / "pki"))

    async def body():
        srv = FakeApiServer(token="right")
        await srv.start(ssl_context=server_context(pki))
        hub = WatchReaderHub(1 << 20, 4)
        bad = KubeApi(load_kube_config(kubeconfig(tmp_path, pki, srv.port, "bad", mutual=False)))
        bad.http.reader_hub = hub
        status = None
        try:
            await bad.watch_pods(lambda d, _ns: None, raw_chunked=True, zero_copy=True)
        except ApiError as exc:
            status = exc.status
        await bad.close()
        srv.token = "t0k"
        good = KubeApi(load_kube_config(kubeconfig(tmp_path, pki, srv.port, "good", mutual=False)))
        good.http.reader_hub = hub
        stream = await good.watch_pods(lambda d, _ns: None, raw_chunked=True, zero_copy=True, timeout_seconds=1)
        await asyncio.wait_for(stream.finished, 10)
        hub.close()
        await good.close()
        await srv.stop()
        return status

    assert run(body()) == 401
