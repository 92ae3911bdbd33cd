"""TCP keep-alive / user-timeout options on every long-lived connection (net/sockopt.py)."""

import asyncio
import socket

from k8s_watcher_amd.net.http import HttpClient
from k8s_watcher_amd.net.sockopt import tune_socket


def _opts(sock):
    return {
        "keepalive": sock.getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE),
        "idle": sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPIDLE),
        "intvl": sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPINTVL),
        "cnt": sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_KEEPCNT),
        "user_timeout": sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_USER_TIMEOUT),
        "nodelay": sock.getsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY),
    }


def test_tune_socket_values():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        assert tune_socket(s, 30)
        o = _opts(s)
        assert o["keepalive"] and o["nodelay"]
        assert (o["idle"], o["intvl"], o["cnt"]) == (30, 10, 3)
        assert o["user_timeout"] == 60_000
    finally:
        s.close()


def test_tune_socket_disabled_and_non_tcp():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        assert tune_socket(s, 0)
        assert not s.getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE)
        assert s.getsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY)
    finally:
        s.close()
    u = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        assert not tune_socket(u, 30)
    finally:
        u.close()
    assert not tune_socket(None)


def test_http_client_connections_are_tuned():
    async def run():
        async def handle(reader, writer):
            await reader.readuntil(b"\r\n\r\n")
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
            await writer.drain()
            await reader.read()
            writer.close()

        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        client = HttpClient(f"http://127.0.0.1:{port}", keepalive=12)
        try:
            resp = await client.request("GET", "/x")
            assert resp.status == 200
            proto = client._all[0]
            return _opts(proto.transport.get_extra_info("socket"))
        finally:
            await client.close()
            srv.close()
            await srv.wait_closed()

    o = asyncio.run(run())
    assert o["keepalive"] and (o["idle"], o["intvl"], o["cnt"]) == (12, 4, 3)
    assert o["user_timeout"] == 24_000


def test_keepalive_settings():
    from k8s_watcher_amd.utils.config import ConfigError, load_settings
    s = load_settings("staging")
    assert s.kubernetes.tcp_keepalive_seconds == 30 and s.clusterapi.tcp_keepalive_seconds == 30
    s = load_settings("staging", overrides={"kubernetes": {"tcp_keepalive_seconds": 0},
                                            "clusterapi": {"tcp_keepalive_seconds": 45}})
    assert s.kubernetes.tcp_keepalive_seconds == 0 and s.clusterapi.tcp_keepalive_seconds == 45
    import pytest
    with pytest.raises(ConfigError):
        load_settings("staging", overrides={"clusterapi": {"tcp_keepalive_seconds": "soon"}})
