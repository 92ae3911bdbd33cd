"""``_kwcore.SinkServer``, the stub clusterapi's native request loop (bench
fixture): same answers and the same verify keys as the asyncio sink."""

import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from conftest import ROOT
from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.testing.stub_sink import _native_sink, payload_key


def _post(body: bytes, path: bytes = b"/api/pods/update", lower: bool = False) -> bytes:
    cl = b"content-length" if lower else b"Content-Length"
    return (b"POST %s HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n%s: %d\r\n\r\n%s"
            % (path, cl, len(body), body))


def _read_responses(sock: socket.socket, n: int, timeout: float = 5.0) -> list:
    sock.settimeout(timeout)
    buf, out = b"", []
    while len(out) < n:
        he = buf.find(b"\r\n\r\n")
        if he >= 0:
            head = buf[:he]
            cl = int(head.lower().split(b"content-length:")[1].split(b"\r\n")[0])
            if len(buf) >= he + 4 + cl:
                out.append((int(head.split(b" ")[1]), buf[he + 4:he + 4 + cl]))
                buf = buf[he + 4 + cl:]
                continue
        chunk = sock.recv(65536)
        assert chunk, "sink closed the connection"
        buf += chunk
    return out


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


BODIES = [
    b'{"name":"a","namespace":"default","uid":"u-1","status":{"phase":"Running","conditions":[]},'
    b'"event_type":"ADDED"}',
    b'{"name":"b","namespace":"default","uid":"u-2","status":{"phase":"Pending"},"metadata":{"annotations":'
    b'{"k8s-watcher.test/generation":"7"}},"event_type":"MODIFIED"}',
    b'{"name":"c","uid":"u-3","status":{"phase":null,"conditions":[]},"event_type":"DELETED"}',
    b'{"no":"fields"}',  # malformed: the key must still match the Python helper byte for byte
]


@pytest.mark.parametrize("reserve", [0, 4096])
def test_native_sink_pipelined_answers_and_keys(reserve):
    """reserve: the key table sized up front (bench --expect-keys), also after a reset."""
    port = _free_port()
    srv = _native_sink(port, True, reserve)
    try:
        with socket.create_connection(("127.0.0.1", port)) as s:
            reqs = [_post(b) for b in BODIES] + [
                b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n",
                _post(b"{}", path=b"/other"),
                _post(BODIES[0], lower=True),
            ]
            wire = b"".join(reqs)
            # split at awkward places: a request carried across reads
            for i in range(0, len(wire), 97):
                s.sendall(wire[i:i + 97])
                time.sleep(0.001)
            got = _read_responses(s, len(reqs))
        assert [st for st, _ in got] == [200] * 4 + [200, 404, 200]
        assert json.loads(got[0][1]) == {"status": "ok"}
        assert json.loads(got[4][1]) == {"status": "healthy"}
        count, keys = srv.snapshot()
        assert count == 5
        want = {}
        for b in BODIES + [BODIES[0]]:
            k = payload_key(b).decode()
            want[k] = want.get(k, 0) + 1
        assert keys == want
        assert srv.stats()["health_checks"] == 1
        count, keys = srv.snapshot(True)  # reset
        assert count == 5 and srv.snapshot() == (0, {})
    finally:
        srv.close()
    with pytest.raises(ValueError):
        srv.snapshot()


def test_native_sink_many_connections():
    port = _free_port()
    srv = _native_sink(port, False)
    try:
        socks = [socket.create_connection(("127.0.0.1", port)) for _ in range(16)]
        for k in range(20):
            for s in socks:
                s.sendall(_post(b'{"uid":"x%d"}' % k) * 3)
        for s in socks:
            assert [st for st, _ in _read_responses(s, 60)] == [200] * 60
            s.close()
        assert srv.stats()["count"] == 16 * 60
        assert srv.snapshot()[1] == {}  # not verifying: no keys kept
    finally:
        srv.close()


def test_sink_process_native_verify_dump(tmp_path):
    """``python -m ...stub_sink --engine native`` with several SO_REUSEPORT
    workers: every worker dumps its counts on SIGUSR1 and on SIGTERM."""
    port = _free_port()
    p = subprocess.Popen([sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port", str(port),
                          "--workers", "2", "--engine", "native", "--verify-dir", str(tmp_path)],
                         cwd=ROOT, stdout=subprocess.PIPE, start_new_session=True)
    try:
        p.stdout.readline()
        for _ in range(200):
            try:
                socket.create_connection(("127.0.0.1", port)).close()
                break
            except OSError:
                time.sleep(0.02)
        time.sleep(0.3)  # both workers bound
        socks = [socket.create_connection(("127.0.0.1", port)) for _ in range(8)]
        for i, s in enumerate(socks):
            s.sendall(_post(BODIES[i % 2]))
        for s in socks:
            assert _read_responses(s, 1)[0][0] == 200
            s.close()
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(10)
        dumps = [json.load(open(tmp_path / f)) for f in os.listdir(tmp_path) if f.endswith(".json")]
        assert len(dumps) == 2
        assert sum(d["count"] for d in dumps) == 8
        total = {}
        for d in dumps:
            for k, v in d["keys"].items():
                total[k] = total.get(k, 0) + v
        assert total == {payload_key(BODIES[0]).decode(): 4, payload_key(BODIES[1]).decode(): 4}
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(5)


def test_native_sink_rejects_bad_fd():
    with pytest.raises(OSError):
        load().SinkServer(-1)
    with pytest.raises(ValueError):
        load().SinkServer(0, b"/api/pods/update", True, -1)


def test_native_sink_reports_stalls_as_a_list():
    """stalls(): serving-loop turns over 20 ms with the thread's rusage deltas
    (none on an idle sink); the bench lines them up with its per-second rows."""
    import socket
    from k8s_watcher_amd.ops.native import load
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    sock.listen(8)
    srv = load().SinkServer(sock.fileno(), b"/api/pods/update", True, 16)
    sock.close()
    try:
        st = srv.stalls()
        assert isinstance(st, list) and all(len(x) == 7 for x in st)
    finally:
        srv.close()
