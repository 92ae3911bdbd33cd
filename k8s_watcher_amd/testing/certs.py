"""Throw-away PKI for TLS tests (``openssl`` CLI): a CA, a server cert for
127.0.0.1/localhost and a client cert, all signed by the CA."""

from __future__ import annotations

import os
import subprocess
from dataclasses import dataclass


@dataclass
class TestPKI:
    dir: str
    ca_crt: str
    server_crt: str
    server_key: str
    client_crt: str
    client_key: str

    def read(self, path: str) -> bytes:
        with open(path, "rb") as fh:
            return fh.read()


def _run(*args: str, cwd: str) -> None:
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True)


def make_pki(directory: str) -> TestPKI:
    os.makedirs(directory, exist_ok=True)
    d = directory
    _run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt",
         "-days", "2", "-subj", "/CN=k8s-watcher-test-ca", cwd=d)
    with open(os.path.join(d, "san.ext"), "w") as fh:
        fh.write("subjectAltName=IP:127.0.0.1,DNS:localhost\n")
    for name, subj, ext in (("server", "/CN=localhost", ["-extfile", "san.ext"]),
                            ("client", "/O=system:masters/CN=watcher", [])):
        _run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out", f"{name}.csr",
             "-subj", subj, cwd=d)
        _run("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
             "-out", f"{name}.crt", "-days", "2", *ext, cwd=d)
    j = lambda n: os.path.join(d, n)  # noqa: E731
    return TestPKI(d, j("ca.crt"), j("server.crt"), j("server.key"), j("client.crt"), j("client.key"))
