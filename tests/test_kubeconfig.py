"""Kubeconfig / in-cluster loading and TLS end to end."""

import base64
import os
import ssl
import sys
import textwrap

import pytest

from conftest import ROOT, run
from k8s_watcher_amd.kube.api import KubeApi
from k8s_watcher_amd.kube.kubeconfig import (ConfigException, list_kube_config_contexts, load_incluster_config,
                                             load_kube_config)
from k8s_watcher_amd.testing.certs import make_pki
from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer


def write(path, text):
    path.write_text(textwrap.dedent(text))
    return str(path)


def two_context_config(tmp_path):
    return write(tmp_path / "config", """
        apiVersion: v1
        kind: Config
        current-context: a
        clusters:
        - name: ca
          cluster: {server: "http://127.0.0.1:1111/"}
        - name: cb
          cluster: {server: "http://127.0.0.1:2222"}
        users:
        - name: ua
          user: {token: tok-a}
        - name: ub
          user: {username: admin, password: pw}
        contexts:
        - name: a
          context: {cluster: ca, user: ua, namespace: team-a}
        - name: b
          context: {cluster: cb, user: ub}
        """)


def test_current_and_explicit_context(tmp_path):
    p = two_context_config(tmp_path)
    ep = load_kube_config(p)
    assert ep.server == "http://127.0.0.1:1111"
    assert ep.auth_headers() == {"Authorization": "Bearer tok-a"}
    assert ep.namespace == "team-a" and ep.context_name == "a"
    ep = load_kube_config(p, context="b")
    assert ep.server == "http://127.0.0.1:2222"
    assert ep.auth_headers()["Authorization"] == "Basic " + base64.b64encode(b"admin:pw").decode()
    with pytest.raises(ConfigException):
        load_kube_config(p, context="missing")


def test_list_contexts_like_library(tmp_path):
    contexts, active = list_kube_config_contexts(two_context_config(tmp_path))
    assert [c["name"] for c in contexts] == ["a", "b"]
    assert active["name"] == "a" and active["context"]["cluster"] == "ca"


def test_missing_file_raises(tmp_path):
    with pytest.raises(ConfigException):
        load_kube_config(str(tmp_path / "nope"))


def test_kubeconfig_env_merge_first_wins(tmp_path, monkeypatch):
    a = write(tmp_path / "a.yaml", """
        current-context: x
        clusters: [{name: c, cluster: {server: "http://first"}}]
        contexts: [{name: x, context: {cluster: c, user: u}}]
        users: [{name: u, user: {token: t1}}]
        """)
    b = write(tmp_path / "b.yaml", """
        current-context: y
        clusters: [{name: c, cluster: {server: "http://second"}}, {name: d, cluster: {server: "http://d"}}]
        contexts: [{name: y, context: {cluster: d, user: u}}]
        users: [{name: u, user: {token: t2}}]
        """)
    monkeypatch.setenv("KUBECONFIG", os.pathsep.join([a, b]))
    ep = load_kube_config()
    assert ep.server == "http://first" and ep.auth_headers()["Authorization"] == "Bearer t1"
    assert load_kube_config(context="y").server == "http://d"


def test_token_file_relative_and_rotation(tmp_path):
    (tmp_path / "tok").write_text("one\n")
    p = write(tmp_path / "cfg", """
        current-context: x
        clusters: [{name: c, cluster: {server: "http://h"}}]
        contexts: [{name: x, context: {cluster: c, user: u}}]
        users: [{name: u, user: {tokenFile: tok}}]
        """)
    ep = load_kube_config(p)
    assert ep.auth_headers() == {"Authorization": "Bearer one"}


def test_exec_credential_plugin(tmp_path):
    plugin = tmp_path / "plugin.py"
    plugin.write_text("import json,os\nprint(json.dumps({'apiVersion':'client.authentication.k8s.io/v1beta1',"
                      "'kind':'ExecCredential','status':{'token':'exec-'+os.environ['X']}}))\n")
    p = write(tmp_path / "cfg", f"""
        current-context: x
        clusters: [{{name: c, cluster: {{server: "http://h"}}}}]
        contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
        users:
        - name: u
          user:
            exec:
              apiVersion: client.authentication.k8s.io/v1beta1
              command: {sys.executable}
              args: ["{plugin}"]
              env: [{{name: X, value: "42"}}]
        """)
    assert load_kube_config(p).auth_headers() == {"Authorization": "Bearer exec-42"}


def test_exec_credential_relative_command(tmp_path):
    # client-go: a command with a path separator resolves against the kubeconfig's directory
    (tmp_path / "bin").mkdir()
    plugin = tmp_path / "bin" / "cred.sh"
    plugin.write_text('#!/bin/sh\necho \'{"kind":"ExecCredential","status":{"token":"rel-tok"}}\'\n')
    plugin.chmod(0o755)
    p = write(tmp_path / "cfg", """
        current-context: x
        clusters: [{name: c, cluster: {server: "http://h"}}]
        contexts: [{name: x, context: {cluster: c, user: u}}]
        users: [{name: u, user: {exec: {command: ./bin/cred.sh, env: [{name: ONLY_NAME}]}}}]
        """)
    assert load_kube_config(p).auth_headers() == {"Authorization": "Bearer rel-tok"}


def test_repo_dummy_kubeconfig():
    """assets/config (C13): plain HTTP to localhost:9988 with a bearer token."""
    ep = load_kube_config(os.path.join(ROOT, "assets", "config"))
    assert ep.server == "http://localhost:9988"
    assert ep.ssl_context is None
    assert ep.auth_headers()["Authorization"].startswith("Bearer ")


def test_incluster(tmp_path):
    pki = make_pki(str(tmp_path / "pki"))
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("sa-token")
    (sa / "ca.crt").write_bytes(pki.read(pki.ca_crt))
    (sa / "namespace").write_text("watchers")
    env = {"KUBERNETES_SERVICE_HOST": "10.0.0.1", "KUBERNETES_SERVICE_PORT": "443"}
    ep = load_incluster_config(str(sa), env)
    assert ep.server == "https://10.0.0.1:443"
    assert ep.auth_headers() == {"Authorization": "Bearer sa-token"}
    assert ep.namespace == "watchers"
    with pytest.raises(ConfigException):
        load_incluster_config(str(sa), {})
    with pytest.raises(ConfigException):
        load_incluster_config(str(tmp_path / "nosa"), env)


def test_tls_with_ca_data_and_client_cert(tmp_path):
    pki = make_pki(str(tmp_path / "pki"))
    b64 = lambda p: base64.b64encode(pki.read(p)).decode()  # noqa: E731
    server_ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    server_ctx.load_cert_chain(pki.server_crt, pki.server_key)
    server_ctx.load_verify_locations(pki.ca_crt)
    server_ctx.verify_mode = ssl.CERT_REQUIRED  # mutual TLS

    async def body():
        srv = FakeApiServer(token="t0k")
        await srv.start(ssl_context=server_ctx)
        cfg = write(tmp_path / "cfg", f"""
            current-context: x
            clusters: [{{name: c, cluster: {{server: "https://127.0.0.1:{srv.port}",
                                           certificate-authority-data: {b64(pki.ca_crt)}}}}}]
            contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
            users:
            - name: u
              user: {{token: t0k, client-certificate-data: {b64(pki.client_crt)},
                      client-key-data: {b64(pki.client_key)}}}
            """)
        api = KubeApi(load_kube_config(cfg))
        ver = await api.get_version()
        await api.close()
        await srv.stop()
        return ver

    assert run(body())["gitVersion"].startswith("v1.33")


def test_tls_server_name_is_verified(tmp_path):
    # tls-server-name: SNI and the certificate check use that name, not the
    # URL host (the server certificate covers "localhost", not "wrong.example")
    from k8s_watcher_amd.net.http import HttpError

    pki = make_pki(str(tmp_path / "pki"))
    server_ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    server_ctx.load_cert_chain(pki.server_crt, pki.server_key)

    async def body(name):
        srv = FakeApiServer()
        await srv.start(ssl_context=server_ctx)
        cfg = write(tmp_path / f"cfg-{name}", f"""
            current-context: x
            clusters: [{{name: c, cluster: {{server: "https://127.0.0.1:{srv.port}",
                                           certificate-authority: {pki.ca_crt}, tls-server-name: {name}}}}}]
            contexts: [{{name: x, context: {{cluster: c, user: u}}}}]
            users: [{{name: u, user: {{}}}}]
            """)
        ep = load_kube_config(cfg)
        assert ep.tls_server_name == name
        api = KubeApi(ep)
        try:
            return await api.get_version()
        finally:
            await api.close()
            await srv.stop()

    assert run(body("localhost"))["gitVersion"].startswith("v1.33")
    with pytest.raises(HttpError, match="CERTIFICATE_VERIFY_FAILED|match"):
        run(body("wrong.example"))


def test_exec_credential_refreshes_in_background_before_expiry(tmp_path):
    import time

    from k8s_watcher_amd.kube.kubeconfig import _ExecCredential

    counter = tmp_path / "n"
    plugin = tmp_path / "plugin.py"
    plugin.write_text(textwrap.dedent(f"""
        import datetime, json
        p = {str(counter)!r}
        try:
            n = int(open(p).read())
        except OSError:
            n = 0
        open(p, "w").write(str(n + 1))
        exp = datetime.datetime.now(datetime.timezone.utc) + datetime.timedelta(seconds=60)
        print(json.dumps({{"kind": "ExecCredential", "status": {{"token": "t%d" % n,
              "expirationTimestamp": exp.strftime("%Y-%m-%dT%H:%M:%SZ")}}}}))
        """))
    cred = _ExecCredential({"command": sys.executable, "args": [str(plugin)]})
    assert cred.headers() == {"Authorization": "Bearer t0"}  # first token: fetched in the foreground
    # 60 s left (< 120 s): the next call answers at once with the current token
    # and refreshes on a thread
    assert cred.headers() == {"Authorization": "Bearer t0"}
    deadline = time.time() + 20
    while cred._bg is not None and time.time() < deadline:
        time.sleep(0.05)
    assert cred.headers()["Authorization"] in ("Bearer t1", "Bearer t2")
    assert int(counter.read_text()) >= 2
