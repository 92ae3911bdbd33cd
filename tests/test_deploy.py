"""Deployment artefacts: RBAC, workloads, Dockerfile and dependency manifests.

The reference claims "Dockerized" (``/root/reference/README.md:9``) but ships
no image, manifest or RBAC; in-cluster it implicitly needs list/watch on pods
and list on namespaces (``pod_watcher.py:146,264``). Here
``engine.service.required_permissions`` is the single source of what a
configuration needs (``--check`` asks the API server about exactly that list)
and ``deploy/k8s/rbac.yaml`` must grant exactly the union over the shipped
workloads: a permission added to the code without RBAC — or RBAC left over
without code — fails this test.
"""

import glob
import os
import re

import pytest
import yaml

from conftest import ROOT
from k8s_watcher_amd.cli import _parser
from k8s_watcher_amd.engine.service import required_permissions
from k8s_watcher_amd.utils.config import deep_merge, load_settings, parse_override

DEPLOY = os.path.join(ROOT, "deploy", "k8s")


def docs():
    out = []
    for path in sorted(glob.glob(os.path.join(DEPLOY, "*.yaml"))):
        with open(path) as fh:
            out += [(os.path.basename(path), d) for d in yaml.safe_load_all(fh) if d]
    return out


def rbac():
    """(cluster rules, {namespace: rules}) bound to the watcher's ServiceAccount."""
    all_docs = [d for _, d in docs()]
    roles = {(d["kind"], d["metadata"].get("namespace"), d["metadata"]["name"]): d
             for d in all_docs if d["kind"] in ("ClusterRole", "Role")}
    cluster, ns_rules = [], {}
    for d in all_docs:
        if d["kind"] not in ("ClusterRoleBinding", "RoleBinding"):
            continue
        subj = d["subjects"][0]
        assert (subj["kind"], subj["name"], subj["namespace"]) == ("ServiceAccount", "k8s-watcher", "k8s-watcher")
        ref = d["roleRef"]
        ns = d["metadata"].get("namespace") if d["kind"] == "RoleBinding" else None
        role = roles[(ref["kind"], ns if ref["kind"] == "Role" else None, ref["name"])]
        if ns is None:
            cluster += role["rules"]
        else:
            ns_rules.setdefault(ns, []).extend(role["rules"])
    return cluster, ns_rules


def workloads():
    return [(f, d) for f, d in docs() if d["kind"] in ("Deployment", "StatefulSet")]


def settings_for(workload, monkeypatch):
    """The Settings the container's args and env produce (shard 0 for a StatefulSet)."""
    spec = workload["spec"]["template"]["spec"]
    c = spec["containers"][0]
    args = _parser().parse_args(c["args"])
    environ = {}
    for e in c.get("env", []):
        if "value" in e:
            environ[e["name"]] = e["value"]
        elif "fieldRef" in e.get("valueFrom", {}):
            path = e["valueFrom"]["fieldRef"]["fieldPath"]
            environ[e["name"]] = {"metadata.namespace": workload["metadata"]["namespace"],
                                  "metadata.name": workload["metadata"]["name"] + "-0"}.get(path, "0")
        else:
            environ[e["name"]] = "secret"
    for k in ("K8S_WATCHER_SHARD_COUNT", "K8S_WATCHER_SHARD_INDEX", "POD_NAMESPACE", "POD_NAME"):
        monkeypatch.delenv(k, raising=False)
        if k in environ:
            monkeypatch.setenv(k, environ[k])
    monkeypatch.setenv("POD_NAMESPACE", workload["metadata"]["namespace"])  # the Lease default
    ov = {}
    for expr in args.overrides:
        ov = deep_merge(ov, parse_override(expr))
    return load_settings(args.environment, config_dir=os.path.join(ROOT, "config"), overrides=ov, environ=environ)


def grants(rule, verb, resource, group, name):
    return (group in rule.get("apiGroups", []) and resource in rule.get("resources", [])
            and verb in rule.get("verbs", [])
            and (not rule.get("resourceNames") or (name is not None and name in rule["resourceNames"])))


def test_every_workload_is_covered_exactly_by_rbac(monkeypatch):
    cluster, ns_rules = rbac()
    needed = set()
    seen_scopes = set()
    for fname, w in workloads():
        assert w["spec"]["template"]["spec"]["serviceAccountName"] == "k8s-watcher", fname
        s = settings_for(w, monkeypatch)
        seen_scopes.add(s.watcher.namespace_scope)
        for verb, res, group, ns, name in required_permissions(s):
            ok = any(grants(r, verb, res, group, name) for r in cluster) or (
                ns is not None and any(grants(r, verb, res, group, name) for r in ns_rules.get(ns, [])))
            assert ok, f"{fname}: RBAC does not grant {verb} {group}/{res} ns={ns} name={name}"
            needed.add((verb, res, group, ns, name))
    # the shipped workloads exercise every watch mode that needs its own permissions
    assert {"client", "discover"} <= seen_scopes
    # nothing granted that no workload needs (least privilege)
    for scope, rules in [(None, cluster)] + [(ns, r) for ns, r in ns_rules.items()]:
        for rule in rules:
            for group in rule["apiGroups"]:
                for res in rule["resources"]:
                    for verb in rule["verbs"]:
                        names = rule.get("resourceNames") or [None]
                        for name in names:
                            used = any(v == verb and r == res and g == group and (scope is None or n == scope)
                                       and (name is None or nm == name)
                                       for v, r, g, n, nm in needed)
                            assert used, f"RBAC grants {verb} {group}/{res} (ns={scope}, name={name}) that no " \
                                         f"workload needs"


def test_check_asks_for_exactly_the_required_permissions():
    """--check (preflight) walks required_permissions; discover adds watch on namespaces."""
    base = load_settings("production", environ={})
    disc = load_settings("production", overrides={"watcher": {"namespace_scope": "discover"}}, environ={})
    assert ("watch", "namespaces", "", None, None) not in required_permissions(base)
    assert ("watch", "namespaces", "", None, None) in required_permissions(disc)
    srv = load_settings("production", overrides={"watcher": {"namespace_scope": "server"}}, environ={})
    assert {p[3] for p in required_permissions(srv) if p[1] == "pods"} == set(srv.watcher.namespaces)


def test_dockerfile_installs_the_declared_dependencies():
    with open(os.path.join(ROOT, "Dockerfile")) as fh:
        df = fh.read()
    assert df.count("pip install --no-cache-dir -r requirements.txt") == 2  # build + runtime stages
    assert "python -m k8s_watcher_amd.ops.native" in df  # the native extension is built into the image
    for src in re.findall(r"^COPY (?!--from)(\S+)", df, flags=re.M):
        assert os.path.exists(os.path.join(ROOT, src.rstrip("/"))), src
    assert 'ENTRYPOINT ["python", "main.py"]' in df


def test_requirements_match_pyproject():
    import tomli
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as fh:
        proj = tomli.load(fh)["project"]
    with open(os.path.join(ROOT, "requirements.txt")) as fh:
        reqs = [ln.split("#")[0].strip() for ln in fh if ln.split("#")[0].strip()]
    assert sorted(reqs) == sorted(proj["dependencies"])
    # every third-party runtime import of the package is declared
    declared = {"yaml": "PyYAML", "dateutil": "python-dateutil", "requests": "requests"}
    pkg = os.path.join(ROOT, "k8s_watcher_amd")
    for path in glob.glob(os.path.join(pkg, "**", "*.py"), recursive=True):
        if os.sep + "testing" + os.sep in path:
            continue  # fixtures: the test extra (numpy)
        with open(path) as fh:
            text = fh.read()
        for mod in re.findall(r"^\s*(?:import|from) (\w+)", text, flags=re.M):
            if mod in ("yaml", "dateutil", "requests"):
                assert any(r.startswith(declared[mod]) for r in reqs), (path, mod)
            assert mod not in ("numpy", "torch", "psutil"), f"{path} imports {mod}: not a runtime dependency"


@pytest.mark.parametrize("extra,mods", [("test", ["pytest", "hypothesis", "numpy", "psutil"]),
                                        ("bench", ["numpy", "psutil", "torch"])])
def test_optional_extras_declared(extra, mods):
    import tomli
    with open(os.path.join(ROOT, "pyproject.toml"), "rb") as fh:
        extras = tomli.load(fh)["project"]["optional-dependencies"][extra]
    for m in mods:
        assert any(e.lower().startswith(m) for e in extras), (extra, m)
