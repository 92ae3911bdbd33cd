"""Synthetic, realistic Pod objects and churn workloads for tests and benchmarks.

There is no cluster, ``kind`` or ``kubectl`` here, so every
scenario is driven from generated objects shaped like real kube-apiserver
output: full metadata including ``managedFields`` and ``ownerReferences``,
a spec with volumes/probes/tolerations, and a status whose conditions and
container states follow the real lifecycle
``Pending → Pending(scheduled) → Running → Succeeded|Failed → deleted``.
A typical object serialises to ≈4-5 KB, which is what makes decode cost
matter at scale.
"""

from __future__ import annotations

import datetime as _dt
import json
import random
import uuid
from typing import Any, Dict, Iterator, List, Optional, Tuple

BASE_TIME = _dt.datetime(2025, 7, 9, 1, 51, 28, tzinfo=_dt.timezone.utc)

NAMESPACES_DEFAULT = ["default", "kube-system", "production", "monitoring",
                      "staging", "batch", "ml-train", "ingress"]


def _clone(obj: Any) -> Any:
    """Deep copy of a JSON document (several times faster than ``copy.deepcopy``)."""
    return json.loads(json.dumps(obj))


def _ts(offset_s: float) -> str:
    return (BASE_TIME + _dt.timedelta(seconds=offset_s)).strftime("%Y-%m-%dT%H:%M:%SZ")


def _uid(rng: random.Random) -> str:
    return str(uuid.UUID(int=rng.getrandbits(128), version=4))


class PodFactory:
    """Deterministic (seeded) generator of pods and their lifecycle states."""

    def __init__(self, seed: int = 0, namespaces: Optional[List[str]] = None,
                 containers: int = 1) -> None:
        self.rng = random.Random(seed)
        self.namespaces = namespaces or NAMESPACES_DEFAULT
        self.containers = containers
        self.counter = 0

    def new_pod(self, namespace: Optional[str] = None, name: Optional[str] = None) -> Dict[str, Any]:
        rng = self.rng
        self.counter += 1
        ns = namespace or self.namespaces[self.counter % len(self.namespaces)]
        app = f"app-{self.counter % 97}"
        rs_hash = f"{rng.getrandbits(40):010x}"[:10]
        name = name or f"{app}-{rs_hash}-{rng.getrandbits(20):05x}"
        t0 = self.counter * 0.5
        uid = _uid(rng)
        containers = []
        for ci in range(self.containers):
            cname = app if ci == 0 else f"sidecar-{ci}"
            containers.append({
                "name": cname,
                "image": f"registry.example.com/team/{app}:v1.{self.counter % 13}.{ci}",
                "ports": [{"containerPort": 8080 + ci, "protocol": "TCP", "name": "http"}],
                "env": [{"name": "APP_ENV", "value": "prod"},
                        {"name": "POD_NAME", "valueFrom": {"fieldRef": {"apiVersion": "v1",
                                                                         "fieldPath": "metadata.name"}}}],
                "resources": {"limits": {"cpu": "2", "memory": "4Gi", "amd.com/gpu": "1"},
                              "requests": {"cpu": "500m", "memory": "1Gi", "amd.com/gpu": "1"}},
                "volumeMounts": [{"name": "kube-api-access", "readOnly": True,
                                  "mountPath": "/var/run/secrets/kubernetes.io/serviceaccount"}],
                "livenessProbe": {"httpGet": {"path": "/healthz", "port": 8080 + ci, "scheme": "HTTP"},
                                  "initialDelaySeconds": 10, "timeoutSeconds": 1, "periodSeconds": 10,
                                  "successThreshold": 1, "failureThreshold": 3},
                "terminationMessagePath": "/dev/termination-log",
                "terminationMessagePolicy": "File",
                "imagePullPolicy": "IfNotPresent",
            })
        pod = {
            "kind": "Pod",
            "apiVersion": "v1",
            "metadata": {
                "name": name,
                "generateName": f"{app}-{rs_hash}-",
                "namespace": ns,
                "uid": uid,
                "resourceVersion": "0",
                "creationTimestamp": _ts(t0),
                "labels": {"app": app, "pod-template-hash": rs_hash, "tier": "backend",
                           "team": f"team-{self.counter % 7}"},
                "annotations": {"kubectl.kubernetes.io/restartedAt": _ts(t0 - 3600),
                                "prometheus.io/scrape": "true",
                                "note": "multi-line\n\"quoted\" été ✓"},
                "ownerReferences": [{"apiVersion": "apps/v1", "kind": "ReplicaSet",
                                     "name": f"{app}-{rs_hash}", "uid": _uid(rng),
                                     "controller": True, "blockOwnerDeletion": True}],
                "managedFields": [
                    {"manager": "kube-controller-manager", "operation": "Update", "apiVersion": "v1",
                     "time": _ts(t0), "fieldsType": "FieldsV1",
                     "fieldsV1": {"f:metadata": {"f:generateName": {}, "f:labels": {".": {}, "f:app": {},
                                                                                     "f:pod-template-hash": {}},
                                                 "f:ownerReferences": {".": {}, f"k:{{\"uid\":\"{uid}\"}}": {}}},
                                  "f:spec": {"f:containers": {f"k:{{\"name\":\"{app}\"}}": {
                                      ".": {}, "f:image": {}, "f:imagePullPolicy": {}, "f:name": {},
                                      "f:ports": {}, "f:resources": {}}}}}},
                    {"manager": "kubelet", "operation": "Update", "apiVersion": "v1", "time": _ts(t0 + 2),
                     "fieldsType": "FieldsV1", "subresource": "status",
                     "fieldsV1": {"f:status": {"f:conditions": {}, "f:containerStatuses": {},
                                               "f:hostIP": {}, "f:phase": {}, "f:podIP": {},
                                               "f:startTime": {}}}},
                ],
            },
            "spec": {
                "volumes": [{"name": "kube-api-access", "projected": {
                    "sources": [{"serviceAccountToken": {"expirationSeconds": 3607, "path": "token"}},
                                {"configMap": {"name": "kube-root-ca.crt",
                                               "items": [{"key": "ca.crt", "path": "ca.crt"}]}}],
                    "defaultMode": 420}}],
                "containers": containers,
                "restartPolicy": "Always",
                "terminationGracePeriodSeconds": 30,
                "dnsPolicy": "ClusterFirst",
                "serviceAccountName": "default",
                "serviceAccount": "default",
                "securityContext": {},
                "schedulerName": "default-scheduler",
                "tolerations": [
                    {"key": "node.kubernetes.io/not-ready", "operator": "Exists", "effect": "NoExecute",
                     "tolerationSeconds": 300},
                    {"key": "node.kubernetes.io/unreachable", "operator": "Exists", "effect": "NoExecute",
                     "tolerationSeconds": 300}],
                "priority": 0,
                "enableServiceLinks": True,
                "preemptionPolicy": "PreemptLowerPriority",
            },
            "status": {"phase": "Pending", "qosClass": "Burstable"},
        }
        return pod

    # ----------------------------------------------------------------- lifecycle
    def scheduled(self, pod: Dict[str, Any]) -> Dict[str, Any]:
        p = _clone(pod)
        n = self.counter
        p["spec"]["nodeName"] = f"mi355x-node-{n % 16:02d}"
        t0 = 1.0
        p["status"] = {
            "phase": "Pending",
            "conditions": [
                {"type": "PodScheduled", "status": "True", "lastProbeTime": None,
                 "lastTransitionTime": _ts(t0)},
                {"type": "Initialized", "status": "True", "lastProbeTime": None,
                 "lastTransitionTime": _ts(t0)},
                {"type": "Ready", "status": "False", "lastProbeTime": None, "lastTransitionTime": _ts(t0),
                 "reason": "ContainersNotReady", "message": f"containers with unready status: [{self._cn(p)}]"},
                {"type": "ContainersReady", "status": "False", "lastProbeTime": None,
                 "lastTransitionTime": _ts(t0), "reason": "ContainersNotReady",
                 "message": f"containers with unready status: [{self._cn(p)}]"},
            ],
            "hostIP": f"10.0.{n % 256}.{(n // 256) % 256}",
            "startTime": _ts(t0),
            "containerStatuses": [
                {"name": c["name"], "state": {"waiting": {"reason": "ContainerCreating"}},
                 "lastState": {}, "ready": False, "restartCount": 0, "image": c["image"], "imageID": "",
                 "started": False} for c in p["spec"]["containers"]],
            "qosClass": "Burstable",
        }
        return p

    def running(self, pod: Dict[str, Any]) -> Dict[str, Any]:
        p = _clone(pod) if "conditions" in (pod.get("status") or {}) else self.scheduled(pod)
        st = p["status"]
        st["phase"] = "Running"
        n = self.counter
        st["podIP"] = f"10.244.{n % 256}.{(n * 7) % 256}"
        st["podIPs"] = [{"ip": st["podIP"]}]
        for c in st["conditions"]:
            if c["type"] in ("Ready", "ContainersReady"):
                c["status"] = "True"
                c.pop("reason", None)
                c.pop("message", None)
                c["lastTransitionTime"] = _ts(5)
        for cs in st["containerStatuses"]:
            cs["state"] = {"running": {"startedAt": _ts(4)}}
            cs["ready"] = True
            cs["started"] = True
            cs["imageID"] = f"registry.example.com/team/app@sha256:{self.rng.getrandbits(256):064x}"
            cs["containerID"] = f"containerd://{self.rng.getrandbits(256):064x}"
        return p

    def terminated(self, pod: Dict[str, Any], failed: bool = False) -> Dict[str, Any]:
        p = self.running(pod) if (pod.get("status") or {}).get("phase") != "Running" else _clone(pod)
        st = p["status"]
        st["phase"] = "Failed" if failed else "Succeeded"
        for c in st["conditions"]:
            if c["type"] in ("Ready", "ContainersReady"):
                c["status"] = "False"
                c["reason"] = "PodCompleted" if not failed else "PodFailed"
                c["lastTransitionTime"] = _ts(60)
        for cs in st["containerStatuses"]:
            cs["state"] = {"terminated": {
                "exitCode": 1 if failed else 0, "reason": "Error" if failed else "Completed",
                "startedAt": _ts(4), "finishedAt": _ts(60),
                "containerID": cs.get("containerID", "containerd://0")}}
            cs["ready"] = False
            cs["started"] = False
        return p

    def deleting(self, pod: Dict[str, Any]) -> Dict[str, Any]:
        p = _clone(pod)
        p["metadata"]["deletionTimestamp"] = _ts(90)
        p["metadata"]["deletionGracePeriodSeconds"] = 0
        return p

    @staticmethod
    def _cn(p: Dict[str, Any]) -> str:
        return " ".join(c["name"] for c in p["spec"]["containers"])

    def lifecycle(self, namespace: Optional[str] = None, failed: Optional[bool] = None
                  ) -> List[Tuple[str, Dict[str, Any]]]:
        """One pod's full churn: ADDED, 3×MODIFIED, DELETED."""
        p0 = self.new_pod(namespace)
        p1 = self.scheduled(p0)
        p2 = self.running(p1)
        if failed is None:
            failed = self.rng.random() < 0.1
        p3 = self.terminated(p2, failed)
        p4 = self.deleting(p3)
        return [("ADDED", p0), ("MODIFIED", p1), ("MODIFIED", p2), ("MODIFIED", p3), ("DELETED", p4)]


def churn_events(n_pods: int, seed: int = 0, namespaces: Optional[List[str]] = None,
                 interleave: int = 64) -> Iterator[Tuple[str, Dict[str, Any]]]:
    """Interleaved lifecycles of ``n_pods`` pods (``interleave`` pods in flight at once)."""
    f = PodFactory(seed, namespaces)
    active: List[List[Tuple[str, Dict[str, Any]]]] = []
    made = 0
    rng = random.Random(seed + 1)
    while made < n_pods or active:
        while made < n_pods and len(active) < interleave:
            active.append(f.lifecycle())
            made += 1
        i = rng.randrange(len(active))
        yield active[i].pop(0)
        if not active[i]:
            active.pop(i)


def event_line(etype: str, obj: Dict[str, Any]) -> bytes:
    return json.dumps({"type": etype, "object": obj}, separators=(",", ":"),
                      ensure_ascii=False).encode("utf-8") + b"\n"
