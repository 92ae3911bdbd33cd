"""Payload extraction (schema §2.3) and filters (C8, C9)."""

import json

import pytest

from k8s_watcher_amd.models.payload import build_core, build_payload_dict, container_state_repr, finish_body
from k8s_watcher_amd.ops.filters import CriticalFilter, NamespaceFilter, is_critical
from k8s_watcher_amd.testing.podgen import PodFactory
from k8s_watcher_amd.utils.timefmt import k8s_time_to_isoformat


def test_full_pod_payload_fields():
    f = PodFactory(seed=5)
    pod = f.running(f.new_pod(namespace="default"))
    p = build_payload_dict(pod, "staging", event_type="MODIFIED")
    assert p["name"] == pod["metadata"]["name"]
    assert p["namespace"] == "default"
    assert p["uid"] == pod["metadata"]["uid"]
    assert p["environment"] == "staging"
    assert p["status"]["phase"] == "Running"
    assert [c["type"] for c in p["status"]["conditions"]] == ["PodScheduled", "Initialized", "Ready",
                                                              "ContainersReady"]
    cs = p["status"]["container_statuses"][0]
    assert cs["ready"] is True and cs["restart_count"] == 0
    assert cs["state"] == {"running": {"startedAt": "2025-07-09T01:51:32Z"}}
    assert p["spec"]["node_name"].startswith("mi355x-node-")
    assert p["spec"]["containers"][0]["image"].startswith("registry.example.com/")
    assert p["metadata"]["labels"]["tier"] == "backend"
    assert p["metadata"]["creation_timestamp"].endswith("+00:00")
    assert p["event_type"] == "MODIFIED"
    assert list(p) == ["name", "namespace", "uid", "environment", "status", "spec", "metadata",
                       "event_timestamp", "event_type"]


def test_status_null_means_unknown():
    pod = {"metadata": {"name": "a", "namespace": "n", "uid": "u"}, "status": None}
    p = build_payload_dict(pod, "development")
    assert p["status"] == {"phase": "Unknown", "conditions": [], "container_statuses": []}
    assert p["spec"] == {"node_name": None, "containers": []}
    assert p["metadata"] == {"labels": {}, "annotations": {}, "creation_timestamp": None}


def test_empty_status_object_has_null_phase():
    p = build_payload_dict({"metadata": {}, "status": {}}, "x")
    assert p["status"] == {"phase": None, "conditions": [], "container_statuses": []}


# Hand-derived from kubernetes==33.1.0: str(V1ContainerState) is
# pprint.pformat(to_dict()) (model_utils to_str); to_dict keeps datetimes that
# ApiClient.deserialize built with dateutil.parser.parse, whose repr carries
# tzinfo=tzutc(); pprint sorts keys and wraps at width 80, one key per line,
# nested dicts aligned after their key (/root/reference/watcher/pod_watcher.py:181).
REPR_RUNNING = ("{'running': {'started_at': datetime.datetime(2025, 7, 9, 1, 51, 32, tzinfo=tzutc())},\n"
                " 'terminated': None,\n"
                " 'waiting': None}")
REPR_WAITING = ("{'running': None,\n"
                " 'terminated': None,\n"
                " 'waiting': {'message': 'Back-off pulling image \"registry.example.com/app:v1\"',\n"
                "             'reason': 'ImagePullBackOff'}}")
# within pprint's width of 80 the dict stays on one line; 81 characters wrap
REPR_EMPTY = "{'running': None, 'terminated': None, 'waiting': None}"
REPR_WAITING_81 = ("{'running': None,\n"
                   " 'terminated': None,\n"
                   " 'waiting': {'message': None, 'reason': ''}}")
REPR_TERMINATED = ("{'running': None,\n"
                   " 'terminated': {'container_id': 'containerd://4f2a',\n"
                   "                'exit_code': 137,\n"
                   "                'finished_at': datetime.datetime(2025, 7, 9, 1, 52, 28, tzinfo=tzutc()),\n"
                   "                'message': 'OOMKilled: memory limit 4Gi',\n"
                   "                'reason': 'OOMKilled',\n"
                   "                'signal': 9,\n"
                   "                'started_at': datetime.datetime(2025, 7, 9, 1, 51, 32, tzinfo=tzutc())},\n"
                   " 'waiting': None}")


@pytest.mark.parametrize("state,text", [
    ({"running": {"startedAt": "2025-07-09T01:51:32Z"}}, REPR_RUNNING),
    ({"waiting": {"reason": "ImagePullBackOff",
                  "message": 'Back-off pulling image "registry.example.com/app:v1"'}}, REPR_WAITING),
    ({}, REPR_EMPTY),
    ({"waiting": {"reason": ""}}, REPR_WAITING_81),
    ({"terminated": {"exitCode": 137, "signal": 9, "reason": "OOMKilled", "message": "OOMKilled: memory limit 4Gi",
                     "startedAt": "2025-07-09T01:51:32Z", "finishedAt": "2025-07-09T01:52:28Z",
                     "containerID": "containerd://4f2a"}}, REPR_TERMINATED),
])
@pytest.mark.parametrize("tz", ["America/New_York", "UTC"])
def test_python_repr_state_matches_library_to_str(state, text, tz, monkeypatch):
    """dateutil (what the library deserialises datetimes with) returns
    ``tzlocal()`` for a ``Z`` timestamp when the process runs in UTC, else
    ``tzutc()``: the reference's text depends on the pod's TZ, and so does ours."""
    import time
    monkeypatch.setenv("TZ", tz)
    time.tzset()
    try:
        if tz == "UTC":
            text = text.replace("tzinfo=tzutc()", "tzinfo=tzlocal()")
        assert container_state_repr(state) == text
    finally:
        monkeypatch.undo()
        time.tzset()
    p = build_payload_dict({"metadata": {}, "status": {"containerStatuses": [{"name": "c", "state": state}]}},
                           "production", state_format="python_repr")
    assert p["status"]["container_statuses"][0]["state"] == container_state_repr(state)


@pytest.mark.parametrize("raw,iso", [
    ("2025-07-09T01:51:28Z", "2025-07-09T01:51:28+00:00"),
    ("2025-07-09T01:51:28.5Z", "2025-07-09T01:51:28.500000+00:00"),
    ("2025-07-09T01:51:28.000000Z", "2025-07-09T01:51:28+00:00"),
    ("2025-07-09T01:51:28.123456789Z", "2025-07-09T01:51:28.123456+00:00"),
    ("2025-07-09T10:51:28+09:00", "2025-07-09T10:51:28+09:00"),
    ("2025-07-09T10:51:28+0900", "2025-07-09T10:51:28+09:00"),
    ("2025-07-09T10:51:28", "2025-07-09T10:51:28"),
    ("garbage", "garbage"),
    (None, None),
])
def test_creation_timestamp_isoformat(raw, iso):
    assert k8s_time_to_isoformat(raw) == iso


def test_core_and_finish_body_roundtrip():
    f = PodFactory(seed=2)
    pod = f.new_pod()
    core = build_core(pod, "production")
    body = finish_body(core, "ADDED", "2025-01-01T00:00:00.000001")
    doc = json.loads(body)
    assert doc["event_type"] == "ADDED" and doc["event_timestamp"] == "2025-01-01T00:00:00.000001"
    assert list(doc)[-2:] == ["event_timestamp", "event_type"]


@pytest.mark.parametrize("etype,has_status,phase,keep", [
    ("DELETED", True, "Running", True),
    ("ADDED", False, None, True),
    ("MODIFIED", True, "Failed", True),
    ("MODIFIED", True, "Succeeded", True),
    ("MODIFIED", True, "Running", False),
    ("ADDED", True, "Pending", False),
    ("ADDED", True, None, False),  # status: {} is truthy in the reference
])
def test_critical_predicate_truth_table(etype, has_status, phase, keep):
    assert is_critical(etype, has_status, phase) is keep
    assert CriticalFilter("production", True)(etype, has_status, phase) is keep
    # inactive outside production or when the switch is off
    assert CriticalFilter("staging", True)(etype, has_status, phase) is True
    assert CriticalFilter("production", False)(etype, has_status, phase) is True


def test_namespace_filter():
    f = NamespaceFilter(["default", "kube-system"])
    assert f("default") and f("kube-system") and not f("batch") and not f(None)
    assert NamespaceFilter([])("anything")
