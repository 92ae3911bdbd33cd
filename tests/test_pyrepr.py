"""state_format: python_repr rendered natively (``ops/csrc/pyrepr.inc``)
against ``models/payload.py::container_state_repr`` — the real pprint and
dateutil, i.e. the reference's ``str(V1ContainerState)``
(``/root/reference/watcher/pod_watcher.py:181``): byte-identical payload cores
for running / waiting / terminated states, messages around pprint's 80-column
boundary and its string wrapping, every timestamp shape, in a UTC process and
not; plus the fused pipeline and a format-2 checkpoint in that mode."""

import json
import time

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from k8s_watcher_amd.ops.decode import PyDecoder
from k8s_watcher_amd.ops.native import NativeDecoder

ascii_text = st.text(alphabet=st.characters(min_codepoint=0, max_codepoint=127), max_size=140)
words = st.lists(st.sampled_from(["Back-off", "pulling", "image", '"registry.example.com/app:v1"', "OOMKilled:",
                                  "memory", "limit", "4Gi", "it's", "a\\b", "x" * 30, "  ", "\n", "\t", "\r\n",
                                  "'quoted'", '"dq"', "\x1c", "\x0b"]), max_size=30).map("".join)
text = st.one_of(ascii_text, words, st.none(), st.just(""))
times = st.one_of(
    st.none(),
    st.builds(lambda y, mo, d, h, mi, s, frac, tz: f"{y:04d}-{mo:02d}-{d:02d}T{h:02d}:{mi:02d}:{s:02d}{frac}{tz}",
              st.integers(1970, 2099), st.integers(1, 12), st.integers(1, 28), st.integers(0, 23),
              st.integers(0, 59), st.integers(0, 59),
              st.sampled_from(["", ".5", ".000000", ".123456789", ".01"]),
              st.sampled_from(["Z", "z", "+00:00", "-00:00", "+0000", "+02:00", "-05:30", ""])),
    st.sampled_from(["2025-02-30T00:00:00Z", "2024-02-29T00:00:00Z", "not a time", "2025-07-09 01:51:32",
                     "2025-07-09T24:00:00Z"]))
ints = st.one_of(st.none(), st.integers(-2 ** 31, 2 ** 31), st.just(137))
odd = st.one_of(st.floats(allow_nan=False, allow_infinity=False), st.booleans(), st.just([1]),
                st.text(min_size=1, max_size=5))  # floats, lists, non-ASCII: the Python fallback

state = st.fixed_dictionaries({}, optional={
    "running": st.one_of(st.none(), st.fixed_dictionaries({}, optional={"startedAt": times})),
    "waiting": st.one_of(st.none(), st.fixed_dictionaries({}, optional={"reason": text, "message": text})),
    "terminated": st.one_of(st.none(), st.fixed_dictionaries({}, optional={
        "exitCode": st.one_of(ints, odd), "signal": ints, "reason": text, "message": st.one_of(text, odd),
        "startedAt": times, "finishedAt": times, "containerID": text})),
})


def cores(pod: dict):
    line = json.dumps({"type": "MODIFIED", "object": pod}).encode() + b"\n"
    py = PyDecoder("production", "python_repr")
    nat = NativeDecoder("production", "python_repr")
    a, b = py.feed(line)[0], nat.feed(line)[0]
    return (a[0], b[0], py.core(a) if a[0] != "INVALID" else None,
            nat.core(b) if b[0] != "INVALID" else None)


@pytest.fixture(params=["America/New_York", "UTC"])
def tz(request, monkeypatch):
    monkeypatch.setenv("TZ", request.param)
    time.tzset()
    yield request.param
    monkeypatch.undo()
    time.tzset()


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                   HealthCheck.function_scoped_fixture])
@given(states=st.lists(state, min_size=1, max_size=3))
def test_native_python_repr_is_byte_identical(tz, states):
    pod = {"metadata": {"name": "p", "namespace": "default", "uid": "u", "resourceVersion": "1"},
           "status": {"phase": "Running",
                      "containerStatuses": [{"name": f"c{i}", "ready": True, "restartCount": 0, "state": s}
                                            for i, s in enumerate(states)]}}
    ta, tb, ca, cb = cores(pod)
    assert ta == tb
    assert ca == cb


@pytest.mark.parametrize("msg_len", range(40, 60))
def test_width_boundary_and_wrapping(tz, msg_len):
    """Around pprint's 80 columns: one line, one key per line, then a message cut into literals."""
    for reason in ("", "ImagePullBackOff"):
        pod = {"status": {"containerStatuses": [{"name": "c", "state": {
            "waiting": {"reason": reason, "message": ("word " * 40)[:msg_len]}}}]}}
        ta, tb, ca, cb = cores(pod)
        assert ca == cb
        pod["status"]["containerStatuses"][0]["state"]["waiting"]["message"] = "y" * (msg_len * 2)
        ta, tb, ca, cb = cores(pod)
        assert ca == cb


def test_common_states_never_need_the_python_formatter():
    """The shapes the API sends are rendered in C++: the fallback is not called."""
    from k8s_watcher_amd.testing.podgen import churn_events, event_line

    def boom(_obj):
        raise AssertionError("python fallback used")

    d = NativeDecoder("production", "python_repr")
    d._d.set_repr("tzutc()", boom)
    data = b"".join(event_line(t, o) for t, o in churn_events(50, seed=4))
    evs = d.feed(data)
    assert evs and all(e[0] != "INVALID" for e in evs)
    assert sum(b"datetime.datetime(" in e[7] for e in evs) > 50


def test_non_object_state_is_invalid_in_both_engines():
    for bad in ("running", [1], {"running": "x"}, {"waiting": 5}):
        pod = {"status": {"containerStatuses": [{"name": "c", "state": bad}]}}
        line = json.dumps({"type": "ADDED", "object": pod}).encode() + b"\n"
        nat = NativeDecoder("production", "python_repr").feed(line)[0]
        assert nat[0] == "INVALID"


def test_pipeline_and_checkpoint_in_python_repr_mode(tmp_path):
    """The fused pipeline renders python_repr natively, and the native cache
    and its format-2 checkpoint work in that mode (they were off before)."""
    from k8s_watcher_amd.engine.checkpoint import load_checkpoint, native_snapshot, write_native
    from k8s_watcher_amd.engine.pipeline import EventPipeline
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.testing.podgen import churn_events, event_line
    from k8s_watcher_amd.utils.config import load_settings

    s = load_settings("staging", overrides={"watcher": {"state_format": "python_repr"}}, environ={})
    out = {}
    for native in (False, True):
        calls = []

        class Rec:
            def submit(self, uid, et, ns, name, core, read_ns, ts):
                calls.append((uid, et, core))

            def flush(self):
                pass

        p = EventPipeline(s, PyDecoder("staging", "python_repr"), Rec(), Metrics())
        p.log_events_setting = False
        if native:
            p.attach_native()
        data = b"".join(event_line(t, o) for t, o in churn_events(60, seed=2))
        if native:
            p.handle_raw(data, 0, framed=False)
        else:
            p.handle_batch(PyDecoder("staging", "python_repr").feed(data), 0)
        out[native] = (calls, p)
    assert out[False][0] == out[True][0] and len(out[True][0]) > 100
    assert any(b"datetime.datetime(" in c for _, _, c in out[True][0])
    p = out[True][1]
    ck = str(tmp_path / "ck")
    snap = native_snapshot(p.cache, None)
    write_native(snap, ck, {"*": "123"}, {})
    loaded = load_checkpoint(ck, native_cache=True)
    assert loaded is not None and len(loaded[1]) == len(p.cache)
