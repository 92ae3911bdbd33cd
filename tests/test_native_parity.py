"""Native decoder (``ops/csrc/kwcore.cpp``) vs the Python engine, field by field.

The C++ engine must be semantically identical to ``models/payload.py`` +
``ops/decode.py``: same event tuple, and a payload core that parses to the
same JSON document. Checked on generated lifecycles, hand-written edge cases
and a hypothesis fuzz over random pod shapes and encodings.
"""

import json

import pytest
from hypothesis import given, settings, strategies as st

from k8s_watcher_amd.ops.decode import E_OBJ, PyDecoder
from k8s_watcher_amd.ops.native import NativeDecoder, load
from k8s_watcher_amd.testing.podgen import churn_events, event_line

ENV = "production"


def both(data: bytes):
    py, nat = PyDecoder(ENV), NativeDecoder(ENV)
    return py, py.feed(data), nat, nat.feed(data)


def assert_same(data: bytes):
    py, a, nat, b = both(data)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x[0] == y[0]
        if x[0] == "INVALID":
            continue
        assert x[1:7] == y[1:7], (x[1:7], y[1:7])
        if x[0] in ("ADDED", "MODIFIED", "DELETED"):
            assert json.loads(py.core(x)) == json.loads(nat.core(y))
        if x[0] == "ERROR":
            assert x[8] == y[8]
    return a, b


def test_generated_churn_parity():
    data = b"".join(event_line(t, o) for t, o in churn_events(300, seed=9))
    a, b = assert_same(data)
    assert len(a) == 1500


def test_split_across_feeds_at_every_boundary():
    data = b"".join(event_line(t, o) for t, o in churn_events(3, seed=1))
    ref = NativeDecoder(ENV).feed(data)
    for cut in range(1, len(data), 97):
        d = NativeDecoder(ENV)
        got = d.feed(data[:cut]) + d.feed(data[cut:])
        assert [g[:7] for g in got] == [r[:7] for r in ref]
        assert [g[7] for g in got] == [r[7] for r in ref]


EDGE_OBJECTS = [
    {"metadata": {"name": "a", "namespace": "ns", "uid": "u1", "resourceVersion": "7"}},
    {"metadata": {"name": "a"}, "status": None, "spec": None},
    {"metadata": None, "status": {}},
    {"metadata": {"name": "é\"\\/\b\f\n\r\t 😀", "labels": None, "annotations": {}}},
    {"metadata": {"labels": {"a": "b", "c": "d\"e"}, "annotations": {"x": "é"},
                  "creationTimestamp": "2025-07-09T10:51:28.25+09:00"}},
    {"metadata": {"creationTimestamp": 12345}},
    {"metadata": {"creationTimestamp": None}},
    {"metadata": {"creationTimestamp": "2025-07-09 10:51:28"}},
    {"metadata": {"creationTimestamp": "not a time"}},
    {"status": {"phase": "Running", "conditions": None, "containerStatuses": None}},
    {"status": {"phase": "Failed", "conditions": [{"type": "Ready"}, {}],
                "containerStatuses": [{"name": "c", "state": None}, {"name": "d", "state": {}},
                                      {"name": "e", "ready": False, "restartCount": 3,
                                       "state": {"waiting": {"reason": "CrashLoopBackOff",
                                                             "message": "back-off 5m0s"}}}]}},
    {"spec": {"nodeName": None, "containers": [{"name": "x"}, {"image": "y"}]}},
    {"spec": {"containers": []}, "status": {"phase": None}},
    {"metadata": {"name": "dup", "uid": "first"}, "extra": [1, 2, {"a": [[]]}], "metadata2": 1},
    {"metadata": {"name": 5, "namespace": True, "uid": None}},
    {"status": {"phase": "Succeeded", "extraList": [{"phase": "Failed"}]}, "kind": "Pod"},
]


@pytest.mark.parametrize("obj", EDGE_OBJECTS)
@pytest.mark.parametrize("etype", ["ADDED", "DELETED"])
def test_edge_objects(obj, etype):
    compact = json.dumps({"type": etype, "object": obj}, separators=(",", ":")).encode() + b"\n"
    spaced = json.dumps({"object": obj, "type": etype}, indent=None, ensure_ascii=True).encode() + b"\n"
    assert_same(compact)
    assert_same(spaced)


def test_bookmark_and_error():
    bm = b'{"type":"BOOKMARK","object":{"kind":"Pod","metadata":{"resourceVersion":"12345"}}}\n'
    err = (b'{"type":"ERROR","object":{"kind":"Status","apiVersion":"v1","status":"Failure",'
           b'"message":"too old resource version: 1 (2)","reason":"Expired","code":410}}\n')
    a, b = assert_same(bm + err)
    assert b[0][0] == "BOOKMARK" and b[0][4] == "12345" and b[0][7] is None
    assert b[1][0] == "ERROR" and b[1][8]["code"] == 410


@pytest.mark.parametrize("line", [
    b"not json", b'{"type":"ADDED"}', b'{"type":"ADDED","object":[]}', b'{"object":{}}',
    b'{"type":"ADDED","object":{"metadata":{"name":"x"}}', b'{"type":"ADDED","object":{}} trailing',
    b'{"type":"ADDED","object":{"metadata":{"name":"unterminated}}}',
])
def test_invalid_lines(line):
    py, a, nat, b = both(line + b"\n")
    assert a[0][0] == "INVALID" and b[0][0] == "INVALID"


def test_blank_lines_and_crlf_ignored():
    obj = {"metadata": {"name": "a", "uid": "u"}}
    data = b"\n  \n" + json.dumps({"type": "ADDED", "object": obj}).encode() + b"\r\n\n"
    _, a, _, b = both(data)
    assert len(a) == len(b) == 1


def test_list_decoding_parity():
    items = [o for t, o in churn_events(20, seed=4) if t == "ADDED"]
    body = json.dumps({"kind": "PodList", "metadata": {"resourceVersion": "99", "continue": "tok"},
                       "items": items}).encode()
    py, nat = PyDecoder(ENV), NativeDecoder(ENV)
    rv1, c1, e1 = py.decode_list(body)
    rv2, c2, e2 = nat.decode_list(body)
    assert (rv1, c1) == (rv2, c2) == ("99", "tok")
    assert [e[:7] for e in e1] == [e[:7] for e in e2]
    assert [json.loads(py.core(x)) for x in e1] == [json.loads(nat.core(y)) for y in e2]
    empty = b'{"kind":"PodList","metadata":{"resourceVersion":"5","continue":""},"items":null}'
    assert nat.decode_list(empty) == ("5", None, []) == py.decode_list(empty)


def test_core_from_summary_parity():
    py, nat = PyDecoder(ENV), NativeDecoder(ENV)
    for args in (("u", "ns", "n", "Running"), ("u", None, "é", None)):
        assert json.loads(py.core_from_summary(*args)) == json.loads(nat.core_from_summary(*args))


def test_scalar_and_simd_paths_agree():
    """Scalar, AVX2 and (where the CPU has it) AVX-512BW block scanners decode
    the same stream to the same events, with and without the light pipeline."""
    mod = load()
    data = b"".join(event_line(t, o) for t, o in churn_events(50, seed=8))
    results = []
    try:
        for level in (False, "avx2", True):
            mod.set_simd(level)
            results.append([s[:8] for s in NativeDecoder(ENV).feed(data)])
    finally:
        mod.set_simd(True)
    assert results[0] == results[1] == results[2]


def test_environment_is_json_escaped():
    d = NativeDecoder('we"ird')
    ev = d.feed(b'{"type":"ADDED","object":{"metadata":{"name":"a"}}}\n')[0]
    assert json.loads(ev[E_OBJ])["environment"] == 'we"ird'


# ----------------------------------------------------------------------------- fuzz

text = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=12)
maybe = lambda s: st.one_of(st.none(), s)  # noqa: E731
scalar = st.one_of(st.none(), st.booleans(), st.integers(-5, 10 ** 6), text)
state_obj = st.one_of(st.none(), st.fixed_dictionaries({}, optional={
    "running": st.fixed_dictionaries({}, optional={"startedAt": text}),
    "waiting": st.fixed_dictionaries({}, optional={"reason": text, "message": text})}))
pod = st.fixed_dictionaries({}, optional={
    "kind": st.just("Pod"),
    "metadata": maybe(st.fixed_dictionaries({}, optional={
        "name": scalar, "namespace": scalar, "uid": scalar, "resourceVersion": scalar,
        "labels": maybe(st.dictionaries(text, text, max_size=3)),
        "annotations": maybe(st.dictionaries(text, text, max_size=3)),
        "creationTimestamp": st.one_of(st.none(), text, st.just("2025-07-09T01:51:28Z"),
                                       st.just("2025-07-09T01:51:28.120Z")),
        "managedFields": st.lists(st.dictionaries(text, scalar, max_size=3), max_size=2)})),
    "spec": maybe(st.fixed_dictionaries({}, optional={
        "nodeName": scalar,
        "containers": maybe(st.lists(st.fixed_dictionaries({}, optional={"name": scalar, "image": scalar}),
                                     max_size=3))})),
    "status": maybe(st.fixed_dictionaries({}, optional={
        "phase": scalar,
        "conditions": maybe(st.lists(st.fixed_dictionaries({}, optional={
            "type": scalar, "status": scalar, "reason": scalar, "message": scalar}), max_size=3)),
        "containerStatuses": maybe(st.lists(st.fixed_dictionaries({}, optional={
            "name": scalar, "ready": scalar, "restartCount": scalar, "state": state_obj}), max_size=3))})),
})


@settings(max_examples=300, deadline=None)
@given(obj=pod, etype=st.sampled_from(["ADDED", "MODIFIED", "DELETED"]), ascii_=st.booleans(),
       spaced=st.booleans())
def test_fuzz_parity(obj, etype, ascii_, spaced):
    seps = (", ", ": ") if spaced else (",", ":")
    line = json.dumps({"type": etype, "object": obj}, ensure_ascii=ascii_, separators=seps).encode("utf-8")
    py, a, nat, b = both(line + b"\n")
    x, y = a[0], b[0]
    assert x[0] == y[0] == etype
    # identity fields: the native engine yields None for non-string values
    for i in (1, 2, 3, 4, 5):
        assert (x[i] if isinstance(x[i], str) else None) == y[i]
    assert x[6] == y[6]
    assert json.loads(py.core(x)) == json.loads(nat.core(y))


# Strings full of brackets, quotes and backslash runs, nested to random depth:
# the block scanners must find the same container end at every SIMD level.
_tricky = st.text(alphabet='{}[]"\\\\ ab:,', min_size=0, max_size=90)
_nested = st.recursive(
    _tricky | st.integers() | st.booleans() | st.none(),
    lambda ch: st.lists(ch, max_size=5) | st.dictionaries(_tricky, ch, max_size=5),
    max_leaves=25)


@settings(max_examples=150, deadline=None)
@given(skipme=_nested, pad=st.integers(min_value=0, max_value=130))
def test_fuzz_block_skipper_all_levels(skipme, pad):
    obj = {"metadata": {"name": "p", "namespace": "default", "uid": "u", "resourceVersion": "1",
                        "labels": {"x" * pad: skipme}, "junk": [skipme, {"a": skipme}]},
           "spec": {"volumes": skipme, "containers": [{"name": "c", "image": "i", "env": skipme}]},
           "status": {"phase": "Running", "junk": skipme}}
    line = json.dumps({"type": "MODIFIED", "object": obj}).encode() + b"\n"
    mod = load()
    out = []
    try:
        for level in (False, "avx2", True):
            mod.set_simd(level)
            out.append([e[:8] for e in NativeDecoder(ENV).feed(line)])
    finally:
        mod.set_simd(True)
    assert out[0] == out[1] == out[2]
    assert out[0] and out[0][0][0] == "MODIFIED"


pod_extra = st.fixed_dictionaries({}, optional={
    "metadata": maybe(st.fixed_dictionaries({}, optional={
        "name": scalar, "uid": scalar, "resourceVersion": scalar,
        "ownerReferences": maybe(st.lists(st.dictionaries(text, scalar, max_size=3), max_size=2))})),
    "status": maybe(st.fixed_dictionaries({}, optional={
        "phase": scalar, "podIP": scalar, "hostIP": scalar, "startTime": scalar, "qosClass": scalar,
        "conditions": maybe(st.lists(st.fixed_dictionaries({}, optional={"type": scalar}), max_size=2))})),
})


@settings(max_examples=200, deadline=None)
@given(obj=pod_extra, mask=st.integers(0, 63), ascii_=st.booleans())
def test_fuzz_extra_fields_parity(obj, mask, ascii_):
    """watcher.payload_extra_fields: same "extra" object from both engines for any mask."""
    from k8s_watcher_amd.ops.decode import PyDecoder
    from k8s_watcher_amd.ops.native import NativeDecoder
    line = json.dumps({"type": "MODIFIED", "object": obj}, ensure_ascii=ascii_).encode("utf-8") + b"\n"
    py, nat = PyDecoder("staging", extra=mask), NativeDecoder("staging", extra=mask)
    x, y = py.feed(line)[0], nat.feed(line)[0]
    assert json.loads(py.core(x)) == json.loads(nat.core(y))
