"""Native JSON validation (``ops/csrc/validate.inc``, ``watcher.validate``)
against CPython's ``json.loads``, under mutation fuzzing of real-shaped pod
watch lines: byte flips, truncations, insertions of structural characters,
bracket-kind swaps, bad literals, broken escapes and broken UTF-8.

* ``_kwcore.json_invalid`` is ``json.loads``' verdict, exactly, at every SIMD
  level (AVX-512 stage 1 + automaton, and the portable scanner);
* ``validate: full``: the native decoders and the fused pipeline mark a line
  INVALID exactly when the Python engine does;
* ``validate: payload`` (the default) and ``full``: every payload core the
  native engine emits is valid JSON — nothing malformed reaches clusterapi.
"""

import json
import random

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from k8s_watcher_amd.engine.pipeline import EventPipeline
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.ops.decode import INVALID, PyDecoder
from k8s_watcher_amd.ops.native import NativeDecoder, load
from k8s_watcher_amd.testing.podgen import churn_events, event_line
from k8s_watcher_amd.utils.config import load_settings

LINES = [event_line(t, o).rstrip(b"\n") for t, o in churn_events(40, seed=21)]

INSERTS = [b"\\u", b"\\", b'"', b",", b":", b"{", b"]", b"tru", b"NaN", b"-", b"01", b"1e", b"\xc3\xa9",
           b"\xed\xa0\x80", b"\xe0\x80\x80", b"\xff", b"\x01", b"\t", b" ", b"\\uZZZZ", b"\\q", b"Infinity"]


def mutate(line: bytes, rng: random.Random, n: int) -> bytes:
    b = bytearray(line)
    for _ in range(n):
        if not b:
            break
        op = rng.randrange(7)
        i = rng.randrange(len(b))
        if op == 0:
            b[i] ^= 1 << rng.randrange(8)
        elif op == 1:
            b = b[:i]
        elif op == 2:
            b[i] = rng.choice(b'{}[],:"\\ 0a-.eE\t\n\x00\x7f\x80')
        elif op == 3:
            del b[i]
        elif op == 4:
            b[i:i] = rng.choice(INSERTS)
        elif op == 5:  # swap a bracket's kind
            j = b.find(b"[" if rng.random() < 0.5 else b"{", i)
            if j >= 0:
                b[j] = ord("{") if b[j] == ord("[") else ord("[")
        else:  # a literal or number made wrong
            for lit, bad in ((b"true", b"tru"), (b"false", b"fals"), (b"null", b"nul"), (b":1", b":01"),
                             (b":0", b":-"), (b'"', b"'")):
                j = b.find(lit, i)
                if j >= 0:
                    b[j:j + len(lit)] = bad
                    break
    return bytes(b)


def py_ok(data: bytes) -> bool:
    try:
        json.loads(data)
        return True
    except ValueError:
        return False


def verdicts(data: bytes):
    mod = load()
    out = []
    try:
        for level in (True, "avx2", False):
            mod.set_simd(level)
            out.append(mod.json_invalid(data) is None)
    finally:
        mod.set_simd(True)
    return out


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(idx=st.integers(0, len(LINES) - 1), seed=st.integers(0, 2 ** 32 - 1), n=st.integers(1, 3))
def test_json_invalid_is_json_loads(idx, seed, n):
    data = mutate(LINES[idx], random.Random(seed), n)
    want = py_ok(data)
    assert verdicts(data) == [want] * 3, data[:300]


@pytest.mark.parametrize("data", [
    b"", b" ", b"1", b"01", b"-", b"-0", b"1.", b"1.5e", b"1e5", b"1E+2", b"-01", b"0.0", b".5", b"NaN", b"-NaN",
    b"-Infinity", b"Infinity", b"nul", b"null ", b"true1", b'"a\\u12"', b'"\\ud800"', b'"\x7f"', '"é"'.encode(),
    b'"\xed\xa0\x80"', b'"\xc0\x80"', b'"\xe2\x82"', b'["\xf4\x90\x80\x80"]', b'"\\u00e9"', b'"\\uD83D\\uDE00"',
    b"[1,]", b'{"a":1,}', b'{"a" 1}', b"{1:2}", b"[1 2]", b"[]", b"{}", b" [ ] ", b"[[[]]]", b"[{]}", b'"\t"',
    b"\t[]\n", b"\x0b[]", b"[1]x", b'"\\x"', b'"\\/"', b"[" * 600 + b"]" * 600, b'"\\' + b"\\" * 63 + b'"',
    b'{"a":1}{"b":2}', b'{"a":[1,{"b":null}],"c":"d"}', b"\xef\xbb\xbf{}",
    # a close with nothing open (read below the validator's stack before round 3's fix)
    b"]", b"}", b"]]", b"}{", b'{"a":1}}', b"[1]]", b' ] ',
])
def test_json_invalid_edge_cases(data):
    assert verdicts(data) == [py_ok(data)] * 3


def _pipeline(env: str, validate: str):
    s = load_settings(env, overrides={"watcher": {"validate": validate}}, environ={})
    calls = []

    class Rec:
        def submit(self, uid, et, ns, name, core, read_ns, ts):
            calls.append(core)

        def flush(self):
            pass

    p = EventPipeline(s, PyDecoder(env), Rec(), Metrics())
    p.log_events_setting = False
    p.attach_native()
    return p, calls


@settings(max_examples=250, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(idx=st.integers(0, len(LINES) - 1), seed=st.integers(0, 2 ** 32 - 1), n=st.integers(1, 3))
def test_full_mode_invalid_iff_python_invalid(idx, seed, n):
    """validate: full — StreamDecoder and the fused Pipeline call a line INVALID
    exactly when PyDecoder (json.loads) does; what they emit is valid JSON."""
    data = mutate(LINES[idx], random.Random(seed), n) + b"\n"
    py = PyDecoder("staging").feed(data)
    py_invalid = not py or py[0][0] == INVALID
    nat = NativeDecoder("staging", validate="full").feed(data)
    assert (not nat or nat[0][0] == INVALID) == py_invalid, data[:300]
    if nat and nat[0][0] != INVALID and nat[0][7] is not None:
        json.loads(nat[0][7])
    p, cores = _pipeline("staging", "full")
    ctrl = p.handle_raw(data, 0, framed=False)
    pipe_invalid = any(c[0] == INVALID for c in ctrl) or (p.metrics.c["events_received"] == 0 and not py_invalid
                                                          and not data.strip())
    if py and py[0][0] in ("ADDED", "MODIFIED", "DELETED"):
        assert not pipe_invalid and p.metrics.c["events_received"] == 1
    else:
        assert p.metrics.c["events_received"] == 0
    for core in cores:
        json.loads(core)


@settings(max_examples=250, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(idx=st.integers(0, len(LINES) - 1), seed=st.integers(0, 2 ** 32 - 1), n=st.integers(1, 3),
       env=st.sampled_from(["staging", "production"]))
def test_payload_mode_never_emits_invalid_json(idx, seed, n, env):
    """validate: payload (default) — whatever the line, every core sent on is valid JSON."""
    data = mutate(LINES[idx], random.Random(seed), n) + b"\n"
    p, cores = _pipeline(env, "payload")
    p.handle_raw(data, 0, framed=False)
    for core in cores:
        json.loads(core)
    nat = NativeDecoder(env).feed(data)
    for ev in nat:
        if ev[0] != INVALID and ev[7] is not None:
            json.loads(ev[7])


def test_payload_mode_rejects_malformed_copied_spans():
    """The cases the round-2 review found: mismatched bracket kinds and a bad
    literal inside labels / annotations were copied into the payload."""
    base = {"metadata": {"name": "a", "namespace": "default", "uid": "u1", "resourceVersion": "1",
                         "labels": {"k": "v"}}, "status": {"phase": "Failed"}}
    good = json.dumps({"type": "ADDED", "object": base}).encode()
    for bad in (good.replace(b'{"k": "v"}', b'{"k": "v"]'), good.replace(b'{"k": "v"}', b'{"k": tru}'),
                good.replace(b'{"k": "v"}', b'{"k": "v\\q"}'), good.replace(b'{"k": "v"}', b'{"k": 01}')):
        assert not py_ok(bad)
        py = PyDecoder("staging").feed(bad + b"\n")
        assert py[0][0] == INVALID
        for mode in ("payload", "full"):
            nat = NativeDecoder("staging", validate=mode).feed(bad + b"\n")
            assert nat[0][0] == INVALID, (mode, bad)
            p, cores = _pipeline("staging", mode)
            ctrl = p.handle_raw(bad + b"\n", 0, framed=False)
            assert [c[0] for c in ctrl] == [INVALID] and cores == []
    p, cores = _pipeline("staging", "payload")
    assert p.handle_raw(good + b"\n", 0, framed=False) == [] and len(cores) == 1
