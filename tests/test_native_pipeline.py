"""The fused native pipeline (``_kwcore.Pipeline``) against the Python
``EventPipeline.handle_batch`` reference: same submits, same cache, same
counters, same control events, for every filter combination."""

import json
import os
import random

import pytest

from conftest import ROOT
from k8s_watcher_amd.engine.pipeline import EventPipeline
from k8s_watcher_amd.metrics import Metrics
from k8s_watcher_amd.ops.decode import PyDecoder
from k8s_watcher_amd.testing.podgen import churn_events, event_line
from k8s_watcher_amd.utils.config import load_settings


class Recorder:
    def __init__(self):
        self.calls = []

    def submit(self, uid, et, ns, name, core, read_ns, ts):
        self.calls.append((uid, et, ns, name, json.loads(core)))

    def flush(self):
        pass


def stream():
    lines = [event_line(t, o) for t, o in churn_events(120, seed=13)]
    lines.insert(7, b'{"type":"BOOKMARK","object":{"kind":"Pod","metadata":{"resourceVersion":"777"}}}\n')
    lines.insert(30, b"this is not json\n")
    lines.insert(45, b'{"type":"ERROR","object":{"kind":"Status","code":500,"message":"boom"}}\n')
    lines.insert(50, b'{"type":"ADDED","object":{"metadata":{"name":"nostatus","namespace":"default","uid":"x1"}}}\n')
    lines.insert(51, b'{"type":"MODIFIED","object":{"metadata":{"name":"nostatus","namespace":"default",'
                     b'"uid":"x1"},"status":{}}}\n')
    return b"".join(lines)


PROFILES = [
    ("staging", {}),
    ("production", {}),
    ("development", {"watcher": {"notify_on": "phase_change"}}),
    ("production", {"watcher": {"notify_on": "phase_change", "namespaces": []}}),
    ("staging", {"watcher": {"shard": {"count": 3, "index": 1}}}),
    ("staging", {"watcher": {"shard": {"count": 2, "index": 0, "key": "uid"}, "namespaces": ["batch"]}}),
]


def run_python(env, ov, data):
    s = load_settings(env, overrides=ov, environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder(env), rec, m)
    p.log_events_setting = False
    ctrl = p.handle_batch(PyDecoder(env).feed(data), 0)
    return rec.calls, p.cache, m.c, p.last_rv, [c[0] for c in ctrl]


def run_native(env, ov, data, framed_chunks=None):
    s = load_settings(env, overrides=ov, environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder(env), rec, m)
    p.log_events_setting = False
    p.attach_native()
    ctrl = []
    if framed_chunks is None:
        ctrl += p.handle_raw(data, 0, framed=False)
    else:
        for piece in framed_chunks:
            ctrl += p.handle_raw(piece, 0, framed=True)
    return rec.calls, p.cache, m.c, p.last_rv, [c[0] for c in ctrl]


def norm_cache(cache):
    return {u: [e[0], e[1], e[2], e[3], json.loads(e[4]) if e[4] else None] for u, e in cache.items()}


@pytest.mark.parametrize("env,ov", PROFILES)
def test_native_pipeline_matches_python(env, ov):
    data = stream()
    a = run_python(env, ov, data)
    b = run_native(env, ov, data)
    assert a[0] == b[0]                       # submits, in order, with identical payload cores
    assert norm_cache(a[1]) == norm_cache(b[1])
    counters = ("events_received", "events_filtered_critical", "events_filtered_namespace", "events_unchanged",
                "events_other_shard", "bookmarks")
    assert {k: a[2][k] for k in counters} == {k: b[2][k] for k in counters}
    assert a[3] == b[3]                       # last resourceVersion
    assert a[4] == b[4] == ["INVALID", "ERROR"]


def test_native_chunked_framing_any_split():
    data = stream()
    lines = data.split(b"\n")[:-1]
    framed = b"".join(b"%x\r\n%s\r\n" % (len(ln) + 1, ln + b"\n") for ln in lines) + b"0\r\n\r\n"
    rng = random.Random(1)
    cuts = sorted(rng.sample(range(1, len(framed)), 60))
    pieces = [framed[i:j] for i, j in zip([0] + cuts, cuts + [len(framed)])]
    a = run_python("production", {}, data)
    b = run_native("production", {}, data, framed_chunks=pieces)
    assert a[0] == b[0] and a[3] == b[3]


def test_native_pipeline_logs_like_python():
    s = load_settings("development", environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder("development"), rec, m)
    lines = []
    p.elog.log = lambda level, msg: lines.append((level, msg))
    p.log_events_setting = True
    p.attach_native()
    ev = b'{"type":"ADDED","object":{"metadata":{"name":"a","namespace":"batch","uid":"u"}}}\n'
    p.handle_raw(ev, 0, framed=False)
    assert lines == [(20, "Pod event detected: ADDED - batch/a")] + \
        ([(10, "Skipping pod batch/a - not in target namespaces")] if p.elog.enabled(10) else [])


def test_light_parse_defers_payload_subtrees():
    """With a filter active the pipeline only walks spec/status arrays for events
    that get a payload: a malformed container list is reported (INVALID) on an
    event that passes the critical filter and never looked at on one that does not."""
    bad_spec = b'"spec":{"containers":[{"name" "c"}]}'
    keep = (b'{"type":"DELETED","object":{"metadata":{"name":"a","namespace":"default","uid":"u1",'
            b'"resourceVersion":"5"},' + bad_spec + b',"status":{"phase":"Running"}}}\n')
    drop = (b'{"type":"MODIFIED","object":{"metadata":{"name":"b","namespace":"default","uid":"u2",'
            b'"resourceVersion":"6"},' + bad_spec + b',"status":{"phase":"Running"}}}\n')
    calls, entries, c, last_rv, ctrl = run_native("production", {}, keep + drop)
    assert ctrl == ["INVALID"]
    assert calls == []
    assert c["events_filtered_critical"] == 1 and "u2" in entries and last_rv == "6"


@pytest.mark.parametrize("threads", [0, 1, 4])
def test_decode_pool_matches_serial(threads):
    """Phase B (decode) on 0..4 worker threads gives exactly the serial result:
    same submits in the same order, same cache, same counters, for feeds of
    every size around the fan-out threshold."""
    data = stream()
    lines = data.split(b"\n")[:-1]
    framed = b"".join(b"%x\r\n%s\r\n" % (len(ln) + 1, ln + b"\n") for ln in lines) + b"0\r\n\r\n"
    rng = random.Random(threads)
    cuts, pos = [], 0
    while pos < len(framed):
        pos += rng.choice([7, 300, 4000, 20000, 60000])
        cuts.append(min(pos, len(framed)))
    pieces = [framed[i:j] for i, j in zip([0] + cuts[:-1], cuts)]
    ref = run_python("production", {"watcher": {"namespaces": []}}, data)
    s = load_settings("production", overrides={"watcher": {"namespaces": [], "decode_threads": threads}},
                      environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder("production"), rec, m)
    p.log_events_setting = False
    p.attach_native()
    assert p.native.decode_threads() == threads
    ctrl = []
    for _ in range(3):  # same stream thrice: the cache sees re-adds of known uids
        p.native.reset()
        for piece in pieces:
            ctrl += p.handle_raw(piece, 0, framed=True)
    assert rec.calls[:len(ref[0])] == ref[0]
    assert len(rec.calls) == 3 * len(ref[0])
    assert norm_cache(p.cache) == norm_cache(ref[1])
    assert [c[0] for c in ctrl] == ["INVALID", "ERROR"] * 3


@pytest.mark.parametrize("spin_us", [0.0, 60.0])
def test_shared_decode_pool_spin_and_stats(spin_us):
    """A shared pool (the service's) with and without idle spinning decodes
    exactly the serial result; its per-worker stats account for the lines the
    workers took, and a pool that does not spin sleeps between feeds."""
    from k8s_watcher_amd.ops.native import load
    import time
    mod = load()
    with pytest.raises(ValueError):
        mod.DecodePool(2, -1.0)
    pool = mod.DecodePool(3, spin_us=spin_us)
    assert pool.spin_us() == spin_us
    data = stream()
    ref = run_python("production", {}, data)
    s = load_settings("production", environ={})
    rec, m = Recorder(), Metrics()
    p = EventPipeline(s, PyDecoder("production"), rec, m)
    p.log_events_setting = False
    p.attach_native(pool)
    lines = data.split(b"\n")
    half = len(lines) // 2
    p.handle_raw(b"\n".join(lines[:half]) + b"\n", 0, framed=False)
    time.sleep(0.01)  # longer than any spin: the workers go to sleep
    p.handle_raw(b"\n".join(lines[half:]), 0, framed=False)
    assert rec.calls == ref[0]
    st = pool.stats()
    assert len(st) == 3
    assert sum(w["lines"] for w in st) <= len(lines)
    assert all(w["spin_s"] >= 0 and w["sleep_s"] >= 0 for w in st)
    if spin_us == 0.0:
        assert all(w["sleeps"] >= 1 for w in st)


def test_decode_pool_lifecycle():
    """Pools are created and joined with their pipelines (no leaked threads).
    Counted in a child process: threads other tests left behind in this
    process may exit while we count."""
    import subprocess
    import sys
    if "libtsan" in os.environ.get("LD_PRELOAD", ""):
        pytest.skip("ThreadSanitizer starts a background thread of its own: exact counts do not hold")
    code = ("import os, sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "from k8s_watcher_amd.ops.native import load\n"
            "from test_native_pipeline import stream\n"
            "mod = load()\n"
            "import time\n"
            "def n(want=None):\n"
            "    # a joined thread can linger in /proc for a moment after pthread_join returns\n"
            "    for _ in range(200):\n"
            "        c = len(os.listdir('/proc/self/task'))\n"
            "        if want is None or c == want: return c\n"
            "        time.sleep(0.005)\n"
            "    return c\n"
            "before = n()\n"
            "for _ in range(20):\n"
            "    pl = mod.Pipeline('production', mod.PodCache(), {}, None, True, False, 1, 0, True, True,"
            " None, False, False, 3)\n"
            "    assert n(before + 3) == before + 3, (n(), before)\n"
            "    pl.feed(stream(), 0)\n"
            "    del pl\n"
            "assert n(before) == before, (n(), before)\n"
            "try:\n"
            "    mod.Pipeline('production', mod.PodCache(), {}, None, True, False, 1, 0, True, True, None,"
            " False, False, 65)\n"
            "except ValueError:\n"
            "    print('ok')\n") % (ROOT, os.path.join(ROOT, "tests"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


def test_decode_pool_create_destroy_race():
    """Workers the OS schedules only after the pool was used or destroyed must
    still see that wake-up (a late-starting worker used to sleep forever and
    hang the destructor's join). Run in a child so a regression fails, not hangs."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from k8s_watcher_amd.ops.native import load\n"
            "m = load()\n"
            "for i in range(300):\n"
            "    p = m.DecodePool(1 + i %% 8)\n"
            "    del p\n"
            "print('ok')\n") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


@pytest.mark.parametrize("mask", [0b111111, 0b010001, 0b100000])
@pytest.mark.parametrize("env,ov", [("staging", {}), ("production", {})])
def test_payload_extra_fields_match_python(mask, env, ov):
    """watcher.payload_extra_fields: the fused pipeline (full and filter-first
    parse, decode pool) emits the same "extra" object as the Python engine."""
    from k8s_watcher_amd.models.payload import EXTRA_FIELDS
    data = stream()
    s = load_settings(env, overrides=ov, environ={})
    s.watcher.payload_extra = mask
    rec_py, rec_nat = Recorder(), Recorder()
    p = EventPipeline(s, PyDecoder(env, extra=mask), rec_py, Metrics())
    p.log_events_setting = False
    p.handle_batch(PyDecoder(env, extra=mask).feed(data), 0)
    q = EventPipeline(s, PyDecoder(env, extra=mask), rec_nat, Metrics())
    q.log_events_setting = False
    q.attach_native()
    q.handle_raw(data, 0, framed=False)
    assert rec_py.calls == rec_nat.calls and rec_py.calls
    want = [n for i, n in enumerate(EXTRA_FIELDS) if mask >> i & 1]
    for call in rec_nat.calls:
        assert list(call[4]["extra"]) == want
    full = [c[4]["extra"] for c in rec_nat.calls if "owner_references" in c[4]["extra"]
            and c[4]["extra"]["owner_references"]]
    if mask >> 5 & 1:
        assert full and full[0]["owner_references"][0]["kind"] == "ReplicaSet"


def test_native_decoder_extra_and_config():
    from k8s_watcher_amd.ops.decode import make_decoder
    from k8s_watcher_amd.utils.config import ConfigError
    line = (b'{"type":"ADDED","object":{"metadata":{"name":"a","namespace":"d","uid":"u","resourceVersion":"7",'
            b'"ownerReferences":[{"kind":"Job","name":"j"}]},"status":{"phase":"Running","podIP":"10.1.2.3",'
            b'"hostIP":"192.168.0.1","startTime":"2025-01-01T00:00:00Z","qosClass":"BestEffort"}}}\n')
    cores = [json.loads(make_decoder(e, "staging", extra=0b111111).core(make_decoder(e, "staging", extra=0b111111)
                                                                          .feed(line)[0])) for e in ("python",)]
    d = make_decoder("native", "staging", extra=0b111111)
    nat = json.loads(d.core(d.feed(line)[0]))
    assert nat == cores[0]
    assert nat["extra"] == {"pod_ip": "10.1.2.3", "host_ip": "192.168.0.1", "start_time": "2025-01-01T00:00:00Z",
                            "qos_class": "BestEffort", "resource_version": "7",
                            "owner_references": [{"kind": "Job", "name": "j"}]}
    s = load_settings("staging", overrides={"watcher": {"payload_extra_fields": ["pod_ip", "owner_references"]}},
                      environ={})
    assert s.watcher.payload_extra == 0b100001
    with pytest.raises(ConfigError):
        load_settings("staging", overrides={"watcher": {"payload_extra_fields": ["nope"]}}, environ={})
