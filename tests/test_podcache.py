"""The native pod cache (``_kwcore.PodCache``, ops/csrc/podcache.inc) behaves
exactly like the Python ``PodCache`` (ops/cache.py) under any sequence of
operations, including None fields, non-ASCII text and checkpoint round trips."""

import json

from hypothesis import given, settings, strategies as st

from k8s_watcher_amd.engine.checkpoint import load_checkpoint, save_checkpoint
from k8s_watcher_amd.ops.cache import MISSING, PodCache, make_pod_cache

uids = st.sampled_from(["u1", "u2", "ü3", None])
texts = st.one_of(st.none(), st.sampled_from(["Running", "Pending", "", "ns-é", "default"]))
cores = st.one_of(st.none(), st.sampled_from([b'{"a":1}', '{"n":"é"}'.encode()]))
ops = st.lists(st.one_of(
    st.tuples(st.just("observe"), st.sampled_from(["ADDED", "MODIFIED", "DELETED"]), uids, texts, texts, texts,
              texts),
    st.tuples(st.just("set_core"), uids, st.sampled_from([b"{}", b'{"x":"y"}'])),
    st.tuples(st.just("put"), uids, texts, texts, texts, texts, cores),
    st.tuples(st.just("pop"), uids),
), max_size=40)


def snapshot(c):
    return sorted(((u or "", u is None), e) for u, e in c.items())


@settings(max_examples=200, deadline=None)
@given(seq=ops)
def test_native_cache_matches_python(seq):
    py, nat = PodCache(), make_pod_cache(True)
    for op in seq:
        name, args = op[0], op[1:]
        r1 = getattr(py, name)(*args)
        r2 = getattr(nat, name)(*args)
        if name == "observe":
            assert (r1 is MISSING) == (r2 is MISSING) and (r1 is MISSING or r1 == r2)
        else:
            assert r1 == r2
        assert len(py) == len(nat)
    assert snapshot(py) == snapshot(nat)
    for u in ("u1", "u2", "ü3", None):
        assert (u in py) == (u in nat)
        assert py.get(u) == nat.get(u)
    recs = sorted(nat.to_records(), key=json.dumps)
    assert recs == sorted(py.to_records(), key=json.dumps)
    again = make_pod_cache(True, recs)
    assert snapshot(again) == snapshot(py)


def test_native_cache_checkpoint_round_trip(tmp_path):
    nat = make_pod_cache(True)
    nat.observe("ADDED", "a", "1", "Running", "default", "p-é")
    nat.set_core("a", '{"name":"p-é"}'.encode())
    nat.observe("ADDED", "b", "2", None, None, None)
    path = str(tmp_path / "ck.json")
    save_checkpoint(path, {"*": "2"}, nat)
    scopes, loaded, _, _ = load_checkpoint(path, native_cache=True)
    assert scopes == {"*": "2"}
    assert type(loaded) is type(nat)
    assert snapshot(loaded) == snapshot(nat)
    _, py, _, _ = load_checkpoint(path)
    assert snapshot(py) == snapshot(nat)


def test_count_namespace_native_matches_python():
    from k8s_watcher_amd.ops.cache import PodCache
    from k8s_watcher_amd.ops.native import load
    caches = [load().PodCache(), PodCache()]
    for c in caches:
        for i in range(30):
            c.put(f"u{i}", str(i), "Running", None if i % 7 == 0 else f"ns{i % 3}", f"p{i}", None)
        c.pop("u4")
    for ns in ("ns0", "ns1", "ns2", "nope", None):
        assert caches[0].count_namespace(ns) == caches[1].count_namespace(ns)
    assert caches[0].count_namespace("nope") == 0
