"""The reference-equivalent baseline (benchmarks/reference_equiv.py) in the
headline bench: its rate must not depend on how much history the replay
fixture has sent before it.

Round 3's fixture answered a watch without a resourceVersion by scanning every
event ever sent in Python while the reference's clock ran, so 24 churn rounds
per step cut the reference to two thirds of its 1-round rate and inflated
``vs_baseline`` ~3x. Now the fixture answers from an index and the clock
starts at the first paced event."""

import os

import pytest

from conftest import run_bench  # noqa: E402

# a wall-clock rate comparison: a noise gate on a shared container, so it runs
# in the box's tier (-m gpu; the host's own CPU share) and not the CPU tier
pytestmark = [pytest.mark.gpu, pytest.mark.perf]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(rounds: int) -> dict:
    d = run_bench(["--steps", "2", "--warmup", "1",
                   "--pods-per-step", "2000", "--rounds-per-step", str(rounds), "--namespaces", "8",
                   "--ref-events", "1500", "--latency-seconds", "0.5", "--latency-seconds-high", "0",
                   "--staging", "off", "--apart", "off", "--no-verify", "--sink-workers", "1",
                   "--no-placement"])
    assert d["_headline"]["reference_equiv_events_per_s"] == d["reference_equiv"]["events_per_s"]
    return d["reference_equiv"]


def test_reference_rate_independent_of_history_length():
    runs = {1: [], 24: []}

    def best() -> dict:
        return {r: max(x["events_per_s"] for x in v) for r, v in runs.items()}

    # interleaved pairs, best of each: this container's load drifts (a shared
    # CPU adds 10-20% noise per run); a third pair only when the first two
    # disagree. Round 3's history walk cost a steady third at 24 rounds.
    for pair in range(3):
        for rounds in (1, 24):
            runs[rounds].append(_bench(rounds))
        b = best()
        if pair >= 1 and b[24] >= 0.85 * b[1]:
            break
    for ref in runs[1] + runs[24]:
        assert ref["events"] == 1500
        # the latency phase paced part of a step: its live pods reach the new
        # watch as ADDED before the replay — handled, not counted
        assert ref["backlog_events_uncounted"] > 0
        # connect -> first paced event: the fixture's answer is O(live pods),
        # not O(history) (round 3: seconds at 24 rounds)
        assert ref["first_event_after_s"] < 0.5, ref
    b = best()
    # 24x the history, no slower (a faster best at 24 rounds is the shared CPU's noise)
    assert b[24] >= 0.85 * b[1], (b, runs)
