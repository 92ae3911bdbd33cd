"""The relist-storm benchmark at small scale (``benchmarks/relist_storm.py``):
every pod watch expires at once after silent churn; every scope relists
through the native Relist and the sink must get exactly the churn, once."""

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.parametrize("initial_sync", ["list", "watch_list"])
@pytest.mark.parametrize("scope,namespaces", [("discover", 40), ("cluster", 8)])
def test_relist_storm_exactly_once(scope, namespaces, initial_sync, tmp_path):
    """``watch_list``: the initial sync and the post-410 resync are WatchList
    streams fed into the native Relist read by read (relist.inc WatchList),
    with the same counts as the LIST path."""
    out = tmp_path / "storm.json"
    res = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "relist_storm.py"), "--scope", scope,
                          "--namespaces", str(namespaces), "--pods", "2000", "--churn", "50", "--page", "37",
                          "--slice-ms", "1", "--initial-sync", initial_sync, "--json-out", str(out)],
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    d = json.loads(out.read_text())
    assert d["initial"]["exactly_once"] and d["initial"]["notified"] == 2000
    st = d["storm"]
    assert st["exactly_once"] and st["expected"] == 150 and st["missing"] == 0 and st["duplicates"] == 0
    r = st["relist"]
    assert r["scopes"] == (namespaces if scope == "discover" else 1)
    assert r["listed"] == 2000 and r["unchanged"] == 2000 - 100
    assert r["added"] == 50 and r["modified"] == 50 and r["deleted"] == 50
    if initial_sync == "watch_list":  # no LIST at all: every sync was a WatchList stream
        assert d["server"]["lists"] == 0 and d["server"]["watch_lists"] == 2 * r["scopes"]
