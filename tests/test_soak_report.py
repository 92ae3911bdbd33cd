"""benchmarks/soak_report.py: the markdown summary of a soak record."""

import json

from benchmarks.soak_report import main, slope


def test_slope_is_least_squares():
    assert slope([0, 1, 2, 3], [1, 3, 5, 7]) == 2.0
    assert slope([0, 1], [0, 1]) is None  # too few points
    assert slope([1, 1, 1], [0, 1, 2]) is None  # no spread in x


def test_report_windows_and_apply_counters(tmp_path, capsys):
    keys = ("apply_partitioned_batches", "apply_partitioned_lines", "apply_tail_submits", "apply_tail_lock_runs",
            "apply_serial_lines", "apply_tail_serial_lines")
    samples = [{"t": 0.0, "pid": 1, "rss_mb": 50.0}]  # an earlier process: not the one reported
    for i in range(0, 3 * 360 + 1):  # the last process: 3 h, a sample every 10 s
        t = 100.0 + i * 10
        h = (t - 100.0) / 3600
        s = {"t": t, "pid": 2, "rss_mb": 60.0 + 0.5 * h, "malloc_in_use_bytes": 40 * 2 ** 20}
        s.update({k: 1000.0 * i for k in keys})
        samples.append(s)
    doc = {"summary": {"complete": True, "elapsed_minutes": 190.0, "minutes": 190.0, "steps": 2000,
                       "steps_by_kind": {"normal": 1900, "kill": 11}, "events_replayed": 100_000_000,
                       "notifications_checked": 20_000_000, "watcher_kills": 11, "steps_failed": 0,
                       "duplicates_outside_kill_steps": 0, "duplicates_in_kill_steps": 3},
           "samples": samples}
    path = tmp_path / "soak.json"
    path.write_text(json.dumps(doc))
    main([str(path), "--title", "Test soak"])
    out = capsys.readouterr().out
    assert out.startswith("# Test soak") and "complete, 190 of 190 minutes" in out
    assert "| failed steps | 0 |" in out and "| duplicates outside / inside kill steps | 0 / 3 |" in out
    assert "pid 2, 3.00 h" in out
    rows = [ln for ln in out.splitlines() if ln.startswith("| from +")]
    assert [r.split("|")[1].strip() for r in rows] == ["from +0.5 h", "from +1 h", "from +2 h"]
    assert all("+0.50" in r and "+0.00" in r for r in rows)  # RSS slope 0.5 MiB/h, the C heap flat
    assert "`apply_tail_lock_runs`" in out and "`apply_tail_serial_lines`" in out
