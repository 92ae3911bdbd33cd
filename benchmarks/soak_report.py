#!/usr/bin/env python3
"""Markdown summary of a ``benchmarks/soak.py --out`` record.

    python -m benchmarks.soak_report profiles/r5/soak_final.json [--title "..."]

Correctness (steps, failures, duplicates), the last process's memory (RSS
and the C heap's in-use bytes, least-squares slopes from +0.5 h, +1 h, +2 h
and +4 h of its life, and the free bytes the allocator keeps — RSS that is
not live data), and the apply-path counters it sampled (which native paths
ran, and that they ran throughout).
"""

from __future__ import annotations

import argparse
import json
from typing import List, Optional


def slope(xs: List[float], ys: List[float]) -> Optional[float]:
    n = len(xs)
    if n < 3:
        return None
    mx, my = sum(xs) / n, sum(ys) / n
    den = sum((x - mx) ** 2 for x in xs)
    return None if den == 0 else sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / den


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--title", default="Soak")
    a = ap.parse_args(argv)
    d = json.load(open(a.path))
    s = d["summary"]
    out = [f"# {a.title}", ""]
    out.append(f"`{a.path}`: {'complete' if s.get('complete') else 'in progress'}, "
               f"{s['elapsed_minutes']:.0f} of {s['minutes']:.0f} minutes.")
    out.append("")
    out.append("| | |")
    out.append("|---|---|")
    out.append(f"| steps | {s['steps']:,} ({', '.join(f'{k} {v}' for k, v in s['steps_by_kind'].items())}) |")
    out.append(f"| events replayed | {s['events_replayed']:,} |")
    out.append(f"| notifications checked at the sink | {s['notifications_checked']:,} |")
    out.append(f"| SIGKILL restarts | {s['watcher_kills']} |")
    out.append(f"| failed steps | {s['steps_failed']} |")
    out.append(f"| duplicates outside / inside kill steps | {s['duplicates_outside_kill_steps']} / "
               f"{s['duplicates_in_kill_steps']} |")
    samples = d["samples"]
    last_pid = samples[-1]["pid"]
    mine = [x for x in samples if x.get("pid") == last_pid]
    t0 = mine[0]["t"]
    out.append("")
    out.append(f"**Last process** (pid {last_pid}, {(mine[-1]['t'] - t0) / 3600:.2f} h, {len(mine)} samples):")
    out.append("")
    out.append("| window | RSS first → last (MiB) | RSS slope (MiB/h) | C heap in use first → last (MiB) | "
               "C heap slope (MiB/h) | C heap free, kept by the allocator, first → last (MiB) |")
    out.append("|---|---|---|---|---|---|")
    for hours in (0.5, 1.0, 2.0, 4.0):
        w = [x for x in mine if x["t"] - t0 >= hours * 3600]
        if len(w) < 3:
            continue
        xs = [(x["t"] - t0) / 3600 for x in w]
        rss = [x["rss_mb"] for x in w]
        heap = [x.get("malloc_in_use_bytes", 0) / 2 ** 20 for x in w]
        free = [x.get("malloc_free_bytes", 0) / 2 ** 20 for x in w]
        rs, hs = slope(xs, rss), slope(xs, heap)
        out.append(f"| from +{hours:g} h | {rss[0]:.1f} → {rss[-1]:.1f} | {rs:+.2f} | {heap[0]:.1f} → {heap[-1]:.1f} "
                   f"| {hs:+.2f} | {free[0]:.1f} → {free[-1]:.1f} |")
    keys = ("apply_partitioned_batches", "apply_partitioned_lines", "apply_tail_submits", "apply_tail_lock_runs",
            "apply_serial_lines", "apply_tail_serial_lines")
    if all(k in mine[-1] for k in keys):
        out.append("")
        out.append("**Apply paths** (cumulative counters of the last process; per hour of its life):")
        out.append("")
        out.append("| counter | at +1 h | at the end | per hour, whole life |")
        out.append("|---|---|---|---|")
        at1 = next((x for x in mine if x["t"] - t0 >= 3600), mine[-1])
        life = max(1e-9, (mine[-1]["t"] - t0) / 3600)
        for k in keys:
            out.append(f"| `{k}` | {int(at1[k]):,} | {int(mine[-1][k]):,} | {mine[-1][k] / life:,.0f} |")
    tr = s.get("transport") or {}
    if tr.get("api_server") == "https" or tr.get("clusterapi") == "https":
        out.append("")
        out.append(f"**Transport**: API server {tr.get('api_server')}, clusterapi {tr.get('clusterapi')}"
                   + (f", a KeyUpdate every {tr['key_update_mib']:g} MiB per connection" if tr.get("key_update_mib") else "")
                   + ".")
        fr = tr.get("front") or {}
        if fr:
            out.append("")
            out.append(f"- TLS front: {fr.get('connections', 0):,} connections, "
                       f"{fr.get('bytes_down', 0) / 1e9:,.1f} GB sealed to the watcher, "
                       f"{fr.get('key_updates', 0):,} KeyUpdates and {fr.get('tickets', 0):,} session tickets sent "
                       f"(half of them split over two records), {fr.get('errors', 0)} errors")
        procs = tr.get("watcher_key_updates_by_process") or []
        if procs:
            ku = [int(p.get("key_updates", 0)) for p in procs]
            nat = sum(int(p.get("streams_native", 0)) for p in procs)
            ossl = sum(int(p.get("streams_openssl", 0)) for p in procs)
            out.append(f"- watcher processes: {len(procs)}, every one followed key updates "
                       f"({min(ku):,}-{max(ku):,} each)" if min(ku) > 0 else
                       f"- watcher processes: {len(procs)}, key updates per process {min(ku):,}-{max(ku):,}")
            out.append(f"- watch streams whose records the hub opened itself: {nat:,}; left on SSL_read: {ossl:,}")
        if "watch_tls_key_updates" in mine[-1]:
            at1 = next((x for x in mine if x["t"] - t0 >= 3600), mine[-1])
            life = max(1e-9, (mine[-1]["t"] - t0) / 3600)
            out.append(f"- last process: {int(at1['watch_tls_key_updates']):,} key updates at +1 h, "
                       f"{int(mine[-1]['watch_tls_key_updates']):,} at the end "
                       f"({mine[-1]['watch_tls_key_updates'] / life:,.0f} per hour)")
    og = s.get("object_growth")
    if og:
        out.append("")
        out.append(f"**Object census**: {json.dumps(og)[:600]}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
