"""In-process ceiling of the fused native pipeline (no sockets, no fixtures).

``bench.py`` is bounded by its replay fixture once the watcher decodes in
parallel (one loopback TCP stream tops out near 3.3 GB/s, see
profiles/decode_threads_gpu_box.md). This script feeds the same prerendered
churn steps straight into ``_kwcore.Pipeline`` — chunk de-framing, decode,
filters, native pod cache, payload cores — from cache-hot buffers of the size
one socket read returns, and reports events/s per decode-thread count, plus
the single-thread stage costs from ``_kwcore.bench_parse`` at each SIMD level.

    python -m benchmarks.pipeline_micro [--pods 10000] [--threads 0,1,2,3,5] [--json out.json]
"""

from __future__ import annotations

import argparse
import json
import sys
import time

from k8s_watcher_amd.ops.native import load
from k8s_watcher_amd.testing.replay_server import Template

READ_SIZE = 4 << 20  # watcher.watch_read_bytes default (bytes per socket read)


def unframe(data: bytes) -> bytes:
    out, p = bytearray(), 0
    while p < len(data):
        nl = data.index(b"\r\n", p)
        size = int(data[p:nl], 16)
        out += data[nl + 2:nl + 2 + size]
        p = nl + 2 + size + 2
    return bytes(out)


def pipeline_rate(mod, data: bytes, n: int, threads: int, critical: bool, reps: int,
                  read_size: int = READ_SIZE, notify: bool = False, probe: dict = None) -> float:
    """``notify``: the production wiring — namespace filter over half the
    namespaces and a native notifier core (never connected: submits queue up,
    which is the apply-side cost of a notification)."""
    chunks = [data[j:j + read_size] for j in range(0, len(data), read_size)]
    best = float("inf")
    for _ in range(reps):
        nsset = notifier = None
        if notify:
            nsset = frozenset(["default", "kube-system", "production", "monitoring"])
            notifier = mod.Notifier(b"POST /x HTTP/1.1\r\nContent-Length: ", 4, 32, 3, 1.0, 2.0, 30.0,
                                    False, False, [502, 503], {})
        pl = mod.Pipeline("production", mod.PodCache(), {}, nsset, critical, False, 1, 0, True, True, notifier,
                          False, False, threads)
        spent = 0
        if probe is not None:
            mod.probe(True)
        for ch in chunks:
            hot = bytearray(ch)  # like a recv buffer: just written, in cache
            t0 = time.perf_counter_ns()
            pl.feed_chunked(hot, 0)
            spent += time.perf_counter_ns() - t0
        if probe is not None:
            got = mod.probe(False)
            if spent < best:
                probe.clear()
                probe.update({k: round(got[k] / max(1, got["lines"]), 1)
                              for k in ("split_ns", "wait_ns", "apply_ns", "run_ns")})
        best = min(best, spent)
        del pl
    return n / (best / 1e9)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--pods", type=int, default=10000)
    ap.add_argument("--threads", default="0,1,2,3,5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--read-size", type=int, default=READ_SIZE, help="bytes per simulated socket read")
    args = ap.parse_args(argv)
    mod = load()
    t = Template("churn", args.pods, 0)
    data, offs = t.render(0, 0, len(t))
    n = len(offs)
    lines = unframe(data)
    res = {"events": n, "bytes_per_event": round(len(lines) / n), "stages_ns_per_event": {}, "pipeline": []}
    for level, name in ((False, "scalar"), ("avx2", "avx2"), (True, "best")):
        mod.set_simd(level)
        row = {}
        for mode, label in ((0, "skip"), (3, "light"), (1, "extract"), (2, "extract+core")):
            secs = min(mod.bench_parse(lines, mode, 1)[0] for _ in range(3))
            row[label] = round(secs / n * 1e9)
        res["stages_ns_per_event"][name] = row
    mod.set_simd(True)
    res["simd"] = mod.cpu_features()
    for th in [int(x) for x in args.threads.split(",")]:
        for critical, notify, profile in ((True, False, "production (critical filter)"),
                                          (False, False, "all events notified"),
                                          (True, True, "production + ns filter + native notifier")):
            pr = {}
            rate = pipeline_rate(mod, data, n, th, critical, args.reps, args.read_size, notify, pr)
            res["pipeline"].append({"decode_threads": th, "profile": profile, "events_per_s": round(rate),
                                    "loop_ns_per_event": pr})
    print(f"# native pipeline ceiling, {n} events x {res['bytes_per_event']} B, SIMD {res['simd']}\n")
    print("| SIMD | skip | light extract | full extract | + payload core |  (ns/event, one thread)")
    print("|---|---|---|---|---|")
    for name, row in res["stages_ns_per_event"].items():
        print(f"| {name} | {row['skip']} | {row['light']} | {row['extract']} | {row['extract+core']} |")
    print("\n| decode threads | profile | events/s | calling thread ns/event: split / decode wait / apply |"
          "\n|---|---|---|---|")
    for r in res["pipeline"]:
        p = r["loop_ns_per_event"]
        print(f"| {r['decode_threads']} | {r['profile']} | {r['events_per_s']:,} | "
              f"{p.get('split_ns')} / {p.get('wait_ns')} / {p.get('apply_ns')} |")
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
