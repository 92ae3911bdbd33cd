#!/usr/bin/env python3
"""Long soak with memory accounting (BASELINE config #5: bookmark/resume across API-server restarts).

    python -m benchmarks.soak --minutes 60 [--pods 10000] [--step-seconds 5] [--out f.json]

A real watcher process (``main.py production --config-dir …``: critical
filter, namespace filter, format-2 checkpoints every 5 s, ``/metrics``) runs
for ``--minutes`` against ``testing/replay_server.py`` (``churn``: ``--pods``
pod lifecycles = 5×pods events per step, one step every ``--step-seconds``)
and the verify-mode stub clusterapi. The schedule mixes, per step:

* normal steps;
* every 7th: the API server drops every watch mid-step (restart): the watcher
  must resume from its resourceVersion — every event exactly once;
* every 11th: compaction mid-step (410): the watcher relists and diffs — the
  intermediate events of that step are gone for good (what a real API server
  does), but every pod's final state (DELETED) must arrive, once;
* every 3rd: a BOOKMARK moves the resume point without events;
* every ``--kill-every`` steps: SIGKILL of the watcher mid-step and a restart
  from the checkpoint — nothing lost; duplicates allowed (re-sent owed
  notifications and events since the checkpoint) and counted.

Every ``--census-minutes`` the watcher's ``/debug/memory`` (``metrics.debug``;
the watcher runs with ``PYTHONTRACEMALLOC=1`` unless ``--no-tracemalloc``) is
taken: live Python objects per type and the top tracemalloc allocation sites.
The summary diffs the census at the end of the last process's first hour with
its last one (``object_growth``), naming what grows outside the C heap. With
``--out`` the summary so far is rewritten every ``--progress-minutes``
(``"complete": false``), so a run cut short still leaves its record.

``--api-tls`` puts the API server behind a TLS 1.3 front
(``testing/tls_front.py``: the native fixture sealer, a KeyUpdate every
``--key-update-mib`` MiB per connection and a NewSessionTicket every
``--ticket-every-mib``, half of them cut over two records), so the
watcher reads its watch over https like production (in-cluster,
``production.yaml``) through its own TLS record layer; ``--tls`` serves the
stub clusterapi over https. The front's drops pass the replay fixture's
aborts on as resets.

Every ``--sample-seconds`` the harness records the watcher's RSS (VmRSS/VmHWM)
and its gauges: cached pods and cache bytes, owed notifications and bytes,
checkpoint stall. The sink's keys are handed over and reset every 50 steps
(SIGUSR2) so neither side grows with the run; each step is judged once the
window has passed it. Output: per-sample series + per-step verdicts + an RSS
slope after warm-up (least squares, MiB/hour).
"""

from __future__ import annotations

import argparse
import asyncio
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import textwrap
import time
from typing import Dict, List, Optional, Set, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from benchmarks.restart_soak import free_port, scrape  # noqa: E402

TARGETS = ("default", "production", "monitoring", "kube-system")  # config/production.yaml


def vm(pid: int) -> Dict[str, float]:
    out = {}
    try:
        with open(f"/proc/{pid}/status") as fh:
            for line in fh:
                if line.startswith(("VmRSS:", "VmHWM:")):
                    out[line.split(":")[0]] = int(line.split()[1]) / 1024
    except OSError:
        pass
    return out


def slope_mib_per_hour(points: List[Tuple[float, float]]) -> Optional[float]:
    if len(points) < 3:
        return None
    n = len(points)
    mx = sum(t for t, _ in points) / n
    my = sum(v for _, v in points) / n
    sxx = sum((t - mx) ** 2 for t, _ in points)
    if sxx == 0:
        return None
    return sum((t - mx) * (v - my) for t, v in points) / sxx * 3600


def rss_segments(samples: List[dict], warmup_minutes: float) -> List[dict]:
    """RSS per watcher process (a SIGKILL restart starts a new one): the
    in-process slope after that process's own warm-up, so restarts at
    different RSS levels do not blur the growth rate."""
    by_pid: Dict[int, List[dict]] = {}
    for x in samples:
        if x.get("rss_mb") and x.get("pid"):
            by_pid.setdefault(x["pid"], []).append(x)
    out = []
    for pid, xs in by_pid.items():
        t0 = xs[0]["t"]
        after = [x for x in xs if x["t"] - t0 >= warmup_minutes * 60]
        out.append({"pid": pid, "minutes": round((xs[-1]["t"] - t0) / 60, 1), "samples": len(xs),
                    "rss_mb_first": xs[0]["rss_mb"], "rss_mb_last": xs[-1]["rss_mb"],
                    "rss_mb_max": max(x["rss_mb"] for x in xs),
                    "slope_mib_per_hour_after_warmup": slope_mib_per_hour([(x["t"], x["rss_mb"]) for x in after])})
    return sorted(out, key=lambda d: -d["minutes"])


def tls_by_process(samples: List[dict]) -> List[dict]:
    """Per watcher process: the TLS record layer's counters at its last
    sample (streams taken over / left on SSL_read, key updates followed)."""
    last: Dict[int, dict] = {}
    for x in samples:
        if x.get("pid") and x.get("watch_tls_records") is not None:
            last[x["pid"]] = x
    return [{"pid": pid, "streams_native": x.get("watch_tls_streams_native"),
             "streams_openssl": x.get("watch_tls_streams_openssl"), "records": x.get("watch_tls_records"),
             "key_updates": x.get("watch_tls_key_updates"), "ring_bytes": x.get("watch_reader_tls_ring_bytes")}
            for pid, x in last.items()]


def memory_at_peak(samples: List[dict]) -> Optional[dict]:
    """The highest-RSS sample, broken down by what the watcher reports holding."""
    xs = [x for x in samples if x.get("rss_mb")]
    if not xs:
        return None
    p = max(xs, key=lambda x: x["rss_mb"])
    mib = lambda k: round((p.get(k) or 0) / 2 ** 20, 1)  # noqa: E731
    parts = {"cache": mib("cache_bytes"), "notifier_owed": mib("notify_outstanding_bytes"),
             "watch_read_buffers": mib("watch_reader_allocated_bytes")}
    out = {"t": p["t"], "rss_mb": p["rss_mb"], "accounted_mib": parts,
           "unaccounted_mib": round(p["rss_mb"] - sum(parts.values()), 1)}
    if p.get("malloc_in_use_bytes") is not None:
        # the C heap as glibc sees it: in use (cache, buffers and everything else
        # malloc'd, Python's large objects included) and free but retained
        out["c_heap_mib"] = {"in_use": mib("malloc_in_use_bytes"), "free_retained": mib("malloc_free_bytes")}
    return out


def object_growth(censuses: List[dict], top: int = 15) -> Optional[dict]:
    """Census of the last process at the end of its first hour (or its first
    one) vs its last: the Python object types and tracemalloc sites that grew."""
    if not censuses:
        return None
    pid = censuses[-1]["pid"]
    mine = [c for c in censuses if c["pid"] == pid]
    if len(mine) < 2:
        return None
    first = next((c for c in mine if c["age_min"] >= 60), mine[0])
    if first is mine[-1]:
        first = mine[0]
    last = mine[-1]
    a, b = first["doc"], last["doc"]
    types = set(a["types"]) | set(b["types"])
    delta = sorted(((k, b["types"].get(k, 0) - a["types"].get(k, 0)) for k in types), key=lambda kv: -kv[1])
    out = {"from": {"age_min": first["age_min"], "rss_mb": first["rss_mb"], "gc_objects": a["gc_objects"],
                    "allocated_blocks": a["allocated_blocks"]},
           "to": {"age_min": last["age_min"], "rss_mb": last["rss_mb"], "gc_objects": b["gc_objects"],
                  "allocated_blocks": b["allocated_blocks"]},
           "hours": round((last["age_min"] - first["age_min"]) / 60, 2),
           "types_grown": [{"type": k, "delta": d} for k, d in delta[:top] if d > 0],
           "types_shrunk": [{"type": k, "delta": d} for k, d in delta[::-1][:5] if d < 0]}
    ta, tb = a.get("tracemalloc"), b.get("tracemalloc")
    if ta and tb:
        sa = {x["site"]: x["bytes"] for x in ta["top"]}
        sb = {x["site"]: x["bytes"] for x in tb["top"]}
        grown = sorted(((k, sb.get(k, 0) - sa.get(k, 0)) for k in set(sa) | set(sb)), key=lambda kv: -kv[1])
        out["tracemalloc"] = {"traced_bytes_from": ta["traced_bytes"], "traced_bytes_to": tb["traced_bytes"],
                              "sites_grown": [{"site": k, "bytes": d} for k, d in grown[:top] if d > 0]}
    return out


class Soak:
    def __init__(self, a) -> None:
        self.a = a
        self.dir = tempfile.mkdtemp(prefix="kw-soak-")
        self.verify_dir = os.path.join(self.dir, "verify")
        os.makedirs(self.verify_dir)
        self.metrics_port = free_port()
        self.sink_port = free_port()
        self.samples: List[dict] = []
        self.watcher: Optional[subprocess.Popen] = None
        self.counts: Dict[int, Dict[str, int]] = {}  # step -> key -> deliveries
        self.verdicts: List[dict] = []
        self.kinds: Dict[int, str] = {}
        # steps inside a SIGKILL's at-least-once window (the kill step and the
        # ones the last checkpoint may predate), whatever else they were (a
        # drop or an expiry there is re-sent too)
        self.rewound: Set[int] = set()
        self.kills = 0
        self.t0 = time.monotonic()
        self.censuses: List[dict] = []
        self.watcher_started = self.t0
        self.front = None

    # ------------------------------------------------------------------ fixtures
    async def start(self) -> None:
        from k8s_watcher_amd.testing.replay_server import Template
        t = time.monotonic()
        self.template = Template("churn", self.a.pods, 0)
        # per event: (uid suffix, type, phase, ns) — what the production profile notifies
        self.expect: List[Tuple[str, str, str, bool]] = []
        import json as _json
        for et, segs, uid in self.template.events:
            obj = _json.loads(self.template.obj(segs, 0, uid, 0))
            phase = (obj.get("status") or {}).get("phase") or ""
            ns = obj["metadata"]["namespace"]
            critical = et == "DELETED" or phase in ("Succeeded", "Failed")
            self.expect.append((uid[8:], et, phase, critical and ns in TARGETS))
        print(f"template: {len(self.expect)} events/step ({time.monotonic() - t:.1f}s)", file=sys.stderr, flush=True)
        spawn = lambda *c: asyncio.create_subprocess_exec(  # noqa: E731
            *c, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            stderr=asyncio.subprocess.DEVNULL, start_new_session=True, cwd=ROOT)
        self.pki = None
        if self.a.api_tls or self.a.tls:
            from k8s_watcher_amd.testing.certs import make_pki
            self.pki = make_pki(os.path.join(self.dir, "pki"))
        sink_tls = ["--tls-cert", self.pki.server_crt, "--tls-key", self.pki.server_key] if self.a.tls else []
        self.replay = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.replay_server",
                                  "--template", "churn", "--pods", str(self.a.pods))
        self.sink = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port",
                                str(self.sink_port), "--workers", str(self.a.sink_workers),
                                "--verify-dir", self.verify_dir, *sink_tls)
        ready = (await asyncio.wait_for(self.replay.stdout.readline(), 900)).decode().split()
        self.api_port, self.E = int(ready[1]), int(ready[2])
        await self.sink.stdout.readline()
        self.front = None
        server = f"http://127.0.0.1:{self.api_port}"
        if self.a.api_tls:
            self.front = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.tls_front",
                                     "--backend", f"127.0.0.1:{self.api_port}", "--cert", self.pki.server_crt,
                                     "--key", self.pki.server_key, "--key-update-mib", str(self.a.key_update_mib),
                                     "--ticket-every-mib", str(self.a.ticket_every_mib))
            front_port = int((await asyncio.wait_for(self.front.stdout.readline(), 60)).decode().split()[1])
            server = f"https://127.0.0.1:{front_port}"
        ca = f", certificate-authority: {self.pki.ca_crt}" if self.a.api_tls else ""
        await asyncio.sleep(0.3)
        cfg = os.path.join(self.dir, "config")
        os.makedirs(cfg)
        with open(os.path.join(self.dir, "kubeconfig"), "w") as fh:
            fh.write(textwrap.dedent(f"""
                current-context: c
                clusters: [{{name: c, cluster: {{server: "{server}"{ca}}}}}]
                contexts: [{{name: c, context: {{cluster: c, user: u}}}}]
                users: [{{name: u, user: {{token: x}}}}]
                """))
        with open(os.path.join(cfg, "base.yaml"), "w") as fh:
            fh.write(textwrap.dedent(f"""
                kubernetes: {{config_file: {os.path.join(self.dir, "kubeconfig")}}}
                clusterapi:
                  health_check_on_start: false
                  retry: {{max_attempts: 10, delay_seconds: 0.2}}
                metrics: {{enabled: true, host: 127.0.0.1, port: {self.metrics_port}, debug: true}}
                watcher:
                  retry: {{max_attempts: 0, delay_seconds: 0.1, max_delay_seconds: 2}}
                  checkpoint: {{path: {os.path.join(self.dir, "state", "checkpoint.bin")}, interval_seconds: 5}}
                """))
        sink_ca = f"ca_file: {self.pki.ca_crt}, " if self.a.tls else ""
        with open(os.path.join(cfg, "production.yaml"), "w") as fh:
            fh.write(textwrap.dedent(f"""
                environment: production
                clusterapi: {{base_url: "{"https" if self.a.tls else "http"}://127.0.0.1:{self.sink_port}", {sink_ca}pool: {{connections: 4, pipeline_depth: 32}}}}
                watcher:
                  namespaces: [{", ".join(TARGETS)}]
                  log_level: WARNING
                  alerts: {{critical_events_only: true}}
                """))
        self.cfg = cfg

    async def front_stats(self) -> Optional[dict]:
        """The TLS front's counters (connections, key updates, tickets, aborts)."""
        if self.front is None:
            return None
        self.front.stdin.write(b"STATS\n")
        await self.front.stdin.drain()
        line = (await asyncio.wait_for(self.front.stdout.readline(), 30)).decode()
        return json.loads(line.split(" ", 1)[1])

    async def cmd(self, line: str) -> int:
        self.replay.stdin.write((line + "\n").encode())
        await self.replay.stdin.drain()
        return int((await self.replay.stdout.readline()).decode().split()[2])

    def start_watcher(self) -> None:
        log = open(os.path.join(self.dir, "watcher.log"), "ab")
        env = dict(os.environ)
        if self.a.tracemalloc:
            env["PYTHONTRACEMALLOC"] = "1"  # one frame per allocation site: /debug/memory's top sites
        self.watcher = subprocess.Popen([sys.executable, os.path.join(ROOT, "main.py"), "production",
                                         "--config-dir", self.cfg], cwd=ROOT, stdout=log, stderr=log,
                                        start_new_session=True, env=env)
        self.watcher_started = time.monotonic()

    def census(self) -> None:
        """The watcher's Python object census (``/debug/memory``)."""
        import urllib.request
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{self.metrics_port}/debug/memory", timeout=30) as r:
                doc = json.loads(r.read())
        except (OSError, ValueError) as exc:
            print(f"census failed: {exc}", file=sys.stderr, flush=True)
            return
        v = vm(self.watcher.pid)
        self.censuses.append({"t": round(time.monotonic() - self.t0, 1), "pid": self.watcher.pid,
                              "age_min": round((time.monotonic() - self.watcher_started) / 60, 1),
                              "rss_mb": v.get("VmRSS"), "doc": doc})

    async def wait_watching(self) -> None:
        for _ in range(6000):
            if await self.cmd("WATCHERS") >= 1 and scrape(self.metrics_port).get("cached_pods") is not None:
                return
            await asyncio.sleep(0.01)
        raise TimeoutError("watcher did not connect")

    # ------------------------------------------------------------------ sampling
    def sample(self, step: int) -> None:
        m = scrape(self.metrics_port)
        v = vm(self.watcher.pid)
        s = {"t": round(time.monotonic() - self.t0, 1), "step": step, "rss_mb": v.get("VmRSS"),
             "hwm_mb": v.get("VmHWM"), "pid": self.watcher.pid}
        for k in ("cached_pods", "cache_bytes", "notify_outstanding", "notify_outstanding_bytes",
                  "watch_reader_allocated_bytes", "watch_reader_held_bytes", "malloc_in_use_bytes", "malloc_free_bytes",
                  "checkpoint_stall_ms", "checkpoint_write_ms", "checkpoint_bytes", "events_received",
                  "notify_delivered", "expired_410", "watch_restarts", "relists", "bookmarks",
                  "apply_partitioned_batches", "apply_partitioned_lines", "apply_tail_serial_lines",
                  "apply_tail_submits", "apply_tail_lock_runs", "apply_serial_batches", "apply_serial_lines",
                  "malloc_arenas", "watch_reader_tls_ring_bytes", "watch_tls_streams_native",
                  "watch_tls_streams_openssl", "watch_tls_records", "watch_tls_key_updates"):
            if k in m:
                s[k] = m[k]
        self.samples.append(s)

    # ------------------------------------------------------------------ verification
    def harvest(self, upto_step: int) -> None:
        """Take the sink's keys (dump + reset) and judge every step < upto_step."""
        for f in glob.glob(os.path.join(self.verify_dir, "sink-*.json")):
            os.unlink(f)
        os.killpg(self.sink.pid, signal.SIGUSR2)
        deadline = time.monotonic() + 120
        while len(glob.glob(os.path.join(self.verify_dir, "sink-*.json"))) < self.a.sink_workers:
            if time.monotonic() > deadline:
                break
            time.sleep(0.05)
        for f in glob.glob(os.path.join(self.verify_dir, "sink-*.json")):
            with open(f) as fh:
                for k, n in json.load(fh)["keys"].items():
                    step = int(k[:8], 16)
                    d = self.counts.setdefault(step, {})
                    d[k] = d.get(k, 0) + n
        for step in sorted(s for s in self.counts if s < upto_step):
            self.judge(step, self.counts.pop(step))

    def judge(self, step: int, got: Dict[str, int]) -> None:
        kind = self.kinds.get(step, "normal")
        prefix = f"{step & 0xFFFFFFFF:08x}"
        want: Set[str] = {f"{prefix}{u}|{et}|{ph}" for u, et, ph, n in self.expect if n}
        dups = sum(v - 1 for v in got.values() if v > 1)
        if kind == "expire":
            # the compacted window is gone for good (a pod born and deleted inside
            # it is unobservable, as with a real API server); every pod that was
            # notified at all must end DELETED — the relist diff sends it
            seen = {k.split("|")[0] for k in got}
            have_del = {k.split("|")[0] for k in got if "|DELETED|" in k}
            missing = len(seen - have_del)
        else:
            missing = len(want - set(got))
        rewound = step in self.rewound
        ok = missing == 0 and (dups == 0 or rewound)
        self.verdicts.append({"step": step, "kind": kind, "ok": ok, "missing": missing, "duplicates": dups,
                              "received": sum(got.values()), "rewound": rewound})

    async def close(self) -> None:
        if self.watcher is not None and self.watcher.poll() is None:
            os.killpg(self.watcher.pid, signal.SIGTERM)
            try:
                self.watcher.wait(20)
            except subprocess.TimeoutExpired:
                os.killpg(self.watcher.pid, signal.SIGKILL)
        for p in (self.replay, self.sink, self.front):
            if p is None:
                continue
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            try:
                await asyncio.wait_for(p.wait(), 10)
            except asyncio.TimeoutError:
                os.killpg(p.pid, signal.SIGKILL)
            t = getattr(p, "_transport", None)
            if t is not None:
                t.close()
        shutil.rmtree(self.dir, ignore_errors=True)


async def amain(a) -> dict:
    s = Soak(a)
    try:
        await s.start()
        s.start_watcher()
        await s.wait_watching()
        await s.cmd("STEP 0")  # warm-up step, judged like the others
        end = time.monotonic() + a.minutes * 60
        step = 1
        last_sample = 0.0
        next_harvest = 50
        events = s.E
        next_census = time.monotonic() + 60.0  # one early census, then every --census-minutes
        next_progress = time.monotonic() + a.progress_minutes * 60
        while time.monotonic() < end:
            if time.monotonic() >= next_census:
                s.census()
                next_census = time.monotonic() + a.census_minutes * 60
            if a.out and time.monotonic() >= next_progress:
                write_out(a.out, {"summary": summarize(s, a, step, events, complete=False),
                                  "samples": s.samples, "verdicts": s.verdicts, "censuses": s.censuses})
                next_progress = time.monotonic() + a.progress_minutes * 60
            t_step = time.monotonic()
            half = s.E // 2
            in_kill_window = a.kill_window_minutes is None or time.monotonic() - s.t0 < a.kill_window_minutes * 60
            if a.kill_every and step % a.kill_every == 0 and in_kill_window:
                s.kinds[step] = "kill"
                # the last checkpoint (every 5 s) may predate these: re-sent after the restart
                for back in range(1, int(5.0 / a.step_seconds) + 3):
                    s.rewound.add(step - back)
                    if s.kinds.get(step - back, "normal") == "normal":
                        s.kinds[step - back] = "pre-kill"
                s.rewound.add(step)
                send = asyncio.ensure_future(s.cmd(f"STEP {step}"))
                await asyncio.sleep(a.step_seconds * 0.1)
                s.sample(step)
                os.killpg(s.watcher.pid, signal.SIGKILL)
                s.watcher.wait()
                s.kills += 1
                s.start_watcher()
                await send
                await s.wait_watching()  # back before the next drop/compaction: a watcher that is
                # down across a compaction legitimately never sees pods born and gone inside it
            elif step % 11 == 0:
                s.kinds[step] = "expire"
                await s.cmd(f"STEP {step} expire={half}")
            elif step % 7 == 0:
                s.kinds[step] = "drop"
                await s.cmd(f"STEP {step} drop={half}")
            else:
                await s.cmd(f"STEP {step}")
            if step % 3 == 0:
                await s.cmd("BOOKMARK")
            events += s.E
            while time.monotonic() < t_step + a.step_seconds:
                if time.monotonic() - last_sample >= a.sample_seconds:
                    last_sample = time.monotonic()
                    s.sample(step)
                    r = s.samples[-1]
                    if s.front is not None:
                        r["front"] = await s.front_stats()
                    print(f"[{r['t']:7.1f}s] step {step} rss {r.get('rss_mb')} MiB cached {r.get('cached_pods')} "
                          f"owed {r.get('notify_outstanding')} ({r.get('notify_outstanding_bytes')} B)",
                          file=sys.stderr, flush=True)
                await asyncio.sleep(0.05)
            if step >= next_harvest:
                s.harvest(step - 10)  # steps well behind the stream are complete
                next_harvest = step + 50
            step += 1
        # let the stream finish, then judge everything
        await asyncio.sleep(max(5.0, a.step_seconds))
        s.sample(step)
        s.census()
        s.harvest(step + 1)
        return {"summary": summarize(s, a, step, events, complete=True), "samples": s.samples,
                "verdicts": s.verdicts, "censuses": s.censuses}
    finally:
        await s.close()


def write_out(path: str, doc: dict) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(doc, fh, indent=1)
    os.replace(tmp, path)


def summarize(s: "Soak", a, step: int, events: int, complete: bool) -> dict:
    after = [x for x in s.samples if x["t"] >= a.warmup_minutes * 60 and x.get("rss_mb")]
    bad = [v for v in s.verdicts if not v["ok"]]
    last = s.samples[-1] if s.samples else {}
    summary = {
        "complete": complete, "elapsed_minutes": round((time.monotonic() - s.t0) / 60, 1),
        "minutes": a.minutes, "steps": step, "events_replayed": events, "pods_per_step": a.pods,
        "watcher_kills": s.kills,
        "steps_by_kind": {k: sum(1 for v in s.verdicts if v["kind"] == k)
                          for k in ("normal", "drop", "expire", "kill", "pre-kill")},
        "steps_failed": len(bad), "failed_examples": bad[:5],
        "duplicates_outside_kill_steps": sum(v["duplicates"] for v in s.verdicts if not v.get("rewound")),
        "duplicates_in_kill_steps": sum(v["duplicates"] for v in s.verdicts if v.get("rewound")),
        "notifications_checked": sum(v["received"] for v in s.verdicts),
        "transport": {"api_server": "https" if a.api_tls else "http", "clusterapi": "https" if a.tls else "http",
                      "key_update_mib": a.key_update_mib if a.api_tls else None,
                      "front": next((x["front"] for x in reversed(s.samples) if x.get("front")), None),
                      "watcher_key_updates_by_process": tls_by_process(s.samples)},
        "rss_mb_after_warmup": {"min": min(x["rss_mb"] for x in after) if after else None,
                                "max": max(x["rss_mb"] for x in after) if after else None,
                                "slope_mib_per_hour": slope_mib_per_hour([(x["t"], x["rss_mb"]) for x in after])},
        "peak_rss_mb_last_process": last.get("hwm_mb"),
        "rss_segments": rss_segments(s.samples, a.warmup_minutes),
        "memory_at_peak": memory_at_peak(s.samples),
        "object_growth": object_growth(s.censuses),
        "last_sample": last,
    }
    return summary


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--minutes", type=float, default=60)
    ap.add_argument("--pods", type=int, default=10000)
    ap.add_argument("--step-seconds", type=float, default=5.0)
    ap.add_argument("--kill-every", type=int, default=60, help="SIGKILL the watcher every N steps (0 = never)")
    ap.add_argument("--kill-window-minutes", type=float, default=None,
                    help="kills only in the first M minutes; the rest is one process (in-process RSS slope)")
    ap.add_argument("--sample-seconds", type=float, default=10.0)
    ap.add_argument("--warmup-minutes", type=float, default=5.0)
    ap.add_argument("--sink-workers", type=int, default=2)
    ap.add_argument("--census-minutes", type=float, default=60.0,
                    help="take the watcher's /debug/memory object census this often (and once at minute 1)")
    ap.add_argument("--no-tracemalloc", dest="tracemalloc", action="store_false",
                    help="run the watcher without PYTHONTRACEMALLOC (object counts only)")
    ap.add_argument("--progress-minutes", type=float, default=15.0,
                    help="with --out: rewrite the summary so far this often")
    ap.add_argument("--api-tls", action="store_true",
                    help="the API server over https (TLS front with key updates): production's transport")
    ap.add_argument("--tls", action="store_true", help="the stub clusterapi over https")
    ap.add_argument("--key-update-mib", type=float, default=64.0,
                    help="with --api-tls: a KeyUpdate every N MiB on each connection")
    ap.add_argument("--ticket-every-mib", type=float, default=256.0,
                    help="with --api-tls: a NewSessionTicket every N MiB on each connection")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    res = asyncio.run(amain(a))
    print(json.dumps(res["summary"], indent=1))
    if a.out:
        write_out(a.out, res)
    return 0 if res["summary"]["steps_failed"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
