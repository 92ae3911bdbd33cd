#!/usr/bin/env python3
"""Crash-restart recovery at scale: SIGKILL the watcher process mid-stream, restart it from its checkpoint.

    python -m benchmarks.restart_soak [--pods 100000] [--rounds 6] [--kills 5] [--out f.json]

The reference keeps its resume point in memory only (``pod_watcher.py:16``):
a restart re-lists and replays every pod as ``ADDED`` (SURVEY §5.3 item 5,
§5.4). Here the watcher is a real separate process (``main.py staging`` with a
config directory pointing at the fixtures) and it is killed with SIGKILL — no
shutdown hook, no final checkpoint — while it is streaming, then started
again:

* fixture: ``testing/replay_server.py`` ``steady`` template, ``--pods`` pods
  served by the initial LIST, then ``--rounds`` rounds that MODIFY every pod
  once (the pod's ``k8s-watcher.test/generation`` annotation = the round), one
  cluster-wide watch with resourceVersion resume (backlog) like kube-apiserver;
* watcher: staging profile (every event notified), format-2 checkpoints every
  ``--checkpoint-interval`` seconds (``engine/checkpoint.py``), ``/metrics``
  polled for the checkpoint stall, write time and size;
* sink: verify mode, counting ``uid|type|phase|generation`` keys.

Pass criteria, reported in the JSON: every pod's every generation delivered
(``lost == 0``, so in particular no final state is lost), and duplicates — the
notifications sent again after a restart — bounded by what the killed process
had handled since its last checkpoint.
"""

from __future__ import annotations

import argparse
import asyncio
import glob
import json
import os
import random
import re
import shutil
import signal
import subprocess
import sys
import tempfile
import textwrap
import time
import urllib.request
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def scrape(port: int) -> Dict[str, float]:
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2) as r:
            text = r.read().decode()
    except OSError:
        return {}
    out = {}
    for line in text.splitlines():
        m = re.match(r"^k8s_watcher_(\w+?)(?:_total)? ([-0-9.e+naninf]+)$", line)
        if m:
            try:
                out[m.group(1)] = float(m.group(2))
            except ValueError:
                pass
    return out


def rss_peak_mb(pid: int) -> Optional[float]:
    try:
        with open(f"/proc/{pid}/status") as fh:
            for line in fh:
                if line.startswith("VmHWM:"):
                    return int(line.split()[1]) / 1024
    except OSError:
        pass
    return None


class Run:
    def __init__(self, a) -> None:
        self.a = a
        self.dir = tempfile.mkdtemp(prefix="kw-restart-")
        self.verify_dir = os.path.join(self.dir, "verify")
        os.makedirs(self.verify_dir)
        self.ck = os.path.join(self.dir, "state", "checkpoint.bin")
        self.metrics_port = free_port()
        self.sink_port = free_port()
        self.samples: List[dict] = []
        self.watcher: Optional[subprocess.Popen] = None
        self.peaks: List[float] = []

    async def start_fixtures(self) -> None:
        spawn = lambda *c: asyncio.create_subprocess_exec(  # noqa: E731
            *c, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            stderr=asyncio.subprocess.DEVNULL, start_new_session=True, cwd=ROOT)
        self.replay = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.replay_server",
                                  "--template", "steady", "--pods", str(self.a.pods), "--namespaces", "default")
        self.sink = await spawn(sys.executable, "-m", "k8s_watcher_amd.testing.stub_sink", "--port",
                                str(self.sink_port), "--workers", str(self.a.sink_workers),
                                "--verify-dir", self.verify_dir)
        ready = (await asyncio.wait_for(self.replay.stdout.readline(), 900)).decode().split()
        assert ready[0] == "READY", ready
        self.api_port, self.E = int(ready[1]), int(ready[2])
        await self.sink.stdout.readline()
        await asyncio.sleep(0.3)
        cfg = os.path.join(self.dir, "config")
        os.makedirs(cfg)
        with open(os.path.join(self.dir, "kubeconfig"), "w") as fh:
            fh.write(textwrap.dedent(f"""
                current-context: c
                clusters: [{{name: c, cluster: {{server: "http://127.0.0.1:{self.api_port}"}}}}]
                contexts: [{{name: c, context: {{cluster: c, user: u}}}}]
                users: [{{name: u, user: {{token: x}}}}]
                """))
        with open(os.path.join(cfg, "base.yaml"), "w") as fh:
            fh.write(textwrap.dedent(f"""
                kubernetes: {{config_file: {os.path.join(self.dir, "kubeconfig")}}}
                clusterapi:
                  base_url: "http://127.0.0.1:{self.sink_port}"
                  health_check_on_start: false
                  retry: {{max_attempts: 10, delay_seconds: 0.2}}
                metrics: {{enabled: true, host: 127.0.0.1, port: {self.metrics_port}}}
                watcher:
                  log_level: WARNING
                  retry: {{max_attempts: 0, delay_seconds: 0.2}}
                  checkpoint: {{path: {self.ck}, interval_seconds: {self.a.checkpoint_interval}}}
                """))
        open(os.path.join(cfg, "staging.yaml"), "w").close()
        self.cfg = cfg

    async def cmd(self, line: str) -> int:
        self.replay.stdin.write((line + "\n").encode())
        await self.replay.stdin.drain()
        return int((await self.replay.stdout.readline()).decode().split()[2])

    def start_watcher(self) -> None:
        log = open(os.path.join(self.dir, "watcher.log"), "ab")
        self.watcher = subprocess.Popen([sys.executable, os.path.join(ROOT, "main.py"), "staging",
                                         "--config-dir", self.cfg], cwd=ROOT, stdout=log, stderr=log,
                                        start_new_session=True)

    def rss_mb(self) -> Optional[float]:
        """Current RSS of the running watcher process (VmRSS), for the memory breakdown."""
        try:
            with open(f"/proc/{self.watcher.pid}/status") as fh:
                for line in fh:
                    if line.startswith("VmRSS:"):
                        return int(line.split()[1]) / 1024
        except (OSError, AttributeError):
            pass
        return None

    def kill_watcher(self) -> None:
        p = self.watcher
        peak = rss_peak_mb(p.pid)
        if peak:
            self.peaks.append(peak)
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()

    async def poll(self, until, timeout: float, what: str) -> dict:
        deadline = time.monotonic() + timeout
        last_print = 0.0
        while True:
            m = scrape(self.metrics_port)
            if m:
                self.samples.append({"t": round(time.monotonic(), 3), "rss_mb": self.rss_mb(),
                                     **{k: m[k] for k in (
                    "checkpoint_stall_ms", "checkpoint_write_ms", "checkpoint_bytes", "checkpoint_owed",
                    "notify_delivered", "events_received", "cached_pods", "cache_bytes",
                    "notify_outstanding_bytes", "watch_reader_allocated_bytes", "malloc_in_use_bytes",
                    "malloc_free_bytes") if k in m}})
            if m and until(m):
                return m
            if time.monotonic() > deadline:
                raise TimeoutError(f"{what}: {m}")
            if time.monotonic() - last_print > 10:
                last_print = time.monotonic()
                print(f"  ... {what}: delivered={m.get('notify_delivered')} received={m.get('events_received')}",
                      file=sys.stderr, flush=True)
            await asyncio.sleep(0.1)

    def sink_keys(self) -> Dict[str, int]:
        for f in glob.glob(os.path.join(self.verify_dir, "sink-*.json")):
            os.unlink(f)
        os.killpg(self.sink.pid, signal.SIGUSR1)
        deadline = time.monotonic() + 120
        while len(glob.glob(os.path.join(self.verify_dir, "sink-*.json"))) < self.a.sink_workers:
            if time.monotonic() > deadline:
                break
            time.sleep(0.05)
        keys: Dict[str, int] = {}
        for f in glob.glob(os.path.join(self.verify_dir, "sink-*.json")):
            with open(f) as fh:
                for k, v in json.load(fh)["keys"].items():
                    keys[k] = keys.get(k, 0) + v
        return keys

    async def close(self) -> None:
        if self.watcher is not None and self.watcher.poll() is None:
            os.killpg(self.watcher.pid, signal.SIGKILL)
            self.watcher.wait()
        for p in (self.replay, self.sink):
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
    from benchmarks.soak import memory_at_peak  # soak.py imports this module
    rng = random.Random(a.seed)
    r = Run(a)
    try:
        await r.start_fixtures()
        P = a.pods
        t0 = time.monotonic()
        r.start_watcher()
        await r.poll(lambda m: m.get("notify_delivered", 0) >= P, 900, "initial list")
        initial_s = time.monotonic() - t0
        await r.poll(lambda m: m.get("checkpoints_written", 0) >= 1, 120, "first checkpoint")
        # rounds are the fixture's steps 0..rounds-1 (its history is contiguous from step 0)
        kill_rounds = sorted(rng.sample(range(a.rounds), min(a.kills, a.rounds)))
        kills = []
        rounds_t0 = time.monotonic()
        for k in range(a.rounds):
            send = asyncio.ensure_future(r.cmd(f"STEP {k}"))
            if k in kill_rounds:
                # kill while the watcher is in the middle of this round's events
                await asyncio.sleep(rng.uniform(0.2, 0.8) * a.round_seconds_hint)
                m = scrape(r.metrics_port)
                r.kill_watcher()
                kills.append({"round": k, "delivered_by_killed_process": m.get("notify_delivered"),
                              "last_checkpoint_pods": m.get("checkpoint_pods"),
                              "seconds_since_its_last_checkpoint": round(time.time() - m["checkpoint_written_at"], 3)
                              if m.get("checkpoint_written_at") else None})
                r.start_watcher()
            await send
            # the round is complete when every pod's generation k arrived at clusterapi
            deadline = time.monotonic() + 900
            while True:
                await asyncio.sleep(1.0)
                keys = r.sink_keys()
                have = sum(1 for key in keys if key.endswith(f"|{k}") and "|MODIFIED|" in key)
                if have >= P:
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(f"round {k}: {have}/{P} pods delivered")
                print(f"  ... round {k}: {have}/{P}", file=sys.stderr, flush=True)
        rounds_s = time.monotonic() - rounds_t0
        m = scrape(r.metrics_port)
        r.kill_watcher()
        keys = r.sink_keys()
        expected = P * (a.rounds + 1)  # initial ADDED + one MODIFIED per round
        by_type: Dict[str, int] = {}
        for key, n in keys.items():
            parts = key.split("|")
            t = f"{parts[1]}|gen{parts[-1]}"
            by_type[t] = by_type.get(t, 0) + n
        per_gen = {}
        for key, n in keys.items():
            gen = key.rsplit("|", 1)[-1]
            per_gen.setdefault(gen, [0, 0])
            per_gen[gen][0] += 1
            per_gen[gen][1] += n - 1
        stalls = [s["checkpoint_stall_ms"] for s in r.samples if "checkpoint_stall_ms" in s]
        writes = [s["checkpoint_write_ms"] for s in r.samples if "checkpoint_write_ms" in s]
        sizes = [s["checkpoint_bytes"] for s in r.samples if "checkpoint_bytes" in s]
        received = sum(keys.values())
        return {
            "pods": P, "rounds": a.rounds, "kills": kills, "initial_list_seconds": round(initial_s, 2),
            "rounds_seconds": round(rounds_s, 2), "notifications_expected": expected,
            "notifications_unique": len(keys), "notifications_received": received,
            "lost": expected - len(keys), "duplicates": received - len(keys),
            "duplicates_per_generation": {g: v[1] for g, v in sorted(per_gen.items())},
            "received_by_type_generation": dict(sorted(by_type.items())),
            "checkpoint_stall_ms_max": max(stalls) if stalls else None,
            "checkpoint_stall_ms_last": stalls[-1] if stalls else None,
            "checkpoint_write_ms_max": max(writes) if writes else None,
            "checkpoint_bytes": max(sizes) if sizes else None,
            "checkpoints_written_last_process": m.get("checkpoints_written"),
            "owed_resent_last_process": m.get("checkpoint_owed_resent"),
            "watcher_peak_rss_mb": max(r.peaks) if r.peaks else None,
            # the highest sampled RSS, split by the cache / owed-notification / read-buffer gauges
            "memory_at_peak": memory_at_peak(r.samples),
            "memory_after_initial_list": memory_at_peak([x for x in r.samples if x["t"] <= t0 + initial_s]),
            "checkpoint_interval_seconds": a.checkpoint_interval,
        }
    finally:
        await r.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--pods", type=int, default=100000)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--kills", type=int, default=4)
    ap.add_argument("--checkpoint-interval", type=float, default=2.0)
    ap.add_argument("--round-seconds-hint", type=float, default=1.0,
                    help="expected duration of one round (kill point = 20-80%% of it)")
    ap.add_argument("--sink-workers", type=int, default=4)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    res = asyncio.run(amain(a))
    line = json.dumps(res, indent=1)
    print(line)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(line + "\n")
    ok = res["lost"] == 0
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
