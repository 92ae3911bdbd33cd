"""Host-tier tests run on the MI355X box (``-m gpu``).

The watcher has no device work; what must hold on the
deployment host is that the in-tree native decoder is the code that runs, the
end-to-end path works there, and the headline bench produces a valid line.
"""

import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, run_bench

pytestmark = pytest.mark.gpu


def test_native_extension_loaded_in_tree():
    from k8s_watcher_amd.ops import native
    mod = native.load()
    assert os.path.realpath(mod.__file__).startswith(os.path.realpath(ROOT))
    assert mod.cpu_features()["avx2"] in (True, False)


def test_smoke_end_to_end():
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.smoke()


def test_bench_line_is_valid():
    line = run_bench(["--steps", "2", "--warmup", "1", "--rounds-per-step", "1", "--apart", "off", "--staging", "off",
                          "--pods-per-step", "1000", "--ref-events", "500", "--latency-seconds", "1", "--latency-seconds-high", "1"])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "vs_baseline"):
        assert key in line
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["steps"] == 2
    assert line["notify_failed"] == 0
    # the watch bytes came through the native reader thread, not asyncio
    assert line["watch_reader_rank0"]["mode"] == "native" and line["watch_reader_rank0"]["reads"] > 0
    assert line["verify"]["exactly_once"]


def test_https_api_server_bench_line_is_valid():
    """An https API server (every real cluster) through the hub's native TLS on the host."""
    line = run_bench(["--steps", "2", "--warmup", "1", "--rounds-per-step", "1", "--apart", "off", "--staging", "off",
                          "--pods-per-step", "1000", "--ref-events", "0", "--latency-seconds", "1",
                          "--latency-rate-high", "0", "--api-tls"])
    assert line["config"]["api_server"] == "https" and line["verify"]["exactly_once"]
    reader = line["watch_reader_rank0"]
    assert reader["mode"] == "native"
    # the hub's own TLS 1.3 record layer carried it, not an SSL_read fallback
    assert reader["tls_taken"] >= 1 and reader["tls_kept"] == 0 and reader["tls_records"] > 0


def test_reader_hub_on_host():
    """The native watch reader's contract (order, EOF, pause, pool backpressure) on the host's CPUs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_reader_hub
    for readers in (1, 3):
        test_reader_hub.test_hub_reads_streams_in_order_and_signals_eof(readers)
    test_reader_hub.test_hub_pause_stops_reading_and_remove_closes()
    test_reader_hub.test_pool_exhaustion_is_backpressure_not_loss()
    test_reader_hub.test_http_stream_adopted_by_hub_end_to_end()
    for depth in (2, 4):
        test_reader_hub.test_read_ahead_is_capped_per_stream(depth)
    test_reader_hub.test_read_ahead_is_capped_in_bytes_over_all_streams()
    # the thread recv()s outside its lock: takes and removals racing it, on the host's cores
    for readers in (1, 3):  # one reader thread, and three sharing the streams
        test_reader_hub.test_take_and_remove_race_the_reader_thread(readers)


def test_hub_framing_and_grouped_dispatch_on_host():
    """Round 3's reader-hub paths on the host's cores: hub-side framing against
    the pipeline's own on random boundaries, grouped dispatch of many bound
    streams, fair-share buffer classes; then a discover-mode bench run with
    1,000 namespace watches, exactly-once, framed by the hub."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_reader_hub
    for seed in (1, 2, 3):
        for buf_bytes in (16 * 1024, 64 * 1024):
            test_reader_hub.test_hub_framing_matches_pipeline_framing_on_random_chunking(seed, buf_bytes)
    test_reader_hub.test_take_dispatch_groups_many_bound_streams_like_serial_feeding()
    test_reader_hub.test_busy_streams_grow_only_to_their_share_of_the_pool()
    line = run_bench(["--steps", "2", "--warmup", "1",
                          "--rounds-per-step", "1", "--apart", "off", "--staging", "off", "--ref-events", "0",
                          "--latency-seconds", "0", "--latency-seconds-high", "0", "--watch-scope", "discover",
                          "--namespaces", "1000"])
    assert line["verify"]["exactly_once"] and line["per_rank"][0]["scopes"] == 1000
    hub = line["watch_reader_rank0"]
    assert hub["mode"] == "native" and hub["framed_reads"] > 0 and hub["hub_dispatch_watches"] == 1000


def test_native_sink_on_host(tmp_path):
    """The bench's native stub clusterapi (_kwcore.SinkServer): pipelined answers, verify keys and
    the SO_REUSEPORT worker processes' dumps, on the host."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_native_sink
    for reserve in (0, 4096):
        test_native_sink.test_native_sink_pipelined_answers_and_keys(reserve)
    test_native_sink.test_native_sink_many_connections()
    test_native_sink.test_sink_process_native_verify_dump(tmp_path)


def test_tls_bench_line_is_valid():
    """production.yaml's https clusterapi through the native TLS notifier core, on the host."""
    line = run_bench(["--steps", "2", "--warmup", "1", "--rounds-per-step", "1", "--apart", "off", "--staging", "off",
                          "--pods-per-step", "1000", "--ref-events", "0", "--latency-seconds", "1", "--latency-rate-high", "0", "--tls"])
    assert line["config"]["clusterapi"] == "https" and line["value"] > 0 and line["notify_failed"] == 0


def test_sharded_ha_and_spool_paths_on_host(tmp_path):
    """Leader election + spool + checkpoint together on the deployment host's CPUs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_ha_soak
    import test_spool
    test_ha_soak.test_graceful_handover_under_churn_keeps_final_state(tmp_path / "ha")
    test_spool.test_shutdown_with_owed_notifications_spools_then_checkpoints(tmp_path / "sp")


def test_round4_paths_on_host():
    """Round 4's paths on the host's cores: the partitioned apply against the
    serial one (every profile), queued reads merged into one pipeline call, a
    bench run at the driver's shape with the zero-copy replay fixture and the
    partitioned apply (exactly-once, both ran), and a WatchList storm through
    the native relist."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_partitioned_apply
    import test_reader_hub
    for env, ov in test_partitioned_apply.PROFILES:
        test_partitioned_apply.test_partitioned_apply_matches_serial(env, ov)
    test_reader_hub.test_take_dispatch_merges_queued_reads_of_one_stream()
    line = run_bench(["--steps", "3", "--warmup", "1",
                          "--rounds-per-step", "4", "--apart", "off", "--staging", "off", "--ref-events", "0",
                          "--latency-seconds", "0", "--latency-seconds-high", "2", "--probe"])
    assert line["verify"]["exactly_once"]
    assert line["loop_probe_rank0"]["partitioned_batches"] > 0
    assert sum(s.get("*", {}).get("bytes", 0) for s in line["fixture_zero_copy"]) > 0
    assert line["latency_high_seconds_rank0"]["rows"] and "rate_dips_rank0" in line
    res = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "relist_storm.py"), "--scope", "cluster",
                          "--namespaces", "16", "--pods", "20000", "--churn", "300", "--initial-sync", "watch_list"],
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    d = json.loads(res.stdout.strip().splitlines()[-1])
    assert d["initial"]["exactly_once"] and d["storm"]["exactly_once"] and d["server"]["lists"] == 0


def test_bench_headline_driver_shape_on_host(tmp_path):
    """The driver's command shape on the host (every phase on, --pods-per-step
    shortened): the last stdout line is the < 4,096-byte headline, stderr is one
    line, every 1k ev/s second with a > 1 ms notification names a cause, and no
    process of the bench outlives it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_bench_headline as tbh
    tbh.check_headline(*tbh.run_driver_shape(tmp_path, extra=("--pods-per-step", "2000")))
