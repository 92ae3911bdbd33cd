"""The batched event logger writes exactly what :mod:`logging` would."""

import io
import logging
import time

import pytest

from k8s_watcher_amd.utils.fastlog import EventLog
from k8s_watcher_amd.utils.logsetup import SERVICE_LOGGER, setup_logging

MSGS = ["Pod event detected: ADDED - default/a", 'quote " back\\slash é\nnewline', "plain"]


@pytest.fixture(autouse=True)
def _restore_root_handlers():
    root = logging.getLogger()
    saved = list(root.handlers)
    yield
    root.handlers[:] = saved


def only_ours():
    """pytest's log capture adds root handlers during each test; production has only ours."""
    root = logging.getLogger()
    root.handlers[:] = [h for h in root.handlers if getattr(h, "_k8s_watcher_amd_handler", False)]


@pytest.mark.parametrize("env", ["development", "staging", "production"])
def test_identical_output(env, monkeypatch):
    fixed = 1_760_000_000.1239
    monkeypatch.setattr(time, "time", lambda: fixed)
    a, b = io.StringIO(), io.StringIO()
    log = setup_logging(env, "DEBUG", stream=a)
    only_ours()
    for m in MSGS:
        log.info(m)
    log.debug("dbg")
    setup_logging(env, "DEBUG", stream=b)
    only_ours()
    el = EventLog(logging.getLogger(SERVICE_LOGGER))
    assert el._handler is not None  # fast path engaged
    for m in MSGS:
        el.log(logging.INFO, m)
    el.log(logging.DEBUG, "dbg")
    el.flush()
    assert a.getvalue() == b.getvalue()


def test_falls_back_with_foreign_handler():
    buf = io.StringIO()
    setup_logging("staging", "INFO", stream=io.StringIO())
    only_ours()
    extra = logging.StreamHandler(buf)
    logging.getLogger(SERVICE_LOGGER).addHandler(extra)
    try:
        el = EventLog(logging.getLogger(SERVICE_LOGGER))
        assert el._handler is None
        el.log(logging.INFO, "via logging")
        el.flush()
        assert "via logging" in buf.getvalue()
    finally:
        logging.getLogger(SERVICE_LOGGER).removeHandler(extra)


MSGS_NATIVE = MSGS + ["ctl \x01\x1f tab\t cr\r ff\x0c bs\x08 del\x7f ✓ 中文", ""]


@pytest.mark.parametrize("env", ["development", "staging", "production"])
def test_native_sink_identical_output(env, tmp_path, monkeypatch):
    """_kwcore.LogSink (ops/csrc/logsink.inc) writes byte for byte what the
    installed logging handler writes, text and production JSON, control
    characters and non-ASCII included."""
    fixed = 1_760_000_000.125
    monkeypatch.setattr(time, "time", lambda: fixed)
    ref, nat = tmp_path / "ref.log", tmp_path / "nat.log"
    log = setup_logging(env, "DEBUG", log_file=str(ref))
    only_ours()
    for m in MSGS_NATIVE:
        log.info(m)
    log.debug("dbg")
    setup_logging(env, "DEBUG", log_file=str(nat))
    only_ours()
    el = EventLog(logging.getLogger(SERVICE_LOGGER))
    sink = el.native_sink
    assert sink is not None  # a real fd in UTF-8: the native path
    sink.set_clock(int(fixed), int(round((fixed - int(fixed)) * 1e9)))
    for m in MSGS_NATIVE:
        sink.log(logging.INFO, m)
    sink.log(logging.DEBUG, "dbg")
    el.flush()
    assert sink.pending() == 0 and sink.stats()["lines"] == len(MSGS_NATIVE) + 1
    logging.getLogger().handlers[0].flush()
    assert nat.read_bytes() == ref.read_bytes()


def test_native_sink_only_for_real_utf8_fds(tmp_path):
    setup_logging("staging", "INFO", stream=io.StringIO())
    only_ours()
    assert EventLog(logging.getLogger(SERVICE_LOGGER)).native_sink is None  # no fd
    fh = open(tmp_path / "latin.log", "w", encoding="latin-1")
    try:
        setup_logging("staging", "INFO", stream=fh)
        only_ours()
        assert EventLog(logging.getLogger(SERVICE_LOGGER)).native_sink is None  # not UTF-8
    finally:
        fh.close()
    assert EventLog(logging.getLogger(SERVICE_LOGGER), native=False).native_sink is None


@pytest.mark.parametrize("env", ["staging", "production"])
def test_native_pipeline_lines_match_python_pipeline(env, tmp_path):
    """The fused pipeline + notifier core writing through the LogSink produce
    the same per-event lines (same order) as the Python pipeline's EventLog."""
    import asyncio
    import re

    from conftest import run
    from k8s_watcher_amd.engine.service import WatcherService
    from k8s_watcher_amd.kube.kubeconfig import KubeEndpoint
    from k8s_watcher_amd.metrics import Metrics
    from k8s_watcher_amd.testing.fake_apiserver import FakeApiServer
    from k8s_watcher_amd.testing.podgen import PodFactory
    from k8s_watcher_amd.testing.stub_sink import StubSink
    from k8s_watcher_amd.utils.config import load_settings

    def lines_of(engine):
        path = tmp_path / f"{engine}.log"

        async def body():
            setup_logging(env, "INFO", log_file=str(path))
            only_ours()
            srv = FakeApiServer()
            await srv.start()
            sink = StubSink()
            await sink.start()
            s = load_settings(env, overrides={
                "clusterapi": {"base_url": sink.url, "health_check_on_start": False,
                               "pool": {"connections": 1}},
                "watcher": {"engine": engine, "log_level": "INFO", "decode_threads": 0,
                            "alerts": {"critical_events_only": False}}})
            svc = WatcherService(s, endpoint=KubeEndpoint(server=srv.url), metrics=Metrics())
            await svc.start()
            if engine == "native":
                assert svc.event_log.native_sink is not None
            f = PodFactory(seed=3, namespaces=["default", "kube-system", "odd \"ns\""])
            for _ in range(6):
                for et, obj in f.lifecycle():
                    srv.apply(et, obj)
            await sink.state.wait_for(30 if env == "staging" else 12, timeout=10)
            await svc.notifier.drain(5)
            svc.stop()
            await svc.shutdown()
            await sink.stop()
            await srv.stop()
        run(body())
        logging.getLogger().handlers[0].flush()
        out = []
        for ln in path.read_text(encoding="utf-8").splitlines():
            if "Pod event detected" in ln or "Successfully notified" in ln:
                out.append(re.sub(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d,\d{3}", "TS", ln))
        return out

    py, nat = lines_of("python"), lines_of("native")
    assert nat and sorted(nat) == sorted(py)
    assert [x for x in nat if "Pod event" in x] == [x for x in py if "Pod event" in x]
