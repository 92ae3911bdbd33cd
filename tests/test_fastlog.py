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
