"""Log formats."""

import io
import json
import logging
import re

from k8s_watcher_amd.utils.logsetup import SERVICE_LOGGER, setup_logging


def _emit(env, level, msg, lvl=logging.INFO):
    buf = io.StringIO()
    log = setup_logging(env, level, stream=buf)
    log.log(lvl, msg)
    return buf.getvalue()


def test_production_json_fields_and_escaping():
    out = _emit("production", "INFO", 'quote " and \\ and\nnewline')
    doc = json.loads(out.strip())
    assert list(doc) == ["timestamp", "level", "logger", "message", "environment"]
    assert doc["level"] == "INFO"
    assert doc["logger"] == SERVICE_LOGGER == "watcher.pod_watcher"
    assert doc["message"] == 'quote " and \\ and\nnewline'
    assert doc["environment"] == "production"
    assert re.match(r"\d{4}-\d{2}-\d{2} \d{2}:\d{2}:\d{2},\d{3}$", doc["timestamp"])


def test_development_format():
    out = _emit("development", "DEBUG", "Pod event detected: ADDED - default/x")
    assert re.match(r"\[DEVELOPMENT\] \d{4}-\d{2}-\d{2} [\d:,]+ - watcher\.pod_watcher - INFO - "
                    r"Pod event detected: ADDED - default/x\n$", out)


def test_level_filtering_and_reconfigure():
    assert _emit("production", "WARNING", "hidden") == ""
    # second setup in the same process replaces the first (reference basicConfig would not)
    out = _emit("staging", "INFO", "shown")
    assert out.startswith("[STAGING]")
