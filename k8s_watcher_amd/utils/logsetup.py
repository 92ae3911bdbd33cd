"""Per-environment log formats (message catalogue §2.4).

Reference (``/root/reference/watcher/pod_watcher.py:77-94``):

* production: one pseudo-JSON line per record with the fields
  ``timestamp, level, logger, message, environment``;
* every other environment: ``[<ENV>] <asctime> - <logger> - <LEVEL> - <message>``;
* the level comes from ``watcher.log_level``.

Differences: the production line is real JSON (the message is escaped, so a
quote in a message no longer breaks the line), and setup replaces only the
handler *this module* installed instead of relying on ``logging.basicConfig``'s
first-call-wins behaviour, so re-configuring in one process works.
"""

from __future__ import annotations

import json
import logging
import sys
from typing import IO, Optional

# Logger names kept from the reference so every log line reads the same.
SERVICE_LOGGER = "watcher.pod_watcher"
NOTIFIER_LOGGER = "watcher.clusterapi_client"

_HANDLER_TAG = "_k8s_watcher_amd_handler"


class JsonLineFormatter(logging.Formatter):
    """Production format: escaped JSON, same field names/order as the reference."""

    def __init__(self, environment: str) -> None:
        super().__init__()
        self.environment = environment

    def format(self, record: logging.LogRecord) -> str:
        msg = record.getMessage()
        if record.exc_info:
            msg = msg + "\n" + self.formatException(record.exc_info)
        doc = {
            "timestamp": self.formatTime(record),
            "level": record.levelname,
            "logger": record.name,
            "message": msg,
            "environment": self.environment,
        }
        return json.dumps(doc, ensure_ascii=False, separators=(",", ":"))


def make_formatter(environment: str) -> logging.Formatter:
    if environment == "production":
        return JsonLineFormatter(environment)
    return logging.Formatter(f"[{environment.upper()}] %(asctime)s - %(name)s - %(levelname)s - %(message)s")


def setup_logging(environment: str, level: str = "INFO", stream: Optional[IO[str]] = None,
                  log_file: Optional[str] = None) -> logging.Logger:
    """Install the environment's handler on the root logger and return the service logger."""
    root = logging.getLogger()
    for h in list(root.handlers):
        if getattr(h, _HANDLER_TAG, False):
            root.removeHandler(h)
            h.close()
    if log_file:
        handler: logging.Handler = logging.FileHandler(log_file, encoding="utf-8")
    else:
        handler = logging.StreamHandler(stream or sys.stderr)
    setattr(handler, _HANDLER_TAG, True)
    handler.setFormatter(make_formatter(environment))
    root.addHandler(handler)
    lvl = logging.getLevelName(str(level).upper())
    if not isinstance(lvl, int):
        raise ValueError(f"unknown log level {level!r}")
    root.setLevel(lvl)
    return logging.getLogger(SERVICE_LOGGER)
