"""Batched per-event log lines with output identical to :mod:`logging`.

In the development/staging profiles the reference writes one INFO line per
pod event (``Pod event detected: ...``, ``pod_watcher.py:223``), and the
notifier one per delivery. Through :mod:`logging` each line costs a
``LogRecord``, a ``findCaller`` stack walk, ``strftime``, a lock round-trip
and a ``flush``. That is ~20 µs of pure overhead per line, more than the
rest of the event's processing.

:class:`EventLog` produces the *same bytes* as the installed handler would
(see ``tests/test_fastlog.py``) and writes a whole batch with one
``write`` + ``flush``:

* it is used only when the output path is exactly what
  :func:`~.logsetup.setup_logging` installed (one tagged handler on the root
  logger, no filters, the logger propagating to root), otherwise every call
  goes through ``logger.log`` unchanged;
* the timestamp prefix is formatted once per millisecond.

When that handler writes to a real file descriptor in UTF-8 and the native
extension is built, :attr:`EventLog.native_sink` is a ``_kwcore.LogSink``
(``ops/csrc/logsink.inc``) for the same fd and format: the native pipeline
and notifier core then format their per-event lines in C++ and never hand
them to Python at all; :meth:`EventLog.flush` writes that batch too.
"""

from __future__ import annotations

import json
import logging
import time
from typing import List, Optional

from .logsetup import _HANDLER_TAG, JsonLineFormatter


class EventLog:
    def __init__(self, logger: logging.Logger, native: bool = True) -> None:
        self.logger = logger
        self._lines: List[str] = []
        self._handler: Optional[logging.Handler] = None
        self._prefix_ms = -1
        self._prefix = {}
        self._native = native
        self.native_sink = None
        self.refresh()

    def refresh(self) -> None:
        """Re-check whether the fast path applies (call after logging is reconfigured)."""
        self._handler = None
        self.native_sink = None
        lg = self.logger
        root = logging.getLogger()
        if lg.handlers or lg.filters or not lg.propagate or root.filters or len(root.handlers) != 1:
            return
        cur = lg.parent
        while cur is not None and cur is not root:
            if cur.handlers or cur.filters or not cur.propagate:
                return
            cur = cur.parent
        h = root.handlers[0]
        if not getattr(h, _HANDLER_TAG, False) or h.filters or not isinstance(h, logging.StreamHandler):
            return
        fmt = h.formatter
        if isinstance(fmt, JsonLineFormatter):
            self._json_env = fmt.environment
        elif fmt is not None and fmt._fmt and fmt._fmt.endswith("%(asctime)s - %(name)s - %(levelname)s - %(message)s") \
                and fmt.datefmt is None and type(fmt) is logging.Formatter:
            self._json_env = None
            self._text_head = fmt._fmt[: -len("%(asctime)s - %(name)s - %(levelname)s - %(message)s")]
        else:
            return
        self._handler = h
        self._prefix_ms = -1
        if self._native:
            self.native_sink = self._make_native_sink(h)

    def _make_native_sink(self, h: logging.StreamHandler):
        stream = h.stream
        try:
            fd = stream.fileno()
        except (AttributeError, OSError, ValueError):
            return None  # StringIO and friends: the Python path
        enc = (getattr(stream, "encoding", None) or "").lower().replace("-", "").replace("_", "")
        if enc != "utf8" or getattr(h, "terminator", "\n") != "\n":
            return None
        try:
            from ..ops.native import NativeUnavailable, load
            mod = load()
        except NativeUnavailable:
            return None
        json_env = self._json_env
        return mod.LogSink(fd, json_env is not None, "" if json_env is not None else self._text_head,
                           self.logger.name, json_env if json_env is not None else "")
    def enabled(self, level: int) -> bool:
        return self.logger.isEnabledFor(level)

    def _stamp(self) -> str:
        now = time.time()
        ms = int(now * 1000)
        if ms != self._prefix_ms:
            self._prefix_ms = ms
            asctime = time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(now))
            self._asctime = "%s,%03d" % (asctime, int((now - int(now)) * 1000))
            self._prefix = {}
        return self._asctime

    def log(self, level: int, msg: str) -> None:
        """Queue one line (caller checked :meth:`enabled`); :meth:`flush` writes them."""
        if self._handler is None:
            self.logger.log(level, msg)
            return
        asctime = self._stamp()
        lvl = logging.getLevelName(level)
        if self._json_env is not None:
            self._lines.append(
                '{"timestamp":"%s","level":"%s","logger":"%s","message":%s,"environment":%s}\n'
                % (asctime, lvl, self.logger.name, json.dumps(msg, ensure_ascii=False),
                   json.dumps(self._json_env, ensure_ascii=False)))
        else:
            head = self._prefix.get(level)
            if head is None:
                head = f"{self._text_head}{asctime} - {self.logger.name} - {lvl} - "
                self._prefix[level] = head
            self._lines.append(head + msg + "\n")

    def flush(self) -> None:
        lines = self._lines
        sink = self.native_sink
        if sink is not None and sink.pending():
            if lines:
                self._write(lines)
            h = self._handler
            if h is not None:
                h.flush()  # nothing of Python's may sit in a buffer ahead of the native lines
            sink.flush()
            return
        if not lines:
            return
        self._write(lines)

    def _write(self, lines: List[str]) -> None:
        self._lines = []
        h = self._handler
        if h is None:
            return
        h.acquire()
        try:
            h.stream.write("".join(lines))
            h.flush()
        except Exception:  # noqa: BLE001 - never let logging break the pipeline
            pass
        finally:
            h.release()
