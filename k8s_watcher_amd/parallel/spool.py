"""Durable spool for notifications clusterapi could not take (``clusterapi.spool``).

Reference: ``ClusterApiClient.update_pod_status`` logs a failure and returns
``False`` (``/root/reference/watcher/clusterapi_client.py:38-53``) — the event
is gone. The notifier pools here retry (``clusterapi.retry``), but a
clusterapi outage longer than the retry budget, or a shutdown with requests
still queued, would still lose state changes. With ``clusterapi.spool.path``
set, such notifications are appended to an on-disk log instead and replayed
in order once clusterapi answers its health check again, across restarts.

Which notifications are spooled: those whose last attempt failed for a
*transient* reason (transport error, timeout, 408/425/429/5xx) and those still
outstanding when the pool closes. A non-retryable answer (e.g. 400) is a
verdict on the payload and is dropped as before. A notification superseded by
a newer one for the same pod is never spooled.

Ordering: a spooled record is replayed only if no *live* notification for the
same pod was submitted after it was spooled (the pools track that per uid);
otherwise it is *stale* and skipped, so a replay never overwrites newer state
at clusterapi. Records from an earlier process are older than anything this
process submits. Delivery stays at-least-once: a crash between a replayed
delivery and the cursor update replays it again.

On-disk format (directory ``path``): segment files ``seg-<n>.spool`` of
records ``<u32 header_len><u32 body_len><header JSON><body>``, where the
header is ``[uid, event_type, namespace, name, seq, epoch]``; ``cursor.json``
holds the position of the first record not yet replayed. A torn record at the
end of the last segment (crash mid-append) is truncated on open.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import struct
import uuid
from collections import Counter
from typing import Dict, Iterable, List, NamedTuple, Optional, Tuple

from ..metrics import Metrics
from ..utils.logsetup import NOTIFIER_LOGGER

_HDR = struct.Struct("<II")
_MAX_HEADER = 1 << 20


class SpoolRecord(NamedTuple):
    uid: str
    etype: str
    ns: str
    name: str
    body: bytes
    seq: int  # notifier seq when spooled in this process; 0 = spooled by an earlier process
    size: int = 0  # bytes on disk


Pos = Tuple[int, int]  # (segment index, byte offset)


class Spool:
    def __init__(self, path: str, max_bytes: int = 1 << 30, segment_bytes: int = 64 << 20,
                 fsync: bool = False, metrics: Optional[Metrics] = None) -> None:
        self.path = path
        self.max_bytes = max_bytes
        self.segment_bytes = segment_bytes
        self.fsync = fsync
        self.metrics = metrics or Metrics()
        self.log = logging.getLogger(NOTIFIER_LOGGER)
        self.epoch = uuid.uuid4().hex[:12]
        os.makedirs(path, exist_ok=True)
        self.uid_counts: Counter = Counter()
        self.count = 0
        self.bytes = 0
        self.cursor: Pos = self._load_cursor()
        segs = self._segments()
        for n in segs:
            if n < self.cursor[0]:
                os.unlink(self._seg_path(n))  # fully replayed before a crash
        segs = [n for n in segs if n >= self.cursor[0]]
        if not segs:
            segs = [self.cursor[0]]
            open(self._seg_path(segs[0]), "ab").close()
        self._scan(segs)
        self.tail = segs[-1]
        self._fh = open(self._seg_path(self.tail), "ab")

    # ------------------------------------------------------------------ files
    def _seg_path(self, n: int) -> str:
        return os.path.join(self.path, f"seg-{n:08d}.spool")

    def _segments(self) -> List[int]:
        out = []
        for f in os.listdir(self.path):
            if f.startswith("seg-") and f.endswith(".spool"):
                try:
                    out.append(int(f[4:-6]))
                except ValueError:
                    pass
        return sorted(out)

    def _load_cursor(self) -> Pos:
        try:
            with open(os.path.join(self.path, "cursor.json")) as fh:
                d = json.load(fh)
            return int(d["segment"]), int(d["offset"])
        except (OSError, ValueError, KeyError, TypeError):
            segs = self._segments()
            return (segs[0] if segs else 0), 0

    def _save_cursor(self) -> None:
        tmp = os.path.join(self.path, "cursor.json.tmp")
        with open(tmp, "w") as fh:
            json.dump({"segment": self.cursor[0], "offset": self.cursor[1]}, fh)
            if self.fsync:
                fh.flush()
                os.fsync(fh.fileno())
        os.replace(tmp, os.path.join(self.path, "cursor.json"))

    def _scan(self, segs: List[int]) -> None:
        """Count pending records from the cursor on; truncate a torn tail."""
        for n in segs:
            start = self.cursor[1] if n == self.cursor[0] else 0
            good = start
            for rec, end in self._iter_segment(n, start):
                self.uid_counts[rec.uid] += 1
                self.count += 1
                good = end
            size = os.path.getsize(self._seg_path(n))
            self.bytes += good - start
            if good < size and n == segs[-1]:
                self.log.warning(f"Spool segment {self._seg_path(n)}: dropping a torn record at {good}")
                with open(self._seg_path(n), "r+b") as fh:
                    fh.truncate(good)

    def _iter_segment(self, n: int, offset: int) -> Iterable[Tuple[SpoolRecord, int]]:
        try:
            fh = open(self._seg_path(n), "rb")
        except FileNotFoundError:
            return
        with fh:
            fh.seek(offset)
            pos = offset
            while True:
                hdr = fh.read(_HDR.size)
                if len(hdr) < _HDR.size:
                    return
                hlen, blen = _HDR.unpack(hdr)
                if hlen > _MAX_HEADER:
                    return
                head = fh.read(hlen)
                body = fh.read(blen)
                if len(head) < hlen or len(body) < blen:
                    return
                try:
                    uid, etype, ns, name, seq, epoch = json.loads(head)
                except (ValueError, TypeError):
                    return
                size = _HDR.size + hlen + blen
                pos += size
                yield SpoolRecord(uid, etype, ns, name, body, int(seq) if epoch == self.epoch else 0, size), pos

    # ------------------------------------------------------------------ API
    def __len__(self) -> int:
        return self.count

    def append(self, records: Iterable[Tuple[str, str, str, str, bytes, int]]) -> List[str]:
        """Append ``(uid, etype, ns, name, body, seq)`` records; returns uids new to the spool.

        Records that would grow the spool past ``max_bytes`` are dropped
        (``spool_dropped``) with an error log, as the reference drops them.
        """
        new_uids = []
        wrote = 0
        for uid, etype, ns, name, body, seq in records:
            head = json.dumps([uid, etype, ns, name, seq, self.epoch], separators=(",", ":")).encode()
            size = _HDR.size + len(head) + len(body)
            if self.bytes + size > self.max_bytes:
                self.metrics.c["spool_dropped"] += 1
                self.log.error(f"Spool full ({self.bytes} bytes): dropping notification about "
                               f"{etype} event for {ns}/{name}")
                continue
            if self._fh.tell() >= self.segment_bytes:
                self._rotate()
            self._fh.write(_HDR.pack(len(head), len(body)))
            self._fh.write(head)
            self._fh.write(body)
            self.bytes += size
            self.count += 1
            wrote += 1
            if self.uid_counts[uid] == 0:
                new_uids.append(uid)
            self.uid_counts[uid] += 1
        if wrote:
            self._fh.flush()
            if self.fsync:
                os.fsync(self._fh.fileno())
        return new_uids

    def _rotate(self) -> None:
        self._fh.flush()
        if self.fsync:
            os.fsync(self._fh.fileno())
        self._fh.close()
        self.tail += 1
        self._fh = open(self._seg_path(self.tail), "ab")

    def read_batch(self, max_records: int) -> Tuple[List[SpoolRecord], Pos]:
        """Up to ``max_records`` records from the cursor, and the position after them."""
        out: List[SpoolRecord] = []
        seg, off = self.cursor
        pos = self.cursor
        while seg <= self.tail:
            for rec, end in self._iter_segment(seg, off):
                out.append(rec)
                pos = (seg, end)
                if len(out) >= max_records:
                    return out, pos
            if seg == self.tail:
                break
            seg, off = seg + 1, 0  # this segment is exhausted
            pos = (seg, 0)
        return out, pos

    def commit(self, pos: Pos, records: List[SpoolRecord]) -> List[str]:
        """Mark ``records`` (a :meth:`read_batch` result) done; returns uids no longer in the spool."""
        gone = []
        for rec in records:
            self.uid_counts[rec.uid] -= 1
            if self.uid_counts[rec.uid] <= 0:
                del self.uid_counts[rec.uid]
                gone.append(rec.uid)
            self.bytes -= rec.size
        self.count -= len(records)
        old_seg = self.cursor[0]
        if self.count == 0:
            # empty: start a fresh segment and drop every old one
            self._fh.close()
            self.tail += 1
            self._fh = open(self._seg_path(self.tail), "ab")
            self.cursor = (self.tail, 0)
            self.bytes = 0
        else:
            self.cursor = pos
        self._save_cursor()
        for n in range(old_seg, self.cursor[0]):
            try:
                os.unlink(self._seg_path(n))
            except FileNotFoundError:
                pass
        return gone

    def close(self) -> None:
        try:
            self._fh.flush()
            if self.fsync:
                os.fsync(self._fh.fileno())
        finally:
            self._fh.close()


class SpoolReplayer:
    """Replays the spool through a notifier pool once clusterapi is healthy again.

    The pool must provide ``health_check()``, ``replay(records) -> int``,
    ``replay_pending()``, ``spool_unwatch(uid)`` and ``flush()`` (both
    :class:`~.notifier.NotifierPool` and :class:`~.native_notifier.NativeNotifierPool` do).
    """

    def __init__(self, spool: Spool, pool, metrics: Metrics, interval: float = 5.0, batch: int = 1000) -> None:
        self.spool = spool
        self.pool = pool
        self.metrics = metrics
        self.interval = interval
        self.batch = batch
        self.log = logging.getLogger(NOTIFIER_LOGGER)

    async def run(self) -> None:
        while True:
            if len(self.spool) and await self.pool.health_check():
                await self.replay_once()
            await asyncio.sleep(self.interval)

    async def replay_once(self) -> bool:
        """Replay until the spool is empty (True) or a replayed notification is spooled again (False)."""
        if len(self.spool):
            self.log.warning(f"Replaying {len(self.spool)} spooled notifications")
        while len(self.spool):
            recs, pos = self.spool.read_batch(self.batch)
            if not recs:
                break
            before = self.metrics.c["notify_spooled"]
            sent = self.pool.replay(recs)
            self.metrics.c["spool_replayed"] += sent
            self.metrics.c["spool_stale_skipped"] += len(recs) - sent
            self.pool.flush()
            while self.pool.replay_pending() > 0:
                await asyncio.sleep(0.005)
            self.pool.flush()  # collect re-spooled records before committing
            for uid in self.spool.commit(pos, recs):
                self.pool.spool_unwatch(uid)
            if self.metrics.c["notify_spooled"] > before:
                return False  # clusterapi failing again: the rest waits for the next health check
        return True


def spool_record_tuple(uid, etype, ns, name, body: bytes, seq: int) -> Tuple[str, str, str, str, bytes, int]:
    return (uid, etype, ns if ns is not None else "None", name if name is not None else "None", body, seq)


__all__ = ["Spool", "SpoolRecord", "SpoolReplayer", "spool_record_tuple"]
