"""Lease-based leader election for running several watcher replicas (HA).

The reference is a single process (``/root/reference/main.py:23-24``,
SURVEY §2.2 "Concurrency: none") with no story for a second replica: two
copies of it would both notify clusterapi about every event. Here replicas
compete for a ``coordination.k8s.io/v1`` Lease and only the holder watches and
notifies; the others wait as candidates and take over when the holder stops
renewing (crash, network partition) or releases the lease on shutdown.

Semantics follow the protocol every Kubernetes controller uses, so the lease
interoperates with ``kubectl get lease`` and other tooling:

* the record is the Lease ``spec`` (``holderIdentity``,
  ``leaseDurationSeconds``, ``acquireTime``, ``renewTime``,
  ``leaseTransitions``); updates are compare-and-swap on
  ``metadata.resourceVersion`` (HTTP 409 = someone else wrote first);
* expiry is judged on the *local* clock from the moment this replica last saw
  the record change — never from the timestamps inside it — so clock skew
  between nodes cannot cause two leaders;
* a leader that cannot renew within ``renew_deadline_seconds`` steps down
  (strictly before its lease can expire for the others);
* an empty ``holderIdentity`` means "released": candidates take it at once.

:class:`LeaderElectedService` wraps :class:`~.service.WatcherService`: one
fresh service per leadership term, torn down (without draining, since a new
leader may already be notifying) when the term ends.
"""

from __future__ import annotations

import asyncio
import datetime as _dt
import logging
import os
import random
import socket
import time
import uuid
from dataclasses import dataclass
from typing import Callable, Dict, Optional

from ..kube.api import ApiError, KubeApi
from ..metrics import Metrics
from ..net.http import HttpError
from ..utils.config import LeaderElectionSettings
from ..utils.logsetup import SERVICE_LOGGER

SA_NAMESPACE_FILE = "/var/run/secrets/kubernetes.io/serviceaccount/namespace"


def micro_time(ts: Optional[float] = None) -> str:
    """Kubernetes ``MicroTime``: RFC 3339 with microseconds, UTC."""
    t = _dt.datetime.fromtimestamp(time.time() if ts is None else ts, tz=_dt.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def default_identity() -> str:
    """``$POD_NAME`` (downward API) or ``<hostname>_<random>`` — unique per process."""
    pod = os.environ.get("POD_NAME")
    if pod:
        return pod
    return f"{socket.gethostname()}_{uuid.uuid4().hex[:8]}"


def default_lease_namespace(sa_file: str = SA_NAMESPACE_FILE) -> str:
    """The pod's own namespace when in-cluster, else ``default``."""
    ns = os.environ.get("POD_NAMESPACE")
    if ns:
        return ns
    try:
        with open(sa_file) as fh:
            return fh.read().strip() or "default"
    except OSError:
        return "default"


@dataclass
class LeaderRecord:
    holder: str = ""
    lease_duration: int = 15
    acquire_time: Optional[str] = None
    renew_time: Optional[str] = None
    transitions: int = 0

    @classmethod
    def from_lease(cls, lease: Dict) -> "LeaderRecord":
        spec = lease.get("spec") or {}
        return cls(holder=spec.get("holderIdentity") or "",
                   lease_duration=int(spec.get("leaseDurationSeconds") or 0),
                   acquire_time=spec.get("acquireTime"), renew_time=spec.get("renewTime"),
                   transitions=int(spec.get("leaseTransitions") or 0))

    def spec(self) -> Dict:
        out: Dict = {"holderIdentity": self.holder, "leaseDurationSeconds": self.lease_duration,
                     "leaseTransitions": self.transitions}
        if self.acquire_time:
            out["acquireTime"] = self.acquire_time
        if self.renew_time:
            out["renewTime"] = self.renew_time
        return out

    def key(self) -> tuple:
        return (self.holder, self.lease_duration, self.acquire_time, self.renew_time, self.transitions)


class LeaderElector:
    """One candidate. Drive it with :meth:`run` (or step it with :meth:`try_acquire_or_renew`)."""

    def __init__(self, api: KubeApi, settings: LeaderElectionSettings, metrics: Optional[Metrics] = None,
                 clock: Callable[[], float] = time.monotonic, rng: Optional[random.Random] = None) -> None:
        if settings.renew_deadline_seconds >= settings.lease_duration_seconds:
            raise ValueError("leader_election: renew_deadline_seconds must be < lease_duration_seconds")
        if settings.retry_period_seconds >= settings.renew_deadline_seconds:
            raise ValueError("leader_election: retry_period_seconds must be < renew_deadline_seconds")
        self.api = api
        self.s = settings
        self.identity = settings.identity or default_identity()
        self.namespace = settings.lease_namespace or default_lease_namespace()
        self.name = settings.lease_name
        self.metrics = metrics or Metrics()
        self.clock = clock
        self.rng = rng or random.Random()
        self.log = logging.getLogger(SERVICE_LOGGER)
        self.observed: Optional[LeaderRecord] = None
        self.observed_rv: Optional[str] = None
        self.observed_at = 0.0
        self.last_renew = 0.0  # local time of our last successful acquire/renew
        self._leader = False
        self.became_leader = asyncio.Event()
        self.lost = asyncio.Event()
        self._stop = asyncio.Event()
        self.metrics.gauges["leader"] = lambda: 1.0 if self._leader else 0.0

    # ------------------------------------------------------------------ state
    @property
    def is_leader(self) -> bool:
        return self._leader

    @property
    def holder(self) -> Optional[str]:
        return self.observed.holder if self.observed else None

    def _observe(self, rec: LeaderRecord, rv: Optional[str]) -> None:
        if self.observed is None or self.observed.key() != rec.key():
            self.observed_at = self.clock()
        self.observed = rec
        self.observed_rv = rv

    def _set_leader(self, leader: bool) -> None:
        if leader == self._leader:
            return
        self._leader = leader
        if leader:
            self.metrics.c["leader_acquired"] += 1
            self.log.info(f"Acquired leadership of lease {self.namespace}/{self.name} as {self.identity}")
            self.lost.clear()
            self.became_leader.set()
        else:
            self.metrics.c["leader_lost"] += 1
            self.log.warning(f"Lost leadership of lease {self.namespace}/{self.name}")
            self.became_leader.clear()
            self.lost.set()

    # ------------------------------------------------------------------ one round
    async def try_acquire_or_renew(self) -> bool:
        """One compare-and-swap round; True if this candidate holds the lease afterwards.

        The whole round (GET, then PUT or POST, with any keep-alive retry)
        runs under ONE deadline, as client-go's ``renew`` does: for a leader,
        what is left of ``renew_deadline_seconds`` since its last successful
        renew; for a candidate, the full deadline. Per-request timeouts alone
        would let a round outlast the lease (each request gets the deadline
        for connect and again for the response), and a candidate takes the
        lease ``lease_duration_seconds`` after the last renew — two leaders.
        The caller (:meth:`run`) steps down when a leader's round fails, so
        a leader stops acting strictly before its lease can expire.
        """
        budget = self.s.renew_deadline_seconds
        if self._leader:
            budget = min(budget, self.last_renew + self.s.renew_deadline_seconds - self.clock())
            if budget <= 0:
                return False
        deadline = time.monotonic() + budget
        try:
            return await asyncio.wait_for(self._round(deadline), budget)
        except asyncio.TimeoutError:
            self.metrics.c["lease_update_errors"] += 1
            self.log.warning(f"Lease {self.namespace}/{self.name} round exceeded its {budget:.2f}s deadline")
            return False

    async def _round(self, deadline: float) -> bool:
        now_wall = time.time()

        def left() -> float:
            return max(0.001, deadline - time.monotonic())

        try:
            lease = await self.api.get_lease(self.namespace, self.name, timeout=left())
            if lease is None:
                rec = LeaderRecord(holder=self.identity, lease_duration=int(round(self.s.lease_duration_seconds)),
                                   acquire_time=micro_time(now_wall), renew_time=micro_time(now_wall))
                body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                        "metadata": {"name": self.name, "namespace": self.namespace}, "spec": rec.spec()}
                created = await self.api.create_lease(self.namespace, body, timeout=left())
                self._observe(rec, (created.get("metadata") or {}).get("resourceVersion"))
                self.last_renew = self.clock()
                return True
            md = lease.get("metadata") or {}
            old = LeaderRecord.from_lease(lease)
            self._observe(old, md.get("resourceVersion"))
            ours = old.holder == self.identity
            if (old.holder and not ours
                    and self.observed_at + max(old.lease_duration, 1) > self.clock()):
                return False  # held by someone else and not expired
            rec = LeaderRecord(holder=self.identity, lease_duration=int(round(self.s.lease_duration_seconds)),
                               renew_time=micro_time(now_wall))
            if ours:
                rec.acquire_time = old.acquire_time
                rec.transitions = old.transitions
            else:
                rec.acquire_time = micro_time(now_wall)
                rec.transitions = old.transitions + 1
            lease = dict(lease)
            lease["metadata"] = dict(md)
            lease["spec"] = rec.spec()
            updated = await self.api.replace_lease(self.namespace, self.name, lease, timeout=left())
            self._observe(rec, (updated.get("metadata") or {}).get("resourceVersion"))
            self.last_renew = self.clock()
            return True
        except ApiError as exc:
            if exc.status == 401 and await self.api.endpoint.refresh_credentials():
                # a standby runs no reflector, so nothing else would refresh its
                # credentials: without this a rotated token locks it out for good
                self.metrics.c["auth_refreshes"] += 1
                self.log.warning("API server answered 401 to a lease request; refreshing credentials")
            if exc.status not in (404, 409):
                self.log.warning(f"Lease {self.namespace}/{self.name} update failed: {exc}")
            self.metrics.c["lease_update_conflicts" if exc.status == 409 else "lease_update_errors"] += 1
            return False
        except (HttpError, OSError, ValueError) as exc:
            self.metrics.c["lease_update_errors"] += 1
            self.log.warning(f"Lease {self.namespace}/{self.name} update failed: {exc}")
            return False

    async def release(self) -> bool:
        """Give the lease up now (empty holder, 1 s duration) so a candidate takes over immediately."""
        if not self._leader or self.observed is None:
            return False
        rec = LeaderRecord(holder="", lease_duration=1, acquire_time=micro_time(), renew_time=micro_time(),
                           transitions=self.observed.transitions)
        body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                "metadata": {"name": self.name, "namespace": self.namespace,
                             "resourceVersion": self.observed_rv}, "spec": rec.spec()}
        self._set_leader(False)
        try:
            await self.api.replace_lease(self.namespace, self.name, body, timeout=self.s.renew_deadline_seconds)
            self.log.info(f"Released lease {self.namespace}/{self.name}")
            return True
        except (ApiError, HttpError, OSError, asyncio.TimeoutError) as exc:
            self.log.warning(f"Could not release lease {self.namespace}/{self.name}: {exc}")
            return False

    # ------------------------------------------------------------------ loop
    def stop(self) -> None:
        self._stop.set()

    async def _sleep(self, seconds: float) -> bool:
        """Sleep unless stopped; True if stopped."""
        waiter = asyncio.ensure_future(self._stop.wait())
        try:
            await asyncio.wait([waiter], timeout=max(0.0, seconds))
        finally:
            waiter.cancel()
        return self._stop.is_set()

    async def run(self) -> None:
        """Acquire, renew, step down on a missed renew deadline, try again; until :meth:`stop`."""
        s = self.s
        self.log.info(f"Leader election: candidate {self.identity} for lease {self.namespace}/{self.name}")
        while not self._stop.is_set():
            ok = await self.try_acquire_or_renew()
            if self._stop.is_set():
                break
            if ok:
                self._set_leader(True)
                if await self._sleep(s.retry_period_seconds):
                    break
                continue
            if self._leader and self.clock() - self.last_renew >= s.renew_deadline_seconds:
                self._set_leader(False)  # could not renew in time: stop acting as leader
            elif self._leader and self.observed is not None and self.observed.holder != self.identity:
                self._set_leader(False)  # someone else holds it now
            # candidates poll with jitter (client-go JitterUntil factor 1.2)
            delay = s.retry_period_seconds * (1.0 if self._leader else 1.0 + 0.2 * self.rng.random())
            if await self._sleep(delay):
                break
        if self._leader:  # hand the lease over at once (client-go ReleaseOnCancel)
            await self.release()
        self._set_leader(False)


def shard_lease(settings) -> LeaderElectionSettings:
    """One lease per shard: with ``watcher.shard.count > 1`` the lease name gets a
    ``-shard-<index>`` suffix, so every shard has its own active replica."""
    import dataclasses
    le = settings.watcher.leader_election
    sh = settings.watcher.shard
    if sh.count <= 1:
        return le
    return dataclasses.replace(le, lease_name=f"{le.lease_name}-shard-{sh.index}")


class LeaderElectedService:
    """Run :class:`WatcherService` only while this replica holds the lease.

    Each leadership term builds a fresh service (list → watch → notify). When
    the term ends — lease lost or not renewed in time — the service stops at
    once and its queued notifications are abandoned rather than drained: the
    new leader lists the cluster itself (at-least-once across the hand-over,
    like the reference's restart-and-replay). A checkpoint on a
    shared volume (``watcher.checkpoint.path``) lets the next leader resume
    from the last quiescent resourceVersion instead.
    """

    def __init__(self, settings, endpoint=None, metrics: Optional[Metrics] = None,
                 notifier_factory=None) -> None:
        from .service import WatcherService
        self.settings = settings
        self.metrics = metrics or Metrics()
        self.notifier_factory = notifier_factory
        self.exit_on_loss = settings.watcher.leader_election.exit_on_loss
        self._probe = WatcherService(settings, endpoint=endpoint, metrics=self.metrics)
        self.endpoint = endpoint
        self.elector: Optional[LeaderElector] = None
        self.service = None
        self.terms = 0
        self._stop = asyncio.Event()
        self.log = logging.getLogger(SERVICE_LOGGER)

    def stop(self) -> None:
        """Graceful: the current term drains its notifier while the lease is
        still renewed; only then is the lease released (``run``'s cleanup)."""
        self._stop.set()
        if self.service is not None:
            self.service.stop()

    async def run(self) -> None:
        from .service import SetupError, WatcherService
        if not await self._probe.setup_k8s_client():
            self.log.error("Failed to setup Kubernetes client")
            raise SetupError("Failed to setup Kubernetes client")
        api = self._probe.api
        assert api is not None
        self.endpoint = self._probe.endpoint
        self.metrics.ready = True  # a standby replica is healthy and ready to take over
        metrics_server = None
        if self.settings.metrics.enabled:  # one server for every term, standby included
            from ..metrics import start_metrics_server
            metrics_server = await start_metrics_server(self.metrics, self.settings.metrics.host,
                                                        self.settings.metrics.port, debug=self.settings.metrics.debug)
        self.elector = LeaderElector(api, shard_lease(self.settings), self.metrics)
        elector_task = asyncio.ensure_future(self.elector.run())
        stopper = asyncio.ensure_future(self._stop.wait())
        try:
            while not self._stop.is_set():
                became = asyncio.ensure_future(self.elector.became_leader.wait())
                await asyncio.wait([became, stopper, elector_task], return_when=asyncio.FIRST_COMPLETED)
                became.cancel()
                if self._stop.is_set() or elector_task.done():
                    break
                self.terms += 1
                svc = WatcherService(self.settings, endpoint=self.endpoint, metrics=self.metrics,
                                     notifier_factory=self.notifier_factory, serve_metrics=False)
                self.service = svc
                lost = asyncio.ensure_future(self.elector.lost.wait())
                run = asyncio.ensure_future(self._term(svc))
                done, _ = await asyncio.wait([run, lost, stopper], return_when=asyncio.FIRST_COMPLETED)
                lost.cancel()
                svc.stop()
                if run in done:
                    self.service = None
                    run.result()  # a watch that failed permanently ends the process (exit 1)
                    break  # the watch ended on its own
                graceful = self._stop.is_set() and not self.elector.lost.is_set()
                await self._end_term(svc, run, graceful)
                self.service = None
                if not self._stop.is_set() and self.exit_on_loss:
                    raise LeadershipLost("leadership lost")
        finally:
            stopper.cancel()
            svc = self.service
            if svc is not None:  # cancelled mid-term: stop watching before giving the lease up
                self.service = None
                svc.stop()
                await svc.shutdown(drain_timeout=0.0, checkpoint=False)
            self.elector.stop()
            try:
                await elector_task
            except Exception:  # noqa: BLE001 - the elector never raises; be defensive at shutdown
                pass
            await api.close()
            if metrics_server is not None:
                metrics_server.close()

    async def _term(self, svc) -> None:
        try:
            await svc.start()
            await svc.wait()
        finally:
            if not self.elector.lost.is_set() and not self._stop.is_set():
                await svc.shutdown()

    async def _end_term(self, svc, run: "asyncio.Future", graceful: bool) -> None:
        # graceful (SIGTERM while leading): drain and checkpoint as a lone
        # watcher would; lease lost: abandon the queue, leave the checkpoint alone.
        # The term's task ends first (svc.stop() was called; a lost lease also
        # cancels it), so a start() still in progress cannot create reflectors
        # after the shutdown below.
        if not graceful and not run.done():
            run.cancel()
        try:
            await run
        except (asyncio.CancelledError, Exception):  # noqa: BLE001 - the term is over either way
            pass
        await svc.shutdown(drain_timeout=10.0 if graceful else 0.0, checkpoint=graceful)


class LeadershipLost(Exception):
    """Leadership ended and ``exit_on_loss`` asks the process to exit (exit status 1)."""
