"""Command-line entry point (``/root/reference/main.py:5-27``).

Same contract as the reference:

* environment precedence: ``argv[1]`` > ``$ENVIRONMENT`` > ``development``;
* anything outside ``development|staging|production`` prints
  ``Error: Unsupported environment '<env>'`` + the supported list, exit 1;
* prints ``Starting k8s-watcher in '<env>' environment``;
* an exception prints ``Error starting watcher: <e>``, exit 1.

Fixes: Kubernetes setup failure exits 1 (reference: 0); SIGTERM stops the
watcher gracefully like SIGINT; the watch ending on its own exits 0. With
``watcher.leader_election.enabled`` the process is one replica of several and
watches only while it holds the Lease (``engine/leader.py``).
Extra flags (all optional, after the environment): ``--config-dir``,
``--set key.path=value`` (repeatable), ``--print-config``, ``--check``
(setup + connectivity only), ``--version``.
"""

from __future__ import annotations

import argparse
import asyncio
import os
import signal
import sys
from typing import List, Optional

from . import __version__
from .utils.config import SUPPORTED_ENVIRONMENTS, ConfigError, deep_merge, dump_effective, load_settings, parse_override
from .utils.logsetup import setup_logging


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="main.py", description="Kubernetes pod-event watcher")
    ap.add_argument("environment", nargs="?", default=None,
                    help="development | staging | production (default: $ENVIRONMENT or development)")
    ap.add_argument("--config-dir", default=None, help="directory holding base.yaml and <env>.yaml")
    ap.add_argument("--set", dest="overrides", action="append", default=[],
                    metavar="KEY=VALUE", help="override a config key, e.g. watcher.notify_on=phase_change")
    ap.add_argument("--print-config", action="store_true", help="print the effective config and exit")
    ap.add_argument("--check", action="store_true", help="set up the client, probe the API and exit")
    ap.add_argument("--version", action="version", version=f"k8s-watcher-amd {__version__}")
    return ap


async def _run_service(settings, check_only: bool) -> int:
    from .engine.leader import LeaderElectedService, LeadershipLost
    from .engine.service import SetupError, WatcherService
    svc = WatcherService(settings)
    if settings.watcher.leader_election.enabled and not check_only:
        svc = LeaderElectedService(settings)
    if check_only:
        ok = await svc.setup_k8s_client()
        if ok:
            ok = await svc.preflight()
        if svc.api is not None:
            await svc.api.close()
        return 0 if ok else 1
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, svc.stop)
        except (NotImplementedError, RuntimeError):
            pass
    try:
        await svc.run()
    except (SetupError, LeadershipLost):
        return 1
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    args = _parser().parse_args(sys.argv[1:] if argv is None else argv)
    environment = os.getenv("ENVIRONMENT", "development")
    if args.environment:
        environment = args.environment
    if environment not in SUPPORTED_ENVIRONMENTS:
        print(f"Error: Unsupported environment '{environment}'")
        print(f"Supported environments: {list(SUPPORTED_ENVIRONMENTS)}")
        return 1
    print(f"Starting k8s-watcher in '{environment}' environment", flush=True)
    try:
        overrides = {}
        for expr in args.overrides:
            overrides = deep_merge(overrides, parse_override(expr))
        settings = load_settings(environment, args.config_dir, overrides)
        if args.print_config:
            dump_effective(settings)
            return 0
        log = setup_logging(environment, settings.watcher.log_level, log_file=settings.watcher.log_file)
        log.info(f"Starting k8s-watcher in {environment} environment")
        return asyncio.run(_run_service(settings, args.check))
    except (ConfigError, Exception) as exc:  # noqa: BLE001 - parity: main.py:25-27
        print(f"Error starting watcher: {exc}")
        return 1


def entrypoint() -> None:
    sys.exit(main())
