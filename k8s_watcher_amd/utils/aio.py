"""asyncio helpers.

:func:`with_timeout` replaces ``asyncio.wait_for`` on the network paths: on
Python 3.10 ``wait_for`` can swallow a cancellation that races with the inner
future's completion (bpo-42130), which would let a cancelled watcher task keep
reconnecting forever. ``asyncio.wait`` based waiting always re-raises.
"""

from __future__ import annotations

import asyncio
from typing import Any, Awaitable, Optional


async def with_timeout(aw: Awaitable[Any], timeout: Optional[float]) -> Any:
    fut = asyncio.ensure_future(aw)
    try:
        done, _ = await asyncio.wait([fut], timeout=timeout)
    except asyncio.CancelledError:
        fut.cancel()
        raise
    if not done:
        fut.cancel()
        raise asyncio.TimeoutError()
    return fut.result()
