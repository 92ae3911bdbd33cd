"""Exponential backoff with jitter driven by a :class:`RetryPolicy`."""

from __future__ import annotations

import random
from typing import Iterator, Optional

from .config import RetryPolicy


class Backoff:
    """Stateful delay generator: ``next_delay()`` grows until ``reset()``."""

    def __init__(self, policy: RetryPolicy, rng: Optional[random.Random] = None) -> None:
        self.policy = policy
        self.attempt = 0
        self._rng = rng or random.Random()

    def reset(self) -> None:
        self.attempt = 0

    def next_delay(self) -> float:
        self.attempt += 1
        base = self.policy.delay(self.attempt)
        j = self.policy.jitter
        if j > 0:
            base *= 1.0 + self._rng.uniform(-j, j)
        return max(0.0, base)

    @property
    def exhausted(self) -> bool:
        """True once ``max_attempts`` consecutive failures have been counted."""
        return self.attempt >= self.policy.max_attempts

    def delays(self) -> Iterator[float]:
        while True:
            yield self.next_delay()
