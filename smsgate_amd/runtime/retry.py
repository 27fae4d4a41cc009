"""Exponential-backoff retry (the reference's ``tenacity`` usage, which is not
installed on the image).

``@retry(attempts=5, wait_min=1, wait_max=20)`` reproduces
``retry(wait=wait_exponential(min=1, max=20), stop=stop_after_attempt(5))``
(writer.py:57; pocketbase.py:69 uses min=2, max=30).  Works on sync and async
callables; after the last attempt it raises :class:`RetryError` chained to the
final exception (tenacity's behaviour, which pocketbase.py:314 relies on).
"""
from __future__ import annotations

import asyncio
import functools
import inspect
import random
import time
from typing import Any, Callable, Optional, Tuple, Type

__all__ = ["RetryError", "retry", "backoff_delays"]


class RetryError(Exception):
    def __init__(self, attempts: int, last: BaseException) -> None:
        super().__init__(f"gave up after {attempts} attempts: {last!r}")
        self.attempts = attempts
        self.last = last


def backoff_delays(attempts: int, wait_min: float, wait_max: float, multiplier: float = 1.0,
                   jitter: float = 0.0):
    """Delays between attempts: ``clamp(multiplier * 2**i, wait_min, wait_max)``."""
    for i in range(attempts - 1):
        d = min(wait_max, max(wait_min, multiplier * (2 ** i)))
        if jitter:
            d += random.uniform(0, jitter)
        yield d


def retry(attempts: int = 5, wait_min: float = 1.0, wait_max: float = 20.0, multiplier: float = 1.0,
          retry_on: Tuple[Type[BaseException], ...] = (Exception,),
          sleep: Optional[Callable[[float], Any]] = None, reraise: bool = False):
    def deco(fn):
        if inspect.iscoroutinefunction(fn):
            @functools.wraps(fn)
            async def aw(*a, **kw):
                delays = list(backoff_delays(attempts, wait_min, wait_max, multiplier))
                for i in range(attempts):
                    try:
                        return await fn(*a, **kw)
                    except retry_on as exc:
                        if i == attempts - 1:
                            if reraise:
                                raise
                            raise RetryError(attempts, exc) from exc
                        d = delays[i]
                        if sleep is not None:
                            r = sleep(d)
                            if inspect.isawaitable(r):
                                await r
                        else:
                            await asyncio.sleep(d)
            return aw

        @functools.wraps(fn)
        def sw(*a, **kw):
            delays = list(backoff_delays(attempts, wait_min, wait_max, multiplier))
            for i in range(attempts):
                try:
                    return fn(*a, **kw)
                except retry_on as exc:
                    if i == attempts - 1:
                        if reraise:
                            raise
                        raise RetryError(attempts, exc) from exc
                    (sleep or time.sleep)(delays[i])
        return sw
    return deco
