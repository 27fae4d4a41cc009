"""Deterministic stand-in for the LLM (tests and the CPU benchmark).

The reference's only parser tests call the live Gemini API
(tests/test_parsers.py:73-86).  :class:`FakeBackend` returns canned answers
keyed by normalised body, a default answer for everything else, or delegates
to another backend; it can also inject latency or failures.  It is the
"mocked-Gemini parser" of BASELINE.json config #1.
"""
from __future__ import annotations

import asyncio
import copy
from typing import Any, Callable, Dict, List, Mapping, Optional, Sequence

from .base import ExtractResult, ParserBackend

__all__ = ["FakeBackend", "DEFAULT_ANSWER"]

#: What the reference's benchmark stub returned (BASELINE.md harness).
DEFAULT_ANSWER: Dict[str, Any] = {
    "txn_type": "debit",
    "date": "06.05.25 14:23",
    "amount": "52.00",
    "currency": "USD",
    "card": "***0018",
    "merchant": "TEST LLC",
    "city": "MOSKOW",
    "address": "TEST STR. 29, 24 AREA",
    "balance": "1842.74",
}


class FakeBackend(ParserBackend):
    name = "fake"

    def __init__(
        self,
        answers: Optional[Mapping[str, Dict[str, Any]]] = None,
        default: Optional[Dict[str, Any]] = DEFAULT_ANSWER,
        fallback: Optional[ParserBackend] = None,
        latency_s: float = 0.0,
        fail: Optional[Callable[[str], Optional[BaseException]]] = None,
        max_batch: int = 256,
    ) -> None:
        self.answers = dict(answers or {})
        self.default = default
        self.fallback = fallback
        self.latency_s = latency_s
        self.fail = fail
        self.max_batch = max_batch
        self.calls = 0
        self.bodies_seen = 0

    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        self.calls += 1
        self.bodies_seen += len(bodies)
        if self.latency_s:
            await asyncio.sleep(self.latency_s)
        out: List[ExtractResult] = []
        missing: List[int] = []
        for i, b in enumerate(bodies):
            if self.fail is not None:
                err = self.fail(b)
                if err is not None:
                    out.append(err)
                    continue
            ans = self.answers.get(b)
            if ans is None and self.fallback is None and self.default is not None:
                ans = self.default
            if ans is None:
                out.append(None)  # type: ignore[arg-type]
                missing.append(i)
            else:
                out.append(copy.copy(ans))
        if missing and self.fallback is not None:
            got = await self.fallback.extract_batch([bodies[i] for i in missing])
            for i, r in zip(missing, got):
                out[i] = r
        for i, r in enumerate(out):
            if r is None:
                from .base import BackendError

                out[i] = BackendError("fake backend has no answer for this body")
        return out
