"""Idempotent persistence targets of the writer stage."""
from __future__ import annotations

import abc
from typing import Sequence

from ..models.domain import ParsedSMS

__all__ = ["Sink"]


class Sink(abc.ABC):
    name: str = "sink"

    async def start(self) -> None:
        pass

    @abc.abstractmethod
    async def upsert_many(self, records: Sequence[ParsedSMS]) -> None:
        """Create-or-update every record, keyed by ``msg_id`` (must be idempotent)."""

    async def upsert(self, record: ParsedSMS) -> None:
        await self.upsert_many([record])

    async def close(self) -> None:
        pass
