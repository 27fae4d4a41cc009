"""In-memory sink (tests, benchmark): last write per ``msg_id`` wins."""
from __future__ import annotations

from typing import Dict, List, Sequence

from ..models.domain import ParsedSMS, as_parsed
from .base import Sink

__all__ = ["MemorySink"]


class MemorySink(Sink):
    name = "memory"

    def __init__(self) -> None:
        self.records: Dict[str, ParsedSMS] = {}
        self.writes = 0

    async def upsert_many(self, records: Sequence[ParsedSMS]) -> None:
        for r in records:
            self.records[r.msg_id] = r
        self.writes += len(records)

    def all(self) -> List[ParsedSMS]:
        return [as_parsed(r) for r in self.records.values()]
