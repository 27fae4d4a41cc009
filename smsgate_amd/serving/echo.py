"""CPU stand-in for :class:`~smsgate_amd.serving.engine.ExtractionEngine` with the
same serving surface (``submit_ids`` / ``step(raw=True)`` / ``busy`` / ``stats``).

Answers every prompt with the token ids of the fake backend's canned answer.  With
``packed`` (default) it also takes whole wire requests (``submit_packed``) and answers
them as one :class:`~smsgate_amd.serving.protocol.PackedAnswer`, like the qa engine.
Used to exercise the replica / distributed harness end to end without a GPU
(``bench.py --cpu-echo-engine`` under ``torch.distributed.run`` with gloo, and
the multi-process tests); it is never a fallback for the GPU engine.
"""
from __future__ import annotations

from typing import Any, List, Tuple

import numpy as np

__all__ = ["EchoEngine"]


class _Stats:
    def __init__(self) -> None:
        self.completed = 0

    def as_dict(self) -> dict:
        return {"completed": self.completed}


class EchoEngine:
    def __init__(self, per_step: int = 300, packed: bool = True) -> None:
        from ..models.tokenizer import load_tokenizer
        from ..parse.backends.fake import DEFAULT_ANSWER
        from .fsm import DEFAULT_FIELDS

        tk = load_tokenizer()
        toks: List[int] = []
        for f in DEFAULT_FIELDS:
            toks += tk.encode(DEFAULT_ANSWER[f.name]) + [tk.sep]
        self.answer = np.asarray(toks, dtype=np.int32)
        self.waiting: List[Tuple[Any, Any]] = []
        self.per_step = per_step
        if not packed:
            self.submit_packed = None  # shadows the method: the engine server's per-message path
        self.seen = 0
        self.stats = _Stats()

    def submit_ids(self, items) -> None:
        self.waiting.extend(items)

    def busy(self) -> bool:
        return bool(self.waiting)

    def submit_packed(self, key: Any, lens, ids) -> None:
        self.waiting.append((key, ("packed", len(lens))))

    def step(self, raw: bool = True):
        from .protocol import PackedAnswer

        out = []
        for k, v in self.waiting[: self.per_step]:
            if isinstance(v, tuple) and v and v[0] == "packed":
                n = v[1]
                out.append((k, PackedAnswer(np.full(n, len(self.answer), dtype=np.uint16), np.tile(self.answer, n))))
                self.seen += n
                self.stats.completed += n
            else:
                out.append((k, self.answer))
                self.seen += 1
                self.stats.completed += 1
        del self.waiting[: self.per_step]
        return out
