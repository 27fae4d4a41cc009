"""The :class:`ParserBackend` boundary — where the reference calls Gemini.

The reference has exactly one extraction call site, ``call_gemini``
(gemini_parser.py:221, :273-292), synchronous and one message at a time. Here
a backend is *batch-first and async*: :meth:`extract_batch` receives the
normalised bodies of many messages and returns, per body, the raw answer dict
(string-valued, like the Gemini JSON) or the exception that message raised.
Blocking backends run off the event loop (fixes R4) and a GPU backend can fill
a decode batch from one call.
"""
from __future__ import annotations

import abc
from typing import Any, Dict, List, Sequence, Union

from ...runtime.errors import TransientError

__all__ = ["ParserBackend", "ExtractResult", "BackendError", "BackendUnavailable"]

ExtractResult = Union[Dict[str, Any], BaseException]


class BackendError(RuntimeError):
    """The backend answered, but not with a usable JSON object."""


class BackendUnavailable(BackendError, TransientError):
    """The backend could not be reached at all (engine process down, socket
    closed).  Not the message's fault: :class:`~smsgate_amd.parse.pipeline.ParsePipeline`
    re-raises it for the whole batch so the stage naks and retries the batch,
    instead of routing every message to the DLQ."""


class ParserBackend(abc.ABC):
    name: str = "abstract"
    #: largest batch the backend wants per call (the stage respects it)
    max_batch: int = 64

    async def start(self) -> None:
        """Acquire resources (HTTP client, GPU weights, …)."""

    async def close(self) -> None:
        """Release resources."""

    @abc.abstractmethod
    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        """One answer (or exception) per body, same order."""

    async def extract(self, body: str) -> Dict[str, Any]:
        res = (await self.extract_batch([body]))[0]
        if isinstance(res, BaseException):
            raise res
        return res
