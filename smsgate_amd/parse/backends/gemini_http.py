"""Google Gemini over plain REST — the reference's extraction call.

The reference uses ``google-genai``'s ``generate_content_stream`` synchronously,
one message at a time, blocking the event loop (gemini_parser.py:273-292;
R4).  ``google-genai`` is not on the image, so this backend speaks the public
REST endpoint ``models/{model}:generateContent`` through ``httpx`` with the
same request: system instruction, the normalised SMS as the user turn,
``temperature=0.1``, ``responseMimeType=application/json`` and the 9-string
response schema (gemini_parser.py:212-220).  The answer text is salvaged with
the same greedy ``{.*}`` extraction (:63-65).

Concurrency: a batch is sent as concurrent requests bounded by
``concurrency`` — the event loop is never blocked.  Failures are returned per
message as :class:`BackendError` (→ DLQ shape b, like ``call_gemini``
re-raising); transient HTTP 429/5xx are retried ``retries`` times with
backoff (the reference had no retry on this call).
"""
from __future__ import annotations

import asyncio
import os
from typing import Any, Dict, List, Optional, Sequence

import httpx

from ..schema import GENERATION_TEMPERATURE, RESPONSE_SCHEMA, SYSTEM_INSTRUCTION
from ..text import extract_json
from .base import BackendError, ExtractResult, ParserBackend

__all__ = ["GeminiHTTPBackend", "build_request"]

API = "https://generativelanguage.googleapis.com/v1beta"


def build_request(body: str) -> Dict[str, Any]:
    return {
        "systemInstruction": {"parts": [{"text": SYSTEM_INSTRUCTION}]},
        "contents": [{"role": "user", "parts": [{"text": body}]}],
        "generationConfig": {
            "temperature": GENERATION_TEMPERATURE,
            "responseMimeType": "application/json",
            "responseSchema": RESPONSE_SCHEMA,
        },
    }


class GeminiHTTPBackend(ParserBackend):
    name = "gemini_http"

    def __init__(self, api_key: Optional[str] = None, model: Optional[str] = None, concurrency: int = 16,
                 retries: int = 2, timeout: float = 60.0, transport: Optional[httpx.AsyncBaseTransport] = None,
                 base_url: str = API, max_batch: int = 64) -> None:
        from ...config import get_settings

        s = get_settings()
        self.api_key = api_key or os.getenv("GEMINI_API_KEY") or s.gemini_api_key
        self.model = model or os.getenv("GEMINI_MODEL") or s.gemini_model
        self.concurrency = concurrency
        self.retries = retries
        self.max_batch = max_batch
        self._timeout = timeout
        self._transport = transport
        self._base = base_url
        self._client: Optional[httpx.AsyncClient] = None
        self._sem: Optional[asyncio.Semaphore] = None

    async def start(self) -> None:
        if self._client is None:
            self._client = httpx.AsyncClient(base_url=self._base, timeout=self._timeout, transport=self._transport)
            self._sem = asyncio.Semaphore(self.concurrency)

    async def close(self) -> None:
        if self._client is not None:
            await self._client.aclose()
            self._client = None

    async def _one(self, body: str) -> ExtractResult:
        if not self.api_key:
            return BackendError("GEMINI_API_KEY is not set")
        assert self._client is not None and self._sem is not None
        url = f"/models/{self.model}:generateContent"
        delay = 1.0
        async with self._sem:
            for attempt in range(self.retries + 1):
                try:
                    r = await self._client.post(url, params={"key": self.api_key}, json=build_request(body))
                    if r.status_code in (429, 500, 502, 503, 504) and attempt < self.retries:
                        await asyncio.sleep(delay)
                        delay *= 2
                        continue
                    r.raise_for_status()
                    data = r.json()
                    text = "".join(p.get("text", "") for c in data.get("candidates", [])[:1]
                                   for p in c.get("content", {}).get("parts", []))
                    try:
                        ans = extract_json(text)
                    except ValueError:
                        return BackendError("Gemini returned malformed JSON")
                    if not isinstance(ans, dict):
                        return BackendError("Gemini returned non-JSON")
                    return ans
                except httpx.HTTPError as exc:
                    if attempt >= self.retries:
                        return BackendError(f"Gemini request failed: {exc}")
                    await asyncio.sleep(delay)
                    delay *= 2
        return BackendError("Gemini request failed")

    async def extract_batch(self, bodies: Sequence[str]) -> List[ExtractResult]:
        await self.start()
        return list(await asyncio.gather(*(self._one(b) for b in bodies)))
