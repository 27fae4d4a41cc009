"""Extraction backends and the registry used by ``PARSER_BACKEND``.

=============  ===================================================================
name           backend
=============  ===================================================================
``fake``       canned answers (tests, CPU benchmark — BASELINE.json config #1)
``regex``      offline rule-based extractor (known bank formats)
``gemini_http`` Google Gemini REST ``generateContent`` over httpx (reference parity)
``local_llm``  schema-constrained extraction LM on MI355X (HIP kernels)
=============  ===================================================================
"""
from __future__ import annotations

from typing import Any

from .base import BackendError, ExtractResult, ParserBackend  # noqa: F401
from .fake import DEFAULT_ANSWER, FakeBackend  # noqa: F401
from .regex import RegexBackend, extract_rule_based  # noqa: F401

__all__ = ["create_backend", "ParserBackend", "BackendError", "FakeBackend", "RegexBackend"]


def create_backend(name: str, **kwargs: Any) -> ParserBackend:
    name = name.lower()
    if name == "fake":
        return FakeBackend(**kwargs)
    if name == "regex":
        return RegexBackend()
    if name in ("gemini", "gemini_http"):
        from .gemini_http import GeminiHTTPBackend

        return GeminiHTTPBackend(**kwargs)
    if name in ("local", "local_llm", "llm"):
        from .local_llm import LocalLLMBackend

        return LocalLLMBackend(**kwargs)
    raise ValueError(f"unknown parser backend {name!r}")
