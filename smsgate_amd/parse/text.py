"""Text-level steps of the parse pipeline: pre-filters, normalisation, JSON salvage.

* :data:`WORKER_SKIP_KEYWORDS` / :func:`worker_should_skip` — the parser
  worker's non-transaction filter (worker.py:112-121). Case-insensitive except
  ``'Daily limit exceeded'``, which the reference matches case-sensitively.
* :data:`LLM_SKIP_KEYWORDS` / :func:`llm_should_skip` — the parser's own OTP
  pre-filter, case-sensitive (gemini_parser.py:198-199).
* :func:`normalize_body` — NBSP→space, bullet→``*``, then
  :func:`mask_card_number_with_prefix` (gemini_parser.py:202-203, 121-137).
* :func:`extract_json` — greedy first-``{`` to last-``}`` salvage of a model
  answer (gemini_parser.py:63-65).
"""
from __future__ import annotations

import json
import re
from typing import Any, Optional

__all__ = [
    "WORKER_SKIP_KEYWORDS",
    "LLM_SKIP_KEYWORDS",
    "worker_should_skip",
    "llm_should_skip",
    "normalize_body",
    "mask_card_number_with_prefix",
    "extract_json",
]

#: Upper-cased substrings that make the worker ack-and-skip a message.
#: D10 (kept for parity): incoming credits ("CREDIT PAYMENT", "C2C RECEIVED")
#: are skipped like OTPs, so they are never stored.
WORKER_SKIP_KEYWORDS = (
    "OTP",
    "CODE:",
    "NOT ENOUGH FUNDS",
    "INSUFFICIENT FUNDS",
    "CREDIT PAYMENT",
    "C2C RECEIVED",
    "PASS:",
    "PASS=",
    "PERSON TO PERSON",
)
_WORKER_SKIP_CASE_SENSITIVE = ("Daily limit exceeded",)

#: Case-sensitive substrings for which the parser returns ``None`` (-> DLQ).
LLM_SKIP_KEYWORDS = ("OTP", "CODE:", "PASS:", "PASS=", "Daily limit exceeded:")

_CARD_RE = re.compile(r"\d{4}\*{3}(\d{4})")
# one alternation scan instead of a generator of ``in`` tests (same semantics)
_WORKER_SKIP_RE = re.compile("|".join(map(re.escape, WORKER_SKIP_KEYWORDS)))
_WORKER_SKIP_CS_RE = re.compile("|".join(map(re.escape, _WORKER_SKIP_CASE_SENSITIVE)))
_LLM_SKIP_RE = re.compile("|".join(map(re.escape, LLM_SKIP_KEYWORDS)))
_JSON_RE = re.compile(r"\{.*\}", re.S)


def worker_should_skip(body: str) -> bool:
    return _WORKER_SKIP_RE.search(body.upper()) is not None or _WORKER_SKIP_CS_RE.search(body) is not None


def llm_should_skip(body: str) -> bool:
    return _LLM_SKIP_RE.search(body) is not None


def mask_card_number_with_prefix(text: str) -> str:
    """``'4083***7538'`` → ``'CARD:7538'`` (every occurrence)."""
    return _CARD_RE.sub(r"CARD:\1", text)


def normalize_body(body: str) -> str:
    return mask_card_number_with_prefix(body.replace("\u00a0", " ").replace("\u2022", "*"))


def extract_json(text: str) -> Optional[Any]:
    m = _JSON_RE.search(text)
    return json.loads(m.group(0)) if m else None
