"""Text-level steps of the parse pipeline: pre-filters, normalisation, JSON salvage.

* :data:`WORKER_SKIP_KEYWORDS` / :func:`worker_should_skip` — the parser
  worker's non-transaction filter (worker.py:112-121). Case-insensitive except
  ``'Daily limit exceeded'``, which the reference matches case-sensitively.
* :data:`LLM_SKIP_KEYWORDS` / :func:`llm_should_skip` — the parser's own OTP
  pre-filter, case-sensitive (gemini_parser.py:198-199).
* keyword matching mode (:func:`set_keyword_match`, env ``PARSER_KEYWORD_MATCH``):
  the reference matches **substrings**, so a purchase at a merchant whose name
  merely *contains* ``OTP`` (``ROTPIOR``, ``KOTPAY``…) is skipped and counted OK
  without ever being parsed (0.38 % of synthetic purchases).  Decision: the
  default is ``"word"`` — a keyword matches only where its alphanumeric edges
  are word boundaries (``OTP`` matches ``Your OTP: 1`` and ``OTP-code``, not
  ``ROTPIOR``); ``"substring"`` restores the reference behaviour exactly
  (parity flag).  Known limit in BOTH modes: a purchase at a merchant literally
  named ``OTP BANK`` is still skipped — the filter has no notion of context, and
  deciding that needs the model (tests/test_parse_helpers.py pins all three).
* :func:`normalize_body` — NBSP→space, bullet→``*``, then
  :func:`mask_card_number_with_prefix` (gemini_parser.py:202-203, 121-137).
* :func:`extract_json` — greedy first-``{`` to last-``}`` salvage of a model
  answer (gemini_parser.py:63-65).
"""
from __future__ import annotations

import json
import os
import re
from typing import Any, Optional

__all__ = [
    "set_keyword_match",
    "keyword_match",
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
_JSON_RE = re.compile(r"\{.*\}", re.S)
KEYWORD_MATCH_MODES = ("word", "substring")


def _keyword_re(words, mode: str) -> "re.Pattern[str]":
    """One alternation scan instead of a generator of ``in`` tests; in ``"word"``
    mode each keyword's alphanumeric edges must sit on word boundaries."""
    def one(k: str) -> str:
        p = re.escape(k)
        if mode == "word":
            p = (r"(?<!\w)" if k[0].isalnum() else "") + p + (r"(?!\w)" if k[-1].isalnum() else "")
        return p

    return re.compile("|".join(one(k) for k in words))


def set_keyword_match(mode: str) -> None:
    """``"word"`` (default) or ``"substring"`` (reference parity) for both filters."""
    global _MODE, _WORKER_SKIP_RE, _WORKER_SKIP_CS_RE, _LLM_SKIP_RE
    if mode not in KEYWORD_MATCH_MODES:
        raise ValueError(f"keyword match mode must be one of {KEYWORD_MATCH_MODES}, not {mode!r}")
    _MODE = mode
    _WORKER_SKIP_RE = _keyword_re(WORKER_SKIP_KEYWORDS, mode)
    _WORKER_SKIP_CS_RE = _keyword_re(_WORKER_SKIP_CASE_SENSITIVE, mode)
    _LLM_SKIP_RE = _keyword_re(LLM_SKIP_KEYWORDS, mode)


# the plain literal alternations: a ~1.7 us scan (the word-boundary patterns cost ~40 us
# on a typical body: the lookarounds defeat the regex engine's literal search), so the
# word patterns only run on the rare body that contains a keyword at all
_WORKER_SUB_RE = _keyword_re(WORKER_SKIP_KEYWORDS, "substring")
_WORKER_SUB_CS_RE = _keyword_re(_WORKER_SKIP_CASE_SENSITIVE, "substring")
_LLM_SUB_RE = _keyword_re(LLM_SKIP_KEYWORDS, "substring")


def keyword_match() -> str:
    return _MODE


_MODE = "word"
set_keyword_match(os.environ.get("PARSER_KEYWORD_MATCH", "word").strip().lower() or "word")


def worker_should_skip(body: str) -> bool:
    u = body.upper()
    if _WORKER_SUB_RE.search(u) is not None and _WORKER_SKIP_RE.search(u) is not None:
        return True
    return _WORKER_SUB_CS_RE.search(body) is not None and _WORKER_SKIP_CS_RE.search(body) is not None


def llm_should_skip(body: str) -> bool:
    return _LLM_SUB_RE.search(body) is not None and _LLM_SKIP_RE.search(body) is not None


def mask_card_number_with_prefix(text: str) -> str:
    """``'4083***7538'`` → ``'CARD:7538'`` (every occurrence).  (The regex scan costs
    ~5.8 us per SMS; a body without ``***`` cannot match.)"""
    if "***" not in text:
        return text
    return _CARD_RE.sub(r"CARD:\1", text)


def normalize_body(body: str) -> str:
    return mask_card_number_with_prefix(body.replace("\u00a0", " ").replace("\u2022", "*"))


def extract_json(text: str) -> Optional[Any]:
    m = _JSON_RE.search(text)
    return json.loads(m.group(0)) if m else None
