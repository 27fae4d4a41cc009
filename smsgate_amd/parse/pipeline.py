"""Batched parse pipeline: pre-filter → normalise → cache → extract → post-process.

Behaviour per message matches ``parse_sms_llm`` (gemini_parser.py:193-271):

1. case-sensitive OTP pre-filter → ``UNMATCHED`` (the worker routes it to the
   DLQ as ``{"reason": "unmatched"}``);
2. body normalisation + card masking; cache key = sha256 of that body;
3. extraction (cache hit or backend call; backend answers are cached *raw*,
   so post-processing fixes apply on replay — SURVEY.md §5.4, D7);
   a backend exception → ``ERROR`` (DLQ shape b);
4. post-processing chain: date (strptime → dateutil → on "String does not
   contain a date" the message timestamp in Asia/Yerevan → body-date repair),
   card (strip ``*``/blanks, first 4), amount/balance via
   :func:`parse_ambiguous_decimal` of ``str(value)`` (so ``None`` fails — D6,
   kept as a contract), :class:`ParsedSmsCore` validation; any failure →
   ``UNMATCHED`` (error captured unless ``txn_type == 'otp'``);
5. ``address == "null"`` → ``""``; a card shorter than 4 chars → ``BROKEN``;
6. build :class:`ParsedSMS` with ``parser_version = "llm-0.2.0"``.

What is different is the execution model: a whole batch of messages is
prepared, looked up in the cache with one query, the misses go to the backend
in one :meth:`ParserBackend.extract_batch` call, and post-processing runs on
the results — the reference did one synchronous HTTPS call per message.
"""
from __future__ import annotations

import enum
import os
import time
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence

from ..models.domain import CORE_FIELDS, PARSER_VERSION_LLM, ParsedSMS, ParsedSmsCore, RawSMS
from ..obs.errors import sentry_capture
from ..obs.metrics import GEMINI_LATENCY, observe_many
from ..runtime.errors import TransientError
from .backends.base import BackendError, ParserBackend
from .cache import MemoryKV, ResponseCache, cache_key
from . import fastpath
from .canonical import canonicalize_answer
from .dates import fix_broken_datetime, parse_custom_datetime, parse_unix_timestamp
from .numeric import parse_ambiguous_decimal
from .text import llm_should_skip, normalize_body

__all__ = ["Outcome", "ParseResult", "ParsePipeline", "BrokenMessage", "postprocess_answer"]

DEFAULT_TZ = "Asia/Yerevan"  # gemini_parser.py:229, Dockerfile TZ
_N_CORE = len(CORE_FIELDS)


# SMSGATE_DEBUG_ANSWERS=DIR: each process appends the first 200 answers that did not
# parse (body, backend answer, outcome) to DIR/answers-<pid>.jsonl (diagnostics)
_DEBUG_DIR = os.environ.get("SMSGATE_DEBUG_ANSWERS", "")
_DEBUG_LEFT = [200]


def _debug_record(body: str, answer: Dict[str, Any], outcome: str) -> None:
    if _DEBUG_LEFT[0] <= 0:
        return
    _DEBUG_LEFT[0] -= 1
    import json

    os.makedirs(_DEBUG_DIR, exist_ok=True)
    with open(os.path.join(_DEBUG_DIR, f"answers-{os.getpid()}.jsonl"), "a") as fh:
        fh.write(json.dumps({"outcome": outcome, "body": body, "answer": answer}, ensure_ascii=False,
                            default=str) + "\n")


_REJECT_TXN = ("otp", "unknown")  # serving/qa.py REJECT_TXN (not imported: parse must not import serving)


def _as_answer(a):
    """A cached / fresh answer as the backend interface's dict: a row of the nine decoded
    field strings (the local extractor's answers) becomes the rejection-nulled dict."""
    if isinstance(a, list) and len(a) == len(CORE_FIELDS):
        return _null_rejection(dict(zip(CORE_FIELDS, a)))
    return a


def _null_rejection(answer: Dict[str, Any]) -> Dict[str, Any]:
    """serving/qa.py null_rejection: a non-transaction class nulls every other field."""
    if answer.get("txn_type") in _REJECT_TXN:
        return {k: (v if k == "txn_type" else None) for k, v in answer.items()}
    return answer


class BrokenMessage(Exception):
    """The SMS parsed but carries no usable card number (gemini_parser.py:20-22)."""


class Outcome(str, enum.Enum):
    PARSED = "parsed"
    UNMATCHED = "unmatched"
    BROKEN = "broken"
    ERROR = "error"


@dataclass
class ParseResult:
    outcome: Outcome
    parsed: Optional[ParsedSMS] = None
    error: Optional[BaseException] = None
    cached: bool = False
    # the native path's PARSED result: the sms.parsed payload itself (parse/fastpath.py;
    # byte-identical to parsed_wire(parsed), future dates already excluded), no ParsedSMS
    wire: Optional[bytes] = None


def postprocess_answer(raw: RawSMS, fixed_body: str, answer: Dict[str, Any], tz: str = DEFAULT_TZ) -> ParseResult:
    """Turn one raw extraction answer into a :class:`ParseResult`."""
    resp = canonicalize_answer(answer)  # currency symbols, day-first slash dates (parse/canonical.py)
    try:
        try:
            resp["date"] = parse_custom_datetime(resp["date"])
        except Exception as exc:
            if "String does not contain a date" in str(exc):
                resp["date"] = parse_unix_timestamp(int(raw.date), tz=tz, aware=False)
        resp["date"] = fix_broken_datetime(raw.body, resp["date"])
        # D8 (kept for parity): a null card raises here, so it lands in the DLQ as
        # "unmatched"; only card *strings* shorter than 4 chars reach BROKEN below.
        card = resp["card"].replace("*", "").replace(" ", "")
        resp["card"] = card = card[:4] if len(card) > 4 else card
        amount = resp["amount"] = parse_ambiguous_decimal(str(resp["amount"]))
        resp["balance"] = parse_ambiguous_decimal(str(resp["balance"]))
        if len(card) < 4:
            # the schema check first (a malformed answer stays UNMATCHED), then BROKEN
            ParsedSmsCore.model_validate(resp)
            return ParseResult(Outcome.BROKEN, error=BrokenMessage("no card number in message"))
        # ONE validation builds the ParsedSMS: it checks every field ParsedSmsCore would
        # (same types; the schema's required keys and amount >= 0 are checked here), so
        # the answer is not validated twice (~3.7 us per message)
        if len(resp) != _N_CORE and any(k not in resp for k in CORE_FIELDS):
            ParsedSmsCore.model_validate(resp)  # raises its "field required" error
        if amount is not None and amount < 0:
            ParsedSmsCore.model_validate(resp)  # raises its "greater than or equal to 0" error
        address = resp["address"]
        parsed = ParsedSMS(
            msg_id=raw.msg_id,
            device_id=raw.device_id,
            sender=raw.sender,
            date=resp["date"],
            raw_body=fixed_body,
            txn_type=resp["txn_type"],
            amount=amount,
            currency=resp["currency"],
            card=card[:4] if len(card) > 4 else card,
            merchant=resp["merchant"],
            city=resp["city"],
            address="" if address == "null" else address,
            balance=resp["balance"],
            parser_version=PARSER_VERSION_LLM,
        )
    except Exception as exc:
        if resp.get("txn_type") != "otp":
            sentry_capture(exc, extras={"raw_body": raw.body[:4096]})
        return ParseResult(Outcome.UNMATCHED, error=exc)
    return ParseResult(Outcome.PARSED, parsed=parsed)


class ParsePipeline:
    """Stateless-per-message, batched parse engine around one backend."""

    def __init__(self, backend: ParserBackend, cache: Optional[ResponseCache] = None,
                 tz: str = DEFAULT_TZ) -> None:
        self.backend = backend
        self.cache = cache if cache is not None else MemoryKV()
        self.tz = tz
        self.backend_calls = 0
        self.backend_seconds = 0.0

    async def parse(self, raw: RawSMS) -> ParseResult:
        return (await self.parse_batch([raw]))[0]

    async def parse_batch(self, raws: Sequence[RawSMS]) -> List[ParseResult]:
        t_start = time.perf_counter()
        n = len(raws)
        results: List[Optional[ParseResult]] = [None] * n
        bodies: List[Optional[str]] = [None] * n
        keys: List[Optional[str]] = [None] * n
        todo: List[int] = []
        for i, raw in enumerate(raws):
            if type(raw) is fastpath.FastRaw:  # no keyword can match; body normalised and keyed natively
                bodies[i] = raw.norm
                keys[i] = raw.key
            else:
                if llm_should_skip(raw.body):
                    results[i] = ParseResult(Outcome.UNMATCHED)
                    continue
                fb = normalize_body(raw.body)
                bodies[i] = fb
                keys[i] = cache_key(fb)
            todo.append(i)
        # the native post-processing needs the answers as rows: backends that give them
        rows_api = getattr(self.backend, "extract_rows", None) if fastpath.available() else None
        rows: Dict[int, List[str]] = {}

        answers: Dict[int, Any] = {}
        cached: set = set()
        if todo:
            hits = self.cache.get_many([keys[i] for i in todo])  # type: ignore[misc]
            miss: List[int] = []
            for i, h in zip(todo, hits):
                if h is None:
                    miss.append(i)
                else:
                    answers[i] = h
                    cached.add(i)
            if miss:
                # One backend call per unique body (duplicates in a batch share it).
                uniq: Dict[str, List[int]] = {}
                for i in miss:
                    uniq.setdefault(bodies[i], []).append(i)  # type: ignore[arg-type]
                ubodies = list(uniq)
                t0 = time.perf_counter()
                try:
                    got = await (rows_api or self.backend.extract_batch)(ubodies)
                except TransientError:
                    raise  # backend unreachable: the stage naks the batch and retries it
                except Exception as exc:  # whole-batch failure
                    got = [exc] * len(ubodies)
                for r in got:
                    if isinstance(r, TransientError):
                        raise r
                self.backend_calls += 1
                self.backend_seconds += time.perf_counter() - t0
                to_cache = []
                for b, r in zip(ubodies, got):
                    if rows_api is not None and isinstance(r, list):
                        for i in uniq[b]:
                            rows[i] = r
                        # the nine decoded strings stand for the answer (cached raw, D7):
                        # _as_answer() makes the backend interface's dict only where the
                        # Python path or a cache reader needs it
                    elif not isinstance(r, BaseException) and not isinstance(r, dict):
                        r = BackendError(f"backend returned {type(r).__name__}, not a JSON object")
                    for i in uniq[b]:
                        answers[i] = r
                    if isinstance(r, (dict, list)):
                        to_cache.append((keys[uniq[b][0]], r))
                if to_cache:
                    self.cache.put_many(to_cache)

        # native post-processing of the fresh answers of natively scanned messages:
        # the sms.parsed payload, an unmatched verdict, or (FALLBACK) the Python path below
        if rows:
            nat = [i for i in todo if i in rows and isinstance(raws[i], fastpath.FastRaw)]
            if nat:
                for i, res in zip(nat, fastpath.postprocess([rows[i] for i in nat], [raws[i] for i in nat])):
                    if isinstance(res, bytes):
                        results[i] = ParseResult(Outcome.PARSED, wire=res)
                    elif res == fastpath.UNMATCHED:  # a non-transaction class: null fields
                        err = AttributeError("'NoneType' object has no attribute 'replace'")
                        if rows[i][0] != "otp":  # (the Python path's capture rule)
                            sentry_capture(err, extras={"raw_body": raws[i].body[:4096]})
                        results[i] = ParseResult(Outcome.UNMATCHED, error=err)

        for i in todo:
            if results[i] is not None:
                continue
            ans = _as_answer(answers[i])
            if isinstance(ans, BaseException):
                sentry_capture(ans, extras={"raw_body": raws[i].body[:4096]})
                results[i] = ParseResult(Outcome.ERROR, error=ans)
            else:
                r = postprocess_answer(raws[i], bodies[i], ans, self.tz)  # type: ignore[arg-type]
                r.cached = i in cached
                results[i] = r
                if _DEBUG_DIR and r.outcome is not Outcome.PARSED:
                    _debug_record(bodies[i], ans, r.outcome.value)
        # One observation per message, like the reference's per-message timer around
        # parse_sms_llm (worker.py:130-133, metrics.py:48-53): _count == messages
        # parsed.  The value is the latency each message experienced — the wall time
        # of the batched parse it was part of.
        observe_many(GEMINI_LATENCY, time.perf_counter() - t_start, n)
        return results  # type: ignore[return-value]
