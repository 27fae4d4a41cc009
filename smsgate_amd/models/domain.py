"""Wire-level domain objects shared by every stage of the pipeline.

These are byte-compatible with the reference's JSON contracts
(``libs/models.py:35-109``, ``libs/llm_core.py:9-19``):

* :class:`RawSMS` travels on ``sms.raw``;
* :class:`ParsedSMS` travels on ``sms.parsed`` / ``sms.processing``
  (naive ISO dates, ``Decimal`` serialised as a string, upper-cased currency,
  exactly-4-char card);
* :class:`ParsedSmsCore` is the mini-schema an extraction backend must fill.

Message identities keep the reference's two quirks (D9): the HTTP gateway uses
``md5(message)`` (api_gateway/main.py:113) and the XML importer uses
``sha1(body)`` (watcher.py:45).
"""
from __future__ import annotations

import datetime as _dt
import hashlib
from decimal import Decimal
from enum import Enum
from typing import Literal, Optional

from pydantic import BaseModel, Field, StringConstraints, field_serializer
from typing_extensions import Annotated

# upper-cased by pydantic-core itself (the reference's validator, `v.upper() if v else v`,
# as a Python callback cost a GIL round trip inside every Rust validation)
_UpperStr = Annotated[str, StringConstraints(to_upper=True)]

__all__ = [
    "TxnType",
    "RawSMS",
    "ParsedSMS",
    "ParsedSmsCore",
    "get_md5_hash",
    "get_sha1_hash",
    "PARSER_VERSION_LLM",
    "CORE_FIELDS",
    "parsed_wire",
    "raw_wire",
    "LazyParsedSMS",
    "as_parsed",
]

PARSER_VERSION_LLM = "llm-0.2.0"  # gemini_parser.py:267


class TxnType(str, Enum):
    """Transaction class an SMS is mapped to."""

    DEBIT = "debit"
    CREDIT = "credit"
    OTP = "otp"
    UNKNOWN = "unknown"


class RawSMS(BaseModel):
    """An ingested, not-yet-understood SMS (``sms.raw`` payload)."""

    msg_id: str
    sender: str = Field(..., min_length=1)
    body: str = Field(..., min_length=1)
    date: str
    device_id: Optional[str] = None
    source: Literal["device", "xml"] = "device"


class ParsedSMS(BaseModel):
    """A fully normalised transaction (``sms.parsed`` payload)."""

    msg_id: str
    device_id: Optional[str]
    sender: str
    date: _dt.datetime
    raw_body: str

    txn_type: TxnType
    amount: Optional[Decimal] = None
    currency: Optional[_UpperStr] = None
    card: Optional[str] = Field(None, min_length=4, max_length=4)

    merchant: Optional[str] = None
    city: Optional[str] = None
    address: Optional[str] = None

    balance: Optional[Decimal] = None

    parser_version: str = "0.1.0"

    # amount / balance: pydantic-core's JSON form of a Decimal is str(v), the reference's
    # serializer (libs/models.py), so no Python callback per field
    @field_serializer("date", when_used="json")
    def _iso(self, v: _dt.datetime) -> str:
        return v.isoformat()


def parsed_wire(p: "ParsedSMS") -> bytes:
    """The ``sms.parsed`` payload: ``p.model_dump_json()`` as UTF-8.  (A hand-built
    dict through ``json.JSONEncoder`` was tried: 12.5 vs 7.9 us per message with
    pydantic-core's serializer on the mixed-layout traffic, Cyrillic included.)"""
    return p.model_dump_json().encode("utf-8")


class LazyParsedSMS:
    """An sms.parsed payload the writer validated natively (parse/fastpath.py
    ``peek_parsed``: the canonical form of a valid ParsedSMS, every field checked); the
    :class:`ParsedSMS` object is built from the same bytes on first use (a sink that
    reads fields, :meth:`model`).  Its attributes are the model's."""
    __slots__ = ("msg_id", "_data", "_model")

    def __init__(self, msg_id: str, data: bytes) -> None:
        self.msg_id = msg_id
        self._data = data
        self._model: Optional[ParsedSMS] = None

    def model(self) -> ParsedSMS:
        if self._model is None:
            self._model = ParsedSMS.model_validate_json(self._data)
        return self._model

    def __getattr__(self, name: str):
        return getattr(self.model(), name)

    def __eq__(self, other) -> bool:
        return self.model() == (other.model() if isinstance(other, LazyParsedSMS) else other)

    __hash__ = None  # type: ignore[assignment]


def as_parsed(r) -> "ParsedSMS":
    """The ParsedSMS of a sink record (a :class:`LazyParsedSMS` or the model itself)."""
    return r.model() if isinstance(r, LazyParsedSMS) else r


def raw_wire(r: "RawSMS") -> bytes:
    """The ``sms.raw`` payload: ``r.model_dump_json()`` as UTF-8 (4.4 vs 6.7 us)."""
    return r.model_dump_json().encode("utf-8")


class ParsedSmsCore(BaseModel):
    """The extraction schema (what an LLM backend must produce)."""

    txn_type: TxnType
    date: _dt.datetime
    amount: Optional[Decimal] = Field(None, ge=0)
    currency: Optional[str]
    card: Optional[str]
    merchant: Optional[str]
    city: Optional[str]
    address: Optional[str]
    balance: Optional[Decimal]


#: Field order of the extraction schema — shared by prompts, FSM decoding and
#: the Gemini response schema (gemini_parser.py:46-61).
CORE_FIELDS = tuple(ParsedSmsCore.model_fields)


def get_md5_hash(text: str) -> str:
    """Gateway message id: hex md5 of the UTF-8 body (libs/models.py:97-109)."""
    return hashlib.md5(text.encode("utf-8")).hexdigest()


def get_sha1_hash(text: str) -> str:
    """XML-import message id: hex sha1 of the UTF-8 body (watcher.py:45)."""
    return hashlib.sha1(text.encode("utf-8")).hexdigest()
