"""SQL schema of the ``sms_data`` table (db/models.py:11-39 of the reference).

Columns (head revision ``dcbadcb88d59`` of the reference's alembic chain):
``id`` int PK; ``msg_id`` unique (nullable); ``original_body``; ``sender`` NOT
NULL; ``datetime`` timestamptz NOT NULL; ``card`` varchar(4) NOT NULL;
``amount`` numeric(14,2) NOT NULL; ``currency`` varchar(3) NOT NULL;
``txn_type`` NOT NULL; ``balance`` numeric(14,2); ``merchant``, ``address``,
``city``, ``device_id``, ``parser_version``.  Indexes on sender, datetime,
txn_type.

Written with SQLAlchemy Core so one definition serves PostgreSQL (production)
and SQLite (tests, single-box deployments); both dialects provide
``INSERT … ON CONFLICT (msg_id) DO UPDATE``.
"""
from __future__ import annotations

from typing import Any, Dict

from sqlalchemy import Column, DateTime, Index, Integer, MetaData, Numeric, String, Table

from ..models.domain import ParsedSMS

__all__ = ["metadata", "sms_data", "parsed_to_row", "UPSERT_EXCLUDED"]

metadata = MetaData()

sms_data = Table(
    "sms_data",
    metadata,
    Column("id", Integer, primary_key=True, autoincrement=True),
    Column("msg_id", String, unique=True, nullable=True),
    Column("original_body", String, nullable=True),
    Column("sender", String, nullable=False),
    Column("datetime", DateTime(timezone=True), nullable=False),
    Column("card", String(4), nullable=False),
    Column("amount", Numeric(14, 2), nullable=False),
    Column("currency", String(3), nullable=False),
    Column("txn_type", String, nullable=False),
    Column("balance", Numeric(14, 2), nullable=True),
    Column("merchant", String, nullable=True),
    Column("address", String, nullable=True),
    Column("city", String, nullable=True),
    Column("device_id", String, nullable=True),
    Column("parser_version", String, nullable=True),
    Index("idx_sms_sender", "sender"),
    Index("idx_sms_datetime", "datetime"),
    Index("idx_sms_txn_type", "txn_type"),
)

#: columns never overwritten by an upsert (upsert.py:22-29)
UPSERT_EXCLUDED = ("id", "msg_id")


def parsed_to_row(p: ParsedSMS) -> Dict[str, Any]:
    """ParsedSMS → row dict: ``date→datetime``, ``raw_body→original_body`` (upsert.py:16-18)."""
    return {
        "msg_id": p.msg_id,
        "original_body": p.raw_body,
        "sender": p.sender,
        "datetime": p.date,
        "card": p.card,
        "amount": p.amount,
        "currency": p.currency,
        "txn_type": p.txn_type.value if hasattr(p.txn_type, "value") else p.txn_type,
        "balance": p.balance,
        "merchant": p.merchant,
        "address": p.address,
        "city": p.city,
        "device_id": p.device_id,
        "parser_version": p.parser_version,
    }
