"""Ordered schema migrations with a version table (the reference uses Alembic,
db/migrations/, six revisions ending at ``dcbadcb88d59``; alembic is not on
the image).

Commands mirror the reference's makefile targets (makefile:40-70):
``upgrade`` (to head or a target), ``downgrade`` (one step / to a target /
``base``), ``current``, ``history``, ``stamp``.  Run as
``python -m smsgate_amd db upgrade`` with ``DATABASE_URL`` (or the
``POSTGRES_*`` settings).

Our chain starts from nothing and reaches the reference's head schema in two
steps; ``stamp-reference`` marks a database that the reference's Alembic chain
already brought to ``dcbadcb88d59`` as being at our head without touching it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

from sqlalchemy import Column, MetaData, String, Table, inspect, text
from sqlalchemy.engine import Connection, Engine

from .schema import sms_data

__all__ = ["Migration", "MIGRATIONS", "current", "upgrade", "downgrade", "stamp", "history", "REFERENCE_HEAD"]

REFERENCE_HEAD = "dcbadcb88d59"
VERSION_TABLE = "smsgate_schema_version"


@dataclass(frozen=True)
class Migration:
    rev: str
    down: Optional[str]
    message: str
    up: Callable[[Connection], None]
    down_fn: Callable[[Connection], None]


def _create_table(c: Connection) -> None:
    cols = [col.copy() for col in sms_data.columns]
    Table("sms_data", MetaData(), *cols).create(c)


def _drop_table(c: Connection) -> None:
    c.execute(text("DROP TABLE IF EXISTS sms_data"))


def _create_indexes(c: Connection) -> None:
    for idx in sms_data.indexes:
        cols = ", ".join(col.name for col in idx.columns)
        c.execute(text(f"CREATE INDEX IF NOT EXISTS {idx.name} ON sms_data ({cols})"))


def _drop_indexes(c: Connection) -> None:
    for idx in sms_data.indexes:
        c.execute(text(f"DROP INDEX IF EXISTS {idx.name}"))


MIGRATIONS: List[Migration] = [
    Migration("0001_sms_data", None, "create sms_data (reference head schema)", _create_table, _drop_table),
    Migration("0002_sms_indexes", "0001_sms_data", "indexes on sender/datetime/txn_type", _create_indexes, _drop_indexes),
]
HEAD = MIGRATIONS[-1].rev


def _version_table(c: Connection) -> Table:
    md = MetaData()
    t = Table(VERSION_TABLE, md, Column("version", String, primary_key=True))
    md.create_all(c)
    return t


def current(engine: Engine) -> Optional[str]:
    with engine.begin() as c:
        t = _version_table(c)
        row = c.execute(t.select()).first()
        return row[0] if row else None


def _set(c: Connection, rev: Optional[str]) -> None:
    t = _version_table(c)
    c.execute(t.delete())
    if rev is not None:
        c.execute(t.insert().values(version=rev))


def _index(rev: Optional[str]) -> int:
    if rev is None:
        return -1
    for i, m in enumerate(MIGRATIONS):
        if m.rev == rev:
            return i
    raise KeyError(f"unknown revision {rev!r}")


def upgrade(engine: Engine, target: str = "head") -> Optional[str]:
    tgt = len(MIGRATIONS) - 1 if target == "head" else _index(target)
    with engine.begin() as c:
        cur = _index(c.execute(_version_table(c).select()).scalar())
        for i in range(cur + 1, tgt + 1):
            MIGRATIONS[i].up(c)
            _set(c, MIGRATIONS[i].rev)
    return current(engine)


def downgrade(engine: Engine, target: str = "-1") -> Optional[str]:
    with engine.begin() as c:
        cur = _index(c.execute(_version_table(c).select()).scalar())
        if target == "base":
            tgt = -1
        elif target.startswith("-"):
            tgt = max(-1, cur - int(target[1:]))
        else:
            tgt = _index(target)
        for i in range(cur, tgt, -1):
            MIGRATIONS[i].down_fn(c)
            _set(c, MIGRATIONS[i].down)
    return current(engine)


def stamp(engine: Engine, rev: str) -> None:
    with engine.begin() as c:
        if rev == REFERENCE_HEAD:
            if "sms_data" not in inspect(c).get_table_names():
                raise RuntimeError("no sms_data table: the database is not at the reference head")
            rev = HEAD
        _set(c, None if rev == "base" else MIGRATIONS[_index(rev)].rev)


def history() -> List[str]:
    return [f"{m.down or '<base>'} -> {m.rev}: {m.message}" for m in MIGRATIONS]
