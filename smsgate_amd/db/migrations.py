"""Ordered schema migrations with a version table (the reference uses Alembic,
db/migrations/, six revisions ending at ``dcbadcb88d59``; alembic is not on
the image).

Commands mirror the reference's makefile targets (makefile:40-70):
``upgrade`` (to head or a target), ``downgrade`` (one step / to a target /
``base``), ``current``, ``history``, ``stamp``.  Run as
``python -m smsgate_amd db upgrade`` with ``DATABASE_URL`` (or the
``POSTGRES_*`` settings).

Our chain starts from nothing and reaches the reference's head schema in two
steps.  A database created by the reference's Alembic chain (an
``alembic_version`` table) is upgraded from **whichever of its six revisions it
is at** — see :data:`REFERENCE_REVISIONS` and :func:`upgrade_from_reference`:
the table is rebuilt into the head schema in one transaction, carrying every
row across the renames the reference made by drop-and-add (and so lost data
on): ``original_body -> raw_body -> original_body`` (f1a93be77048,
007078d0ce44), ``datetime -> date -> datetime`` (f1a93be77048, dcbadcb88d59),
and ``original_key -> msg_id`` with the unique constraint moved
(f1ebe9c5dea6).  ``stamp dcbadcb88d59`` still marks a reference-head database
as ours without touching it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

from sqlalchemy import Column, MetaData, String, Table, inspect, text
from sqlalchemy.engine import Connection, Engine

from .schema import sms_data

__all__ = ["Migration", "MIGRATIONS", "current", "upgrade", "downgrade", "stamp", "history", "REFERENCE_HEAD",
           "REFERENCE_REVISIONS", "reference_revision", "upgrade_from_reference"]

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


# The reference's Alembic chain (db/migrations/versions/*.py), oldest first, and for
# each revision the SQL expression (over that revision's sms_data columns) of each
# head column whose name or existence changed.  Columns not listed keep their name.
#   ab372595639c  create: original_key (unique), original_body, datetime, ...
#   f1a93be77048  + raw_body, date, msg_id (index), device_id, parser_version;
#                 - datetime, original_body   (the reference dropped the data)
#   80b70406bdea  - msg_id
#   f1ebe9c5dea6  + msg_id (unique), - original_key
#   007078d0ce44  + original_body, - raw_body
#   dcbadcb88d59  + datetime, - date          (head)
REFERENCE_REVISIONS: Dict[str, Dict[str, str]] = {
    "ab372595639c": {"msg_id": "original_key", "original_body": "original_body", "datetime": "datetime",
                     "device_id": "NULL", "parser_version": "NULL"},
    "f1a93be77048": {"msg_id": "COALESCE(msg_id, original_key)", "original_body": "raw_body", "datetime": "date",
                     "device_id": "device_id", "parser_version": "parser_version"},
    "80b70406bdea": {"msg_id": "original_key", "original_body": "raw_body", "datetime": "date",
                     "device_id": "device_id", "parser_version": "parser_version"},
    "f1ebe9c5dea6": {"msg_id": "msg_id", "original_body": "raw_body", "datetime": "date",
                     "device_id": "device_id", "parser_version": "parser_version"},
    "007078d0ce44": {"msg_id": "msg_id", "original_body": "original_body", "datetime": "date",
                     "device_id": "device_id", "parser_version": "parser_version"},
    REFERENCE_HEAD: {"msg_id": "msg_id", "original_body": "original_body", "datetime": "datetime",
                     "device_id": "device_id", "parser_version": "parser_version"},
}


def reference_revision(c: Connection) -> Optional[str]:
    """The reference Alembic revision of this database, or None (no ``alembic_version``)."""
    if "alembic_version" not in inspect(c).get_table_names():
        return None
    return c.execute(text("SELECT version_num FROM alembic_version")).scalar()


def upgrade_from_reference(c: Connection, rev: str) -> int:
    """Rebuild ``sms_data`` of a database at reference revision ``rev`` into the head
    schema, keeping every row; returns the number of rows carried over.

    Rows whose ``msg_id`` would collide (possible at f1a93be77048, where msg_id was
    not unique) keep the newest (highest ``id``).  Afterwards ``alembic_version``
    says ``dcbadcb88d59`` (the schema *is* the reference head's) and our version
    table says :data:`HEAD`."""
    if rev not in REFERENCE_REVISIONS:
        raise KeyError(f"unknown reference revision {rev!r}")
    mapping = REFERENCE_REVISIONS[rev]
    head_cols = [col.name for col in sms_data.columns]
    sel = ", ".join(f"{mapping.get(n, n)} AS {n}" for n in head_cols)
    key = mapping["msg_id"]
    # carry the rows aside, then recreate sms_data under its own name: the primary key,
    # the unique constraint and (Postgres) the id sequence get the names Alembic's chain
    # gave them (sms_data_pkey, sms_data_id_seq), not the names of a renamed copy
    c.execute(text(
        f"CREATE TABLE sms_data__carry AS SELECT {sel} FROM sms_data "
        f"WHERE ({key}) IS NULL OR id IN (SELECT MAX(id) FROM sms_data GROUP BY {key})"))
    c.execute(text("DROP TABLE sms_data"))
    _create_table(c)
    c.execute(text(f"INSERT INTO sms_data ({', '.join(head_cols)}) SELECT {', '.join(head_cols)} FROM sms_data__carry"))
    c.execute(text("DROP TABLE sms_data__carry"))
    n = int(c.execute(text("SELECT COUNT(*) FROM sms_data")).scalar() or 0)
    _reset_id_sequence(c)
    _create_indexes(c)
    c.execute(text("UPDATE alembic_version SET version_num = :v"), {"v": REFERENCE_HEAD})
    _set(c, HEAD)
    return n


def _reset_id_sequence(c: Connection) -> None:
    """After rows were inserted with explicit ids: move Postgres' serial sequence past
    MAX(id), so the writer's INSERT (which never passes ``id``) does not collide with
    a carried row.  SQLite's INTEGER PRIMARY KEY continues from MAX(rowid) by itself."""
    if c.dialect.name == "postgresql":
        c.execute(text("SELECT setval(pg_get_serial_sequence('sms_data', 'id'), "
                       "COALESCE(MAX(id), 1), MAX(id) IS NOT NULL) FROM sms_data"))


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
        cur_rev = c.execute(_version_table(c).select()).scalar()
        if cur_rev is None:
            ref = reference_revision(c)
            if ref is not None and "sms_data" in inspect(c).get_table_names():
                # a database the reference's Alembic chain created: carry it to our head
                upgrade_from_reference(c, ref)
                cur_rev = HEAD
        cur = _index(cur_rev)
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
