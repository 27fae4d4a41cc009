"""Response cache keyed by ``sha256(normalised body)``.

The reference keeps raw LLM answers in a ``diskcache`` directory
(``.gemini_cache``, gemini_parser.py:33, :207-222) so replays never pay the
LLM again while post-processing fixes still apply.
``diskcache`` is not on the image, so :class:`SqliteKV` is a small sqlite3 KV
(WAL mode, one table, JSON values) with the same role; :class:`MemoryKV` is an
LRU for tests and benchmarks.  Both expose batched ``get_many``/``put_many``
so the parser stage does one round trip per batch, not per message.
"""
from __future__ import annotations

import hashlib
import json
import sqlite3
import threading
from collections import OrderedDict
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

__all__ = ["cache_key", "ResponseCache", "MemoryKV", "SqliteKV", "open_cache"]


def cache_key(fixed_body: str) -> str:
    return hashlib.sha256(fixed_body.encode()).hexdigest()


class ResponseCache:
    def get_many(self, keys: Sequence[str]) -> List[Optional[Any]]:
        raise NotImplementedError

    def put_many(self, items: Iterable[Tuple[str, Any]]) -> None:
        raise NotImplementedError

    def get(self, key: str) -> Optional[Any]:
        return self.get_many([key])[0]

    def put(self, key: str, value: Any) -> None:
        self.put_many([(key, value)])

    def __contains__(self, key: str) -> bool:
        return self.get(key) is not None

    def __len__(self) -> int:
        raise NotImplementedError

    def close(self) -> None:
        pass


class MemoryKV(ResponseCache):
    def __init__(self, capacity: int = 1 << 20) -> None:
        self._d: "OrderedDict[str, Any]" = OrderedDict()
        self._cap = capacity
        self._lock = threading.Lock()

    def get_many(self, keys: Sequence[str]) -> List[Optional[Any]]:
        with self._lock:
            out = []
            for k in keys:
                v = self._d.get(k)
                if v is not None:
                    self._d.move_to_end(k)
                out.append(v)
            return out

    def put_many(self, items: Iterable[Tuple[str, Any]]) -> None:
        with self._lock:
            for k, v in items:
                self._d[k] = v
                self._d.move_to_end(k)
            while len(self._d) > self._cap:
                self._d.popitem(last=False)

    def __len__(self) -> int:
        return len(self._d)


class SqliteKV(ResponseCache):
    def __init__(self, path: str | Path) -> None:
        self._path = str(path)
        self._lock = threading.Lock()
        self._db = sqlite3.connect(self._path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("PRAGMA synchronous=NORMAL")
        self._db.execute("CREATE TABLE IF NOT EXISTS kv (k TEXT PRIMARY KEY, v TEXT NOT NULL)")

    def get_many(self, keys: Sequence[str]) -> List[Optional[Any]]:
        if not keys:
            return []
        found: Dict[str, Any] = {}
        with self._lock:
            for i in range(0, len(keys), 500):
                chunk = list(keys[i:i + 500])
                q = "SELECT k, v FROM kv WHERE k IN (%s)" % ",".join("?" * len(chunk))
                for k, v in self._db.execute(q, chunk):
                    found[k] = json.loads(v)
        return [found.get(k) for k in keys]

    def put_many(self, items: Iterable[Tuple[str, Any]]) -> None:
        rows = [(k, json.dumps(v, ensure_ascii=False, default=str)) for k, v in items]
        if not rows:
            return
        with self._lock:
            self._db.execute("BEGIN")
            self._db.executemany("INSERT OR REPLACE INTO kv (k, v) VALUES (?, ?)", rows)
            self._db.execute("COMMIT")

    def __len__(self) -> int:
        with self._lock:
            return int(self._db.execute("SELECT COUNT(*) FROM kv").fetchone()[0])

    def items(self) -> List[Tuple[str, Any]]:
        with self._lock:
            return [(k, json.loads(v)) for k, v in self._db.execute("SELECT k, v FROM kv ORDER BY k")]

    def close(self) -> None:
        with self._lock:
            self._db.close()


def open_cache(spec: Optional[str]) -> ResponseCache:
    """``None``/``''``/``memory`` → :class:`MemoryKV`; anything else is a sqlite path."""
    if not spec or spec == "memory" or spec == ":memory:":
        return MemoryKV()
    return SqliteKV(spec)
