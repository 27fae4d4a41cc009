"""Process-wide settings, read from the environment and an optional ``.env`` file.

Parity with ``libs/config.py:25-113`` of the reference: the same field names
(environment variable = upper-cased field name, matched case-insensitively),
the same defaults, the computed ``database_url``/``database_url_async`` DSNs,
the ``backup_dir`` mkdir side effect (config.py:59-62) and a cached singleton
:func:`get_settings`.

Deliberate differences (documented fixes):

* ``pydantic-settings`` is not installed on the target image, so the loader
  is a ~60-line in-repo replacement (:func:`read_env_file` + :meth:`Settings.load`).
* Fields that were *required* in the reference (``pb_email``, ``tg_bot_token``,
  ``postgres_*``, ``log_dir`` …) have harmless defaults, so a service that does
  not need PocketBase/Telegram/Postgres can start without them.  Services
  that do need them validate at their own start-up.
* ``nats_dsn`` keeps its reference name; its default points at the in-repo bus
  (``memory://``) instead of the stale ``redis://`` URL (config.py:27).
* ``database_url_override`` (``DATABASE_URL``) lets the SQL sink run on SQLite
  where no Postgres driver exists (asyncpg/psycopg2 are not on the image).
"""
from __future__ import annotations

import json
import os
import threading
from pathlib import Path
from typing import Any, Dict, Mapping, Optional

from pydantic import BaseModel, ConfigDict, computed_field, model_validator

__all__ = ["Settings", "get_settings", "reset_settings", "read_env_file"]


def read_env_file(path: str | os.PathLike[str]) -> Dict[str, str]:
    """Parse a dotenv file: ``KEY=VALUE`` lines, ``#`` comments, optional quotes.

    Keys are lower-cased (settings matching is case-insensitive).  Missing files
    yield an empty mapping.
    """
    p = Path(path)
    if not p.is_file():
        return {}
    out: Dict[str, str] = {}
    for raw in p.read_text(encoding="utf-8").splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[len("export "):].lstrip()
        key, sep, val = line.partition("=")
        if not sep:
            continue
        val = val.strip()
        if len(val) >= 2 and val[0] == val[-1] and val[0] in "\"'":
            val = val[1:-1]
        elif " #" in val:
            val = val.split(" #", 1)[0].rstrip()
        out[key.strip().lower()] = val
    return out


class Settings(BaseModel):
    """All knobs of every service (field name == env var name, case-insensitive)."""

    model_config = ConfigDict(extra="ignore", validate_default=True)

    # ── message bus (reference: NATS JetStream) ─────────────────────────────
    nats_dsn: str = "memory://"
    bus_dir: Path = Path("./.bus-data")
    stream_max_age_s: float = 3 * 24 * 3600.0  # nats_utils.py:75
    ack_wait_s: float = 30.0

    # ── PocketBase ──────────────────────────────────────────────────────────
    pb_url: str = "http://127.0.0.1:8090"
    pb_email: str = ""
    pb_password: str = ""

    # ── Sentry ──────────────────────────────────────────────────────────────
    sentry_dsn: Optional[str] = None
    enable_sentry: bool = False
    gemini_api_key: Optional[str] = None
    gemini_model: str = "gemini-2.5-flash-preview-05-20"  # gemini_parser.py:27

    # ── parser backend selection (new: the reference hard-wires Gemini) ─────
    parser_backend: str = "gemini_http"
    parser_cache_path: str = ".gemini_cache.sqlite"
    parser_concurrency: int = 8
    parser_batch_size: int = 64
    # keyword skip filters: "word" (default; a keyword must stand as a word) or
    # "substring" (the reference's exact behaviour, worker.py:112-121) -- parse/text.py
    parser_keyword_match: str = "word"
    llm_model: str = "smollm-135m"
    llm_checkpoint: Optional[str] = None
    llm_device: str = "cuda"

    # ── XML-backup watcher ──────────────────────────────────────────────────
    backup_dir: Path = Path("./backups")
    xml_scan_interval_s: float = 10.0  # watcher.py:31

    # ── ngrok / API gateway ─────────────────────────────────────────────────
    enable_ngrok: bool = False
    ngrok_authtoken: Optional[str] = None
    ngrok_domain: Optional[str] = None
    api_host: Optional[str] = "0.0.0.0"
    api_port: Optional[int] = 9001

    # ── Prometheus ports ────────────────────────────────────────────────────
    api_metrics_port: int = 9101
    parser_metrics_port: int = 9102
    pbwriter_metrics_port: int = 9103

    # ── Telegram notifier ───────────────────────────────────────────────────
    tg_bot_token: str = ""
    tg_chat_ids: str = ""
    check_interval_seconds: int = 3600  # dashboard/main.py:72

    log_dir: str = "./.logs"

    # ── SQL persistence ─────────────────────────────────────────────────────
    postgres_user: str = "postgres"
    postgres_password: str = ""
    postgres_db: str = "smsgate"
    postgres_host: str = "localhost"
    postgres_port: int = 5432
    database_url_override: Optional[str] = None

    mcp_host: str = "0.0.0.0"
    mcp_port: int = 9122  # mcp_server/server.py:125

    @model_validator(mode="after")
    def _make_dirs(self) -> "Settings":
        # Same side effect as config.py:59-62.
        self.backup_dir.mkdir(parents=True, exist_ok=True)
        return self

    @computed_field  # type: ignore[prop-decorator]
    @property
    def database_url(self) -> str:
        if self.database_url_override:
            return self.database_url_override
        return (
            "postgresql+psycopg2://"
            f"{self.postgres_user}:{self.postgres_password}"
            f"@{self.postgres_host}:{self.postgres_port}/{self.postgres_db}"
        )

    @computed_field  # type: ignore[prop-decorator]
    @property
    def database_url_async(self) -> str:
        if self.database_url_override:
            return self.database_url_override
        return (
            "postgresql+asyncpg://"
            f"{self.postgres_user}:{self.postgres_password}"
            f"@{self.postgres_host}:{self.postgres_port}/{self.postgres_db}"
        )

    @property
    def allowed_chat_ids(self) -> set[int]:
        return {int(c.strip()) for c in self.tg_chat_ids.split(",") if c.strip()}

    @classmethod
    def load(
        cls,
        env: Optional[Mapping[str, str]] = None,
        env_file: str | os.PathLike[str] | None = ".env",
        **overrides: Any,
    ) -> "Settings":
        """Build settings: defaults < ``.env`` < process environment < overrides."""
        values: Dict[str, Any] = {}
        if env_file is not None:
            values.update(read_env_file(env_file))
        src = os.environ if env is None else env
        names = set(cls.model_fields)
        aliases = {"database_url": "database_url_override"}
        for k, v in src.items():
            lk = k.lower()
            lk = aliases.get(lk, lk)
            if lk in names:
                values[lk] = v
        for k, v in list(values.items()):
            if k in aliases:
                values[aliases[k]] = values.pop(k)
        values = {k: v for k, v in values.items() if k in names}
        # Empty strings in .env mean "unset" for optional fields.
        for k in list(values):
            if values[k] == "" and cls.model_fields[k].default is None:
                values.pop(k)
        values.update(overrides)
        return cls.model_validate(values)

    def dump(self) -> str:
        return json.dumps(self.model_dump(), indent=2, default=str)


_lock = threading.Lock()
_settings: Optional[Settings] = None


def get_settings() -> Settings:
    """Process-wide singleton (config.py:110-113)."""
    global _settings
    if _settings is None:
        with _lock:
            if _settings is None:
                _settings = Settings.load()
    return _settings


def reset_settings(new: Optional[Settings] = None) -> None:
    """Replace (or drop) the cached singleton — for tests and CLI overrides."""
    global _settings
    with _lock:
        _settings = new


if __name__ == "__main__":  # config.py:120-123
    print(get_settings().dump())
