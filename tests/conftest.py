"""Shared fixtures. GPU tests are marked ``@pytest.mark.gpu`` and run on an MI355X box."""
from __future__ import annotations

import asyncio
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("SMSGATE_TRACE", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


def run(coro):
    return asyncio.run(coro)


@pytest.fixture
def arun():
    return run


@pytest.fixture(autouse=True)
def _isolate_settings(tmp_path, monkeypatch):
    """Each test gets fresh settings rooted in a temp dir (no stray ./backups)."""
    from smsgate_amd import config

    monkeypatch.setenv("BACKUP_DIR", str(tmp_path / "backups"))
    monkeypatch.setenv("LOG_DIR", str(tmp_path / "logs"))
    # the parse pipeline's response cache: one per test (a shared file would let one
    # test's cached answer skip another test's backend call)
    monkeypatch.setenv("PARSER_CACHE_PATH", str(tmp_path / "parser_cache.sqlite"))
    config.reset_settings()
    from smsgate_amd import bus

    bus.reset_connections()
    yield
    config.reset_settings()
    bus.reset_connections()


REFERENCE_CASES = [
    (
        "APPROVED PURCHASE DB SALE: TEST LLC, MOSKOW, "
        "TEST STR. 29, 24 AREA,06.05.25 14:23,card ***0018. "
        "Amount:52.00 USD, Balance:1842.74 USD",
        dict(merchant="TEST LLC", city="MOSKOW", address="TEST STR. 29, 24 AREA", amount="52.00",
             balance="1842.74", date=(2025, 5, 6, 14, 23), card="0018", currency="USD"),
    ),
    (
        "APPROVED PURCHASE DB SALE: TEST, MOSKOW,"
        "06.05.25 15:11,card ***0018. Amount:3460.00 USD, "
        "Balance:1800.74 USD",
        dict(merchant="TEST", city="MOSKOW", address="", amount="3460.00", balance="1800.74",
             date=(2025, 5, 6, 15, 11), card="0018", currency="USD"),
    ),
    (
        "DEBIT ACCOUNT&#10;27,252.00 AMD&#10;4083***7538,&#10;AMERIABANK API GATE, AM"
        "&#10;10.06.2025 20:51&#10;BALANCE: 391,469.09 AMD",
        dict(merchant="AMERIABANK API GATE", city="AM", address="", amount="27252.00", balance="391469.09",
             date=(2025, 6, 10, 20, 51), card="7538", currency="AMD"),
    ),
]


async def drain(bus, subject):
    """Read (and ack) everything currently on ``subject`` as JSON."""
    import json

    sub = await bus.subscribe(subject, "inspect-" + subject.replace(".", "-"))
    out = []
    while True:
        got = await sub.fetch(100, 0.05)
        if not got:
            return out
        for m in got:
            await m.ack()
            out.append(json.loads(m.data))
