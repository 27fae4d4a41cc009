"""XML backup importer (services/xml_watcher/watcher.py parity).

Every ``XML_SCAN_INTERVAL_S`` (10 s, watcher.py:31) scans ``BACKUP_DIR/*.xml``
(SMS Backup & Restore format: ``<smses><sms address=… date=<ms> body=…/>``),
maps each ``<sms>`` to ``RawSMS(source="xml", device_id="xml_backup",
msg_id=sha1(body), sender=address, date=UTC ISO)`` (watcher.py:35-54),
publishes them to ``sms.raw`` and moves the file to ``processed/``
(watcher.py:57-62, :84).  A failing file is reported and retried next scan.

Differences: parsing runs off the loop (``asyncio.to_thread``, as the
reference did), publishing is one batched round trip per file instead of two
broker RPCs per message, and the move is idempotent (an existing target is
replaced instead of crashing ``shutil.move``).  The stream is ensured once.
"""
from __future__ import annotations

import asyncio
import logging
import os
import shutil
import xml.etree.ElementTree as ET
from datetime import datetime, timezone
from pathlib import Path
from typing import Iterable, List, Optional

from ..bus.base import SUBJECT_RAW, Bus
from ..models.domain import RawSMS, get_sha1_hash
from ..obs.errors import sentry_capture

__all__ = ["iter_sms", "XmlWatcher", "move_to_processed"]

log = logging.getLogger("xml_watcher")


def iter_sms(xml_path: Path) -> Iterable[RawSMS]:
    root = ET.parse(xml_path).getroot()
    for elem in root.findall("sms"):
        body = elem.get("body", "")
        date_ms = int(elem.get("date", "0"))
        yield RawSMS(
            source="xml",
            device_id="xml_backup",
            msg_id=get_sha1_hash(body),
            sender=elem.get("address", ""),
            date=datetime.fromtimestamp(date_ms / 1000, tz=timezone.utc).isoformat(),
            body=body,
        )


def move_to_processed(src: Path, processed_dir: Path) -> Path:
    processed_dir.mkdir(parents=True, exist_ok=True)
    dst = processed_dir / src.name
    if dst.exists():
        dst.unlink()
    shutil.move(str(src), str(dst))
    return dst


class XmlWatcher:
    def __init__(self, bus: Bus, backup_dir: Path, interval_s: float = 10.0) -> None:
        self.bus = bus
        self.backup_dir = Path(backup_dir)
        self.processed_dir = self.backup_dir / "processed"
        self.interval_s = interval_s
        self.imported = 0
        self.failed_files = 0

    async def process_file(self, path: Path) -> int:
        try:
            msgs: List[RawSMS] = await asyncio.to_thread(lambda: list(iter_sms(path)))
            if msgs:
                await self.bus.publish_many([(SUBJECT_RAW, m.model_dump_json().encode()) for m in msgs])
            move_to_processed(path, self.processed_dir)
            self.imported += len(msgs)
            log.info("imported %d message(s) from %s", len(msgs), path)
            return len(msgs)
        except Exception as exc:  # noqa: BLE001 — retried on the next scan
            self.failed_files += 1
            sentry_capture(exc, extras={"file": str(path)})
            log.exception("failed to import %s", path)
            return 0

    async def scan_once(self) -> int:
        n = 0
        for f in sorted(self.backup_dir.glob("*.xml")):
            n += await self.process_file(f)
        return n

    async def run(self, stop: Optional[asyncio.Event] = None) -> None:
        await self.bus.ensure_stream()
        stop = stop or asyncio.Event()
        while not stop.is_set():
            await self.scan_once()
            try:
                await asyncio.wait_for(stop.wait(), self.interval_s)
            except asyncio.TimeoutError:
                pass


def write_backup_xml(path: os.PathLike, items: Iterable[tuple]) -> None:
    """Write an SMS-backup XML file: ``items`` of (address, date_ms, body) — used by tests/tools."""
    root = ET.Element("smses")
    for addr, date_ms, body in items:
        ET.SubElement(root, "sms", {"address": addr, "date": str(date_ms), "body": body, "type": "1"})
    ET.ElementTree(root).write(path, encoding="utf-8", xml_declaration=True)
