"""PocketBase → chart → Telegram notifier (services/dashboard/main.py parity).

* every ``CHECK_INTERVAL_SECONDS`` (3600 s): fetch ``sms_data`` records with
  ``datetime > last_ts − 7 days`` (dashboard/main.py:207-210); if the newest
  record is newer than ``last_ts``, build a stacked daily-amount-per-merchant
  bar chart (plotly; HTML + JPG via kaleido) and send the photo — caption
  "Обновлённая статистика платежей" plus the last known balance — and the HTML
  document to every allowed chat (:146-246), then persist ``last_ts``;
* concurrently long-poll ``getUpdates`` (timeout 30 s) and answer chats not in
  ``TG_CHAT_IDS`` with "⛔️ У вас нет доступа к этому боту. Ваш chat_id: <id>"
  (:255-286), persisting the update ``offset``.

Fixes: one in-memory state object shared by both loops and written atomically
(temp file + rename) — the reference's two tasks each kept their own copy and
the Telegram task overwrote ``last_ts`` with its stale start-up value (R1/D13);
a corrupt state file falls back to defaults instead of crashing; a failed JPG
export (kaleido unavailable) still sends the HTML report.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import tempfile
from datetime import datetime, timedelta, timezone
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Set, Tuple

import httpx
from dateutil import parser as dt_parse

__all__ = ["NotifierState", "build_chart", "TelegramClient", "Notifier", "DENY_TEXT"]

log = logging.getLogger("notifier")

DENY_TEXT = "⛔️ У вас нет доступа к этому боту. Ваш chat_id: {chat_id}"
CAPTION = "Обновлённая статистика платежей"


class NotifierState:
    def __init__(self, path: Path) -> None:
        self.path = Path(path)
        self.data: Dict[str, Any] = self._load()

    def _default(self) -> Dict[str, Any]:
        return {"last_ts": (datetime.now(timezone.utc) - timedelta(days=7)).isoformat(), "offset": 0}

    def _load(self) -> Dict[str, Any]:
        if self.path.exists():
            try:
                d = json.loads(self.path.read_text())
                if isinstance(d, dict) and "last_ts" in d:
                    d.setdefault("offset", 0)
                    return d
            except ValueError:
                log.warning("state file %s corrupt; starting from defaults", self.path)
        return self._default()

    def save(self) -> None:
        self.path.parent.mkdir(parents=True, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=str(self.path.parent), prefix=".state-")
        with os.fdopen(fd, "w") as f:
            json.dump(self.data, f, indent=2)
        os.replace(tmp, self.path)

    @property
    def last_ts(self) -> datetime:
        return dt_parse.isoparse(self.data["last_ts"])


def build_chart(records: List[Mapping[str, Any]], title: str, out_dir: Path,
                want_image: bool = True) -> Tuple[Path, Optional[Path], Optional[Tuple[float, str]]]:
    import pandas as pd
    import plotly.express as px

    df = pd.DataFrame(records)
    if df.empty:
        raise ValueError("no records to chart")
    df["merchant"] = df.get("merchant", pd.Series(dtype=object)).fillna("Unknown").replace(
        {"": "Unknown", "null": "Unknown"})
    df["amount"] = pd.to_numeric(df["amount"], errors="coerce")
    df["datetime"] = pd.to_datetime(df["datetime"], errors="coerce", utc=True)
    df["balance"] = pd.to_numeric(df["balance"], errors="coerce") if "balance" in df.columns else pd.NA
    df = df.dropna(subset=["amount", "datetime"])
    if df.empty:
        raise ValueError("no chartable records")
    df["date"] = df["datetime"].dt.date
    daily = df.groupby(["date", "merchant"])["amount"].sum().reset_index().sort_values("date")
    fig = px.bar(daily, x="date", y="amount", color="merchant",
                 labels={"date": "Дата", "amount": "Сумма", "merchant": "Продавец"}, height=600)
    fig.update_layout(title_text=title, xaxis_tickangle=-45)
    out_dir.mkdir(parents=True, exist_ok=True)
    html = out_dir / "payments_by_day.html"
    fig.write_html(str(html))
    img: Optional[Path] = None
    if want_image:
        try:
            img = out_dir / "payments_by_day.jpg"
            fig.write_image(str(img), format="jpg", scale=2)
        except Exception as exc:  # kaleido missing/broken: the HTML report still goes out
            log.warning("chart image export failed: %s", exc)
            img = None
    last_balance = None
    if df["balance"].notna().any():
        row = df.loc[df["datetime"].idxmax()]
        if pd.notna(row["balance"]):
            last_balance = (float(row["balance"]), str(row.get("currency", "") or ""))
    return html, img, last_balance


class TelegramClient:
    def __init__(self, token: str, transport: Optional[httpx.AsyncBaseTransport] = None, timeout: float = 60.0):
        self._c = httpx.AsyncClient(base_url=f"https://api.telegram.org/bot{token}", timeout=timeout,
                                    transport=transport)

    async def call(self, method: str, **kw) -> httpx.Response:
        r = await self._c.post(f"/{method}", **kw)
        r.raise_for_status()
        return r

    async def get_updates(self, offset: int, timeout: int = 30) -> List[Dict[str, Any]]:
        params = {"timeout": timeout}
        if offset:
            params["offset"] = offset
        r = await self._c.get("/getUpdates", params=params)
        r.raise_for_status()
        return r.json().get("result", [])

    async def close(self) -> None:
        await self._c.aclose()


class Notifier:
    def __init__(self, pb, tg: TelegramClient, allowed: Set[int], state: NotifierState, out_dir: Path,
                 interval_s: float = 3600.0, collection: str = "sms_data") -> None:
        self.pb, self.tg, self.allowed, self.state = pb, tg, allowed, state
        self.out_dir = Path(out_dir)
        self.interval_s = interval_s
        self.collection = collection
        self.reports_sent = 0
        self.denied: List[int] = []

    async def _send_file(self, method: str, field: str, path: Path, caption: str = "") -> None:
        data = path.read_bytes()
        for chat in sorted(self.allowed):
            try:
                await self.tg.call(method, data={"chat_id": chat, "caption": caption}, files={field: (path.name, data)})
            except httpx.HTTPError as exc:
                log.error("telegram %s to %s failed: %s", method, chat, exc)

    async def run_cycle(self) -> bool:
        last_ts = self.state.last_ts
        since = (last_ts + timedelta(microseconds=1) - timedelta(days=7)).strftime("%Y-%m-%d %H:%M:%S.%f")
        records = await self.pb.get_records_since(self.collection, since)
        if not records:
            return False
        dts = []
        for r in records:
            try:
                d = dt_parse.isoparse(str(r.get("datetime")).replace(" ", "T"))
                dts.append(d if d.tzinfo else d.replace(tzinfo=timezone.utc))
            except (ValueError, TypeError):
                continue
        if not dts or max(dts) <= last_ts:
            return False
        html, img, bal = build_chart(records, "Статистика платежей по дням", self.out_dir)
        caption = CAPTION
        if bal:
            caption += f"\nПоследний баланс: {bal[0]:,.2f} {bal[1]}".replace(",", " ")
        if img is not None:
            await self._send_file("sendPhoto", "photo", img, caption)
            await self._send_file("sendDocument", "document", html)
        else:
            await self._send_file("sendDocument", "document", html, caption)
        self.state.data["last_ts"] = max(dts).isoformat()
        self.state.save()
        self.reports_sent += 1
        return True

    async def handle_updates(self, updates: List[Dict[str, Any]]) -> None:
        for upd in updates:
            self.state.data["offset"] = upd["update_id"] + 1
            msg = upd.get("message") or upd.get("edited_message")
            if msg:
                chat = msg["chat"]["id"]
                if chat not in self.allowed:
                    self.denied.append(chat)
                    try:
                        await self.tg.call("sendMessage", data={"chat_id": chat, "text": DENY_TEXT.format(chat_id=chat)})
                    except httpx.HTTPError as exc:
                        log.error("deny message failed: %s", exc)
        if updates:
            self.state.save()

    async def listen(self, stop: asyncio.Event) -> None:
        while not stop.is_set():
            try:
                await self.handle_updates(await self.tg.get_updates(int(self.state.data.get("offset", 0))))
            except httpx.HTTPError as exc:
                log.warning("getUpdates failed: %s", exc)
                await asyncio.sleep(5)

    async def run(self, stop: Optional[asyncio.Event] = None) -> None:
        stop = stop or asyncio.Event()
        listener = asyncio.create_task(self.listen(stop))
        try:
            while not stop.is_set():
                try:
                    await self.run_cycle()
                except Exception:  # noqa: BLE001
                    log.exception("report cycle failed")
                try:
                    await asyncio.wait_for(stop.wait(), self.interval_s)
                except asyncio.TimeoutError:
                    pass
        finally:
            listener.cancel()
