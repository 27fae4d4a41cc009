"""PocketBase → chart → Telegram notifier (services/dashboard/main.py parity).

* every ``CHECK_INTERVAL_SECONDS`` (3600 s): fetch ``sms_data`` records with
  ``datetime > last_ts − 7 days`` (dashboard/main.py:207-210); if the newest
  record is newer than ``last_ts``, build a stacked daily-amount-per-merchant
  bar chart (inline-SVG HTML + a Pillow JPG) and send the photo — caption
  "Обновлённая статистика платежей" plus the last known balance — and the HTML
  document to every allowed chat (:146-246), then persist ``last_ts``;
* concurrently long-poll ``getUpdates`` (timeout 30 s) and answer chats not in
  ``TG_CHAT_IDS`` with "⛔️ У вас нет доступа к этому боту. Ваш chat_id: <id>"
  (:255-286), persisting the update ``offset``.

Fixes: one in-memory state object shared by both loops and written atomically
(temp file + rename) — the reference's two tasks each kept their own copy and
the Telegram task overwrote ``last_ts`` with its stale start-up value (R1/D13);
a corrupt state file falls back to defaults instead of crashing; the chart needs no
plotting stack or headless browser (SVG + Pillow), and a failed JPG still sends the
HTML report.
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

__all__ = ["NotifierState", "build_chart", "daily_totals", "TelegramClient", "Notifier", "DENY_TEXT"]

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


# stacked-bar palette (one colour per merchant, cycled) and the report's axis labels
_PALETTE = ("#4C78A8", "#F58518", "#54A24B", "#E45756", "#72B7B2", "#EECA3B", "#B279A2", "#FF9DA6",
            "#9D755D", "#BAB0AC")
_LABELS = {"x": "Дата", "y": "Сумма", "legend": "Продавец"}
_FONT_PATHS = ("/usr/share/fonts/truetype/dejavu/DejaVuSans.ttf",)


def _number(v: Any) -> Optional[float]:
    try:
        x = float(str(v).replace(" ", "").replace(",", "."))
    except (TypeError, ValueError):
        return None
    return x if x == x and abs(x) != float("inf") else None


def _when(v: Any) -> Optional[datetime]:
    try:
        d = dt_parse.isoparse(str(v).replace(" ", "T"))
    except (TypeError, ValueError, OverflowError):
        return None
    return d if d.tzinfo else d.replace(tzinfo=timezone.utc)


def daily_totals(records: List[Mapping[str, Any]]):
    """(days, merchants, {(day, merchant): amount}, last balance) of the chartable records.

    A record counts when its amount is a number and its datetime parses (UTC when naive);
    an empty or missing merchant is "Unknown".  Merchants are ordered by their total,
    largest first (the legend and the stacking order).  The last balance is the one on
    the newest record, if that record has one."""
    totals: Dict[Tuple[Any, str], float] = {}
    per_merchant: Dict[str, float] = {}
    newest: Optional[Tuple[datetime, Mapping[str, Any]]] = None
    for r in records:
        amt, when = _number(r.get("amount")), _when(r.get("datetime"))
        if amt is None or when is None:
            continue
        m = str(r.get("merchant") or "").strip()
        m = "Unknown" if m in ("", "null", "None") else m
        key = (when.date(), m)
        totals[key] = totals.get(key, 0.0) + amt
        per_merchant[m] = per_merchant.get(m, 0.0) + amt
        if newest is None or when > newest[0]:
            newest = (when, r)
    if not totals:
        raise ValueError("no chartable records")
    days = sorted({d for d, _ in totals})
    merchants = sorted(per_merchant, key=lambda k: (-per_merchant[k], k))
    balance = None
    if newest is not None:
        b = _number(newest[1].get("balance"))
        if b is not None:
            balance = (b, str(newest[1].get("currency") or ""))
    return days, merchants, totals, balance


def _layout(days, merchants, totals, width: int, height: int):
    """Bar rectangles in pixel space: [(x, y, w, h, colour)], the y-axis ticks
    [(y_pixel, value)], the plot box (left, top, right, bottom) and each day's x centre.
    Negative totals (refunds) are drawn down from the zero line."""
    left, top, right, bottom = 80, 50, width - 200, height - 110
    pos = [sum(max(totals.get((d, m), 0.0), 0.0) for m in merchants) for d in days]
    neg = [sum(min(totals.get((d, m), 0.0), 0.0) for m in merchants) for d in days]
    hi, lo = max(pos + [0.0]), min(neg + [0.0])
    span = (hi - lo) or 1.0
    step = 10 ** max(0, len(str(int(span / 5))) - 1) if span >= 5 else 1
    while span / step > 8:
        step *= 2
    hi_t = step * -(-hi // step)
    lo_t = -step * -(-(-lo) // step)
    span = (hi_t - lo_t) or 1.0

    def y_of(v: float) -> float:
        return bottom - (v - lo_t) / span * (bottom - top)

    slot = (right - left) / max(len(days), 1)
    bw = slot * 0.7
    bars, centres = [], []
    for i, d in enumerate(days):
        cx = left + slot * (i + 0.5)
        centres.append(cx)
        up = down = 0.0
        for k, m in enumerate(merchants):
            v = totals.get((d, m), 0.0)
            if not v:
                continue
            base = up if v > 0 else down
            y0, y1 = y_of(base), y_of(base + v)
            bars.append((cx - bw / 2, min(y0, y1), bw, abs(y1 - y0), _PALETTE[k % len(_PALETTE)]))
            if v > 0:
                up += v
            else:
                down += v
    ticks, t = [], lo_t
    while t <= hi_t + 1e-9:
        ticks.append((y_of(t), t))
        t += step
    return bars, ticks, (left, top, right, bottom), centres


def _fmt(v: float) -> str:
    return f"{v:,.0f}".replace(",", " ") if abs(v) >= 100 or v == int(v) else f"{v:.2f}"


def _svg(days, merchants, totals, title: str, width: int = 1000, height: int = 600) -> str:
    from html import escape
    bars, ticks, (l, t, r, b), centres = _layout(days, merchants, totals, width, height)
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" '
           f'font-family="DejaVu Sans, Arial, sans-serif" font-size="12">',
           f'<text x="{width / 2:.0f}" y="28" text-anchor="middle" font-size="18">{escape(title)}</text>']
    for y, v in ticks:
        out.append(f'<line x1="{l}" x2="{r}" y1="{y:.1f}" y2="{y:.1f}" stroke="#ddd"/>'
                   f'<text x="{l - 6}" y="{y + 4:.1f}" text-anchor="end">{_fmt(v)}</text>')
    for x, y, w, h, c in bars:
        out.append(f'<rect x="{x:.1f}" y="{y:.1f}" width="{w:.1f}" height="{h:.1f}" fill="{c}"/>')
    for cx, d in zip(centres, days):
        out.append(f'<text transform="translate({cx:.1f},{b + 14}) rotate(-45)" text-anchor="end">{d.isoformat()}</text>')
    out.append(f'<text x="{(l + r) / 2:.0f}" y="{height - 12}" text-anchor="middle">{_LABELS["x"]}</text>')
    out.append(f'<text transform="translate(18,{(t + b) / 2:.0f}) rotate(-90)" text-anchor="middle">{_LABELS["y"]}</text>')
    out.append(f'<text x="{r + 20}" y="{t}" font-weight="bold">{_LABELS["legend"]}</text>')
    for k, m in enumerate(merchants[:25]):
        y = t + 18 * (k + 1)
        out.append(f'<rect x="{r + 20}" y="{y - 10}" width="12" height="12" fill="{_PALETTE[k % len(_PALETTE)]}"/>'
                   f'<text x="{r + 38}" y="{y}">{escape(m[:22])}</text>')
    out.append("</svg>")
    return "\n".join(out)


def _raster(days, merchants, totals, title: str, path: Path, scale: int = 2) -> None:
    """The same chart as a JPEG through Pillow (no browser / kaleido)."""
    from PIL import Image, ImageDraw, ImageFont
    W, H = 1000, 600
    bars, ticks, (l, t, r, b), centres = _layout(days, merchants, totals, W, H)

    def font(sz: int):
        for fp in _FONT_PATHS:
            if os.path.exists(fp):
                return ImageFont.truetype(fp, sz * scale)
        return ImageFont.load_default(size=sz * scale)
    f12, f18 = font(12), font(18)
    img = Image.new("RGB", (W * scale, H * scale), "white")
    g = ImageDraw.Draw(img)
    S = lambda *v: [x * scale for x in v]  # noqa: E731
    g.text(S(W / 2, 12), title, fill="black", font=f18, anchor="mt")
    for y, v in ticks:
        g.line(S(l, y, r, y), fill="#dddddd", width=scale)
        g.text(S(l - 6, y), _fmt(v), fill="black", font=f12, anchor="rm")
    for x, y, w, h, c in bars:
        g.rectangle(S(x, y, x + w, y + max(h, 0.5)), fill=c)
    for cx, d in zip(centres, days):
        lab = Image.new("RGBA", (int(f12.getlength(d.isoformat())) + 4, 16 * scale), (255, 255, 255, 0))
        ImageDraw.Draw(lab).text((0, 0), d.isoformat(), fill="black", font=f12)
        lab = lab.rotate(45, expand=True)
        img.paste(lab, (int(cx * scale) - lab.width, int((b + 6) * scale)), lab)
    g.text(S((l + r) / 2, H - 12), _LABELS["x"], fill="black", font=f12, anchor="mb")
    ylab = Image.new("RGBA", (int(f12.getlength(_LABELS["y"])) + 4, 16 * scale), (255, 255, 255, 0))
    ImageDraw.Draw(ylab).text((0, 0), _LABELS["y"], fill="black", font=f12)
    ylab = ylab.rotate(90, expand=True)
    img.paste(ylab, (10 * scale, int((t + b) / 2 * scale) - ylab.height // 2), ylab)
    g.text(S(r + 20, t), _LABELS["legend"], fill="black", font=f12, anchor="ls")
    for k, m in enumerate(merchants[:25]):
        y = t + 18 * (k + 1)
        g.rectangle(S(r + 20, y - 10, r + 32, y + 2), fill=_PALETTE[k % len(_PALETTE)])
        g.text(S(r + 38, y), m[:22], fill="black", font=f12, anchor="ls")
    img.save(str(path), format="JPEG", quality=90)


def build_chart(records: List[Mapping[str, Any]], title: str, out_dir: Path,
                want_image: bool = True) -> Tuple[Path, Optional[Path], Optional[Tuple[float, str]]]:
    """Daily spend per merchant as a stacked bar chart (dashboard/main.py:146-197 parity:
    one bar per day, one segment per merchant, the last balance for the caption).

    Rendered here without a plotting stack: an HTML page holding an inline SVG, and the
    same layout rasterised to ``payments_by_day.jpg`` with Pillow, so the photo goes out
    wherever the service runs (the reference's JPG needed a headless browser).  Returns
    (html path, jpg path or None, (balance, currency) or None)."""
    if not records:
        raise ValueError("no records to chart")
    days, merchants, totals, balance = daily_totals(records)
    out_dir.mkdir(parents=True, exist_ok=True)
    html = out_dir / "payments_by_day.html"
    from html import escape
    html.write_text("<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\"><title>" + escape(title)
                    + "</title></head><body>\n" + _svg(days, merchants, totals, title) + "\n</body></html>\n",
                    encoding="utf-8")
    img: Optional[Path] = None
    if want_image:
        try:
            img = out_dir / "payments_by_day.jpg"
            _raster(days, merchants, totals, title, img)
        except Exception as exc:  # Pillow missing / no usable font: the HTML report still goes out
            log.warning("chart image export failed: %s", exc)
            img = None
    return html, img, balance


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
