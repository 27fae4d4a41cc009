"""Optional public tunnel for the gateway (the reference's ngrok integration,
services/api_gateway/main.py:64-100: ``ENABLE_NGROK`` / ``NGROK_AUTHTOKEN`` /
``NGROK_DOMAIN``, started before uvicorn, stopped on shutdown).

Uses the ``ngrok`` Python SDK when importable, else the ``ngrok`` CLI (public
URL read back from its local API on :4040), else logs a warning and runs
without a tunnel — neither is on the MI355X image, and the reference imported
the SDK unconditionally (it is not even in its requirements.txt).
"""
from __future__ import annotations

import logging
import shutil
import subprocess
import time
from typing import Any, Optional

log = logging.getLogger("tunnel")

__all__ = ["Tunnel", "open_tunnel"]


class Tunnel:
    def __init__(self, url: Optional[str], handle: Any = None, proc: Optional[subprocess.Popen] = None) -> None:
        self.url, self._handle, self._proc = url, handle, proc

    def close(self) -> None:
        if self._handle is not None:
            try:
                import ngrok  # type: ignore

                ngrok.disconnect(self.url)
            except Exception as exc:  # noqa: BLE001
                log.debug("ngrok disconnect: %s", exc)
        if self._proc is not None and self._proc.poll() is None:
            self._proc.terminate()
            try:
                self._proc.wait(5)
            except subprocess.TimeoutExpired:
                self._proc.kill()


def _cli_url(timeout: float = 10.0) -> Optional[str]:
    import httpx

    end = time.monotonic() + timeout
    while time.monotonic() < end:
        try:
            r = httpx.get("http://127.0.0.1:4040/api/tunnels", timeout=1.0)
            for t in r.json().get("tunnels", []):
                if t.get("public_url", "").startswith("https://"):
                    return t["public_url"]
        except Exception:  # noqa: BLE001 - the agent is still starting
            pass
        time.sleep(0.3)
    return None


def open_tunnel(settings, port: int) -> Optional[Tunnel]:
    if not settings.enable_ngrok:
        return None
    try:
        import ngrok  # type: ignore
    except ImportError:
        ngrok = None
    if ngrok is not None:
        kw = {"authtoken": settings.ngrok_authtoken} if settings.ngrok_authtoken else {"authtoken_from_env": True}
        if settings.ngrok_domain:
            kw["domain"] = settings.ngrok_domain
        listener = ngrok.forward(port, **kw)
        url = listener.url() if callable(getattr(listener, "url", None)) else str(listener)
        log.info("ngrok tunnel %s -> :%d", url, port)
        return Tunnel(url, handle=listener)
    exe = shutil.which("ngrok")
    if exe:
        cmd = [exe, "http", str(port), "--log", "stdout"]
        if settings.ngrok_authtoken:
            cmd += ["--authtoken", settings.ngrok_authtoken]
        if settings.ngrok_domain:
            cmd += ["--domain", settings.ngrok_domain]
        proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        url = _cli_url()
        log.info("ngrok CLI tunnel %s -> :%d", url, port)
        return Tunnel(url, proc=proc)
    log.warning("ENABLE_NGROK is set but neither the ngrok SDK nor the ngrok CLI is available; no tunnel")
    return None
