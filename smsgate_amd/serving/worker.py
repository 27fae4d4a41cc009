"""Engine worker thread: continuous batching across concurrent async callers.

The asyncio side (parser stage) submits batches of bodies and awaits a future;
one dedicated thread owns the GPU engine and runs admit → decode-chunk →
harvest steps, so requests arriving while others decode join the running
batch instead of waiting for it to drain. Kernel launches and graph replays
release the GIL, so CPU post-processing on the event loop overlaps the GPU.
"""
from __future__ import annotations

import asyncio
import queue
import threading
import traceback
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

__all__ = ["EngineWorker"]


@dataclass
class _Req:
    bodies: Sequence[str]
    done_cb: Callable[[List[Any]], None]
    results: List[Any] = field(default_factory=list)
    remaining: int = 0


class EngineWorker:
    def __init__(self, engine_factory: Callable[[], Any], name: str = "extract-engine") -> None:
        self._factory = engine_factory
        self._q: "queue.Queue[Optional[_Req]]" = queue.Queue()
        self._thread = threading.Thread(target=self._main, name=name, daemon=True)
        self._ready = threading.Event()
        self._stop = False
        self.engine = None
        self.error: Optional[BaseException] = None

    def start(self, timeout: Optional[float] = None) -> None:
        self._thread.start()
        self._ready.wait(timeout)
        if self.error is not None:
            raise RuntimeError("engine failed to start") from self.error

    def stop(self) -> None:
        self._stop = True
        self._q.put(None)
        self._thread.join(timeout=30)

    def submit(self, bodies: Sequence[str], done_cb: Callable[[List[Any]], None]) -> None:
        self._q.put(_Req(bodies, done_cb))

    async def extract(self, bodies: Sequence[str]) -> List[Any]:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def cb(res: List[Any]) -> None:
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(res))

        self.submit(bodies, cb)
        return await fut

    def _main(self) -> None:
        try:
            self.engine = self._factory()
        except BaseException as exc:  # noqa: BLE001
            self.error = exc
            traceback.print_exc()
            self._ready.set()
            return
        self._ready.set()
        eng = self.engine
        inflight: Dict[int, _Req] = {}
        next_id = 0
        while not self._stop:
            # drain new requests (block only when idle)
            try:
                req = self._q.get(block=not eng.busy(), timeout=None if not eng.busy() else 0)
            except queue.Empty:
                req = None
            while req is not None:
                rid = next_id
                next_id += 1
                req.results = [None] * len(req.bodies)
                req.remaining = len(req.bodies)
                inflight[rid] = req
                if req.remaining == 0:
                    inflight.pop(rid).done_cb([])
                else:
                    eng.submit_many([((rid, i), b) for i, b in enumerate(req.bodies)])
                try:
                    req = self._q.get_nowait()
                except queue.Empty:
                    req = None
            if self._stop:
                break
            try:
                finished = eng.step()
            except BaseException as exc:  # noqa: BLE001 — fail every waiting caller loudly
                traceback.print_exc()
                for r in inflight.values():
                    r.done_cb([exc] * len(r.bodies))
                inflight.clear()
                eng.waiting.clear()
                eng.active.clear()
                continue
            for (rid, i), ans in finished:
                r = inflight.get(rid)
                if r is None:
                    continue
                r.results[i] = ans
                r.remaining -= 1
                if r.remaining == 0:
                    inflight.pop(rid)
                    r.done_cb(r.results)
