"""Low-overhead CPU sampling profiler for the host pipeline processes.

cProfile instruments every call (a ~1 µs hook on each of the millions of small calls a
parser process makes per second) and counts time a call spends *blocked* -- a socket
write waiting for buffer space, an epoll wait -- as that call's own time, so its
per-message table over-states both the cheap Python calls and the waits.

This sampler instead arms ``ITIMER_PROF`` (it ticks with the process's CPU time, user +
system, every thread): every ``interval`` seconds of CPU the main thread's Python stack
is recorded.  A blocked process consumes no CPU and takes no samples; a sample that
lands while the main thread sits in ``select`` / ``epoll`` is CPU some other thread of
the process used (the engine client's reader thread).  Native calls are charged to the
Python line that made them.  The kernel checks CPU-time timers at its scheduler tick,
so a shorter interval than the tick silently yields fewer samples: every sample is
therefore weighted by the process CPU time actually consumed while the sampler ran
(``time.process_time``) / samples, not by the nominal interval.

    s = CpuSampler(); s.start(); ...; s.stop(); s.dump(path, msgs=n)
"""
from __future__ import annotations

import json
import os
import signal
import time
from collections import Counter
from typing import Dict, Optional

__all__ = ["CpuSampler", "merge_samples"]


class CpuSampler:
    def __init__(self, interval: float = 0.002, depth: int = 48) -> None:
        self.interval = interval
        self.depth = depth
        self.leaf: Counter = Counter()  # "file:line func" of the innermost frame
        self.incl: Counter = Counter()  # "file func" of every frame on the stack (once per sample)
        self.samples = 0
        self.cpu_s = 0.0  # process CPU time while sampling
        self._t0 = 0.0
        self._old = None
        self._on = False

    @staticmethod
    def _where(code, line: Optional[int] = None) -> str:
        f = code.co_filename
        parts = f.replace("\\", "/").split("/")
        short = "/".join(parts[-2:]) if len(parts) > 1 else f
        return f"{short}:{line} {code.co_name}" if line is not None else f"{short} {code.co_name}"

    def _handler(self, signum, frame) -> None:
        if frame is None:
            return
        self.samples += 1
        self.leaf[self._where(frame.f_code, frame.f_lineno)] += 1
        seen = set()
        f, d = frame, 0
        while f is not None and d < self.depth:
            k = self._where(f.f_code)
            if k not in seen:
                seen.add(k)
                self.incl[k] += 1
            f, d = f.f_back, d + 1

    def start(self) -> None:
        if self._on:
            return
        self._old = signal.signal(signal.SIGPROF, self._handler)
        self._t0 = time.process_time()
        signal.setitimer(signal.ITIMER_PROF, self.interval, self.interval)
        self._on = True

    def stop(self) -> None:
        if not self._on:
            return
        signal.setitimer(signal.ITIMER_PROF, 0.0, 0.0)
        self.cpu_s += time.process_time() - self._t0
        signal.signal(signal.SIGPROF, self._old or signal.SIG_DFL)
        self._on = False

    def as_dict(self, msgs: int = 0) -> Dict:
        return {"interval_s": self.interval, "samples": self.samples, "cpu_s": round(self.cpu_s, 4), "msgs": msgs,
                "pid": os.getpid(),
                "leaf": dict(self.leaf), "incl": dict(self.incl)}

    def dump(self, path: str, msgs: int = 0) -> None:
        with open(path, "w") as fh:
            json.dump(self.as_dict(msgs), fh)


def merge_samples(docs) -> Dict:
    """Sum several processes' :meth:`CpuSampler.as_dict` (same interval)."""
    out = {"interval_s": None, "samples": 0, "cpu_s": 0.0, "msgs": 0, "leaf": Counter(), "incl": Counter(),
           "procs": 0}
    for d in docs:
        out["interval_s"] = d["interval_s"]
        out["samples"] += d["samples"]
        out["cpu_s"] += d.get("cpu_s", d["samples"] * d["interval_s"])
        out["msgs"] += d["msgs"]
        out["leaf"].update(d["leaf"])
        out["incl"].update(d["incl"])
        out["procs"] += 1
    return out
