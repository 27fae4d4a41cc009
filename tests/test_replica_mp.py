"""Multi-process replica on CPU: spawned parser workers ↔ EngineServer over pipes.

A CPU stand-in engine answers every prompt with the token encoding of a fixed
valid answer, so the whole parser → remote engine → post-processing → routing
path runs across real process boundaries without a GPU.
"""
import numpy as np

from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.parallel.replica import Coordinator, spawn_parser_workers
from smsgate_amd.parse.backends.fake import DEFAULT_ANSWER
from smsgate_amd.serving.fsm import DEFAULT_FIELDS


class CpuEchoEngine:
    def __init__(self):
        tk = load_tokenizer()
        toks = []
        for f in DEFAULT_FIELDS:
            toks += tk.encode(DEFAULT_ANSWER[f.name]) + [tk.sep]
        self.answer = np.asarray(toks, dtype=np.int32)
        self.waiting = []
        self.active = {}
        self._pending = None
        self.seen = 0

    def submit_ids(self, items):
        self.waiting.extend(items)

    def busy(self):
        return bool(self.waiting)

    def step(self, raw=True):
        out = [(k, self.answer) for k, _ in self.waiting[:300]]
        self.seen += len(out)
        del self.waiting[:300]
        return out


def test_replica_two_workers_end_to_end():
    procs, conns = spawn_parser_workers(2, rank=0, cfg={"batch": 64, "concurrency": 2})
    eng = CpuEchoEngine()
    coord = Coordinator(eng, conns)
    try:
        coord.wait_all("ready", timeout=120)
        dt, counts = coord.run_phase([[11, 12], [21, 22]], n_per_step=150)
    finally:
        coord.shutdown(procs)
    assert sum(counts.values()) == 2 * 2 * 150
    # OTP/credit-style synthetic messages are skipped before the engine
    assert eng.seen < 600 and eng.seen > 300
    assert counts["ok"] > 0 and dt > 0
    assert all(not p.is_alive() for p in procs)
