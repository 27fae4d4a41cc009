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
    assert counts["ok"] + counts["fail"] + counts["skip"] == 2 * 2 * 150
    assert counts["sink_stored"] + counts["writer_no_merchant"] == counts["parsed"]  # writer saw every parse
    # OTP/credit-style synthetic messages are skipped before the engine
    assert eng.seen < 600 and eng.seen > 300
    assert counts["ok"] > 0 and dt > 0
    assert all(not p.is_alive() for p in procs)


def test_bench_two_ranks_torchrun_gloo(tmp_path):
    """The bench's DP harness end to end on CPU: torch.distributed.run with 2 ranks
    (gloo, 127.0.0.1), each rank a Coordinator + 2 spawned parser workers around the
    CPU echo engine; barrier-bracketed timing, MAX over ranks, ONE JSON line."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--cpu-echo-engine", "--msgs-per-step", "256", "--cpu-workers", "2"]
    r = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 512
    assert out["value"] > 0 and out["steps"] == 2 and out["scaling"] == "weak"
    rt = out["routing"]  # outcomes summed over both ranks
    assert rt["parsed"] + rt["keyword_skipped"] + rt["broken"] + rt["dlq"] == 512 * 2
