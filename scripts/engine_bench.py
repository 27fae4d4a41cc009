"""Engine-level cost split on one MI355X: a full decode step (graph replay, all
rows active) at several batch sizes, and prefill throughput (tokens/s)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd.parse.backends.local_llm import build_engine  # noqa: E402
from smsgate_amd.serving.engine import _Pending  # noqa: E402
from smsgate_amd.utils.synth import generate_bodies  # noqa: E402


def main():
    S = int(os.environ.get("SLOTS", "8192"))
    eng = build_engine("smollm-135m", device="cuda", random_init=True, answer_format="copy", max_slots=S, steps_per_graph=2)
    res = {"slots": S}
    bodies = generate_bodies(S, seed=5)
    ids = eng.tok.message_ids(bodies, 128)
    # prefill all rows (chunked like the engine does)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = list(range(S))
    items = [_Pending(i, x) for i, x in enumerate(ids)]
    ntok = 0
    o = 0
    while o < S:
        chunk, t = [], 0
        while o < S and (not chunk or t + len(items[o].ids) <= eng.cfg.prefill_max_tokens):
            chunk.append(o)
            t += len(items[o].ids)
            o += 1
        eng._prefill([rows[i] for i in chunk], [items[i] for i in chunk])
        ntok += t
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res.update(prefill_tokens=ntok, prefill_s=round(dt, 4), prefill_us_per_token=round(dt / ntok * 1e6, 3),
               prefill_us_per_seq=round(dt / S * 1e6, 2))
    for i in range(S):
        eng.active[i] = i
    eng.done[:S] = 0
    for B in (2048, 4096, 8192):
        if B > S:
            continue
        g = eng.graphs[eng._bucket(B)]
        for _ in range(3):
            g.replay()
            eng.done[:S] = 0
            eng.out_len[:S] = 0
            eng.state[:S] = eng.fsm.start_state
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 10
        a.record()
        for _ in range(n):
            g.replay()
        b.record()
        b.synchronize()
        per_step = a.elapsed_time(b) / (n * eng.cfg.steps_per_graph) * 1000
        res[f"decode_step_us_B{B}"] = round(per_step, 1)
        res[f"decode_us_per_row_B{B}"] = round(per_step / B, 3)
        eng.done[:S] = 0
        eng.out_len[:S] = 0
        eng.state[:S] = eng.fsm.start_state
    # per message: ~prefill + 58 decode row-steps at B=S
    if f"decode_us_per_row_B{S}" in res:
        per_msg = res["prefill_us_per_seq"] + 58 * res[f"decode_us_per_row_B{S}"]
        res["gpu_us_per_msg_est"] = round(per_msg, 2)
        res["gpu_bound_msgs_per_s_est"] = round(1e6 / per_msg, 0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
