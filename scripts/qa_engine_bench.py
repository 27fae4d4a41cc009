#!/usr/bin/env python3
"""Engine-only throughput of the one-forward (qa) format: the 135M architecture
(random init: the compute does not depend on the weights' values -- one forward per
message whatever the answer), formats traffic tokenised up front, batches submitted
the way the engine server receives them (512-message requests), timed with a GPU
synchronise on both sides.  Prints one JSON line: msgs/s, GPU-busy estimate, tokens
per message, batch sizes.  ``--profile`` adds a short untimed pass for rocprofv3."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=65536)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--queries", type=int, default=9)
    p.add_argument("--max-slots", type=int, default=8192)
    p.add_argument("--qa-max-tokens", default="262144", help="comma list: one JSON line per value (a sweep)")
    p.add_argument("--split-prefill", type=int, default=0, help="EngineConfig.qa_split_prefill")
    p.add_argument("--request", type=int, default=512)
    p.add_argument("--packed", type=int, default=1, choices=[0, 1],
                   help="1: each request one engine unit (submit_packed, the engine server's path)")
    p.add_argument("--prefill-attn", default="auto,st32,st32pf",
                   help="comma list of EngineConfig.prefill_attn values (ops.set_prefill_impl): one line each")
    a = p.parse_args()

    import numpy as np
    import torch

    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights, qa_config
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.serving.engine import EngineConfig
    from smsgate_amd.serving.qa_engine import QAEngine
    from smsgate_amd.utils.synth import generate_traffic

    tok = load_tokenizer()
    cfg = qa_config(CONFIGS["smollm-135m"], queries=a.queries)
    w = ExtractorWeights(cfg, device="cuda", seed=0)
    w.requires_grad_(False)
    bodies = [normalize_body(s.body) for s in generate_traffic(a.n, seed=1, traffic="formats")]
    ids = [np.asarray(x, dtype=np.int32) for x in tok.message_ids(bodies, 128)]
    tokens = sum(len(x) for x in ids) / len(ids)
    lens = np.asarray([len(x) for x in ids], dtype=np.int32)

    def run_once(eng) -> float:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = 0
        k = 0
        while done < len(ids):
            # keep ~8 requests waiting, like 8 parser processes with one request in flight each
            while k < len(ids) and len(eng.waiting) * (a.request if a.packed else 1) < 8 * a.request:
                part = range(k, min(k + a.request, len(ids)))
                if a.packed:
                    eng.submit_packed(k, lens[part.start:part.stop], np.concatenate([ids[i] for i in part]))
                else:
                    eng.submit_ids([(i, ids[i]) for i in part])
                k += a.request
            out = eng.step(raw=True)
            done += sum(len(v.lens) for _, v in out) if a.packed else len(out)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    import itertools

    for mt, pa in itertools.product((int(x) for x in str(a.qa_max_tokens).split(",")), a.prefill_attn.split(",")):
        eng = QAEngine(w, tok, EngineConfig(max_slots=a.max_slots, qa_max_tokens=mt, qa_split_prefill=a.split_prefill,
                                            prefill_attn=pa))
        run_once(eng)  # warm-up (allocator, first launches)
        eng.reset_stats()
        times = [run_once(eng) for _ in range(a.reps)]
        st = eng.stats
        out = {"metric": "qa_engine_msgs_per_s", "value": round(a.n / min(times), 1),
               "runs_s": [round(t, 3) for t in times], "n": a.n, "queries": a.queries,
               "prompt_tokens_per_msg": round(tokens, 2), "rows_per_msg": round(tokens + a.queries, 2),
               "batches": st.prefill_batches, "msgs_per_batch": round(st.prefill_seqs / max(1, st.prefill_batches), 1),
               "gpu_idle_s": round(st.gpu_idle_s, 4), "host_prefill_s": round(st.prefill_s, 3),
               "harvest_wait_s": round(st.harvest_wait_s, 3),
               "config": {"prefill_attn": pa, "packed": bool(a.packed), "max_slots": a.max_slots, "qa_max_tokens": mt,
                          "qa_split_prefill": a.split_prefill}}
        print(json.dumps(out), flush=True)
        del eng
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
