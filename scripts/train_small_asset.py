#!/usr/bin/env python3
"""Train the bundled ``small`` extractor (models/assets/extractor-small.safetensors) with
the flagship recipe (models/train.py FLAGSHIP_RECIPE: qa answers, non-transactions,
fresh examples) and score it through the HIP qa engine: the reference CASES, held-out
formats / values, held-out non-transactions (the bundled checkpoint
and the smoke test ran the round-4 copy-format stack).  One JSON line on stdout."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/extractor-small.safetensors")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--eval-n", type=int, default=500)
    a = p.parse_args()
    import torch

    from smsgate_amd.models.evaluate import (evaluate_engine, evaluate_negatives, golden_case_mismatches,
                                             golden_case_results)
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights
    from smsgate_amd.models.train import ExamplePool, recipe, train_extractor
    from smsgate_amd.parse.backends.local_llm import build_engine

    tc = recipe("small", a.steps, log_every=500, data_parallel=False)
    t0 = time.time()
    data = ExamplePool(tc.n_examples, seed=tc.seed, families=tc.families, workers=12, answer_format=tc.answer_format,
                       negatives=tc.negatives).get()
    w = train_extractor(tc, device="cuda", data=data, log=lambda s: print(f"[small] {s}", file=sys.stderr, flush=True))
    train_s = time.time() - t0
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    w.save(a.out)
    w2 = ExtractorWeights.load(a.out, CONFIGS["small"], device=torch.device("cuda"))  # the file, as served
    eng = build_engine("small", weights=w2, max_slots=1024)
    res = {"model": "small", "steps": tc.steps, "batch": tc.batch, "train_s": round(train_s, 1),
           "bytes": os.path.getsize(a.out)}
    for name, fam, seed in (("heldout_formats", "heldout", 4243), ("heldout_values", "heldout_values", 4245),
                            ("train_formats", "train", 4242)):
        q = evaluate_engine(eng, n=a.eval_n, seed=seed, vocab_name="heldout", families=fam)
        res[name] = {k: q[k] for k in ("exact", "published_wrong_rate", "declined_rate", "by_family")}
    res["negatives_heldout"] = evaluate_negatives(eng, n=a.eval_n, seed=4246, families="neg_heldout")
    bad = golden_case_mismatches(golden_case_results(eng))
    res["reference_cases"] = {"passed": 3 - len({b.split(".")[0].split(":")[0] for b in bad}), "mismatches": bad}
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
