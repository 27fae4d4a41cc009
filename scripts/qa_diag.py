#!/usr/bin/env python3
"""Diagnostics of one trained sample of the flagship recipe: train (models/train.py
``recipe()``, one seed), then dump, for the scored sets, every item's prompt ids, gold
answer and the head's raw fp32 scores (models/evaluate.py TorchQAExtractor.scores) to
an .npz -- so decode rules and confidence measures can be studied offline on the CPU
(serving/qa.py qa_decode_ref) without retraining.  Optionally saves the serving
weights."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SETS = (("heldout_formats", "heldout", 4243), ("heldout_values", "heldout_values", 4245),
        ("validation", "train", 7001), ("negatives_heldout", "neg_heldout", 4246))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--eval-n", type=int, default=500)
    p.add_argument("--workers", type=int, default=6)
    p.add_argument("--overrides", default="")
    p.add_argument("--out", default="gpurun_out/qa_diag_seed0.npz")
    p.add_argument("--save-weights", default="")
    a = p.parse_args()
    import numpy as np
    import torch

    from smsgate_amd.models.evaluate import TorchQAExtractor
    from smsgate_amd.models.train import ExamplePool, recipe, train_extractor
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.utils.synth import generate

    kw = json.loads(a.overrides) if a.overrides else {}
    for k, v in kw.pop("env", {}).items():
        os.environ[k] = str(v)
    tc = recipe(None, a.steps, seed=a.seed, log_every=500, data_parallel=False, **kw)
    t0 = time.time()
    data = ExamplePool(tc.n_examples, seed=tc.seed, families=tc.families, workers=a.workers,
                       answer_format=tc.answer_format, negatives=tc.negatives).get()
    w = train_extractor(tc, device="cuda", data=data, log=lambda s: print(f"[diag] {s}", flush=True))
    del data
    if a.save_weights:
        w.save(a.save_weights)
    eng = TorchQAExtractor(w, batch=256, min_conf=0.0)
    out = {}
    meta = {"seed": a.seed, "train_s": round(time.time() - t0, 1), "overrides": a.overrides, "sets": {}}
    for name, fam, seed in SETS:
        items = [s for s in generate(a.eval_n, seed=seed, vocab_name="heldout", families=fam)
                 if s.answer is not None]
        bodies = [normalize_body(s.body) for s in items]
        msgs = eng.tok.message_ids(bodies, 128)
        cls, st, nl, en = eng.scores(msgs)
        L = max(len(m) for m in msgs)
        ids = np.full((len(msgs), L), -1, dtype=np.int32)
        for i, m in enumerate(msgs):
            ids[i, :len(m)] = m
        out[f"{name}_ids"] = ids
        out[f"{name}_cls"] = cls.astype(np.float32)
        out[f"{name}_start"] = st.astype(np.float32)
        out[f"{name}_null"] = nl.astype(np.float32)
        out[f"{name}_end"] = en.astype(np.float32)
        meta["sets"][name] = [{"body": s.body, "family": s.family, "answer": s.answer, "ts": s.timestamp}
                              for s in items]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **out)
    with open(a.out.replace(".npz", ".json"), "w") as fh:
        json.dump(meta, fh, ensure_ascii=False, default=str)
    print(json.dumps({"out": a.out, "train_s": meta["train_s"]}), flush=True)
    del eng, w
    torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
