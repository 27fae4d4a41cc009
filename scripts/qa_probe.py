#!/usr/bin/env python3
"""Quality probe of the answer formats (VERDICT r04 next #2a: size the one-forward
span extractor with the training stack before building its engine).

For each ``--formats`` entry: train the flagship with the bench's recipe
(``bench.py _train_plan``: steps x batch fresh examples of the training families,
12 % non-transactions), then score it

* held-out formats (6 layouts never trained on), training formats, held-out value
  styles (utils/synth.py VALUE_FAMILIES) -- exact after the real post-processing;
* non-transactions: the share of held-out / training negative families that would be
  published on sms.parsed (``false_parsed_rate``);
* the reference's three CASES.

qa / qa17 are served by the PyTorch reference path (models/evaluate.py
TorchQAExtractor: the same decode rules as the HIP kernel), span / copy by the HIP
engine.  One JSON line per format on stdout and in ``--out``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--formats", default="qa,qa17")
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--negatives", type=float, default=0.12)
    p.add_argument("--eval-n", type=int, default=500)
    p.add_argument("--model", default="smollm-135m")
    p.add_argument("--out", default="gpurun_out/qa_probe.jsonl")
    p.add_argument("--save-dir", default="")
    p.add_argument("--variants", default="",
                   help="';'-separated training variants of the FIRST format, each 'key=value,...' over steps, "
                        "negatives, lr, fused, proc (procedural family weight, SMSGATE_PROC_WEIGHT), labels (pseudo-word label share, SMSGATE_SYNTH_LABELS), seed (training sample); e.g. "
                        "'steps=4000;steps=6000;proc=6'")
    a = p.parse_args()
    if a.variants:
        return _variants(a)

    from smsgate_amd.models.train import ExamplePool, TrainConfig

    fmts = a.formats.split(",")
    pools = {f: ExamplePool(a.steps * a.batch, seed=0, families="train", workers=12, answer_format=f,
                            negatives=a.negatives) for f in fmts[:1]}
    import torch

    from smsgate_amd.models.evaluate import (TorchQAExtractor, evaluate_engine, evaluate_negatives,
                                             golden_case_mismatches, golden_case_results)
    from smsgate_amd.models.train import train_extractor

    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for i, fmt in enumerate(fmts):
        t0 = time.time()
        data = pools.pop(fmt).get()
        if i + 1 < len(fmts):  # the next format's examples build while this one trains
            pools[fmts[i + 1]] = ExamplePool(a.steps * a.batch, seed=0, families="train", workers=12,
                                             answer_format=fmts[i + 1], negatives=a.negatives)
        tc = TrainConfig(model=a.model, steps=a.steps, batch=a.batch, lr=a.lr, n_examples=a.steps * a.batch,
                         log_every=500, data_parallel=False, families="train", answer_format=fmt,
                         negatives=a.negatives)
        w = train_extractor(tc, device="cuda", data=data, log=lambda s: print(f"[{fmt}] {s}", flush=True))
        train_s = time.time() - t0
        if a.save_dir:
            os.makedirs(a.save_dir, exist_ok=True)
            w.save(os.path.join(a.save_dir, f"{a.model}-{fmt}.safetensors"))
        if fmt.startswith("qa"):
            eng = TorchQAExtractor(w, batch=256)
        else:
            from smsgate_amd.parse.backends.local_llm import build_engine

            eng = build_engine(a.model, weights=w, answer_format=fmt, max_slots=1024)
        t1 = time.time()
        res = {"format": fmt, "steps": a.steps, "batch": a.batch, "negatives": a.negatives,
               "train_s": round(train_s, 1)}
        for name, fam in (("heldout_formats", "heldout"), ("train_formats", "train"),
                          ("heldout_values", "heldout_values")):
            q = evaluate_engine(eng, n=a.eval_n, seed=4243, vocab_name="heldout", families=fam)
            res[name] = {"exact": round(q["exact"], 4), "parse_rate": round(q["parse_rate"], 4),
                         "field_acc": {k: round(v, 4) for k, v in q["field_acc"].items()},
                         "by_family": q.get("by_family")}
        for name, fam in (("negatives_heldout", "neg_heldout"), ("negatives_train", "neg_train")):
            res[name] = evaluate_negatives(eng, n=a.eval_n, families=fam)
        bad = golden_case_mismatches(golden_case_results(eng))
        res["reference_cases"] = {"passed": 3 - len({b.split(".")[0].split(":")[0] for b in bad}), "mismatches": bad}
        res["eval_s"] = round(time.time() - t1, 1)
        line = json.dumps(res)
        print(line, flush=True)
        with open(a.out, "a") as fh:
            fh.write(line + "\n")
        del eng, w
        torch.cuda.empty_cache()
    return 0


def _variants(a) -> int:
    """One format, several training recipes, each trained and scored like main()."""
    import torch

    from smsgate_amd.models.evaluate import TorchQAExtractor, evaluate_engine, evaluate_negatives
    from smsgate_amd.models.train import ExamplePool, TrainConfig, train_extractor

    fmt = a.formats.split(",")[0]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for spec in a.variants.split(";"):
        kv = dict(x.split("=") for x in spec.split(",") if x)
        steps = int(kv.get("steps", a.steps))
        neg = float(kv.get("negatives", a.negatives))
        for key, env in (("proc", "SMSGATE_PROC_WEIGHT"), ("labels", "SMSGATE_SYNTH_LABELS")):
            if key in kv:
                os.environ[env] = kv[key]
            else:
                os.environ.pop(env, None)
        t0 = time.time()
        seed = int(kv.get("seed", 0))  # the training sample (data and init); the bench trains seed 0
        data = ExamplePool(steps * a.batch, seed=seed, families="train", workers=12, answer_format=fmt,
                           negatives=neg).get()
        tc = TrainConfig(model=a.model, steps=steps, batch=a.batch, lr=float(kv.get("lr", a.lr)),
                         n_examples=steps * a.batch, log_every=1000, data_parallel=False, families="train",
                         answer_format=fmt, negatives=neg, fused=bool(int(kv.get("fused", 1))), seed=seed)
        t1 = time.time()
        w = train_extractor(tc, device="cuda", data=data, log=lambda s: print(f"[{spec}] {s}", flush=True))
        res = {"format": fmt, "variant": spec, "steps": steps, "negatives": neg, "data_s": round(t1 - t0, 1),
               "train_s": round(time.time() - t1, 1)}
        eng = TorchQAExtractor(w, batch=256)
        for name, fam in (("heldout_formats", "heldout"), ("train_formats", "train"),
                          ("heldout_values", "heldout_values")):
            q = evaluate_engine(eng, n=a.eval_n, seed=4243, vocab_name="heldout", families=fam)
            res[name] = {"exact": round(q["exact"], 4), "parse_rate": round(q["parse_rate"], 4),
                         "by_family": q.get("by_family")}
        res["negatives_heldout"] = evaluate_negatives(eng, n=a.eval_n, families="neg_heldout")
        line = json.dumps(res)
        print(line, flush=True)
        with open(a.out, "a") as fh:
            fh.write(line + "\n")
        del eng, w, data
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
