"""Training-recipe / decoding probe for the extractor's held-out quality (GPU).

Each ``--run`` is a JSON dict of :class:`~smsgate_amd.models.train.TrainConfig`
overrides; every run trains the model, then scores held-out SMS through the HIP
engine once per ``--engine`` variant (JSON dict of EngineConfig overrides), and
prints one JSON line per (run, engine variant) with the field accuracies, the
first wrong answers (truth vs extracted) and the reference's three CASES.

    python scripts/quality_probe.py --run '{"steps": 2000, "batch": 128}' \\
        --run '{"steps": 2000, "batch": 128, "n_examples": 256000}' \\
        --engine '{}' --engine '{"copy_constrain": false}' --out gpurun_out/quality.jsonl
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _errors(items, answers, limit):
    from smsgate_amd.models.evaluate import _FIELDS, _norm_truth, _post

    out = []
    for it, ans in zip(items, answers):
        p = _post(it.body, it.timestamp, ans)
        truth = _norm_truth(it.answer)
        if p is None:
            out.append({"body": it.body, "unparsed": ans})
        else:
            bad = {f: [truth[f], (ans or {}).get(f)] for f in ("merchant", "city", "address")
                   if (getattr(p, f) or "") != truth[f]}
            if bad:
                out.append({"body": it.body, "wrong": bad})
        if len(out) >= limit:
            break
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="smollm-135m")
    p.add_argument("--run", action="append", default=[])
    p.add_argument("--engine", action="append", default=[])
    p.add_argument("--eval-n", type=int, default=1000)
    p.add_argument("--errors", type=int, default=20)
    p.add_argument("--save", default="", help="save the last run's weights here")
    p.add_argument("--load", default="", help="skip training: evaluate this checkpoint")
    p.add_argument("--out", default="")
    a = p.parse_args()
    import torch

    from smsgate_amd.models.evaluate import golden_case_results, score_answers
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import TrainConfig, train_extractor
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine
    from smsgate_amd.utils.synth import generate

    items = [s for s in generate(a.eval_n, seed=4242, vocab_name="heldout") if s.answer is not None]
    bodies = [normalize_body(s.body) for s in items]
    runs = [json.loads(r) for r in a.run] or [{}]
    engines = [json.loads(e) for e in a.engine] or [{}]
    for run in runs:
        t0 = time.perf_counter()
        if a.load:
            w = ExtractorWeights.load(a.load, CONFIGS[a.model], device=torch.device("cuda"))
            train_s = 0.0
        else:
            cfg = TrainConfig(model=a.model, log_every=200, data_parallel=False, **run)
            w = train_extractor(cfg, device="cuda", log=lambda s: print(s, file=sys.stderr, flush=True))
            train_s = time.perf_counter() - t0
        w.requires_grad_(False)
        for ek in engines:
            eng = ExtractionEngine(w, load_tokenizer(), EngineConfig(**{"max_slots": 1024,
                                                                        "buckets": (64, 256, 1024), **ek}))
            t1 = time.perf_counter()
            answers = eng.run(bodies)
            dec_s = time.perf_counter() - t1
            q = score_answers(items, answers)
            rec = {"run": run, "engine": ek, "train_s": round(train_s, 1), "eval_s": round(dec_s, 2),
                   "exact": round(q["exact"], 4), "parse_rate": round(q["parse_rate"], 4), "n": q["n"],
                   "field_acc": {k: round(v, 4) for k, v in q["field_acc"].items()},
                   "golden": golden_case_results(eng), "errors": _errors(items, answers, a.errors)}
            line = json.dumps(rec)
            print(line, flush=True)
            if a.out:
                os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
                with open(a.out, "a") as f:
                    f.write(line + "\n")
            del eng
            torch.cuda.empty_cache()
        if a.save:
            w.save(a.save)


if __name__ == "__main__":
    main()
