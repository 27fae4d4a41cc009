"""Train the extractor on the TRAINING template families and score it, during and
after training, on SMS layouts it never saw (utils/synth.py HELDOUT_FAMILIES).

One JSON line per evaluation (``--jsonl``): step, seconds, exact / field accuracy
on the training families (held-out vocabulary), on the held-out families (with the
regex backend's score on the same items and a per-family breakdown) and the
reference's three CASES.  ``--out`` saves the final bf16 weights (safetensors).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="smollm-135m")
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--examples", type=int, default=0, help="0 = steps x batch")
    p.add_argument("--eval-every", type=int, default=500)
    p.add_argument("--eval-n", type=int, default=600)
    p.add_argument("--workers", type=int, default=12)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--families", default="train")
    p.add_argument("--out", default="")
    p.add_argument("--jsonl", default="gpurun_out/family_probe.jsonl")
    p.add_argument("--tag", default="")
    p.add_argument("--format", default="copy", choices=["copy", "span"])
    a = p.parse_args()

    from smsgate_amd.models.train import ExamplePool, TrainConfig, train_extractor

    n = a.examples or a.steps * a.batch
    t0 = time.perf_counter()
    pool = ExamplePool(n, seed=a.seed, families=a.families, workers=a.workers,  # before the GPU is touched
                       answer_format=a.format)

    import torch

    from smsgate_amd.models.evaluate import evaluate_engine, golden_case_mismatches, golden_case_results
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine

    os.makedirs(os.path.dirname(a.jsonl) or ".", exist_ok=True)
    t_train = [0.0]

    def evaluate(step, w):
        te = time.perf_counter()
        eng = ExtractionEngine(w, load_tokenizer(), EngineConfig(max_slots=1024, buckets=(64, 256, 1024)))
        tr = evaluate_engine(eng, n=a.eval_n // 2, seed=4242, vocab_name="heldout", families="train")
        ho = evaluate_engine(eng, n=a.eval_n, seed=4243, vocab_name="heldout", families="heldout", with_regex=True)
        leg = evaluate_engine(eng, n=a.eval_n // 2, seed=4244, vocab_name="heldout")
        bad = golden_case_mismatches(golden_case_results(eng))
        # a few wrong answers per held-out family: what the model gets wrong, field by field
        from smsgate_amd.models.evaluate import _expected, _post
        from smsgate_amd.parse.text import normalize_body
        from smsgate_amd.utils.synth import generate

        items = [x for x in generate(240, seed=4245, vocab_name="heldout", families="heldout") if x.answer]
        got = eng.run([normalize_body(x.body) for x in items])
        fails = {}
        for x, g in zip(items, got):
            p = _post(x.body, x.timestamp, g)
            want = _expected(x)
            diff = {}
            if p is None:
                diff = {"unparsed": g}
            else:
                for k in want:
                    v = getattr(p, k)
                    v = v.value if hasattr(v, "value") else v
                    if str(v) != str(want[k]):
                        diff[k] = [str(v), str(want[k])]
            if diff and len(fails.setdefault(x.family, [])) < 2:
                fails[x.family].append({"body": x.body[:160], "diff": diff})
        rec = {"tag": a.tag, "model": a.model, "format": a.format, "step": step, "train_s": round(time.perf_counter() - t0, 1),
               "batch": a.batch, "lr": a.lr,
               "train_formats": {"exact": round(tr["exact"], 4), "by_family": tr["by_family"]},
               "legacy_mix_exact": round(leg["exact"], 4),
               "heldout_formats": {"exact": round(ho["exact"], 4), "regex_exact": round(ho["regex_exact"], 4),
                                   "field_acc": {k: round(v, 4) for k, v in ho["field_acc"].items()},
                                   "by_family": ho["by_family"]},
               "cases_mismatches": bad, "heldout_failures": fails, "eval_s": round(time.perf_counter() - te, 1)}
        print(json.dumps(rec), flush=True)
        with open(a.jsonl, "a") as f:
            f.write(json.dumps(rec) + "\n")
        del eng
        torch.cuda.empty_cache()

    data = pool.get()
    print(f"examples: {len(data)} in {time.perf_counter() - t0:.1f}s", flush=True)
    cfg = TrainConfig(model=a.model, steps=a.steps, batch=a.batch, lr=a.lr, warmup=a.warmup, n_examples=n,
                      seed=a.seed, log_every=200, eval_every=a.eval_every, families=a.families, data_parallel=False,
                      answer_format=a.format)
    w = train_extractor(cfg, device="cuda", log=lambda s: print(s, flush=True), on_eval=evaluate, data=data)
    evaluate(a.steps, w)
    if a.out:
        w.save(a.out)
        print(f"saved {a.out}", flush=True)


if __name__ == "__main__":
    main()
