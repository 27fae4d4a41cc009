"""Training curve of the extractor: train on the GPU, and every --eval-every steps
decode held-out SMS (vocabulary disjoint from training) through the HIP engine
and the real post-processing; print one JSON line per evaluation.

    python scripts/train_curve.py --model smollm-135m --batch 128 --steps 1500 --eval-every 250
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
    p.add_argument("--steps", type=int, default=1500)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--examples", type=int, default=60000)
    p.add_argument("--eval-every", type=int, default=250)
    p.add_argument("--eval-n", type=int, default=600)
    p.add_argument("--out", default="")
    a = p.parse_args()
    import torch

    from smsgate_amd.models.evaluate import evaluate_engine, golden_case_results
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import TrainConfig, train_extractor
    from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine

    t0 = time.perf_counter()
    paused = [0.0]

    def ev(step, w):
        t = time.perf_counter()
        eng = ExtractionEngine(w, load_tokenizer(), EngineConfig(max_slots=1024, buckets=(64, 1024),
                                                                  use_graphs=False))
        r = evaluate_engine(eng, n=a.eval_n)
        gold = golden_case_results(eng)
        del eng
        torch.cuda.empty_cache()
        paused[0] += time.perf_counter() - t
        print(json.dumps({"step": step, "train_s": round(time.perf_counter() - t0 - paused[0], 1), **r,
                          "golden_ok": [g is not None for g in gold], "golden": gold}), flush=True)

    cfg = TrainConfig(model=a.model, steps=a.steps, batch=a.batch, lr=a.lr, warmup=a.warmup,
                      n_examples=a.examples, eval_every=a.eval_every, log_every=100)
    w = train_extractor(cfg, device="cuda", log=lambda s: print(s, flush=True), on_eval=ev)
    ev(a.steps, w)
    if a.out:
        w.save(a.out)


if __name__ == "__main__":
    main()
