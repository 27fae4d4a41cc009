#!/usr/bin/env python3
"""Quality of the flagship training recipe over several training samples, on ONE GPU.

VERDICT r05 weak #1 / next #1: the bench's quality is one training sample (seed 0) and
the samples differ by points, so every training-mix change is judged on the mean over
seeds 0-3.  The recipe's training step is launch-bound at batch 128 (~100 TFLOP/s of a
2.5 PFLOP/s part), so the seeds train CONCURRENTLY: one child process per seed, each
with its own HIP queues, sharing the GPU (the parent never touches the GPU; children are
started before any of them initialises it).

Each child trains models/train.py ``recipe()`` (the bench's TrainConfig) with its seed
(data and init), then scores it with the PyTorch reference extractor
(models/evaluate.py TorchQAExtractor, the HIP kernel's decode rules) WITHOUT abstention
and keeps every answer's confidence, so the parent can sweep the abstention threshold:

* held-out formats / values, training formats (held-out names): exact, published-wrong;
* held-out / training negatives: the share published on sms.parsed;
* a VALIDATION set for the threshold: training layouts, held-out names, its own seed --
  the threshold is chosen on it, never on a held-out set.

Output: one JSON line per seed (``--out``) and a summary line with the seed means per
threshold.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SETS = (("heldout_formats", "heldout", 4243), ("heldout_values", "heldout_values", 4245),
        ("train_formats", "train", 4242), ("validation", "train", 7001))
NEG_SETS = (("negatives_heldout", "neg_heldout", 4246), ("negatives_train", "neg_train", 4247))
TAUS = (0.0, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)


def child(a) -> int:
    import torch

    from smsgate_amd.models.evaluate import TorchQAExtractor, evaluate_engine
    from smsgate_amd.models.train import ExamplePool, recipe, train_extractor
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.utils.synth import generate
    from smsgate_amd.models.evaluate import _post

    kw = json.loads(a.overrides) if a.overrides else {}
    for k, v in kw.pop("env", {}).items():
        os.environ[k] = str(v)
    tc = recipe(a.model, a.steps, a.batch, seed=a.seed, log_every=500, data_parallel=False, **kw)
    t0 = time.time()
    data = ExamplePool(tc.n_examples, seed=tc.seed, families=tc.families, workers=a.workers,
                       answer_format=tc.answer_format, negatives=tc.negatives).get()
    t1 = time.time()
    log = open(os.path.join(a.log_dir, f"seed{a.seed}.log"), "a")
    w = train_extractor(tc, device=a.device, data=data, log=lambda s: (log.write(s + "\n"), log.flush()))
    del data
    t2 = time.time()
    eng = TorchQAExtractor(w, batch=256, min_conf=0.0)
    res = {"seed": a.seed, "tag": a.tag, "overrides": a.overrides, "data_s": round(t1 - t0, 1),
           "train_s": round(t2 - t1, 1)}
    for name, fam, seed in SETS:
        q = evaluate_engine(eng, n=a.eval_n, seed=seed, vocab_name="heldout", families=fam, per_item=True)
        fams = [s.family for s in generate(a.eval_n, seed=seed, vocab_name="heldout", families=fam)
                if s.answer is not None]
        res[name] = {"exact": q["exact"], "published_wrong_rate": q["published_wrong_rate"],
                     "by_family": q["by_family"], "items": q["items"], "conf": q["conf"], "families": fams}
    for name, fam, seed in NEG_SETS:
        items = generate(a.eval_n, seed=seed, vocab_name="heldout", families=fam)
        answers = eng.run([normalize_body(s.body) for s in items])
        pub = [_post(s.body, s.timestamp, ans) is not None for s, ans in zip(items, answers)]
        res[name] = {"published": pub, "conf": [round(float(c), 5) for c in eng.last_conf],
                     "families": [s.family for s in items]}
    res["eval_s"] = round(time.time() - t2, 1)
    with open(a.child_out, "w") as fh:
        json.dump(res, fh)
    del eng, w
    torch.cuda.empty_cache()
    return 0


def _at(entry, tau):
    """(exact, published_wrong) rates of a scored set with abstention at ``tau``."""
    n = max(1, len(entry["items"]))
    ok = sum(1 for (p, e), c in zip(entry["items"], entry["conf"]) if p and e and c >= tau)
    wrong = sum(1 for (p, e), c in zip(entry["items"], entry["conf"]) if p and not e and c >= tau)
    return ok / n, wrong / n


def _fam_at(entry, tau):
    out = {}
    for f, (p, e), c in zip(entry["families"], entry["items"], entry["conf"]):
        k = out.setdefault(f, [0, 0, 0])
        k[0] += 1
        k[1] += bool(p and e and c >= tau)
        k[2] += bool(p and not e and c >= tau)
    return {f: (v[1] / v[0], v[2] / v[0]) for f, v in sorted(out.items())}


def summarise(results, taus=TAUS):
    """Seed means per threshold (exact / published-wrong per set, negatives published)."""
    import statistics as st

    out = {"seeds": [r["seed"] for r in results], "by_tau": {}}
    for tau in taus:
        row = {}
        for name, _, _ in SETS:
            ex = [_at(r[name], tau) for r in results]
            row[name] = {"exact": round(st.mean(e for e, _ in ex), 4), "wrong": round(st.mean(w for _, w in ex), 4),
                         "exact_per_seed": [round(e, 4) for e, _ in ex]}
            if name == "heldout_values":
                fams = [_fam_at(r[name], tau) for r in results]
                row[name]["by_family"] = {f: round(st.mean(fa[f][0] for fa in fams), 4) for f in fams[0]}
                row[name]["wrong_by_family"] = {f: round(st.mean(fa[f][1] for fa in fams), 4) for f in fams[0]}
        for name, _, _ in NEG_SETS:
            row[name] = round(st.mean(sum(p and c >= tau for p, c in zip(r[name]["published"], r[name]["conf"]))
                                      / max(1, len(r[name]["published"])) for r in results), 4)
        out["by_tau"][str(tau)] = row
    return out


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--seeds", default="0,1,2,3")
    p.add_argument("--model", default=None)
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--batch", type=int, default=None)
    p.add_argument("--eval-n", type=int, default=500)
    p.add_argument("--workers", type=int, default=4, help="example-building processes per seed")
    p.add_argument("--overrides", default="", help="JSON TrainConfig overrides (plus 'env': {...})")
    p.add_argument("--tag", default="recipe")
    p.add_argument("--variants", default="", help="JSON list of {tag, overrides}: several recipes at once")
    p.add_argument("--out", default="gpurun_out/qa_seeds.jsonl")
    p.add_argument("--log-dir", default="gpurun_out/qa_seeds_logs")
    p.add_argument("--device", default="cuda")
    p.add_argument("--child", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--child-out", default="")
    a = p.parse_args()
    os.makedirs(a.log_dir, exist_ok=True)
    if a.child:
        return child(a)
    seeds = [int(s) for s in a.seeds.split(",")]
    # --variants '[{"tag": "lr5e4", "overrides": {"lr": 5e-4}}, ...]': every variant x every
    # seed trains concurrently (one child each), one summary line per variant
    variants = json.loads(a.variants) if a.variants else [{"tag": a.tag, "overrides": a.overrides}]
    for v in variants:
        if isinstance(v.get("overrides"), dict):
            v["overrides"] = json.dumps(v["overrides"])
    procs = []
    for v in variants:
        v["seeds"] = [int(x) for x in v.get("seeds", seeds)]  # a variant may name its own seeds
        for s in v["seeds"]:
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--seed", str(s), "--eval-n", str(a.eval_n),
                   "--workers", str(a.workers), "--tag", v["tag"], "--device", a.device, "--log-dir", a.log_dir,
                   "--child-out", os.path.join(a.log_dir, f"{v['tag']}-seed{s}.json")]
            for k in ("model", "steps", "batch"):
                if getattr(a, k) is not None:
                    cmd += [f"--{k}", str(getattr(a, k))]
            if v.get("overrides"):
                cmd += ["--overrides", v["overrides"]]
            procs.append(((v["tag"], s), subprocess.Popen(cmd)))
    rcs = {key: pr.wait() for key, pr in procs}
    ok = True
    for v in variants:
        results = []
        vr = {s: rcs[(v["tag"], s)] for s in v["seeds"]}
        for s in v["seeds"]:
            path = os.path.join(a.log_dir, f"{v['tag']}-seed{s}.json")
            if vr[s] == 0 and os.path.exists(path):
                results.append(json.load(open(path)))
        if not results:
            print(json.dumps({"tag": v["tag"], "error": "no seed finished", "rcs": vr}))
            ok = False
            continue
        summ = summarise(results)
        summ.update(tag=v["tag"], overrides=v.get("overrides", ""), rcs=vr,
                    train_s=[r["train_s"] for r in results], data_s=[r["data_s"] for r in results])
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "a") as fh:
            fh.write(json.dumps(summ) + "\n")
        print(json.dumps({"tag": v["tag"], **{k: summ["by_tau"][k] for k in ("0.0",)}}), flush=True)
        ok &= all(x == 0 for x in vr.values())
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
