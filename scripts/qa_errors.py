#!/usr/bin/env python3
"""Error analysis of a trained extractor: the held-out SMS it gets wrong, field by
field (body, the answer after post-processing, the generator's expected values), and
the non-transactions it lets through.  Loads a checkpoint (e.g. the bench's weights
cache from the same GPU call) and serves it through its engine.

    python scripts/qa_errors.py --weights /tmp/smsgate_bench_weights/<file> > errors.jsonl
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--weights", default="")
    p.add_argument("--n", type=int, default=600)
    p.add_argument("--per-family", type=int, default=6)
    a = p.parse_args()
    import torch

    from smsgate_amd.models.evaluate import _expected, _post, _same
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights
    from smsgate_amd.parse.backends.local_llm import build_engine
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.utils.synth import generate

    path = a.weights or sorted(glob.glob("/tmp/smsgate_bench_weights/*.safetensors"), key=os.path.getmtime)[-1]
    w = ExtractorWeights.load(path, CONFIGS["smollm-135m"], device=torch.device("cuda"))
    eng = build_engine("smollm-135m", weights=w, max_slots=2048)
    fields = ("txn_type", "date", "amount", "currency", "card", "merchant", "city", "address", "balance")
    shown = {}
    for sel, seed in (("heldout", 4243), ("train", 4242), ("heldout_values", 4245), ("neg_heldout", 4246)):
        items = generate(a.n, seed=seed, vocab_name="heldout", families=sel)
        answers = eng.run([normalize_body(s.body) for s in items])
        for it, ans in zip(items, answers):
            if shown.get(it.family, 0) >= a.per_family:
                continue
            p_ = _post(it.body, it.timestamp, ans)
            if it.kind == "negative":
                if p_ is None:
                    continue
                rec = {"set": sel, "family": it.family, "body": it.body, "answer": ans, "error": "false parse"}
            else:
                if p_ is None:
                    rec = {"set": sel, "family": it.family, "body": it.body, "answer": ans, "error": "not parsed"}
                else:
                    want = _expected(it)
                    got = {"txn_type": p_.txn_type.value, "date": p_.date, "amount": p_.amount,
                           "currency": p_.currency, "card": p_.card, "merchant": p_.merchant, "city": p_.city,
                           "address": p_.address, "balance": p_.balance}
                    bad = {f: [str(got[f]), str(want[f])] for f in fields if not _same(f, got[f], want[f])}
                    if not bad:
                        continue
                    rec = {"set": sel, "family": it.family, "body": it.body, "wrong": bad}
            shown[it.family] = shown.get(it.family, 0) + 1
            print(json.dumps(rec, ensure_ascii=False, default=str), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
