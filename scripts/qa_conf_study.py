#!/usr/bin/env python3
"""Offline study of abstention rules on a qa_diag.py dump (CPU only): decode every
scored set with the host reference decoder (serving/qa.py qa_decode_ref), score the
answers through the real post-processing (models/evaluate.py score_answers), compute
several candidate confidence measures per answer and print, per measure and
threshold, exact / published-wrong / declined per set (and held-out negatives
published).  The threshold the engine serves (EngineConfig.qa_min_conf) is chosen from
this table on the VALIDATION set (training layouts, held-out vocabulary), then read off
the held-out sets."""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Dict, List

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def _lse(x: np.ndarray) -> float:
    m = float(x.max())
    return m + float(np.log(np.exp(x - m).sum()))


def measures(cls, st, nl, en, body, flags, lay, c: int, raw) -> Dict[str, float]:
    """Candidate confidences of one decoded answer (``raw``: spans before absorption)."""
    from smsgate_amd.serving.qa import REJECT_TXN, TXN_TYPES, _pair_mask, qa_confidence

    n = len(body) - 1
    cl = np.asarray(cls, dtype=np.float64)
    p_cls = float(np.exp(cl[c] - _lse(cl)))
    srt = np.sort(cl)
    out = {"full_min": qa_confidence(cls, st, nl, en, n, c, raw), "cls": p_cls,
           "cls_margin": float(srt[-1] - srt[-2])}
    if TXN_TYPES[c] in REJECT_TXN:
        for k in ("pair_min", "pair_margin", "pair_prod", "field_margin_min"):
            out[k] = p_cls if not k.endswith("margin") and not k.endswith("margin_min") else out["cls_margin"]
        return out
    fb = flags[np.asarray(body[:n], dtype=np.int64)]
    pair_min, prod, marg = p_cls, p_cls, out["cls_margin"]
    for f, (bits, cap, s_need, e_need) in enumerate(lay.rules()):
        s_ = np.asarray(st[f][:n], dtype=np.float64)
        e_ = np.asarray(en[f][:n], dtype=np.float64)
        e_ = e_ - _lse(e_)  # log softmax of the end over the body
        vs, pairs = _pair_mask(fb, n, bits, cap, s_need, e_need)
        nul = float(nl[f])
        if pairs.any():
            sc = np.where(pairs, s_[:, None] + e_[None, :], -np.inf).ravel()
            cand = np.concatenate([sc[np.isfinite(sc)], [nul]])
        else:
            cand = np.asarray([nul])
        a, z = raw[f]
        chosen = nul if a < 0 else float(s_[a] + e_[z])
        p = float(np.exp(chosen - _lse(cand)))  # the decoded decision among the VALID ones
        srt2 = np.sort(cand)
        m2 = float(srt2[-1] - srt2[-2]) if len(cand) > 1 else 30.0
        pair_min, prod, marg = min(pair_min, p), prod * p, min(marg, m2)
    out.update(pair_min=pair_min, pair_prod=prod, pair_margin=marg)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dumps", nargs="+")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from smsgate_amd.models.evaluate import score_answers
    from smsgate_amd.models.extractor import SPAN_PTR0
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import DEFAULT_FIELDS
    from smsgate_amd.serving.qa import null_rejection, qa_decode_ref, qa_expand, qa_layout, qa_token_flags
    from smsgate_amd.utils.synth import generate

    from scripts.qa_diag import SETS

    tok = load_tokenizer()
    names = [f.name for f in DEFAULT_FIELDS]
    table: Dict[str, Dict[str, List]] = {}
    for path in a.dumps:
        z = np.load(path)
        meta = json.load(open(path.replace(".npz", ".json")))
        for name, fam, seed in SETS:
            ids = z[f"{name}_ids"]
            msgs = [list(r[r >= 0]) for r in ids]
            cls, st, nl, en = (z[f"{name}_{k}"] for k in ("cls", "start", "null", "end"))
            n_pos = st.shape[-1]
            lay = qa_layout(SPAN_PTR0, n_pos, 9)
            flags = qa_token_flags(tok, lay.vocab)
            items = [s for s in generate(500, seed=seed, vocab_name="heldout", families=fam) if s.answer is not None]
            assert [s.body for s in items] == [d["body"] for d in meta["sets"][name]], name
            dec = qa_decode_ref(cls, st, nl, en, msgs, flags, lay)
            toks = [qa_expand(tok, lay, c, sp, m) for (c, sp), m in zip(dec, msgs)]
            answers = [null_rejection(dict(zip(names, v))) for v in tok.decode_fields(toks, len(names))]
            if fam.startswith("neg"):  # non-transactions: every published answer is wrong
                from smsgate_amd.models.evaluate import _post

                pubs = [_post(it.body, it.timestamp, ans) is not None for it, ans in zip(items, answers)]
                sc = {"items": [(p_, False) for p_ in pubs], "exact": 0.0,
                      "published_wrong_rate": sum(pubs) / len(pubs), "declined_rate": 0.0}
            else:
                sc = score_answers(items, answers, by_family=True, per_item=True)
            # raw spans (before absorption) for the measures: decode once more without absorption
            raw = []
            for m, body in enumerate(msgs):
                raw.append(_raw_spans(cls[m], st[m], nl[m], en[m], body, flags, lay))
            rows = table.setdefault(name, {"pub": [], "ok": [], "fam": [], "neg": [], "m": []})
            for i, (it, (pub, ok)) in enumerate(zip(items, sc["items"])):
                rows["pub"].append(pub)
                rows["ok"].append(ok)
                rows["fam"].append(it.family)
                rows["m"].append(measures(cls[i], st[i], nl[i], en[i], msgs[i], flags, lay, dec[i][0], raw[i]))
            print(f"{path} {name}: exact {sc['exact']:.4f} wrong {sc['published_wrong_rate']:.4f} "
                  f"declined {sc['declined_rate']:.4f}", flush=True)
    report = {}
    keys = list(next(iter(table.values()))["m"][0].keys())
    for key in keys:
        vals = np.concatenate([[r[key] for r in t["m"]] for t in table.values()])
        qs = sorted(set(np.quantile(vals, np.linspace(0.0, 0.3, 31)).round(6)))
        rep = []
        for tau in [0.0] + list(qs):
            row = {"tau": float(tau)}
            for name, t in table.items():
                keep = np.asarray([r[key] >= tau for r in t["m"]])
                pub, ok = np.asarray(t["pub"]), np.asarray(t["ok"])
                N = len(pub)
                row[name] = (round(float((ok & keep).mean()), 4), round(float((pub & ~ok & keep).mean()), 4))
                if name == "heldout_values":
                    fams = np.asarray(t["fam"])
                    row["hv_min_family"] = round(min(float((ok & keep)[fams == f].mean()) for f in set(t["fam"])), 4)
            rep.append(row)
        report[key] = rep
        print(f"== {key}")
        for row in rep[:: max(1, len(rep) // 12)]:
            print("  ", json.dumps(row))
    if a.out:
        json.dump(report, open(a.out, "w"))
    return 0


def _raw_spans(cls, st, nl, en, body, flags, lay):
    from smsgate_amd.serving.qa import REJECT_TXN, TXN_TYPES, _pair_mask

    c = int(np.argmax(np.asarray(cls, dtype=np.float32)))
    if TXN_TYPES[c] in REJECT_TXN:
        return [(-1, -1)] * lay.n_copy
    n = len(body) - 1
    fb = flags[np.asarray(body[:n], dtype=np.int64)]
    out = []
    for f, (bits, cap, s_need, e_need) in enumerate(lay.rules()):
        s_ = np.asarray(st[f][:n], dtype=np.float32)
        e_ = np.asarray(en[f][:n], dtype=np.float32)
        vs, pairs = _pair_mask(fb, n, bits, cap, s_need, e_need)
        if not pairs.any() or np.float32(nl[f]) >= s_[vs].max():
            out.append((-1, -1))
            continue
        k = int(np.argmax(np.where(pairs, s_[:, None] + e_[None, :], -np.inf)))
        out.append((k // n, k % n))
    return out


if __name__ == "__main__":
    sys.exit(main())
