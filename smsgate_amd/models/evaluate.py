"""Score a trained extractor through the HIP serving engine and the real parse
post-processing.

Two numbers matter and they are different things:

* **parse rate** — the share of LLM-routed messages whose answer survives the
  reference's post-processing chain (date, card, decimals, ``ParsedSmsCore``
  validation: gemini_parser.py:224-268) and would be published on
  ``sms.parsed``.  This is what the headline benchmark's routing reports;
* **field accuracy** — exact match of each extracted value against the
  generator's ground truth (after the same post-processing for amounts / card /
  date), on SMS whose merchant / city / street vocabulary is disjoint from the
  training pools (:func:`~smsgate_amd.utils.synth.vocab` ``"heldout"``).
"""
from __future__ import annotations

from decimal import Decimal
from typing import Any, Dict, List, Optional, Sequence

__all__ = ["score_answers", "evaluate_engine", "golden_case_results", "golden_case_mismatches",
           "REFERENCE_EXPECTED"]

_FIELDS = ("txn_type", "date", "amount", "currency", "card", "merchant", "city", "address", "balance")


def _post(raw_body: str, ts: int, ans: Optional[Dict[str, Any]]):
    from ..models.domain import RawSMS
    from ..parse.pipeline import Outcome, postprocess_answer
    from ..parse.text import normalize_body

    if ans is None:
        return None
    raw = RawSMS(msg_id="e", device_id="d", sender="BANK", date=str(ts), body=raw_body, source="device")
    r = postprocess_answer(raw, normalize_body(raw_body), ans)
    return r.parsed if r.outcome is Outcome.PARSED else None


def _norm_truth(truth: Dict[str, Optional[str]]) -> Dict[str, str]:
    from ..parse.numeric import parse_ambiguous_decimal

    t = {k: (truth.get(k) or "") for k in _FIELDS}
    t["card"] = t["card"].replace("*", "").replace(" ", "")[:4]
    for k in ("amount", "balance"):
        t[k] = str(parse_ambiguous_decimal(t[k])) if t[k] else ""
    return t


def score_answers(items: Sequence[Any], answers: Sequence[Optional[Dict[str, Any]]]) -> Dict[str, Any]:
    """``items``: :class:`~smsgate_amd.utils.synth.SynthSMS` with answers;
    ``answers``: the raw extractor answers in the same order."""
    n = len(items)
    parsed = 0
    hits = {f: 0 for f in _FIELDS}
    whole = 0
    for it, ans in zip(items, answers):
        p = _post(it.body, it.timestamp, ans)
        if p is None:
            continue
        parsed += 1
        truth = _norm_truth(it.answer)
        got = {"txn_type": p.txn_type.value if hasattr(p.txn_type, "value") else str(p.txn_type),
               "date": (ans or {}).get("date", "") or "", "amount": str(Decimal(p.amount)) if p.amount is not None else "",
               "currency": p.currency or "", "card": p.card or "", "merchant": p.merchant or "", "city": p.city or "",
               "address": p.address or "", "balance": str(Decimal(p.balance)) if p.balance is not None else ""}
        ok = True
        for f in _FIELDS:
            same = str(got[f]).strip() == str(truth[f]).strip()
            hits[f] += same
            ok &= same
        whole += ok
    d = max(1, n)
    return {"n": n, "parse_rate": parsed / d, "field_acc": {f: hits[f] / d for f in _FIELDS}, "exact": whole / d}


def evaluate_engine(engine, n: int = 500, seed: int = 987654, vocab_name: str = "heldout") -> Dict[str, Any]:
    """Decode ``n`` generated SMS (LLM-routed kinds only) and score them."""
    from ..parse.text import normalize_body
    from ..utils.synth import generate

    items = [s for s in generate(n, seed=seed, vocab_name=vocab_name) if s.answer is not None]
    answers = engine.run([normalize_body(s.body) for s in items])
    out = score_answers(items, answers)
    out["vocab"] = vocab_name
    return out


def golden_case_results(engine) -> List[Optional[Dict[str, Any]]]:
    """The reference's three CASES (tests/test_parsers.py:11-58) through the
    engine and post-processing: the ParsedSMS fields, or None if unparsed."""
    from ..parse.text import normalize_body
    from ..utils.synth import reference_cases

    bodies = reference_cases()
    answers = engine.run([normalize_body(b) for b in bodies])
    out: List[Optional[Dict[str, Any]]] = []
    for b, a in zip(bodies, answers):
        p = _post(b, 1746541380, a)
        out.append(None if p is None else p.model_dump(mode="json"))
    return out


# the expected values of the reference's CASES (tests/test_parsers.py:11-58, asserted
# field by field like :73-86); dates as the ISO strings ParsedSMS serialises
REFERENCE_EXPECTED = (
    dict(merchant="TEST LLC", city="MOSKOW", address="TEST STR. 29, 24 AREA", amount="52.00", balance="1842.74",
         date="2025-05-06T14:23", card="0018", currency="USD", txn_type="debit"),
    dict(merchant="TEST", city="MOSKOW", address="", amount="3460.00", balance="1800.74",
         date="2025-05-06T15:11", card="0018", currency="USD", txn_type="debit"),
    dict(merchant="AMERIABANK API GATE", city="AM", address="", amount="27252.00", balance="391469.09",
         date="2025-06-10T20:51", card="7538", currency="AMD", txn_type="debit"),
)


def golden_case_mismatches(results: Sequence[Optional[Dict[str, Any]]]) -> List[str]:
    """Every field of :func:`golden_case_results` that differs from the
    reference's expectation, as ``"case<i>.<field>: got != want"`` (empty = all
    three CASES pass)."""
    bad: List[str] = []
    for i, (got, want) in enumerate(zip(results, REFERENCE_EXPECTED), 1):
        if got is None:
            bad.append(f"case{i}: not parsed")
            continue
        for k, v in want.items():
            g = got.get(k)
            if k in ("amount", "balance"):
                same = g is not None and Decimal(str(g)) == Decimal(v)
            elif k == "date":
                same = str(g or "").startswith(v)
            else:
                same = (g or "") == v
            if not same:
                bad.append(f"case{i}.{k}: {g!r} != {v!r}")
    return bad
