"""Score a trained extractor through the HIP serving engine and the real parse
post-processing.

Two numbers matter and they are different things:

* **parse rate** — the share of LLM-routed messages whose answer survives the
  reference's post-processing chain (date, card, decimals, ``ParsedSmsCore``
  validation: gemini_parser.py:224-268) and would be published on
  ``sms.parsed``.  This is what the headline benchmark's routing reports;
* **field accuracy** — each stored value (after the real post-processing
  chain) against the generator's expected value, on SMS whose merchant / city /
  street vocabulary is disjoint from the training pools
  (:func:`~smsgate_amd.utils.synth.vocab` ``"heldout"``) — and, for
  ``families="heldout"``, in template families never trained on
  (:data:`~smsgate_amd.utils.synth.HELDOUT_FAMILIES`).
"""
from __future__ import annotations

from decimal import Decimal
from typing import Any, Dict, List, Optional, Sequence, Tuple

__all__ = ["score_answers", "evaluate_engine", "regex_answers", "golden_case_results", "golden_case_mismatches",
           "TorchQAExtractor", "evaluate_negatives",
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


def _expected(it: Any) -> Dict[str, Any]:
    """The final values a correct parse must produce: the generator's own
    ``expected`` (utils/synth.py), independent of the pipeline under test."""
    exp = getattr(it, "expected", None)
    if exp is not None:
        return exp
    from ..parse.numeric import parse_ambiguous_decimal
    from ..parse.dates import parse_custom_datetime

    t = {k: (it.answer.get(k) or "") for k in _FIELDS}
    return dict(txn_type=t["txn_type"], date=parse_custom_datetime(t["date"]),
                amount=parse_ambiguous_decimal(t["amount"]), currency=t["currency"],
                card=t["card"].replace("*", "").replace(" ", "")[-4:], merchant=t["merchant"], city=t["city"],
                address=t["address"], balance=parse_ambiguous_decimal(t["balance"]))


def _same(field: str, got: Any, want: Any) -> bool:
    if field in ("amount", "balance"):
        return got is not None and want is not None and Decimal(got) == Decimal(want)
    if field == "date":
        return got == want
    return str(got or "").strip() == str(want or "").strip()


def score_answers(items: Sequence[Any], answers: Sequence[Optional[Dict[str, Any]]],
                  by_family: bool = False, per_item: bool = False) -> Dict[str, Any]:
    """``items``: :class:`~smsgate_amd.utils.synth.SynthSMS` with answers;
    ``answers``: the raw extractor answers in the same order.  Every field is
    compared AFTER the real post-processing chain (the stored ``ParsedSMS``
    value: datetime, Decimal, ISO currency, 4-digit card) with the generator's
    expected value; ``exact`` = all nine fields right.  ``published_wrong_rate``: the
    share that would be published on sms.parsed with a wrong field (parsed, not
    exact) -- the cost a wrong answer has and a declined one (``declined_rate``:
    answered as a non-transaction, dead-lettered) does not.  ``by_family``: also the
    exact rate per template family (and ``wrong_by_family``); ``per_item``: also the
    (published, exact) flags of every item (calibration)."""
    from ..serving.qa import REJECT_TXN

    n = len(items)
    parsed = 0
    declined = 0
    hits = {f: 0 for f in _FIELDS}
    whole = 0
    fam_n: Dict[str, int] = {}
    fam_ok: Dict[str, int] = {}
    fam_wrong: Dict[str, int] = {}
    flags: List[Tuple[bool, bool]] = []
    for it, ans in zip(items, answers):
        fam = getattr(it, "family", "legacy")
        fam_n[fam] = fam_n.get(fam, 0) + 1
        declined += bool(ans) and ans.get("txn_type") in REJECT_TXN
        p = _post(it.body, it.timestamp, ans)
        if p is None:
            flags.append((False, False))
            continue
        parsed += 1
        want = _expected(it)
        got = {"txn_type": p.txn_type.value if hasattr(p.txn_type, "value") else str(p.txn_type),
               "date": p.date, "amount": p.amount, "currency": p.currency, "card": p.card,
               "merchant": p.merchant, "city": p.city, "address": p.address, "balance": p.balance}
        ok = True
        for f in _FIELDS:
            same = _same(f, got[f], want[f])
            hits[f] += same
            ok &= same
        whole += ok
        fam_ok[fam] = fam_ok.get(fam, 0) + ok
        fam_wrong[fam] = fam_wrong.get(fam, 0) + (not ok)
        flags.append((True, ok))
    d = max(1, n)
    out = {"n": n, "parse_rate": parsed / d, "field_acc": {f: hits[f] / d for f in _FIELDS}, "exact": whole / d,
           "published_wrong_rate": (parsed - whole) / d, "declined_rate": declined / d}
    if by_family:
        out["by_family"] = {f: round(fam_ok.get(f, 0) / c, 4) for f, c in sorted(fam_n.items())}
        out["wrong_by_family"] = {f: round(fam_wrong.get(f, 0) / c, 4) for f, c in sorted(fam_n.items())}
    if per_item:
        out["items"] = flags
    return out


def regex_answers(items: Sequence[Any]) -> List[Dict[str, Any]]:
    """The rule-based backend's answers for ``items`` (the "could a regex do it?" baseline)."""
    from ..parse.backends.regex import UNKNOWN_ANSWER, extract_rule_based

    return [extract_rule_based(it.body) or dict(UNKNOWN_ANSWER) for it in items]


def evaluate_engine(engine, n: int = 500, seed: int = 987654, vocab_name: str = "heldout",
                    families: Any = None, with_regex: bool = False, per_item: bool = False) -> Dict[str, Any]:
    """Decode ``n`` generated SMS (LLM-routed kinds only) and score them.
    ``families``: None = the legacy mix, else template families (``"heldout"`` = the
    layouts never trained on); ``with_regex`` adds the regex backend's score on the
    same items (``regex_exact``)."""
    from ..parse.text import normalize_body
    from ..utils.synth import generate

    items = [s for s in generate(n, seed=seed, vocab_name=vocab_name, families=families) if s.answer is not None]
    answers = engine.run([normalize_body(s.body) for s in items])
    out = score_answers(items, answers, by_family=families is not None, per_item=per_item)
    if per_item and getattr(engine, "last_conf", None) is not None and len(engine.last_conf) == len(items):
        out["conf"] = [round(float(c), 5) for c in engine.last_conf]
    out["vocab"] = vocab_name
    if families is not None:
        out["families"] = families if isinstance(families, str) else list(families)
    if with_regex:
        out["regex_exact"] = score_answers(items, regex_answers(items))["exact"]
    return out


class TorchQAExtractor:
    """A qa-format model (serving/qa.py) served by the PyTorch reference forward and
    the host reference decoder -- the engine interface's ``run`` without the HIP path
    (quality probes, CPU tests; serving/qa_engine.py is the GPU engine)."""

    def __init__(self, weights, tokenizer=None, max_body: int = 128, batch: int = 256,
                 compute_dtype=None, min_conf: Optional[float] = None) -> None:
        import torch

        from ..serving.engine import QA_MIN_CONF

        from ..serving.qa import qa_layout, qa_token_flags
        from .extractor import SPAN_PTR0
        from .tokenizer import load_tokenizer

        self.w = weights
        self.tok = tokenizer or load_tokenizer()
        cfg = weights.cfg
        if cfg.qa_queries <= 0:
            raise ValueError("TorchQAExtractor: not a qa-format model")
        self.lay = qa_layout(SPAN_PTR0, cfg.span_positions, cfg.qa_queries)
        self.flags = qa_token_flags(self.tok, self.lay.vocab)
        self.max_body = max_body
        self.batch = batch
        self.compute_dtype = compute_dtype or torch.float32
        # abstention threshold (serving/qa.py qa_decode_ref); the confidence of every
        # answer of the last run() is kept in ``last_conf`` (calibration)
        self.min_conf = QA_MIN_CONF if min_conf is None else float(min_conf)
        self.last_conf: List[float] = []

    def scores(self, msgs: Sequence[Sequence[int]]):
        """The head's fp32 scores of ``msgs`` (``body <ans>`` ids): (cls [M, 4],
        start [M, nf, n_pos], null [M, nf], end [M, nf, n_pos]) numpy arrays."""
        import numpy as np
        import torch

        from ..parse.schema import EXTRACTOR_PROMPT
        from ..serving.qa import qa_logits
        from .extractor import reference_forward
        from .train import qa_batch

        prefix = self.tok.prefix_ids(EXTRACTOR_PROMPT)
        dev = self.w.embed.device
        parts = []
        for k in range(0, len(msgs), self.batch):
            part = [list(m) for m in msgs[k:k + self.batch]]
            exs = [(m, (0, [(-1, -1)] * self.lay.n_copy)) for m in part]
            ids, add, qpos, _ = qa_batch(prefix, exs, self.tok.pad, dev, self.lay)
            with torch.no_grad():
                h = reference_forward(self.w, ids, compute_dtype=self.compute_dtype, return_hidden=True, add_ids=add)
                parts.append([t.float().cpu().numpy() for t in qa_logits(h, self.w.embed, qpos, self.lay)])
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(4))

    def decode_ids(self, msgs: Sequence[Sequence[int]]):
        """(class, spans) per message (``body <ans>`` ids)."""
        from ..serving.qa import qa_decode_ref

        out = []
        self.last_conf = []
        for k in range(0, len(msgs), self.batch):
            part = [list(m) for m in msgs[k:k + self.batch]]
            cls, st, nl, en = self.scores(part)
            out += qa_decode_ref(cls, st, nl, en, part, self.flags, self.lay, self.min_conf, self.last_conf)
        return out

    def run(self, bodies: Sequence[str]) -> List[Dict[str, Optional[str]]]:
        from ..serving.fsm import DEFAULT_FIELDS
        from ..serving.qa import null_rejection, qa_expand

        msgs = self.tok.message_ids(list(bodies), self.max_body)
        dec = self.decode_ids(msgs)
        toks = [qa_expand(self.tok, self.lay, c, sp, m) for (c, sp), m in zip(dec, msgs)]
        names = [f.name for f in DEFAULT_FIELDS]
        return [null_rejection(dict(zip(names, vals))) for vals in self.tok.decode_fields(toks, len(names))]


def evaluate_negatives(engine, n: int = 500, seed: int = 4244, vocab_name: str = "heldout",
                       families: Any = "neg_heldout") -> Dict[str, Any]:
    """Non-transaction SMS (utils/synth.py NEG_FAMILIES) through the extractor and the
    real post-processing: ``false_parsed_rate`` = the share that would be published on
    sms.parsed (the reference routes them to the DLQ as unmatched), per family too."""
    from ..parse.text import normalize_body
    from ..utils.synth import generate

    items = generate(n, seed=seed, vocab_name=vocab_name, families=families)
    answers = engine.run([normalize_body(s.body) for s in items])
    fam_n: Dict[str, int] = {}
    fam_bad: Dict[str, int] = {}
    bad = 0
    txn: Dict[str, int] = {}
    for it, ans in zip(items, answers):
        fam_n[it.family] = fam_n.get(it.family, 0) + 1
        t = str((ans or {}).get("txn_type"))
        txn[t] = txn.get(t, 0) + 1
        parsed = _post(it.body, it.timestamp, ans) is not None
        bad += parsed
        fam_bad[it.family] = fam_bad.get(it.family, 0) + parsed
    return {"n": len(items), "false_parsed_rate": bad / max(1, len(items)), "families": families,
            "by_family": {f: round(fam_bad.get(f, 0) / c, 4) for f, c in sorted(fam_n.items())},
            "txn_type": dict(sorted(txn.items()))}


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
