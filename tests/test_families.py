"""Template families of the synthetic SMS generator.

The local extractor replaces a format-agnostic Gemini prompt
(/root/reference/libs/gemini_parser.py:37-61), so it is scored on SMS layouts it
never saw in training.  These CPU tests pin the ground the GPU evaluation stands on:

* the split is by family (>= 20 training families, held-out families disjoint);
* every family's gold answer, run through the real post-processing chain, gives the
  generator's ``expected`` values (so a correct extraction scores 1.0);
* every gold answer is reachable by the copy-constrained schema decoder and fits the
  per-field token caps (so a perfect model is not blocked by the FSM);
* the rule-based regex backend fails the held-out families (<= 0.3 exact): the set
  measures something a fixed-template parser cannot do.
"""
from __future__ import annotations

from collections import Counter

import pytest

from smsgate_amd.models.domain import RawSMS
from smsgate_amd.models.evaluate import score_answers
from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.models.train import answer_tokens
from smsgate_amd.parse.backends.regex import UNKNOWN_ANSWER, extract_rule_based
from smsgate_amd.parse.canonical import CURRENCY_ALIASES
from smsgate_amd.parse.pipeline import Outcome, postprocess_answer
from smsgate_amd.parse.text import normalize_body, worker_should_skip
from smsgate_amd.serving.fsm import DEFAULT_FIELDS, build_fsm
from smsgate_amd.utils import synth
from smsgate_amd.utils.synth import FAMILIES, HELDOUT_FAMILIES, TRAIN_FAMILIES, generate


@pytest.fixture(scope="module")
def tk_fsm():
    tk = load_tokenizer()
    return tk, build_fsm(tk, (tk.vocab_size + 63) // 64 * 64)


def test_split_is_by_family():
    assert len(TRAIN_FAMILIES) >= 20 and len(HELDOUT_FAMILIES) >= 5
    assert not set(TRAIN_FAMILIES) & set(HELDOUT_FAMILIES)
    assert {"legacy_purchase", "legacy_account"} <= set(TRAIN_FAMILIES)
    tr = {s.family for s in generate(3000, seed=3, families="train")}
    ho = {s.family for s in generate(1000, seed=3, families="heldout")}
    assert tr == set(TRAIN_FAMILIES) and ho == set(HELDOUT_FAMILIES)
    # the three languages and both transaction types occur
    assert {f.lang for f in FAMILIES} == {"en", "ru", "tr"} and {f.txn for f in FAMILIES} == {"debit", "credit"}


def test_generator_symbols_agree_with_parse_aliases():
    for code, sym in synth._SYMBOL.items():
        assert CURRENCY_ALIASES[sym] == code
    for code, word in synth._WORD.items():
        assert CURRENCY_ALIASES[word.rstrip(".").upper()] == code


def _got(p):
    return dict(txn_type=p.txn_type.value, date=p.date, amount=p.amount, currency=p.currency, card=p.card,
                merchant=p.merchant, city=p.city, address=p.address, balance=p.balance)


@pytest.mark.parametrize("which", ["train", "heldout"])
def test_gold_answers_postprocess_to_expected(which):
    bad = Counter()
    for s in generate(3000, seed=17, vocab_name="heldout", families=which):
        raw = RawSMS(msg_id="e", device_id="d", sender="B", date=str(s.timestamp), body=s.body, source="device")
        r = postprocess_answer(raw, normalize_body(s.body), s.answer)
        assert r.outcome is Outcome.PARSED, (s.family, s.body, r.error)
        got = _got(r.parsed)
        for k, v in s.expected.items():
            bad[(s.family, k)] += got[k] != v
    assert not +bad, +bad


@pytest.mark.parametrize("which", ["train", "heldout"])
def test_score_of_gold_answers_is_one(which):
    items = generate(400, seed=23, vocab_name="heldout", families=which)
    res = score_answers(items, [s.answer for s in items])
    assert res["exact"] == 1.0 and res["parse_rate"] == 1.0, res


def _walk_ok(fsm, ids, body):
    s, prev = fsm.start_state, body[-1]
    for t in ids:
        if not fsm.copy_mask_host(s, prev, body)[t]:
            return False
        s, prev = fsm.step_host(s, t), t
    return s == fsm.done_state


@pytest.mark.parametrize("which", ["train", "heldout", "heldout_values"])
def test_gold_answers_reachable_by_qa_decoder(which):
    """Every gold value is a span the served (qa) decoder can produce: in its field's
    token class, at word boundaries, with the field kind's edge tokens and inside the
    field's token cap -- so a perfect model is never blocked by the decode rules."""
    from smsgate_amd.models.train import answer_fsm
    from smsgate_amd.serving.qa import qa_targets

    tk = load_tokenizer()
    spec = answer_fsm(tk, "qa")
    bad = Counter()
    longest = Counter()
    for s in generate(1500, seed=29, vocab_name="heldout", families=which):
        b = normalize_body(s.body)
        enc = tk.encode_offsets([b])[0]
        t = qa_targets(tk, spec.lay, spec.flags, s.answer, b, enc, len(tk.message_ids([b], 128)[0]))
        if t is None:
            bad[s.family] += 1
            continue
        for f, (a, z) in zip(DEFAULT_FIELDS[1:], t[1]):
            longest[f.name] = max(longest[f.name], z - a + 1 if a >= 0 else 0)
    assert not bad, bad
    for f in DEFAULT_FIELDS[1:]:  # at most ~3/4 of a cap is used: headroom for longer real values
        assert longest[f.name] <= max(2, int(0.75 * f.cap) + 1), (f.name, longest[f.name], f.cap)


@pytest.mark.parametrize("which", [["legacy_purchase", "legacy_account", "legacy_credit"]])
def test_gold_answers_reachable_by_copy_fsm(tk_fsm, which):
    """The copy format (the autoregressive engine's) on the reference's own formats."""
    tk, fsm = tk_fsm
    bad = Counter()
    for s in generate(600, seed=29, vocab_name="heldout", families=which):
        b = normalize_body(s.body)
        enc = tk.encode_offsets([b])[0]
        ids = answer_tokens(tk, fsm, s.answer, b, enc)
        if ids is None or not _walk_ok(fsm, ids, tk.message_ids([b], 128)[0]):
            bad[s.family] += 1
    assert not bad, bad


def test_bodies_fit_the_prompt_budget(tk_fsm):
    tk, _ = tk_fsm
    items = generate(3000, seed=31, vocab_name="heldout", families="all")
    lens = [len(e) for e in tk.encode_batch([normalize_body(s.body) for s in items])]
    assert max(lens) <= 110 and sum(lens) / len(lens) < 50  # max_body_tokens is 128


def test_transactions_pass_the_word_keyword_filter():
    items = generate(5000, seed=37, vocab_name="heldout", families="all")
    assert sum(worker_should_skip(s.body) for s in items) == 0


def test_regex_backend_fails_heldout_families():
    """The held-out set only counts if a fixed-template parser cannot do it."""
    ho = generate(600, seed=41, vocab_name="heldout", families="heldout")
    legacy = generate(300, seed=41, vocab_name="heldout", families=["legacy_purchase", "legacy_account"])

    def regex_exact(items):
        return score_answers(items, [extract_rule_based(s.body) or dict(UNKNOWN_ANSWER) for s in items])["exact"]

    assert regex_exact(ho) <= 0.3
    assert regex_exact(legacy) == 1.0


def test_procedural_layouts_never_draw_a_heldout_signature():
    import random

    r = random.Random(5)
    seen = set()
    for lang in ("en", "ru", "tr"):
        for _ in range(20000):
            order, multi = synth._proc_layout(r, lang)
            assert (lang, order, multi) not in synth._HELDOUT_SIGNATURES
            seen.add((lang, order, multi))
    assert len(seen) > 500  # and they are diverse
    # each held-out family's own layout is one of the excluded signatures
    assert len(synth._HELDOUT_SIGNATURES) == 5 and {s[0] for s in synth._HELDOUT_SIGNATURES} == {"en", "ru", "tr"}


# ------------------------------------------------ non-transactions (VERDICT r04 missing #1)
def test_negative_families_split_and_pass_the_keyword_filters():
    """>= 8 non-transaction families in EN / RU / translit, split by family; every body
    passes BOTH keyword filters (the worker's and the parser's OTP pre-filter), so the
    extractor itself must reject it."""
    from smsgate_amd.parse.text import llm_should_skip
    from smsgate_amd.utils.synth import NEG_FAMILIES, NEG_HELDOUT_FAMILIES, NEG_TRAIN_FAMILIES, is_negative

    assert len(NEG_TRAIN_FAMILIES) >= 8 and len(NEG_HELDOUT_FAMILIES) >= 4
    assert not set(NEG_TRAIN_FAMILIES) & set(NEG_HELDOUT_FAMILIES)
    assert {f.lang for f in NEG_FAMILIES} == {"en", "ru", "tr"}
    assert {f.txn for f in NEG_FAMILIES} == {"unknown", "otp"}
    items = generate(4000, seed=43, vocab_name="heldout", families="neg_all")
    assert {s.family for s in items} == set(NEG_TRAIN_FAMILIES + NEG_HELDOUT_FAMILIES)
    assert all(is_negative(s.family) and s.kind == "negative" for s in items)
    assert not [s.body for s in items if worker_should_skip(s.body) or llm_should_skip(s.body)]
    # never mixed into a transaction selector unless asked
    assert not [s for s in generate(2000, seed=44, families="all") if is_negative(s.family)]
    mixed = generate(4000, seed=45, families="all", negatives=0.1)
    share = sum(is_negative(s.family) for s in mixed) / len(mixed)
    assert 0.08 < share < 0.12
    assert {s.family for s in generate(3000, seed=46, families="train", negatives=0.5)
            if is_negative(s.family)} == set(NEG_TRAIN_FAMILIES)


def test_negative_gold_answers_end_unmatched():
    """Gemini's shape for a non-transaction (txn_type unknown / otp, null fields) goes
    down the reference's D6 path: str(None) -> ValueError -> UNMATCHED (-> DLQ)."""
    for s in generate(1500, seed=47, vocab_name="heldout", families="neg_all"):
        assert s.answer["txn_type"] in ("unknown", "otp") and all(
            v is None for k, v in s.answer.items() if k != "txn_type")
        raw = RawSMS(msg_id="e", device_id="d", sender="B", date=str(s.timestamp), body=s.body, source="device")
        assert postprocess_answer(raw, normalize_body(s.body), s.answer).outcome is Outcome.UNMATCHED


def test_training_examples_include_negatives():
    from smsgate_amd.models.train import answer_fsm, make_examples

    tk = load_tokenizer()
    fsm = answer_fsm(tk, "qa")
    ex = make_examples(tk, fsm, 2000, seed=5, negatives=0.2)
    classes = Counter(c for _, (c, _) in ex)
    assert classes[3] + classes[2] > 250 and classes[0] > 1000, classes  # unknown / otp, debit


# ------------------------------------------------ held-out VALUE styles
# Each held-out value style is one COMBINATION of value-grammar axes (VERDICT r05 next
# #1a): the training pools have every axis -- 12-hour clocks, month-first order, Russian
# genitive month names -- in other combinations, never the held-out one
_HV_PATTERNS = {
    "en_12h": r"\b[A-Z][a-z]{2} \d{1,2}, \d{4} \d{1,2}:\d{2} (AM|PM)\b",
    "ru_month": r"\b\d{1,2} (января|февраля|марта|апреля|мая|июня|июля|августа|сентября|октября|ноября|декабря) "
                r"\d{4} \d{2}:\d{2}",
    "code_glued": r"\b(AMD|USD|EUR|RUB|GEL|GBP)\d",
    "apos": r"\d'\d{3}",
    "x_mask": r"(?<![A-Za-z0-9])x\d{4}\b",
    "dots_mask": r"(?<!\.)\.\.\d{4}\b",
}


def test_heldout_value_styles_never_appear_in_training():
    """The held-out value styles are rendered only by the heldout_values families: no
    language pool offers them, no other family declares them, and no generated
    training / negative body contains one."""
    import re

    from smsgate_amd.utils.synth import (HELDOUT_VALUE_STYLES, NEG_FAMILIES, VALUE_FAMILIES, _PROC_POOLS,
                                         _STYLE_POOLS)

    held = {s for v in HELDOUT_VALUE_STYLES.values() for s in v}
    for pools in _STYLE_POOLS.values():
        assert not held & {s for v in pools.values() for s in v}
    assert not held & {s for p in _PROC_POOLS.values() for v in p.values() for s in v}
    for f in FAMILIES + NEG_FAMILIES:
        assert not held & set(f.dates + f.money + f.cards + f.numbers), f.name
    assert all(f.heldout and f.split == "values" for f in VALUE_FAMILIES)
    pats = {k: re.compile(p) for k, p in _HV_PATTERNS.items()}
    train = generate(20000, seed=48, vocab_name="train", families="train", negatives=0.12, training=True)
    hits = Counter(k for s in train for k, p in pats.items() if p.search(s.body))
    assert not hits, hits
    # ... and each held-out value family shows its style
    hv = generate(2000, seed=49, vocab_name="heldout", families="heldout_values")
    seen = Counter(k for s in hv for k, p in pats.items() if p.search(s.body))
    assert {"en_12h", "ru_month", "code_glued", "apos"} <= set(seen), seen
    assert seen["x_mask"] + seen["dots_mask"] > 0, seen


def test_heldout_value_gold_answers_postprocess_to_expected():
    bad = Counter()
    for s in generate(2000, seed=50, vocab_name="heldout", families="heldout_values"):
        raw = RawSMS(msg_id="e", device_id="d", sender="B", date=str(s.timestamp), body=s.body, source="device")
        r = postprocess_answer(raw, normalize_body(s.body), s.answer)
        assert r.outcome is Outcome.PARSED, (s.family, s.body, r.error)
        got = _got(r.parsed)
        for k, v in s.expected.items():
            bad[(s.family, k)] += got[k] != v
    assert not +bad, +bad


def test_russian_month_dates_canonicalise():
    from smsgate_amd.parse.canonical import canonical_date_text

    assert canonical_date_text("6 июня 2025 14:23") == "2025-06-06 14:23"
    assert canonical_date_text("22 марта 2025") == "2025-03-22"
    assert canonical_date_text("1 мая 2024 г. 09:05") == "2024-05-01 09:05"
    assert canonical_date_text("06.05.25 14:23") == "06.05.25 14:23"  # dotted: the reference chain's
    assert canonical_date_text("6 foo 2025") == "6 foo 2025"
    # the training grammar's other Russian-month combinations, and the Latin transliteration
    assert canonical_date_text("6 июня 2025 в 14:23") == "2025-06-06 14:23"
    assert canonical_date_text("14:23 6 июня 2025") == "2025-06-06 14:23"
    assert canonical_date_text("06 июн. 2025 14:23") == "2025-06-06 14:23"
    assert canonical_date_text("6 iyunya 2025 14:23") == "2025-06-06 14:23"
    assert canonical_date_text("14:23 6 June 2025") == "14:23 6 June 2025"  # English: dateutil's


def test_value_grammar_covers_every_axis_of_the_heldout_styles():
    """The held-out value styles are interpolations of the training grammar: each of
    their axes occurs in training bodies, in other combinations."""
    import re

    train = generate(20000, seed=51, vocab_name="train", families="train", training=True)
    axes = {
        "12h clock": r"\d{1,2}:\d{2} ?(AM|PM|am|pm)\b",
        "month-first, comma": r"\b[A-Z][a-z]{2} \d{1,2}, \d{4}\b",
        "Russian genitive month": r"\d \b(января|февраля|марта|апреля|мая|июня|июля|августа|сентября|октября|ноября|"
                                  r"декабря)\b",
        "Russian month, then a 24-hour time": r"\d{1,2} [а-я]+\.? \d{4}( г\.| в)? \d{2}:\d{2}",
        "x glyph mask": r"\b[xX]{2,4} ?\d{4}\b",
        "dot mask": r"(\.\.\.|…)\d{4}\b",
    }
    for name, pat in axes.items():
        assert sum(bool(re.search(pat, s.body)) for s in train) > 50, name


def test_training_stream_is_pinned(monkeypatch):
    """The in-run training data is a fixed function of the seed: the bench's quality
    numbers reproduce from run to run (training on the box is deterministic too).  A
    default-off experiment knob must not draw from the generator's RNG.  Round 5 hit
    this: an unconditional draw for SMSGATE_SYNTH_LABELS changed every later example and
    moved held-out formats from 99.0 to 95.2 %.  Update the fingerprint only on a
    deliberate change to the training distribution."""
    import hashlib

    monkeypatch.delenv("SMSGATE_SYNTH_LABELS", raising=False)
    monkeypatch.delenv("SMSGATE_PROC_WEIGHT", raising=False)
    h = hashlib.sha256()
    for s in generate(400, seed=5, families="train"):
        h.update(s.body.encode())
        h.update(repr(sorted((s.answer or {}).items())).encode())
    assert h.hexdigest()[:16] == "47169bc036094f72"  # round 6: widened value grammar + credit phrasing


def test_heldout_credit_layout_is_an_interpolation():
    """hv_en_credit ("Incoming payment X credited to card Y. Sender: M, C. D. Bal B") stays
    unseen as a whole -- its header phrase is in no training body and its segment order
    is a held-out signature -- while its parts are trained: "credited" after an amount,
    "to card", a sender label, in other procedural credit layouts."""
    import re

    train = generate(20000, seed=51, vocab_name="train", families="train", negatives=0.12, training=True)
    assert not [s.body for s in train if "Incoming payment" in s.body]
    credit = [s.body for s in train if s.family == "proc_en_credit"]
    assert any(re.search(r"\d credited\b", b) for b in credit)
    assert any("to card" in b for b in credit) and any("Sender" in b for b in credit)
