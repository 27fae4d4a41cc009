"""The schema FSM's per-field token caps never cut a value.

Every generated answer — training vocabulary and the held-out vocabulary whose
merchant / city / street names the model never saw — is written the way the
extractor writes it (the body's own tokens) and must be reproducible by the
constrained decoder; the truncation rate is pinned at 0 (required < 0.5 %).
Also pins that answers copy the body's tokens (the speculative drafter's premise).
"""
from __future__ import annotations

import pytest

from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.models.train import answer_tokens
from smsgate_amd.parse.text import normalize_body
from smsgate_amd.serving.fsm import DEFAULT_FIELDS, build_fsm
from smsgate_amd.utils.synth import _GOLDEN_VOCAB, generate, reference_cases, vocab


@pytest.fixture(scope="module")
def tk_fsm():
    tk = load_tokenizer()
    return tk, build_fsm(tk, (tk.vocab_size + 63) // 64 * 64)


@pytest.mark.parametrize("vocab_name", ["train", "heldout"])
def test_caps_truncate_nothing(tk_fsm, vocab_name):
    tk, fsm = tk_fsm
    items = [s for s in generate(6000, seed=31337, vocab_name=vocab_name) if s.answer is not None]
    bodies = [normalize_body(s.body) for s in items]
    encs = tk.encode_offsets(bodies)
    over = {f.name: 0 for f in DEFAULT_FIELDS}
    rejected = 0
    for s, b, e in zip(items, bodies, encs):
        if answer_tokens(tk, fsm, s.answer, b, e) is None:
            rejected += 1
            for f in DEFAULT_FIELDS:
                v = s.answer.get(f.name) or ""
                if f.kind != "enum" and v and len(tk.value_span_ids(v, b, *e)) > f.cap:
                    over[f.name] += 1
    assert rejected / len(items) < 0.005, (rejected, over)
    assert rejected == 0, over


def test_vocabularies_are_disjoint_and_exclude_golden_words():
    tr, ho = vocab("train"), vocab("heldout")
    for a, b in ((tr.words, ho.words), (tr.cities, ho.cities), (tr.streets, ho.streets)):
        assert not set(a) & set(b)
    for v in (tr, ho):
        assert not (set(v.words) | set(v.cities) | set(v.streets)) & _GOLDEN_VOCAB
    # and the tokenizer has no whole-word token for a golden word: they split like unseen names
    tk = load_tokenizer()
    strings = set(tk.token_strings)
    for w in _GOLDEN_VOCAB - {"AM"}:
        assert w not in strings and " " + w not in strings, w


def test_answers_copy_body_tokens(tk_fsm):
    tk, fsm = tk_fsm
    body = normalize_body(reference_cases()[0])
    ids, offs = tk.encode_offsets([body])[0]
    for value in ("TEST LLC", "MOSKOW", "TEST STR. 29, 24 AREA", "52.00", "***0018", "1842.74", "USD"):
        span = tk.value_span_ids(value, body, ids, offs)
        assert tk.decode(span).strip() == value
        n = len(span)
        assert any(ids[i:i + n] == span for i in range(len(ids) - n + 1)), value  # a contiguous body span
