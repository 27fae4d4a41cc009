"""Span-pointer answer format (serving/fsm.py build_span_fsm, VERDICT r03 next #2a):
every copied field is two pointers into the SMS body instead of its tokens.

CPU checks: every gold answer of every template family is expressible and walks the
FSM under the copy rules; expanding a span answer gives exactly the copy-format
answer (what ops.span_commit writes on the GPU); the host masks' start / end rules;
a tiny span model trains."""
import re
from collections import Counter

import numpy as np
import pytest

from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.models.train import answer_fsm, answer_span_tokens, answer_tokens
from smsgate_amd.parse.text import normalize_body
from smsgate_amd.serving.fsm import PTR_END, PTR_START
from smsgate_amd.utils.synth import generate


@pytest.fixture(scope="module")
def fsms():
    tk = load_tokenizer()
    return tk, answer_fsm(tk, "span"), answer_fsm(tk, "copy")


def test_shape(fsms):
    tk, f, _ = fsms
    assert f.span and f.ptr0 == 8192 and f.n_pos == 130 and f.vocab == 8448
    assert f.max_steps() == 8 + 1 + 2 * 8  # enum (+ <sep>) and two pointers per copied field
    assert f.max_answer_tokens() == sum(x.cap for x in f.fields) + len(f.fields)
    kinds = Counter(int(k) & 0xFF for k in f.copy_kind)
    assert kinds[PTR_START] == 8 and kinds[PTR_END] == 8


# round 6's glued card masks ("XX1234", "...1234", "XXXX XXXX XXXX 1234"): the span / copy
# formats' word boundaries do not split letters or dots from digits, so these values are
# not expressible there; the served qa format's are (tests/test_families.py
# test_gold_answers_reachable_by_qa_decoder).  The autoregressive formats are kept for the
# reference's own formats and the layouts of rounds 3-5.
_GLUED_MASK = re.compile(r"(?:[xX]{2,4} ?|\.\.\.|…|(?:(?:XXXX|xxxx|\*\*\*\*) ){3})(\d{4})\b")


@pytest.mark.parametrize("families", ["train", "heldout", None])
def test_gold_answers_expressible_and_expand_to_copy_format(fsms, families):
    tk, f, fc = fsms
    bad = Counter()
    lens = []
    skipped = 0
    n = 0
    for s in generate(1200, seed=31, vocab_name="heldout", families=families):
        if s.answer is None:
            continue
        n += 1
        if _GLUED_MASK.search(s.body):
            skipped += 1
            continue
        b = normalize_body(s.body)
        enc = tk.encode_offsets([b])[0]
        msg = tk.message_ids([b], 128)[0]
        sp = answer_span_tokens(tk, f, s.answer, b, enc, len(msg))
        if sp is None:
            bad[s.family] += 1
            continue
        lens.append(len(sp))
        assert f.expand_span_answer(sp, msg) == answer_tokens(tk, fc, s.answer, b, enc), s.body
    assert not bad, bad
    assert skipped < 0.4 * n and (families is not None or skipped == 0), (skipped, n)
    assert np.mean(lens) <= 19  # vs ~36 answer tokens in copy format (scripts/span_sim.py)


def test_host_masks(fsms):
    tk, f, _ = fsms
    body = "Purchase 1,234.50 USD at SHOP NAME, card *1234"
    msg = tk.message_ids([body], 128)[0]
    strings = [tk.token_strings[t] for t in msg]
    # the amount field's start / end states
    amt = f.fields.index(next(x for x in f.fields if x.name == "amount"))
    a_start = [s for s in range(f.num_states) if f.field_of_state[s] == amt and f.copy_kind[s] & 0xFF == PTR_START][0]
    a_end = int(f.next_tok[a_start])
    m = f.copy_mask_host(a_start, -1, msg)
    ok = {j for j in range(len(msg)) if m[f.ptr0 + j]}
    assert m[f.sep_token]
    # a number starts at its first token only; words are not numbers
    j1 = next(j for j, t in enumerate(strings) if t.strip().startswith("1"))
    assert j1 in ok and 0 not in ok  # "Purchase" is no number
    assert j1 + 1 not in ok and j1 + 2 not in ok  # never inside "1,234.50" (" 1," "234" ".50")
    assert len(msg) - 1 not in ok  # never the closing <ans>
    e = f.copy_mask_host(a_end, f.ptr0 + j1, msg)
    ends = [j for j in range(len(msg)) if e[f.ptr0 + j]]
    assert ends and all(j >= j1 for j in ends)
    # the amount cannot end inside "1,234.50": its last pointer is the number's last token
    assert tk.decode(msg[j1:ends[-1] + 1]).strip() == "1,234.50"
    assert not e[f.sep_token]


def test_tiny_span_model_trains_on_cpu():
    import torch

    from smsgate_amd.models.train import TrainConfig, train_extractor

    torch.manual_seed(0)
    w = train_extractor(TrainConfig(model="tiny", steps=3, batch=4, n_examples=48, ema=0, log_every=0,
                                    answer_format="span", families=None), device="cpu", log=lambda s: None)
    assert w.cfg.span_positions == 130 and w.embed.shape[0] >= 8192 + 130
    assert torch.isfinite(w.embed.float()).all()


def test_checkpoint_carries_its_answer_format(tmp_path):
    """A span checkpoint loads as a span model whatever config the caller passes, a
    copy-format checkpoint (the round-4 small extractor) as a copy model, and the
    bundled small extractor as a qa model."""
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights, span_config
    from smsgate_amd.parse.backends.local_llm import bundled_checkpoint

    w = ExtractorWeights(span_config(CONFIGS["tiny"]), device="cpu", seed=1)
    p = str(tmp_path / "span.safetensors")
    w.save(p)
    got = ExtractorWeights.load(p, CONFIGS["tiny"])
    assert got.cfg.span_positions == 130 and got.embed.shape[0] == 8448
    copy = ExtractorWeights.load(bundled_checkpoint("small-copy"), span_config(CONFIGS["small"]))
    assert copy.cfg.span_positions == 0 and copy.cfg.qa_queries == 0 and copy.cfg.vocab == 8192
    small = ExtractorWeights.load(bundled_checkpoint("small"), CONFIGS["small"])
    assert small.cfg.qa_queries == 9 and small.cfg.span_positions == 130


def test_dates_and_numbers_never_start_inside_a_card_mask(fsms):
    """'Карта **** 7492 17.05.24 ...': the digits after a mask are the card's -- a date or
    an amount cannot start there (the held-out ru_karta_first layout's typical miss)."""
    tk, f, _ = fsms
    msg = tk.message_ids(["Карта **** 7492 17.05.24 покупка на сумму 41,76 AMD"], 128)[0]
    strings = [tk.token_strings[t] for t in msg]
    j_card = next(j for j, t in enumerate(strings) if t.strip() == "****") + 1  # " 7" of " 7" "492"
    j_date = next(j for j, t in enumerate(strings) if t.strip().startswith("17"))
    by_field = {x.name: i for i, x in enumerate(f.fields)}
    for name, allowed in (("date", False), ("amount", False), ("card", True)):
        st = [s for s in range(f.num_states)
              if f.field_of_state[s] == by_field[name] and int(f.copy_kind[s]) & 0xFF == PTR_START][0]
        m = f.copy_mask_host(st, -1, msg)
        assert bool(m[f.ptr0 + j_card]) is allowed, name
    date_st = [s for s in range(f.num_states)
               if f.field_of_state[s] == by_field["date"] and int(f.copy_kind[s]) & 0xFF == PTR_START][0]
    assert f.copy_mask_host(date_st, -1, msg)[f.ptr0 + j_date]


def test_a_start_is_offered_only_with_an_end(fsms):
    """the end state has no <sep>, so a start whose word runs on into a glued
    out-of-class token ("1500р", "17.05.24г") must not be offered -- else the kernel's
    empty end set decodes <sep> and span_commit ends the whole answer.  Every offered
    start has at least one end; the glued amount is not offered, the later fields are."""
    tk, f, _ = fsms
    body = "Покупка 1500р MARKET, YEREVAN. 17.05.24г Карта *1234. Баланс 200 RUB"
    msg = tk.message_ids([body], 128)[0]
    strings = [tk.token_strings[t] for t in msg]
    fi = {x.name: k for k, x in enumerate(f.fields)}
    starts = {name: [s for s in range(f.num_states) if f.field_of_state[s] == fi[name]
                     and f.copy_kind[s] & 0xFF == PTR_START][0] for name in ("amount", "date", "balance", "card")}
    j1500 = next(j for j, t in enumerate(strings) if t.strip() == "15")  # " 15" "00" "р"
    m = f.copy_mask_host(starts["amount"], -1, msg)
    assert not m[f.ptr0 + j1500]  # "1500" + "р": no number end after it
    for name, st in starts.items():
        cand = [j for j in range(len(msg)) if f.copy_mask_host(st, -1, msg)[f.ptr0 + j]]
        for j in cand:
            e = f.copy_mask_host(int(f.next_tok[st]), f.ptr0 + j, msg)
            assert e[f.ptr0:f.ptr0 + len(msg)].any(), (name, j, strings[j])
    # the balance (after the glued tokens) is still reachable
    jb = next(j for j, t in enumerate(strings) if t.strip() == "200")
    assert f.copy_mask_host(starts["balance"], -1, msg)[f.ptr0 + jb]
    # property: over generated bodies (glued currencies included) no start lacks an end
    items = generate(300, seed=61, vocab_name="heldout", families="all", negatives=0.1)
    for s in items:
        m2 = tk.message_ids([normalize_body(s.body)], 128)[0]
        for st in starts.values():
            for j in np.nonzero(f.copy_mask_host(st, -1, m2)[f.ptr0:f.ptr0 + len(m2)])[0]:
                assert f.copy_mask_host(int(f.next_tok[st]), f.ptr0 + int(j), m2)[f.ptr0:f.ptr0 + len(m2)].any()
