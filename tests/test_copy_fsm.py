"""CPU checks of the copy-constrained schema FSM (serving/fsm.py): the state
kinds, the host reference mask, and that every gold answer -- synthetic SMS of
both vocabularies and the reference's three CASES (tests/test_parsers.py:11-58)
-- is reachable under the constraint, so the constraint can only remove wrong
answers, never the right one."""
import pytest

from conftest import REFERENCE_CASES
from smsgate_amd.models.tokenizer import load_tokenizer
from smsgate_amd.models.train import answer_tokens
from smsgate_amd.parse.text import normalize_body
from smsgate_amd.serving.fsm import COPY_NEXT, COPY_NONE, COPY_START, DEFAULT_FIELDS, build_fsm
from smsgate_amd.utils.synth import generate


@pytest.fixture(scope="module")
def tk_fsm():
    tk = load_tokenizer()
    return tk, build_fsm(tk, (tk.vocab_size + 127) // 128 * 128)


def test_copy_state_kinds(tk_fsm):
    _, fsm = tk_fsm
    ck = fsm.copy_kind
    assert ck[fsm.done_state] == COPY_NONE and ck[fsm.start_state] == COPY_NONE  # txn_type: enum
    for fi, f in enumerate(fsm.fields):
        states = [s for s in range(fsm.num_states) if fsm.field_of_state[s] == fi]
        kinds = [int(ck[s]) for s in states]
        if not f.copy:
            assert set(kinds) == {COPY_NONE}
            continue
        # chain: one start state, cap - 1 continuation states, the only-<sep> cap state
        assert kinds == [COPY_START] + [COPY_NEXT] * (f.cap - 1) + [COPY_NONE], f.name
    assert [f.name for f in DEFAULT_FIELDS if f.copy] == ["date", "amount", "currency", "card", "merchant", "city",
                                                          "address", "balance"]


def test_host_mask_semantics(tk_fsm):
    tk, fsm = tk_fsm
    body = tk.message_ids([normalize_body(REFERENCE_CASES[0][0])], 128)[0]
    merchant = fsm.fields.index(next(f for f in fsm.fields if f.name == "merchant"))
    s0 = next(s for s in range(fsm.num_states) if fsm.field_of_state[s] == merchant)
    m0 = set(fsm.copy_mask_host(s0, tk.sep, body).nonzero()[0])
    t_, est = tk.encode(" T")[0], tk.encode("EST")[0]
    # a value starts at a word boundary: " T" may start one, "EST" (always inside "TEST") may not
    assert t_ in m0 and est not in m0 and tk.sep in m0
    assert m0 <= {t for t in body if fsm.allowed[s0, t]} | {tk.sep}
    # after " T" only "EST" may follow -- and the value may not end inside the word
    assert set(fsm.copy_mask_host(s0 + 1, t_, body).nonzero()[0]) == {est}
    # after "EST" the word is complete: " L" / " STR" / "," continue or <sep> ends it
    after = set(fsm.copy_mask_host(s0 + 1, est, body).nonzero()[0])
    assert tk.sep in after and tk.encode(" L")[0] in after
    # a token absent from the body: nothing (the kernels then fall back to <sep>)
    absent = next(i for i in range(fsm.vocab) if i not in body and fsm.allowed[s0 + 1, i])
    assert not fsm.copy_mask_host(s0 + 1, absent, body).any()
    # non-copy state: the schema mask unchanged
    assert (fsm.copy_mask_host(fsm.start_state, 0, body) == fsm.allowed[fsm.start_state]).all()


def _walk_ok(fsm, ids, body):
    s, prev = fsm.start_state, body[-1]
    for t in ids:
        if not fsm.copy_mask_host(s, prev, body)[t]:
            return False
        s, prev = fsm.step_host(s, t), t
    return s == fsm.done_state


@pytest.mark.parametrize("vocab_name", ["train", "heldout"])
def test_every_gold_answer_is_reachable(tk_fsm, vocab_name):
    tk, fsm = tk_fsm
    items = [s for s in generate(600, seed=11, vocab_name=vocab_name) if s.answer]
    bad = 0
    for s in items:
        b = normalize_body(s.body)
        ids = answer_tokens(tk, fsm, s.answer, b)
        assert ids is not None
        bad += not _walk_ok(fsm, ids, tk.message_ids([b], 128)[0])
    assert bad == 0


def test_reference_cases_reachable(tk_fsm):
    tk, fsm = tk_fsm
    for body, exp in REFERENCE_CASES:
        b = normalize_body(body)
        # the LLM answer shape: card as in the body, amounts / date as written there
        card = "CARD:" + exp["card"] if "CARD:" + exp["card"] in b else "***" + exp["card"]
        amount = next(a for a in ("27,252.00", exp["amount"]) if a in b)
        balance = next(a for a in ("391,469.09", exp["balance"]) if a in b)
        date = next(d for d in ("06.05.25 14:23", "06.05.25 15:11", "10.06.2025 20:51") if d in b)
        ans = dict(txn_type="debit", date=date, amount=amount, currency=exp["currency"], card=card[-4:],
                   merchant=exp["merchant"], city=exp["city"], address=exp["address"], balance=balance)
        ids = answer_tokens(tk, fsm, ans, b)
        assert ids is not None and _walk_ok(fsm, ids, tk.message_ids([b], 128)[0]), body


def test_model_text_line_breaks(tk_fsm):
    """``&#10;`` (the reference export's line break) reaches the model as ONE token, and
    copied values still decode to the body's own text."""
    tk, fsm = tk_fsm
    body = "DEBIT ACCOUNT&#10;111,264.44 RUB&#10;CARD:4579,&#10;S1X1GWT5, TIOVINVU&#10;25.02.2023 19:39"
    ids = tk.encode(body)
    assert len(ids) <= len(tk.tk.encode(body, add_special_tokens=False).ids) - 7
    assert "&#" not in tk.decode(ids) and tk.decode(ids).count("\n") == 4
    enc = tk.encode_offsets([body])[0]
    for v in ("TIOVINVU", "111,264.44", "S1X1GWT5"):
        assert tk.decode(tk.value_span_ids(v, body, *enc)).strip() == v


def test_sparse_argmax_eligibility():
    """The candidate-sparse arg-max needs small allowed sets outside the copy states: the
    default schema qualifies (enum / <sep>-only states), schema-only decoding (every text
    field a free class) does not."""
    import dataclasses

    from smsgate_amd import ops
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.serving.fsm import DEFAULT_FIELDS, build_fsm

    tok = load_tokenizer()
    assert ops.sparse_argmax_ok(build_fsm(tok, 8192))
    free = tuple(dataclasses.replace(f, copy=False) for f in DEFAULT_FIELDS)
    assert not ops.sparse_argmax_ok(build_fsm(tok, 8192, free))
