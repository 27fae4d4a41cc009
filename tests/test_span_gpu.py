"""Span-pointer answer format on the GPU (csrc/spec_kernels.hip: sparse_argmax_kernel's
pointer kinds, span_commit_kernel) against the host references of serving/fsm.py and
an fp32 PyTorch reference, and end to end: a span model decodes through the engine
(pointer rows added to the prompt, answers expanded to copy format on the GPU) and
learns the task."""
import random

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd import ops  # noqa: E402
from smsgate_amd.models.tokenizer import load_tokenizer  # noqa: E402
from smsgate_amd.models.train import answer_fsm, make_examples  # noqa: E402
from smsgate_amd.parse.text import normalize_body  # noqa: E402
from smsgate_amd.utils.synth import generate, reference_cases  # noqa: E402

DEV = "cuda"
i32 = dict(dtype=torch.int32, device=DEV)


def _key(tok):  # an arg-max key naming `tok` (what sparse_argmax writes)
    return (1 << 40) | (0xFFFFFFFF - tok)


@pytest.fixture(scope="module")
def span_data():
    tok = load_tokenizer()
    fsm = answer_fsm(tok, "span").to_device(DEV)
    exs = make_examples(tok, fsm, 500, seed=13, vocab_name="heldout", families="train")[:256]
    exs += make_examples(tok, fsm, 200, seed=14, vocab_name="heldout", families=None)[:64]
    n, LB = len(exs), 130
    body = torch.zeros(n, LB, **i32)
    blen = torch.zeros(n, **i32)
    for r, (m, _) in enumerate(exs):
        body[r, :len(m)] = torch.tensor(m)
        blen[r] = len(m)
    return tok, fsm, exs, body, blen


@pytest.mark.parametrize("H", [256, 576])
def test_sparse_argmax_pointer_rows(span_data, H):
    """Rows at every point of gold span answers: the kernel's choice is allowed by the
    host rules (start: boundary + class; end: cap, class run, boundary) and its logit
    is the allowed maximum of the fp32 reference (to bf16 rounding)."""
    tok, fsm, exs, body, blen = span_data
    n = len(exs)
    g = torch.Generator().manual_seed(5)
    states, prevs = [], []
    for m, a in exs:
        L = int(torch.randint(0, len(a), (1,), generator=g))
        s = fsm.start_state
        for x in a[:L]:
            s = fsm.step_host(s, x)
        states.append(s)
        prevs.append(a[L - 1] if L else m[-1])
    state, prev, slot = torch.tensor(states, **i32), torch.tensor(prevs, **i32), torch.arange(n, **i32)
    h = (torch.randn(n, H, generator=g) * 2).to(torch.bfloat16).to(DEV)
    nw = (torch.rand(H, generator=g) + 0.5).to(torch.bfloat16).to(DEV)
    w = (torch.randn(fsm.vocab, H, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    best = torch.zeros(n, dtype=torch.int64, device=DEV)
    ops.sparse_argmax(h, ops.fold_norm(w, nw), state, fsm, best, prev, slot, body, blen, 1e-5)
    torch.cuda.synchronize()
    ref = ops.ref_gemm(h, w, norm_eps=1e-5, norm_w=nw)
    kinds = {0: 0, 3: 0, 4: 0}
    for r in range(n):
        allowed = torch.tensor(fsm.copy_mask_host(states[r], prevs[r], exs[r][0]), device=DEV)
        t = (0xFFFFFFFF - (int(best[r]) & 0xFFFFFFFF)) if int(best[r]) else fsm.sep_token
        assert bool(allowed[t]), (r, t, int(fsm.copy_kind[states[r]]))
        top = ref[r].masked_fill(~allowed, float("-inf")).max()
        assert float(ref[r, t]) >= float(top) - 0.02 * abs(float(top)) - 0.02, (r, t)
        kinds[int(fsm.copy_kind[states[r]]) & 0xFF] += 1
    assert all(v > 10 for v in kinds.values()), kinds  # every kind of state was exercised


def test_span_commit_expands_like_host(span_data):
    """Feeding the gold pointer answers through span_commit (from the prefill's row
    map, then step by step) writes exactly the copy-format answer, ends every row, and
    leaves each row's state / last token / position as the host FSM says."""
    tok, fsm, exs, body, blen = span_data
    n = len(exs)
    steps = max(len(a) for _, a in exs)
    state = torch.full((n,), fsm.done_state, **i32)
    tok_io, done = torch.zeros(n, **i32), torch.ones(n, **i32)
    out_buf = torch.full((n, fsm.max_answer_tokens()), -7, **i32)
    out_len = torch.zeros(n, **i32)
    pos = torch.tensor([len(m) - 1 for m, _ in exs], **i32)
    perm = list(range(n))
    random.Random(0).shuffle(perm)  # prefill: key row i -> state row perm[i]
    rows = torch.tensor(perm, **i32)
    state[rows.long()] = fsm.start_state
    done[rows.long()] = 0
    slot_of_key = rows.clone()
    best = torch.tensor([_key(exs[perm[i]][1][0]) for i in range(n)], dtype=torch.int64, device=DEV)
    ops.span_commit(best, fsm, state, tok_io, out_buf, out_len, done, pos, slot_of_key, body, blen, n, row_map=rows)
    for k in range(1, steps):
        best = torch.tensor([_key(a[k]) if k < len(a) else 0 for _, a in exs], dtype=torch.int64, device=DEV)
        ops.span_commit(best, fsm, state, tok_io, out_buf, out_len, done, pos, torch.arange(n, **i32), body, blen, n)
    torch.cuda.synchronize()
    for r, (m, a) in enumerate(exs):
        want = fsm.expand_span_answer(a, m)
        assert out_buf[r, :int(out_len[r])].tolist() == want, r
        assert int(done[r]) == 1 and int(state[r]) == fsm.done_state and int(tok_io[r]) == a[-1]
        assert int(pos[r]) == len(m) - 1 + len(a) - 1  # one KV position per emitted token but the last


def _span_engine(w, **kw):
    from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine

    return ExtractionEngine(w, load_tokenizer(), EngineConfig(**{"max_slots": 512, "buckets": (64, 512), **kw}))


def _ref_greedy(w, fsm, tok, bodies):
    """fp32 PyTorch greedy decode of span weights ``w`` under the host rules: the
    answers and every step's logits."""
    from smsgate_amd.models.extractor import ExtractorWeights, reference_forward
    from smsgate_amd.parse.schema import EXTRACTOR_PROMPT

    msgs = tok.message_ids(bodies, 128)
    prefix = tok.prefix_ids(EXTRACTOR_PROMPT)
    wf = ExtractorWeights(w.cfg, device=DEV, dtype=torch.float32, seed=None)
    wf.load_state_dict({k: v.float() for k, v in w.state_dict().items()})
    refs, ref_logits = [], []
    with torch.no_grad():
        for m in msgs:
            seq = prefix + m
            add = [-1] * len(prefix) + [fsm.ptr0 + j for j in range(len(m))]
            st, prev, ans, lgs = fsm.start_state, m[-1], [], []
            while st != fsm.done_state and len(ans) < fsm.max_steps():
                logits = reference_forward(wf, torch.tensor([seq], device=DEV),
                                           add_ids=torch.tensor([add], device=DEV))[0, -1, : fsm.vocab]
                allowed = torch.tensor(fsm.copy_mask_host(st, prev, m), device=DEV)
                lgs.append((logits, allowed))
                t = int(logits.masked_fill(~allowed, float("-inf")).argmax())
                ans.append(t)
                seq.append(t)
                add.append(-1)
                st, prev = fsm.step_host(st, t), t
            refs.append(ans)
            ref_logits.append(lgs)
    return msgs, refs, ref_logits


def _tol(scale: float) -> float:
    return 0.05 * scale + 0.05  # bf16 forward vs fp32 (the logits bound asserted below)


def test_span_engine_matches_fp32_reference_decode():
    """Random-init span model vs a plain fp32 PyTorch greedy decode under the host
    rules: teacher-forced on the reference's answers, the engine's logits (pointer rows
    added to the prompt inputs, pointer ids fed back as decode inputs, the lm_head over
    tokenizer + pointer rows) match at every step within bf16 rounding."""
    from smsgate_amd.models.extractor import CONFIGS, ExtractorWeights, span_config

    cfg = span_config(CONFIGS["small"])
    w = ExtractorWeights(cfg, device=DEV, dtype=torch.bfloat16, seed=3)
    eng = _span_engine(w, use_graphs=False)
    assert eng.span and not eng.spec and eng.Lmax == 160 and eng.V_dec == 8448
    tok, fsm = eng.tok, eng.fsm
    bodies = [normalize_body(s.body) for s in generate(24, seed=8, vocab_name="heldout", families="train") if s.answer]
    bodies += [normalize_body(b) for b in reference_cases()]
    msgs, refs, ref_logits = _ref_greedy(w, fsm, tok, bodies)
    L = max(len(a) for a in refs)
    forced = [a + [fsm.sep_token] * (L - len(a)) for a in refs]
    outs = eng.debug_logits(bodies, [f[:L - 1] for f in forced])
    for b, lgs in enumerate(ref_logits):
        for step, (ref, _) in enumerate(lgs):
            got = outs[step][b, : fsm.vocab].float()
            scale = ref.abs().max().item()
            err = (got - ref).abs().max().item()
            assert err <= _tol(scale), (b, step, err, scale)


def test_span_engine_answers_match_fp32_reference(span_small):
    """The trained span model through the engine vs the fp32 PyTorch greedy decode: at
    least 90 % of the answers identical, and EVERY disagreement explained -- at the first
    step where the engine's (teacher-forced) choice differs, the fp32 top-2 margin
    between the two tokens is within bf16 rounding of the engine's forward."""
    eng = _span_engine(span_small, use_graphs=False)
    tok, fsm = eng.tok, eng.fsm
    items = [s for s in generate(120, seed=9, vocab_name="heldout") if s.answer]  # the mix it was trained on
    bodies = [normalize_body(s.body) for s in items] + [normalize_body(b) for b in reference_cases()]
    msgs, refs, ref_logits = _ref_greedy(span_small, fsm, tok, bodies)
    got = eng.run(bodies)
    L = max(len(a) for a in refs)
    forced = [a + [fsm.sep_token] * (L - len(a)) for a in refs]
    outs = eng.debug_logits(bodies, [f[:L - 1] for f in forced])
    same = 0
    for b, (m, a, g) in enumerate(zip(msgs, refs, got)):
        vals = fsm.split_fields(fsm.expand_span_answer(a, m))
        if {f.name: tok.decode(v).strip() for f, v in zip(fsm.fields, vals)} == g:
            same += 1
            continue
        explained = False
        for step, (ref, allowed) in enumerate(ref_logits[b]):
            e = outs[step][b, : fsm.vocab].float().masked_fill(~allowed, float("-inf"))
            te = int(e.argmax())
            if te != a[step]:
                margin = float(ref[a[step]] - ref[te])
                assert 0 <= margin <= _tol(float(ref.abs().max())), (b, step, margin)
                explained = True
                break
        assert explained, (b, g, a)
    assert same >= 0.9 * len(bodies), (same, len(bodies))


@pytest.fixture(scope="module")
def span_small():
    """A small span model trained 2 500 steps on the legacy mix (~30 s)."""
    from smsgate_amd.models.train import TrainConfig, train_extractor

    w = train_extractor(TrainConfig(model="small", steps=2500, lr=2e-3, n_examples=30000, log_every=0, families=None,
                                    answer_format="span"), device="cuda")
    w.requires_grad_(False)
    return w


def test_span_model_learns_extraction(span_small):
    """The small span model decodes held-out SMS through the engine as well as the
    copy-format test model (test_train_gpu.py)."""
    from smsgate_amd.models.train import field_accuracy

    w = span_small
    assert w.cfg.span_positions == 130
    eng = _span_engine(w)
    held = [s for s in generate(300, seed=424242, vocab_name="heldout") if s.answer is not None]
    acc = field_accuracy(eng.run([normalize_body(s.body) for s in held]), [s.answer for s in held])
    for f in ("txn_type", "date", "currency"):
        assert acc[f] >= 0.95, acc
    assert sum(acc[f] for f in acc if f != "all") / 9 >= 0.8, acc


def test_span_templates_keep_answers(span_small):
    """Message-start templates (KV of a common opening computed once, copied into each
    matching message's slot) leave span answers unchanged: the opening's keys carry
    the pointer rows of positions 0..k-1 in both cases."""
    import dataclasses

    from smsgate_amd.utils.synth import generate_traffic

    bodies = [normalize_body(s.body) for s in generate_traffic(1200, seed=17, traffic="formats")]
    outs, stats = [], []
    for slots in (0, 16):
        eng = _span_engine(span_small, template_slots=slots, template_every=128, template_min_count=4)
        outs.append(eng.run(bodies))
        stats.append(dataclasses.replace(eng.stats))
        del eng
    bad = [(b, x, y) for b, x, y in zip(bodies, *outs) if x != y]
    print("TEMPLATES", stats[1].templates, stats[1].template_tokens, "mismatches", len(bad), "of", len(bodies))
    for b, x, y in bad[:8]:
        print("MISMATCH", repr(b[:120]), {k: (x[k], y[k]) for k in x if x[k] != y[k]})
    assert stats[1].templates > 0 and stats[1].template_tokens > 0.5 * len(bodies)
    assert not bad, len(bad)  # 0 of 1 200 in every logged run (profiles/r04_span_pytest.log)


def test_span_engine_survives_nan_filled_allocator_blocks(span_small):
    """Regression: finished rows in a decode bucket skip attention, so their rows of the
    attention output must not carry the allocator block's old contents into the next
    layer (NaN keys / values in their slots poisoned the slot's next message).  An
    engine built after NaN-filled memory went back to the caching allocator answers
    like one built on fresh memory, with rows reused many times."""
    from smsgate_amd.utils.synth import generate_traffic

    bodies = [normalize_body(s.body) for s in generate_traffic(1500, seed=23, traffic="formats")]
    kw = dict(max_slots=128, buckets=(64, 128), use_graphs=True)
    eng = _span_engine(span_small, **kw)
    clean = eng.run(bodies)
    del eng
    torch.cuda.synchronize()
    junk = torch.full((1 << 30,), float("nan"), dtype=torch.bfloat16, device=DEV)  # 2 GB of NaN
    del junk  # back to the caching allocator: the next engine's buffers / graph pools reuse it
    eng = _span_engine(span_small, **kw)
    dirty = eng.run(bodies)
    same = sum(a == b for a, b in zip(clean, dirty))
    assert same == len(bodies), same  # a partial regression of the NaN leak fails too


def test_embed_rows_add_matches_torch():
    """The fused prompt-row kernel == torch's bf16 gather + gather + add, bit for bit."""
    g = torch.Generator().manual_seed(9)
    table = torch.randn(8448, 576, generator=g).to(torch.bfloat16).to(DEV)
    ids = torch.randint(0, 8192, (3001,), generator=g, dtype=torch.int32).to(DEV)
    pos = torch.randint(0, 130, (3001,), generator=g, dtype=torch.int32).to(DEV)
    got = ops.embed_rows_add(ids, pos, table, 8192)
    ref = table[ids.long()] + table[pos.long() + 8192]
    assert torch.equal(got, ref)


def test_sparse_argmax_never_picks_a_start_without_an_end():
    """ADVICE r04 on the GPU: rows whose hidden state points straight at a start that has
    no end ("15" of "1500р", glued) get another allowed token from the kernel -- the host
    rule (serving/fsm.py _span_candidates) and the kernel agree."""
    tok = load_tokenizer()
    fsm = answer_fsm(tok, "span").to_device(DEV)
    bodies = ["Покупка 1500р MARKET, YEREVAN. Карта *1234. Баланс 200 RUB",
              "Оплата 99р SHOP 17.05.24г карта *4321 остаток 5 RUB"]
    msgs = tok.message_ids(bodies, 128)
    fi = next(k for k, x in enumerate(fsm.fields) if x.name == "amount")
    st = [s for s in range(fsm.num_states) if fsm.field_of_state[s] == fi and fsm.copy_kind[s] & 0xFF == 3][0]
    H = 576
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(fsm.vocab, H, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    rows, glued = [], []
    for m in msgs:
        strings = [tok.token_strings[t] for t in m]
        j = next(j for j, t in enumerate(strings) if t.strip() in ("15", "99"))
        assert not fsm.copy_mask_host(st, -1, m)[fsm.ptr0 + j]
        rows.append(w[fsm.ptr0 + j].float() * 20)
        glued.append(fsm.ptr0 + j)
    n = len(msgs)
    h = torch.stack(rows).to(torch.bfloat16)
    body = torch.zeros(n, 130, **i32)
    blen = torch.zeros(n, **i32)
    for r, m in enumerate(msgs):
        body[r, :len(m)] = torch.tensor(m)
        blen[r] = len(m)
    best = torch.zeros(n, dtype=torch.int64, device=DEV)
    state = torch.full((n,), st, **i32)
    ops.sparse_argmax(h, ops.fold_norm(w, torch.ones(H, dtype=torch.bfloat16, device=DEV)), state, fsm, best,
                      torch.tensor([m[-1] for m in msgs], **i32), torch.arange(n, **i32), body, blen, 1e-5)
    torch.cuda.synchronize()
    for r, m in enumerate(msgs):
        t = (0xFFFFFFFF - (int(best[r]) & 0xFFFFFFFF)) if int(best[r]) else fsm.sep_token
        assert t != glued[r] and fsm.copy_mask_host(st, -1, m)[t], (r, t)
