"""Copy-constrained decoding on the GPU (csrc/spec_kernels.hip copy_mask_kernel, the
EPI 4 arg-max epilogue, fsm_sample / spec_verify with row masks) against plain
PyTorch references, and the engine-level guarantee: every copied value is a
chain of body bigrams, with and without speculative decoding."""
import random

import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd import ops  # noqa: E402
from smsgate_amd.parse.text import normalize_body  # noqa: E402
from smsgate_amd.serving.fsm import COPY_NEXT, COPY_NONE, COPY_START, build_fsm  # noqa: E402
from smsgate_amd.utils.synth import generate, reference_cases  # noqa: E402

DEV = "cuda"
i32 = dict(dtype=torch.int32, device=DEV)


def _setup(n_rows, seed=0):
    """FSM over the decode vocabulary, a few prompt bodies in KV slots, and ``n_rows``
    rows in random states (every copy kind) with plausible previous tokens."""
    from smsgate_amd.models.tokenizer import load_tokenizer

    tk = load_tokenizer()
    V = (tk.vocab_size + 127) // 128 * 128
    fsm = build_fsm(tk, V).to_device(DEV)
    bodies = [normalize_body(s.body) for s in generate(12, seed=seed, vocab_name="heldout") if s.answer]
    bodies += [normalize_body(b) for b in reference_cases()]
    msgs = tk.message_ids(bodies, 128)
    S, LB = len(msgs) + 1, 130
    body = torch.zeros(S, LB, **i32)
    blen = torch.zeros(S, **i32)
    for k, m in enumerate(msgs):
        body[k, :len(m)] = torch.tensor(m)
        blen[k] = len(m)
    rng = random.Random(seed)
    kinds = fsm.copy_kind
    by_kind = {k: [s for s in range(fsm.num_states) if kinds[s] == k] for k in (COPY_NONE, COPY_START, COPY_NEXT)}
    st, pv, sl = [], [], []
    for r in range(n_rows):
        k = r % 3
        st.append(rng.choice(by_kind[k]))
        slot = rng.randrange(len(msgs))
        sl.append(slot)
        m = msgs[slot]
        # mostly a token of the body (a copy in progress), sometimes anything
        pv.append(rng.choice(m[1:-1]) if rng.random() < 0.85 else rng.randrange(tk.vocab_size))
    return fsm, body, blen, torch.tensor(st, **i32), torch.tensor(pv, **i32), torch.tensor(sl, **i32)


@pytest.mark.parametrize("n", [1, 5, 301])
def test_copy_masks_match_reference(n):
    fsm, body, blen, st, pv, sl = _setup(n, seed=n)
    words = fsm.vocab // 32
    sentinel = 0x5A5A5A5A
    out = torch.full((n + 2, words), sentinel, **i32)
    ops.copy_masks(fsm, st, pv, sl, body, blen, out, n)
    torch.cuda.synchronize()
    ref = ops.ref_copy_masks(fsm, st, pv, sl, body, blen)
    got = ops.unpack_masks(out[:n]).cpu()
    kinds = fsm.copy_kind[st.cpu().numpy()]
    for r in range(n):
        if kinds[r] == COPY_NONE:
            assert torch.all(out[r] == sentinel)  # non-copy rows are never written
        else:
            assert torch.equal(got[r], ref[r]), r
            if kinds[r] == COPY_START:
                assert got[r, fsm.sep_token]  # an empty value is always possible
    assert torch.all(out[n:] == sentinel)


@pytest.mark.parametrize("cfg", [0, 3, 17])
@pytest.mark.parametrize("M", [1, 77, 700])
def test_gemm_argmax_copy_rows(cfg, M):
    """EPI 4 with row masks == fp32 masked arg-max of the same bf16 logits (copy rows
    by their own mask, the others by their state's), and == fsm_sample with the masks."""
    fsm, body, blen, st, pv, sl = _setup(M, seed=100 + M)
    K = 576
    g = torch.Generator(device="cpu").manual_seed(7)
    a = (torch.randn(M, K, generator=g)).to(torch.bfloat16).to(DEV)
    w = (torch.randn(fsm.vocab, K, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    rm = torch.zeros(M, fsm.vocab // 32, **i32)
    ops.copy_masks(fsm, st, pv, sl, body, blen, rm)
    best = torch.zeros(M, dtype=torch.int64, device=DEV)
    ops.gemm_argmax(a, w, st, fsm, best, norm_eps=1e-5, cfg=cfg, row_masks=rm)
    logits = ops.gemm(a, w, norm_eps=1e-5)
    tok = torch.zeros(M, **i32)
    zeros = [torch.zeros(M, **i32) for _ in range(4)]
    st_s = st.clone()
    ops.fsm_sample(logits, fsm, st_s, tok, torch.zeros(M, 4, **i32), zeros[0], zeros[1], zeros[2], zeros[3], 0.0, 0,
                   row_masks=rm)
    tok_b = torch.zeros(M, **i32)
    st_b = st.clone()
    ops.fsm_commit(best, fsm, st_b, tok_b, torch.zeros(M, 4, **i32), torch.zeros(M, **i32), torch.zeros(M, **i32),
                   torch.zeros(M, **i32), M)
    assert torch.equal(tok, tok_b) and torch.equal(st_s, st_b)
    allowed = ops.ref_copy_masks(fsm, st, pv, sl, body, blen)
    lf = logits.float().cpu()
    for r in range(M):
        if allowed[r].any():
            assert int(tok_b[r]) == int(lf[r].masked_fill(~allowed[r], float("-inf")).argmax()), r
    with pytest.raises(ValueError):  # wrong mask width is refused before any launch
        ops.gemm_argmax(a, w, st, fsm, best, norm_eps=1e-5, row_masks=rm[:, :-1].contiguous())


def _engine(spec_k, **kw):
    from smsgate_amd.parse.backends.local_llm import build_engine, bundled_checkpoint

    return build_engine("small", bundled_checkpoint("small-copy"), device=DEV, answer_format="copy", max_slots=512,
                        buckets=(64, 512), use_graphs=False, spec_k=spec_k,
                        decode_attn_small_rows=0, lm_head_fused=True, split_decode=0, **kw)


def _raw_run(eng, bodies):
    eng.submit_ids(list(enumerate(eng.tok.message_ids(bodies, eng.cfg.max_body_tokens))))
    out = {}
    while eng.busy():
        for k, toks in eng.step(raw=True):
            out[k] = [int(t) for t in toks]
    return [out[i] for i in range(len(bodies))]


@pytest.mark.parametrize("random_init", [True, False])
def test_engine_values_are_body_bigram_chains(random_init):
    """Random weights (answers are noise) or the bundled trained model: every copied
    value starts with a body token and continues along body bigrams -- the model
    cannot write a token sequence the SMS does not contain.  Speculative decoding
    gives the same tokens."""
    bodies = [normalize_body(s.body) for s in generate(160, seed=31, vocab_name="heldout") if s.answer]
    bodies += [normalize_body(b) for b in reference_cases()]
    kw = {"random_init": True} if random_init else {}
    eng = _engine(0, **kw)
    outs = _raw_run(eng, bodies)
    msgs = eng.tok.message_ids(bodies, eng.cfg.max_body_tokens)
    fsm = eng.fsm
    n_vals = 0
    for m, toks in zip(msgs, outs):
        bigrams = set(zip(m[:-1], m[1:]))
        vals = fsm.split_fields(toks)
        for f, v in zip(fsm.fields, vals):
            if not f.copy or not v:
                continue
            n_vals += 1
            assert v[0] in m, (f.name, v)
            for x, y in zip(v[:-1], v[1:]):
                assert (x, y) in bigrams, (f.name, v)
    if not random_init:  # (random weights mostly end a value at once: <sep> beats the few body tokens)
        assert n_vals > len(bodies)
    spec = _raw_run(_engine(4, **kw), bodies)
    assert spec == outs


def test_copy_off_is_the_old_decoder():
    """copy_constrain=False serves exactly the schema-only decoder (no row masks)."""
    bodies = [normalize_body(b) for b in reference_cases()]
    eng = _engine(0, copy_constrain=False)
    assert not eng.copy and not hasattr(eng, "copy_rows")
    assert len(eng.run(bodies)) == 3


@pytest.mark.parametrize("H", [128, 576])
def test_sparse_argmax_matches_dense_masked_argmax(H):
    """ops.sparse_argmax (candidates only) == the dense lm_head GEMM's masked arg-max
    (copy masks + EPI 4) on rows in every kind of state: the chosen token is allowed,
    its logit is the allowed maximum of an fp32 reference (to bf16 rounding), and the
    two kernels pick the same token except at bf16 near-ties."""
    from smsgate_amd import ops
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import make_examples
    from smsgate_amd.serving.fsm import build_fsm

    tok = load_tokenizer()
    V = (tok.vocab_size + 127) // 128 * 128
    fsm = build_fsm(tok, V).to_device("cuda")
    assert ops.sparse_argmax_ok(fsm)
    exs = make_examples(tok, fsm, 400, seed=11, vocab_name="heldout")[:256]
    n, LB = len(exs), 160
    i32 = dict(dtype=torch.int32, device="cuda")
    body = torch.zeros(n, LB, **i32)
    blen = torch.zeros(n, **i32)
    states, prevs = [], []
    g = torch.Generator().manual_seed(3)
    for r, (m, a) in enumerate(exs):
        body[r, :len(m)] = torch.tensor(m)
        blen[r] = len(m)
        L = int(torch.randint(0, len(a), (1,), generator=g))  # any point of the gold answer
        s = fsm.start_state
        for x in a[:L]:
            s = fsm.step_host(s, x)
        states.append(s)
        prevs.append(a[L - 1] if L else fsm.start_state)
    state = torch.tensor(states, **i32)
    prev = torch.tensor(prevs, **i32)
    slot = torch.arange(n, **i32)
    h = (torch.randn(n, H, generator=g) * 2).to(torch.bfloat16).cuda()
    nw = (torch.rand(H, generator=g) + 0.5).to(torch.bfloat16).cuda()
    w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16).cuda()
    wf = ops.fold_norm(w, nw)
    sparse = torch.zeros(n, dtype=torch.int64, device="cuda")
    ops.sparse_argmax(h, wf, state, fsm, sparse, prev, slot, body, blen, 1e-5)
    masks = torch.zeros(n, V // 32, **i32)
    ops.copy_masks(fsm, state, prev, slot, body, blen, masks, n)
    dense = torch.zeros(n, dtype=torch.int64, device="cuda")
    ops.gemm_argmax(h, wf, state, fsm, dense, norm_eps=1e-5, row_masks=masks)
    torch.cuda.synchronize()
    ref = ops.ref_gemm(h, w, norm_eps=1e-5, norm_w=nw)  # fp32 logits
    tid = lambda k: (0xFFFFFFFF - (int(k) & 0xFFFFFFFF)) if int(k) else fsm.sep_token  # noqa: E731
    same = 0
    for r in range(n):
        allowed = torch.tensor(fsm.copy_mask_host(states[r], prevs[r], exs[r][0]), device="cuda")
        ts, td = tid(sparse[r]), tid(dense[r])
        assert bool(allowed[ts]) or not allowed.any(), (r, ts)
        top = ref[r].masked_fill(~allowed, float("-inf")).max()
        assert float(ref[r, ts]) >= float(top) - 0.02 * abs(float(top)) - 0.02, (r, ts, float(ref[r, ts]), float(top))
        same += ts == td
    assert same >= 0.97 * n, same
