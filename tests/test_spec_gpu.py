"""Speculative decoding (csrc/spec_kernels.hip): prompt-lookup drafts from the SMS
body, verified in one forward, give the SAME greedy answers as one-token decode
and emit several tokens per row per forward on trained weights."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd.parse.text import normalize_body  # noqa: E402
from smsgate_amd.utils.synth import generate, reference_cases  # noqa: E402


def _engine(spec_k, use_graphs, **kw):
    from smsgate_amd.parse.backends.local_llm import build_engine, bundled_checkpoint

    # one attention kernel and our own lm_head GEMM in both modes: identical per-row arithmetic
    return build_engine("small", bundled_checkpoint("small-copy"), device="cuda", max_slots=512, buckets=(64, 512), use_graphs=use_graphs,
                        spec_k=spec_k, decode_attn_small_rows=0, lm_head_fused=True, split_decode=0, **kw)


@pytest.mark.parametrize("use_graphs,policy", [(False, 0), (False, 1), (True, 1)])
def test_spec_matches_plain_greedy_decode(use_graphs, policy):
    bodies = [normalize_body(s.body) for s in generate(400, seed=2024, vocab_name="heldout") if s.answer]
    bodies += [normalize_body(b) for b in reference_cases()]
    base = _engine(0, use_graphs).run(bodies)
    eng = _engine(4, use_graphs, spec_policy=policy)
    spec = eng.run(bodies)
    assert spec == base
    st = eng.spec_stats()
    assert st["spec_tokens_per_row_step"] >= 2.0, st


def test_spec_draft_budget_clamps_without_changing_answers():
    """A draft budget far below demand clamps drafts (later rows get fewer), never answers."""
    bodies = [normalize_body(s.body) for s in generate(300, seed=7, vocab_name="heldout") if s.answer]
    base = _engine(0, False).run(bodies)
    eng = _engine(6, False, spec_draft_frac=0.25)
    assert eng.run(bodies) == base
    assert 1.0 < eng.spec_stats()["spec_tokens_per_row_step"]


def test_spec_plan_budget_water_filling():
    """spec_plan: with an unlimited budget every row keeps its drafts; with a tight
    one the counts are water-filled (each row min(nd, c) or one more) and packed."""
    import random

    from smsgate_amd import ops
    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import make_examples
    from smsgate_amd.serving.fsm import build_fsm

    tok = load_tokenizer()
    V = 49152
    fsm = build_fsm(tok, V).to_device("cuda")
    exs = make_examples(tok, fsm, 400, seed=5, vocab_name="heldout")[:300]
    B, K, LB, max_out = len(exs), 6, 160, 160
    rng = random.Random(0)
    i32 = dict(dtype=torch.int32, device="cuda")
    body = torch.zeros(B + 1, LB, **i32)
    blen = torch.zeros(B + 1, **i32)
    out_buf = torch.zeros(B, max_out, **i32)
    out_len = torch.zeros(B, **i32)
    tok_buf = torch.zeros(B, **i32)
    state = torch.zeros(B, **i32)
    for r, (m, a) in enumerate(exs):
        body[r, :len(m)] = torch.tensor(m)
        blen[r] = len(m)
        L = rng.randint(1, len(a) - 1)
        out_buf[r, :L] = torch.tensor(a[:L])
        out_len[r] = L
        tok_buf[r] = a[L - 1]
        s = fsm.start_state
        for x in a[:L]:
            s = fsm.step_host(s, x)
        state[r] = s
    strings = tok.token_strings
    delim = torch.tensor([(("," in t) or ("&#" in t) or (";" in t)) and i != tok.sep for i, t in enumerate(strings)]
                         + [False] * (V - len(strings)), dtype=torch.uint8, device="cuda")
    pos = torch.arange(B, **i32) + 30
    slot = torch.arange(B, **i32)
    done = torch.zeros(B, **i32)
    done[::7] = 1  # finished rows take no pseudo-row
    live = (done == 0).cpu()

    def plan(T_cap):
        bufs = [torch.zeros(T_cap, **i32) for _ in range(5)]
        rs, nd, meta = torch.zeros(B, **i32), torch.zeros(B, **i32), torch.zeros(1, **i32)
        draft = torch.zeros(B * ops.SPEC_MAX_K, **i32)
        ops.spec_plan(fsm, state, bufs[4], K, T_cap, tok.sep, B, tok_buf, pos, slot, done, out_buf, out_len, body,
                      blen, delim, draft, bufs[0], bufs[1], bufs[2], bufs[3], rs, nd, meta)
        torch.cuda.synchronize()
        return rs.cpu(), nd.cpu(), int(meta.cpu()[0]), bufs[0].cpu()

    def starts(nd):
        n = torch.where(nd >= 0, 1 + nd, torch.zeros_like(nd))
        return torch.cumsum(n, 0) - n

    rs, full, used, xt = plan(B * (1 + K))
    assert torch.equal(full < 0, ~live)
    nlive = int(live.sum())
    assert int(full[live].sum()) > nlive  # plenty of drafts to clamp
    assert used == nlive + int(full[live].sum())
    assert torch.equal(rs[live], starts(full)[live])
    cap = nlive // 2
    rs, nd, used, xt = plan(B + cap)  # budget: T_cap - live rows = B - nlive + cap
    budget = B - nlive + cap
    nd, full = nd[live], full[live]
    assert used == nlive + int(nd.sum()) and int(nd.sum()) == min(budget, int(full.sum()))
    assert torch.all((nd >= 0) & (nd <= full))
    clamped = nd < full
    c = int(nd[clamped].min())
    assert torch.all(nd >= torch.minimum(full, torch.full_like(full, c))) and int(nd.max()) <= c + 1
    assert torch.equal(rs[live], starts(nd))
    assert torch.equal(xt[rs[live].long()], tok_buf.cpu()[live])  # each live row's first pseudo-row = its last token
