"""Speculative decoding (csrc/spec_kernels.hip): prompt-lookup drafts from the SMS
body, verified in one forward, give the SAME greedy answers as one-token decode
and emit several tokens per row per forward on trained weights."""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd.parse.text import normalize_body  # noqa: E402
from smsgate_amd.utils.synth import generate, reference_cases  # noqa: E402


def _engine(spec_k, use_graphs, **kw):
    from smsgate_amd.parse.backends.local_llm import build_engine

    # one attention kernel and our own lm_head GEMM in both modes: identical per-row arithmetic
    return build_engine("small", device="cuda", max_slots=512, buckets=(64, 512), use_graphs=use_graphs,
                        spec_k=spec_k, decode_attn_small_rows=0, lm_head_fused=True, split_decode=0, **kw)


@pytest.mark.parametrize("use_graphs", [False, True])
def test_spec_matches_plain_greedy_decode(use_graphs):
    bodies = [normalize_body(s.body) for s in generate(400, seed=2024, vocab_name="heldout") if s.answer]
    bodies += [normalize_body(b) for b in reference_cases()]
    base = _engine(0, use_graphs).run(bodies)
    eng = _engine(4, use_graphs)
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
