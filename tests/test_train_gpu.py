"""The local extractor actually learns the task: train on synthetic SMS (fwd+bwd on
the GPU), then decode through the HIP serving engine and score field accuracy on
held-out synthetic SMS.  Also: the bundled trained (qa-format) checkpoint extracts
correctly and rejects non-transactions."""
import os

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from smsgate_amd.models.tokenizer import load_tokenizer  # noqa: E402
from smsgate_amd.models.train import TrainConfig, field_accuracy, train_extractor  # noqa: E402
from smsgate_amd.parse.text import normalize_body  # noqa: E402
from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine  # noqa: E402
from smsgate_amd.utils.synth import generate  # noqa: E402


def _score(w, n=300):
    eng = ExtractionEngine(w, load_tokenizer(), EngineConfig(max_slots=512, buckets=(64, 512)))
    held = [s for s in generate(n, seed=424242, vocab_name="heldout") if s.answer is not None]
    pred = eng.run([normalize_body(s.body) for s in held])
    return field_accuracy(pred, [s.answer for s in held])


def test_training_learns_extraction():
    # the legacy mix (the reference's two formats): what the small model learns in 2 500 steps;
    # the template-family generalisation of the 135M flagship is scored by bench.py
    w = train_extractor(TrainConfig(model="small", steps=2500, lr=2e-3, n_examples=30000, log_every=0, families=None),
                        device="cuda")
    acc = _score(w)
    for f in ("txn_type", "date", "currency"):
        assert acc[f] >= 0.95, acc
    assert sum(acc[f] for f in acc if f != "all") / 9 >= 0.8, acc


def test_bundled_checkpoint_extracts():
    """The bundled small extractor is a qa-format model trained with the flagship recipe
    (scripts/train_small_asset.py): through the HIP qa engine it extracts held-out
    layouts with held-out names, rejects held-out non-transactions and parses the
    reference CASES."""
    from smsgate_amd.models.evaluate import evaluate_engine, evaluate_negatives, golden_case_mismatches, \
        golden_case_results
    from smsgate_amd.parse.backends.local_llm import bundled_checkpoint, build_engine

    path = bundled_checkpoint("small")
    assert path is not None and os.path.exists(path)
    eng = build_engine("small", device="cuda", max_slots=1024)
    assert type(eng).__name__ == "QAEngine"
    q = evaluate_engine(eng, n=300, seed=4243, vocab_name="heldout", families="heldout")
    assert q["exact"] >= 0.95 and q["published_wrong_rate"] <= 0.03, q
    neg = evaluate_negatives(eng, n=300, seed=4246, families="neg_heldout")
    assert neg["false_parsed_rate"] <= 0.01, neg
    assert not golden_case_mismatches(golden_case_results(eng))
