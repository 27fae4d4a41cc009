"""The reference's three golden CASES (tests/test_parsers.py:11-58, asserted like
:73-86) through the local_llm backend with the bundled trained checkpoint and the
full parse pipeline.  The checkpoint was trained on vocabularies that contain none
of the golden words (TEST, LLC, MOSKOW, AMERIABANK, API, GATE, AM —
tests/test_fsm_caps.py pins that), so this is an out-of-vocabulary test of the
extractor's copying, not a memorisation check."""
from datetime import datetime
from decimal import Decimal

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]

from conftest import REFERENCE_CASES  # noqa: E402
from smsgate_amd.models import RawSMS, TxnType  # noqa: E402
from smsgate_amd.parse.backends.local_llm import LocalLLMBackend, build_engine, bundled_checkpoint  # noqa: E402
from smsgate_amd.parse.pipeline import ParsePipeline  # noqa: E402


@pytest.fixture(scope="module")
def pipeline():
    eng = build_engine("small", bundled_checkpoint("small-copy"), device="cuda", max_slots=64, buckets=(64,), spec_k=0)
    return ParsePipeline(LocalLLMBackend.from_engine(eng))


@pytest.mark.parametrize("fmt,spec_k", [("qa", 0), ("copy", 0), ("copy", 4)])
def test_reference_cases_local_llm(pipeline, fmt, spec_k, arun):
    """qa: the bundled one-forward checkpoint (the default ``small`` weights); copy: the
    round-4 autoregressive checkpoint, without and with speculative drafts."""
    if fmt == "qa":
        eng = build_engine("small", device="cuda", max_slots=64)
        assert type(eng).__name__ == "QAEngine"
        pipe = ParsePipeline(LocalLLMBackend.from_engine(eng))
    elif spec_k:
        eng = build_engine("small", bundled_checkpoint("small-copy"), device="cuda", max_slots=64, buckets=(64,), spec_k=spec_k)
        pipe = ParsePipeline(LocalLLMBackend.from_engine(eng))
    else:
        pipe = pipeline
    raws = [RawSMS(msg_id=f"g{i}", device_id="d", sender="BANK", date="1746541380", body=b, source="device")
            for i, (b, _) in enumerate(REFERENCE_CASES)]
    results = arun(pipe.parse_batch(raws))
    for (body, exp), res in zip(REFERENCE_CASES, results):
        p = res.parsed
        assert p is not None, (body, res)
        assert p.txn_type == TxnType.DEBIT
        assert (p.merchant, p.city, p.address, p.card, p.currency) == (
            exp["merchant"], exp["city"], exp["address"], exp["card"], exp["currency"]), p
        assert p.amount == Decimal(exp["amount"]) and p.balance == Decimal(exp["balance"])
        assert p.date == datetime(*exp["date"])
