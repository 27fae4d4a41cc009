"""Train the extractor on synthetic SMS (GPU), then score it through the HIP serving
engine on held-out synthetic SMS and the reference's three golden cases."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="small")
    p.add_argument("--steps", type=int, default=800)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--lr", type=float, default=2e-3)
    p.add_argument("--examples", type=int, default=40000)
    p.add_argument("--eval", type=int, default=500)
    p.add_argument("--out", default="")
    a = p.parse_args()
    import asyncio

    import torch

    from smsgate_amd.models.tokenizer import load_tokenizer
    from smsgate_amd.models.train import TrainConfig, field_accuracy, train_extractor
    from smsgate_amd.parse.text import normalize_body
    from smsgate_amd.serving.engine import EngineConfig, ExtractionEngine
    from smsgate_amd.utils.synth import generate

    t0 = time.perf_counter()
    w = train_extractor(TrainConfig(model=a.model, steps=a.steps, batch=a.batch, lr=a.lr, n_examples=a.examples),
                        device="cuda", log=lambda s: print(s, flush=True))
    train_s = time.perf_counter() - t0
    if a.out:
        w.save(a.out)
    eng = ExtractionEngine(w, load_tokenizer(), EngineConfig(max_slots=1024, buckets=(64, 256, 1024)))
    held = [s for s in generate(a.eval, seed=987654) if s.answer is not None]
    pred = eng.run([normalize_body(s.body) for s in held])
    acc = field_accuracy(pred, [s.answer for s in held])

    # the reference's golden cases through the whole parse pipeline
    from smsgate_amd.models import RawSMS
    from smsgate_amd.parse.backends.local_llm import LocalLLMBackend
    from smsgate_amd.parse.pipeline import ParsePipeline
    from smsgate_amd.utils.synth import reference_cases

    async def golden():
        be = LocalLLMBackend.from_engine(eng) if hasattr(LocalLLMBackend, "from_engine") else None
        if be is None:
            return None
        pipe = ParsePipeline(be)
        out = []
        for i, body in enumerate(reference_cases()):
            r = await pipe.parse(RawSMS(msg_id=f"g{i}", device_id="d", sender="BANK", date="2025-05-06T00:00:00",
                                        body=body, source="device"))
            out.append(None if r.parsed is None else r.parsed.model_dump(mode="json"))
        await be.close()
        return out

    gold = asyncio.run(golden())
    print(json.dumps({"model": a.model, "steps": a.steps, "train_s": round(train_s, 1), "accuracy": acc,
                      "golden": gold}), flush=True)


if __name__ == "__main__":
    main()
