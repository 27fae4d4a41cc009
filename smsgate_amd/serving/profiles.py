"""Named engine configurations: ONE source of defaults for ``bench.py`` and
``engine-server`` (and so for the compose deployment, which serves the profile
the headline bench measured).

* ``throughput`` — the headline bench's configuration: 8 192 rows, two decode
  steps per graph, admission at 12.5 % free rows, up to six drafts per row
  (profiles/r02s3_admit_frac_ab*.jsonl, r02s3_spec_k_ab.jsonl);
* both learn up to 32 message-start templates (``EngineConfig.template_slots``): 16 of
  them left 3.2 of ~50 prompt tokens per message uncomputed, +1.8 % msgs/s interleaved
  (profiles/r03_ab_templates2.jsonl; a 16 384-row engine lost 12 % there); 32 reach 4.0
  of the 4.1 tokens an oracle choice would save (replay of 20 k purchase SMS through
  the learning policy);
* ``latency`` — the serving-latency configuration: 4 096 rows, otherwise the
  throughput profile's knobs (two steps per graph, 12.5 % admission, six drafts);
  p50 25.9 / 31.7 / 41.5 / 49.9 ms at 1 k / 6 k / 10 k / 14 k msgs/s offered, against
  29.3 / 37.6 / 42.8 / 52.2 ms for the round-2 latency profile (``latency_r2``: four
  steps per graph, 25 % admission, four drafts) in the same call
  (profiles/r03s2b_latency_{latency,latency_r2,throughput}.json).

The one-forward qa engine (serving/qa_engine.py, the default extractor since round 5)
reads only its ``qa_*`` knobs and ``max_slots``:

* both profiles: packed batches of up to 262 144 rows (~5 000 messages), a second batch
  in flight once 65 536 rows wait (profiles/r05_qa_min_tokens_ab.jsonl).  Under Poisson
  arrivals that gives p50 / p99 of 1.4 / 1.7 ms at 1 k msgs/s, 1.7 / 2.0 ms at 10 k and
  5.4 / 6.5 ms at 40 k (profiles/r06_latency_qa_throughput.json): a batch is launched as
  soon as the GPU is free, so at these loads it holds what arrived during one forward.
  Smaller batches (16 384 rows, a second in flight from 2 048) were slower at every
  load -- 3.9 ms p99 at 10 k, 13.0 ms at 40 k (profiles/r06_latency_qa_latency.json) --
  so the latency profile serves the throughput profile's qa knobs.

Everything not listed keeps the :class:`~smsgate_amd.serving.engine.EngineConfig`
default.
"""
from __future__ import annotations

from typing import Any, Dict

__all__ = ["PROFILES", "profile_kwargs", "BUCKETS"]

BUCKETS = (64, 128, 256, 512, 1024, 2048, 4096, 8192)

PROFILES: Dict[str, Dict[str, Any]] = {
    "throughput": dict(max_slots=8192, steps_per_graph=2, admit_min_fraction=0.125, spec_k=6, spec_draft_frac=1.25,
                       buckets=BUCKETS, split_decode=4096, split_prefill=8192, copy_constrain=True,
                       template_slots=32, qa_max_tokens=262144, qa_min_tokens=65536),
    "latency": dict(max_slots=4096, steps_per_graph=2, admit_min_fraction=0.125, spec_k=6, spec_draft_frac=1.25,
                    buckets=BUCKETS[:-1], split_decode=4096, split_prefill=8192, copy_constrain=True,
                    template_slots=32, qa_max_tokens=262144, qa_min_tokens=65536),
    # the round-2 latency profile (4 steps per graph, 25 % admission, 4 drafts): with the
    # round-3 kernels it was behind the throughput profile at every load
    # (profiles/r03s2_latency_{latency,throughput}.json, r03s2b_latency_latency_r2.json)
    "latency_r2": dict(max_slots=4096, steps_per_graph=4, admit_min_fraction=0.25, spec_k=4, spec_draft_frac=1.25,
                       buckets=BUCKETS[:-1], split_decode=4096, split_prefill=8192, copy_constrain=True,
                       template_slots=32),
}


def profile_kwargs(name: str, **overrides: Any) -> Dict[str, Any]:
    """EngineConfig keyword arguments of profile ``name`` with ``overrides`` applied
    (None values are ignored, so unset CLI flags keep the profile's value)."""
    if name not in PROFILES:
        raise KeyError(f"unknown engine profile {name!r} (one of {sorted(PROFILES)})")
    kw = dict(PROFILES[name])
    kw.update({k: v for k, v in overrides.items() if v is not None})
    if "max_slots" in overrides and overrides["max_slots"] is not None:
        kw["buckets"] = tuple(b for b in kw["buckets"] if b <= kw["max_slots"]) or (kw["max_slots"],)
    return kw
