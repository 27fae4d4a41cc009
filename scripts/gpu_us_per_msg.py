#!/usr/bin/env python3
"""GPU time per LLM-routed message from a rocprofv3 ``*_kernel_stats.csv`` of a bench
run (VERDICT r03 next #2's measure: round 3 = 36.8 us, profiles/PERF.md).

    python scripts/gpu_us_per_msg.py <kernel_stats.csv | results.db> <bench JSON line file> [--out f.json]

Messages = (warmup + steps) x msgs_per_step_per_gpu x llm share of the profiled run
(run it with ``--eval-n 0 --ingest bus``: no quality evaluation, one ingest phase, and
weights from the cache, so the profile holds the serving kernels only).  Kernel time
is split into GEMMs, attention, the lm_head arg-max / commit, speculative planning
and the rest.

Two measures: the SUM of kernel durations (round 4's measure) and, from a results.db,
the BUSY time -- the union of the kernels' [start, end) intervals.  With two streams
in flight (the engine runs its prefill halves on two) kernels overlap and each one
runs longer while it shares the CUs, so the sum over-counts the GPU time a message
costs; the busy time is the wall-clock the GPU spent on it.  ``--msgs N`` instead of a
bench JSON: an engine-only run of N messages (scripts/qa_engine_bench.py)."""
import argparse
import csv
import json


def _group(name: str) -> str:
    n = name.lower()
    if "gemm" in n or "cijk" in n:
        return "gemm"
    if "attn" in n:
        return "attention"
    if "argmax" in n or "commit" in n or "fsm_" in n:
        return "lm_head_argmax_commit"
    if "spec_" in n:
        return "spec_plan_verify"
    return "other"


def _busy_ns(db):
    """(union of the kernel intervals in ns, number of streams) of a results.db, or
    (None, None) when it has no per-dispatch ``kernels`` view."""
    try:
        iv = sorted(db.execute("SELECT start, end FROM kernels"))
    except Exception:  # noqa: BLE001 -- a stats-only database
        return None, None
    if not iv:
        return None, None
    streams = db.execute("SELECT COUNT(DISTINCT stream_id) FROM kernels").fetchone()[0]
    busy, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + ce - cs, streams


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("stats")
    p.add_argument("bench", nargs="?", default="")
    p.add_argument("--msgs", type=float, default=0.0)
    p.add_argument("--out", default="")
    a = p.parse_args(argv)
    if a.stats.endswith(".db"):  # rocprofv3's SQLite output (no --output-format csv): its top_kernels view, us
        import sqlite3

        db = sqlite3.connect(a.stats)
        rows = [{"Name": n, "TotalDurationNs": float(t) * 1e3}
                for n, t in db.execute("SELECT name, total_duration FROM top_kernels")]
        busy, streams = _busy_ns(db)
    else:
        rows = list(csv.DictReader(open(a.stats)))
        busy, streams = None, None
    if a.msgs:
        b, msgs = {}, a.msgs
    else:
        line = [x for x in open(a.bench).read().splitlines() if x.startswith("{")][-1]
        b = json.loads(line)
        per_step = b["config"]["msgs_per_step_per_gpu"]
        msgs = (b["steps"] + b["warmup"]) * per_step * float(b.get("llm_parsed_share", 1.0))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    groups = {}
    for r in rows:
        g = _group(r["Name"])
        groups[g] = groups.get(g, 0.0) + float(r["TotalDurationNs"])
    out = {"kernel_s": round(tot / 1e9, 3), "llm_msgs": int(msgs), "gpu_us_per_msg": round(tot / 1e3 / msgs, 2),
           "by_group_us_per_msg": {k: round(v / 1e3 / msgs, 2) for k, v in sorted(groups.items(), key=lambda x: -x[1])},
           "bench_value": b.get("value"), "answer_format": b.get("answer_format"), "traffic": b.get("traffic")}
    if busy is not None:
        out["gpu_busy_us_per_msg"] = round(busy / 1e3 / msgs, 2)
        out["streams"] = streams
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(out, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
