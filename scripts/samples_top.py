#!/usr/bin/env python3
"""Top-N of a bench CPU sampling profile (``bench.py --profile-cpu DIR``, the default
``--profile-mode sample``; smsgate_amd/utils/sampler.py): CPU µs per message by
innermost Python line (self) and by function on the stack (inclusive), parser
processes aggregated, the rank process separately.

    python scripts/samples_top.py DIR [--bench bench.json] [-n 25]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smsgate_amd.utils.sampler import merge_samples  # noqa: E402


def _table(doc, msgs: float, n: int) -> str:
    cpu = doc.get("cpu_s") or doc["samples"] * doc["interval_s"]
    us = cpu * 1e6 / max(1, doc["samples"]) / max(1.0, msgs)  # each sample's share of the measured CPU time
    tot = doc["samples"] * us
    lines = [f"  {doc['samples']} samples over {cpu:.2f} s of process CPU = {tot:.1f} us/msg over "
             f"{int(msgs)} msgs ({doc.get('procs', 1)} process(es))",
             "  self us/msg  innermost line"]
    for k, c in sorted(doc["leaf"].items(), key=lambda x: -x[1])[:n]:
        lines.append(f"  {c * us:11.2f}  {k}")
    lines.append("  incl us/msg  function on the stack")
    for k, c in sorted(doc["incl"].items(), key=lambda x: -x[1])[:n]:
        lines.append(f"  {c * us:11.2f}  {k}")
    return "\n".join(lines)


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--bench", default="")
    p.add_argument("-n", type=int, default=25)
    a = p.parse_args()
    parsers = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(a.dir, "parser-*.samples.json")))]
    bench_msgs = 0
    if a.bench:
        d = json.loads([x for x in open(a.bench) if x.startswith("{")][-1])
        bench_msgs = d["steps"] * d["config"]["msgs_per_step_per_gpu"]
    print(f"# CPU sampling profile of the timed bus phase ({a.dir}): ITIMER_PROF samples of the main "
          "thread's stack; waits take no samples")
    if parsers:
        m = merge_samples(parsers)
        print("\n## parser processes\n" + _table(m, m["msgs"] or bench_msgs, a.n))
    for f in sorted(glob.glob(os.path.join(a.dir, "rank*.samples.json"))):
        d = json.load(open(f))
        print(f"\n## {os.path.basename(f)}\n" + _table(d, d["msgs"] or bench_msgs, a.n))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
