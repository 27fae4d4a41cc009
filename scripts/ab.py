#!/usr/bin/env python3
"""Interleaved A/B driver for bench.py (replaces round 1's per-experiment ab_*.sh).

Each ``--arm NAME=ARGS`` is a set of extra ``bench.py`` arguments; the arms run
interleaved (A B A B …) ``--repeats`` times so box drift hits every arm alike,
each run under its own time limit.  Every run's JSON line (plus arm name and
wall time) is appended to ``--out``; a per-arm summary (mean / min / max msgs/s)
is printed at the end.  Stops at the first failing run.

    python scripts/ab.py --out gpurun_out/ab_spec.jsonl --repeats 2 \\
        --arm "spec0=--spec-k 0" --arm "spec4=--spec-k 4" --common "--steps 10 --warmup 2 --eval-n 0"
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--arm", action="append", required=True, help="NAME=extra bench.py args")
    p.add_argument("--common", default="", help="args for every arm")
    p.add_argument("--repeats", type=int, default=2)
    p.add_argument("--timeout", type=int, default=600, help="seconds per run")
    p.add_argument("--script", default="bench.py")
    p.add_argument("--out", required=True)
    a = p.parse_args(argv)
    arms = []
    for spec in a.arm:
        name, _, args = spec.partition("=")
        arms.append((name, shlex.split(args)))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    results = {name: [] for name, _ in arms}
    for rep in range(a.repeats):
        for name, args in arms:
            cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", a.script, *shlex.split(a.common), *args]
            t0 = time.time()
            # the run's stderr streams into a log next to --out (progress stays visible)
            with open(a.out + ".stderr.log", "a") as err:
                r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=err, text=True)
            line = next((x for x in reversed(r.stdout.splitlines()) if x.startswith("{")), None)
            if r.returncode != 0 or line is None:
                print(f"[ab] {name} run {rep} failed (rc {r.returncode}); stderr in {a.out}.stderr.log", flush=True)
                return r.returncode or 1
            d = json.loads(line)
            d.update(arm=name, repeat=rep, wall_s=round(time.time() - t0, 1), args=args)
            with open(a.out, "a") as f:
                f.write(json.dumps(d) + "\n")
            results[name].append(float(d.get("value", 0.0)))
            print(f"[ab] {name} #{rep}: {d.get('value')} {d.get('unit', '')}", flush=True)
    for name, vals in results.items():
        print(f"[ab] {name}: mean {sum(vals) / len(vals):.1f}  min {min(vals):.1f}  max {max(vals):.1f}  n={len(vals)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
