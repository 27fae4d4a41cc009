#!/usr/bin/env python3
"""Shrink a ``rocprofv3 --kernel-trace --stats`` output directory to what is worth keeping.

The kernel trace of a bench run holds one row per dispatch (millions for a full
run), far more than gpurun copies back.  This streams it once and writes, next to
the stats CSV, ``<prefix>_grid_hist.csv``: per (kernel, grid size, workgroup size)
the dispatch count and total / mean duration -- enough to recover each GEMM's
row-count distribution (grid = tiles) -- then deletes the trace.

    python scripts/prof_summary.py gpurun_out/prof_r03a [--keep-trace]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def _col(header, *names):
    for n in names:
        if n in header:
            return header.index(n)
    raise KeyError(f"none of {names} in {header}")


def summarise(trace: str) -> str:
    agg = defaultdict(lambda: [0, 0])
    with open(trace, newline="") as f:
        rd = csv.reader(f)
        h = next(rd)
        kn = _col(h, "Kernel_Name")
        gx = _col(h, "Grid_Size_X", "Grid_Size")
        wx = _col(h, "Workgroup_Size_X", "Workgroup_Size")
        t0, t1 = _col(h, "Start_Timestamp"), _col(h, "End_Timestamp")
        for row in rd:
            k = (row[kn], int(row[gx]), int(row[wx]))
            a = agg[k]
            a[0] += 1
            a[1] += int(row[t1]) - int(row[t0])
    out = trace.replace("_kernel_trace.csv", "_grid_hist.csv")
    total = sum(v[1] for v in agg.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size", "Workgroup_Size", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for (name, g, wg), (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, g, wg, n, ns, round(ns / n, 1), round(100.0 * ns / total, 3)])
    return out


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("dir")
    p.add_argument("--keep-trace", action="store_true")
    a = p.parse_args()
    traces = glob.glob(os.path.join(a.dir, "**", "*_kernel_trace.csv"), recursive=True)
    for t in traces:
        print(summarise(t))
        if not a.keep_trace:
            os.remove(t)
    for pat in ("*_agent_info.csv",):  # (large, machine description only)
        for f in glob.glob(os.path.join(a.dir, "**", pat), recursive=True):
            os.remove(f)
    return 0 if traces else 1


if __name__ == "__main__":
    sys.exit(main())
