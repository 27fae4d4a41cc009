#!/usr/bin/env python3
"""Top-N functions (own time) of the bench's per-process cProfile dumps
(``bench.py --profile-cpu DIR``): the parser processes aggregated, and the rank
process, with the messages of the profiled phase to put them per message.

    python scripts/cprof_top.py DIR [--bench bench.json] [--n 20] > profiles/cprof_top.txt
"""
import argparse
import glob
import io
import json
import os
import pstats


def _top(files, n, msgs):
    st = pstats.Stats(*files, stream=io.StringIO())
    rows = []
    for (fn, line, name), (cc, nc, tt, ct, _) in st.stats.items():
        rows.append((tt, ct, nc, f"{os.path.basename(fn)}:{line}({name})"))
    rows.sort(reverse=True)
    total = sum(r[0] for r in rows)
    out = [f"  total own time {total:.2f} s" + (f" = {total / msgs * 1e6:.1f} us/msg over {msgs} msgs" if msgs else "")]
    out.append(f"  {'own s':>8} {'cum s':>8} {'calls':>9} {'us/msg':>7}  function")
    for tt, ct, nc, name in rows[:n]:
        per = f"{tt / msgs * 1e6:7.2f}" if msgs else "      -"
        out.append(f"  {tt:8.3f} {ct:8.3f} {nc:9d} {per}  {name}")
    return "\n".join(out)


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--bench", default="")
    p.add_argument("--n", type=int, default=20)
    a = p.parse_args()
    msgs = 0
    parsers = sorted(glob.glob(os.path.join(a.dir, "parser-*.pstats")))
    # the messages the parser processes actually parsed while profiling (each dumps its
    # count next to its stats: only the timed bus phase is profiled)
    side = [p[: -len(".pstats")] + ".json" for p in parsers]
    if side and all(os.path.exists(s) for s in side):
        msgs = sum(json.load(open(s))["msgs"] for s in side)
    elif a.bench:
        d = json.loads([x for x in open(a.bench) if x.startswith("{")][-1])
        msgs = d["steps"] * d["config"]["msgs_per_step_per_gpu"]  # the profiled (timed) phase
    ranks = sorted(glob.glob(os.path.join(a.dir, "rank*.pstats")))
    print(f"# cProfile of the timed phase ({a.dir}); own time excludes callees; blocking waits (poll / epoll /"
          " event sync) are idle, not CPU")
    if parsers:
        print(f"\n## parser processes ({len(parsers)} aggregated)\n" + _top(parsers, a.n, msgs))
    for r in ranks:
        print(f"\n## {os.path.basename(r)}\n" + _top([r], a.n, msgs))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
