"""GPU idle-gap analysis of a rocprofv3 kernel trace: busy fraction over the run,
the largest gaps, and which kernels border them.  Usage: trace_gaps.py kernel_trace.csv"""
import csv
import sys
from collections import Counter


def main(path: str) -> None:
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    ev.sort()
    # skip the first 40% (build / warm-up / graph capture): analyse the tail
    t0 = ev[int(len(ev) * 0.4)][0]
    ev = [e for e in ev if e[0] >= t0]
    span = ev[-1][1] - ev[0][0]
    busy, cur_s, cur_e = 0, ev[0][0], ev[0][1]
    gaps = []
    prev_name = ev[0][2]
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    print(f"kernels={len(ev)} span={span/1e6:.1f} ms busy={busy/1e6:.1f} ms ({100*busy/span:.1f}%)")
    big = [g for g in gaps if g[0] > 20_000]
    print(f"gaps>20us: n={len(big)} total={sum(g[0] for g in big)/1e6:.1f} ms; "
          f"all gaps total={sum(g[0] for g in gaps)/1e6:.1f} ms (n={len(gaps)})")
    for g in sorted(gaps, reverse=True)[:15]:
        print(f"  {g[0]/1e3:9.1f} us  after {g[1]!r} before {g[2]!r}")
    c = Counter((g[1][:30], g[2][:30]) for g in big)
    for k, v in c.most_common(8):
        print("  ", v, k)


if __name__ == "__main__":
    main(sys.argv[1])
