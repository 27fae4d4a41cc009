"""Summarize a rocprofv3 kernel_stats.csv (group GEMMs, print top kernels)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
agg = {}
for r in rows:
    n = r['Name']
    key = 'GEMM(hipBLASLt)' if 'Cijk' in n else n.split('(')[0].replace('void ', '')[:70]
    a = agg.setdefault(key, [0, 0.0])
    a[0] += int(r['Calls']); a[1] += float(r['TotalDurationNs'])
print(f"total kernel time {tot/1e6:.1f} ms")
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:15]:
    print(f"{k:72s} calls={c:>7} total_ms={t/1e6:9.2f} avg_us={t/c/1e3:8.2f} pct={100*t/tot:5.1f}")
