"""Average counters per kernel family from a rocprofv3 counter_collection.csv."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    n = "fused" if "gemm_fused" in n else ("blas" if "Cijk" in n else None)
    if n:
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
