"""Average counters per kernel (template instantiation) from a rocprofv3 counter_collection.csv."""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "gemm_fused" in n:
            m = re.search(r"gemm_fused_kernel<([^>]*)>", n)
            n = "fused<" + (m.group(1) if m else "?") + ">"
        elif "Cijk" in n:
            n = "blas:" + n.split("_MT")[1].split("_")[0] if "_MT" in n else "blas"
        else:
            continue
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
