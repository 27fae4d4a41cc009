"""Average counters per kernel (template instantiation) from rocprofv3 counter_collection.csv files.

Default: the fused GEMMs and hipBLASLt kernels.  ``--match SUBSTR``: every
kernel whose name contains SUBSTR (e.g. ``attn``; "" = all); ``--by-grid``: one line
per (kernel, grid size), so one instantiation at two shapes stays apart."""
import collections
import csv
import re
import sys

args = sys.argv[1:]
match = None
by_grid = "--by-grid" in args
args = [a for a in args if a != "--by-grid"]
if args and args[0] == "--match":
    match, args = args[1], args[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in args:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if match is not None:
            if match not in n:
                continue
            n = n.replace("(anonymous namespace)::", "").split("(")[0]
        elif "gemm_fused" in n:
            m = re.search(r"gemm_fused_kernel<([^>]*)>", n)
            n = "fused<" + (m.group(1) if m else "?") + ">"
        elif "Cijk" in n:
            n = "blas:" + n.split("_MT")[1].split("_")[0] if "_MT" in n else "blas"
        else:
            continue
        if by_grid:
            n = f"{n} grid={r['Grid_Size']}"
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
