#!/bin/bash
# Round 5: parser processes per GPU after the per-connection senders -- 10 (default) /
# 12 / 14, interleaved twice; trained weights reused from the first run's cache
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05aa
mkdir -p $O
for w in 10 12 14 10 12 14; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 2 --cpu-workers $w > $O/b_$w.tmp 2>> $O/bench.err \
    || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
  python - "$w" <<'PY' >> $O/ab.jsonl
import json, sys
d = json.loads(open(f"gpurun_out/r05aa/b_{sys.argv[1]}.tmp").read().strip().splitlines()[-1])
print(json.dumps({"cpu_workers": int(sys.argv[1]), "value": d["value"], "http": d["http_ingest"]["value"],
                  "cpu_us": d["cpu"]["cpu_us_per_msg"], "http_cpu_us": d["http_ingest"]["cpu"]["cpu_us_per_msg"]}))
PY
  tail -1 $O/ab.jsonl
done
