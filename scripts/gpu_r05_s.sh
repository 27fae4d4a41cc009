#!/bin/bash
# Round 5: engine batching policy in the full bench -- the second in-flight batch once
# 32 k / 64 k (default) / 128 k rows wait; interleaved, trained weights reused from the
# first run's cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05s
mkdir -p $O
for mt in 65536 131072 32768 65536 131072 32768; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 12 --warmup 2 --qa-min-tokens $mt > $O/b_$mt.tmp 2>> $O/bench.err \
    || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
  python - "$mt" <<'PY' >> $O/ab.jsonl
import json, sys
d = json.loads(open(f"gpurun_out/r05s/b_{sys.argv[1]}.tmp").read().strip().splitlines()[-1])
print(json.dumps({"qa_min_tokens": int(sys.argv[1]), "value": d["value"], "http": (d.get("http_ingest") or {}).get("value"),
                  "cpu_us": (d.get("cpu") or {}).get("cpu_us_per_msg")}))
PY
  tail -1 $O/ab.jsonl
done
