#!/bin/bash
# Round 5 (round-6 guidance): twice the procedural layouts' weight in the training mix,
# on the four training samples of r05_qa_probe6_seeds.jsonl (+ seed 0 of the current
# recipe as the baseline for that sample)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05kk
mkdir -p $O
timeout -k 10 1500 python -u scripts/qa_probe.py --formats qa \
  --variants "seed=0;proc=6,seed=0;proc=6,seed=1;proc=6,seed=2;proc=6,seed=3" \
  --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -40 $O/probe.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05kk/probe.jsonl"):
    d = json.loads(l)
    print(d["variant"], {k: d[k]["exact"] for k in ("heldout_formats", "train_formats", "heldout_values") if k in d},
          d["negatives_heldout"]["false_parsed_rate"])
PY
