#!/bin/bash
# Round 5: training-mix A/B -- unseen pseudo-word labels and "#1234" masks in the
# procedural families (SMSGATE_SYNTH_LABELS) vs none; qa format, the bench's recipe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 1100 python -u scripts/qa_probe.py --formats qa --variants "labels=0;labels=0.2" \
  --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -40 $O/probe.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05r/probe.jsonl"):
    d = json.loads(l)
    print(d["variant"], {k: d[k]["exact"] for k in ("heldout_formats", "train_formats", "heldout_values") if k in d},
          d.get("negatives_heldout", d.get("quality_negatives")))
PY
