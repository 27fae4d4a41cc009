#!/bin/bash
# Round 5: how much the quality moves with the training sample -- the bench's recipe on
# three other seeds (data and init), scored by the host reference decoder (the kernel's
# rules, colon rule included)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05ii
mkdir -p $O
timeout -k 10 1100 python -u scripts/qa_probe.py --formats qa --variants "seed=1;seed=2;seed=3" \
  --out $O/probe.jsonl > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -40 $O/probe.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05ii/probe.jsonl"):
    d = json.loads(l)
    print(d["variant"], {k: d[k]["exact"] for k in ("heldout_formats", "train_formats", "heldout_values") if k in d},
          d["negatives_heldout"]["false_parsed_rate"])
PY
