#!/bin/bash
# Round 5: phase length -- the bus phase at 20 and at 60 steps (the fill / drain of the
# pipeline is a fixed cost per phase)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r05hh
mkdir -p $O
for st in 20 60 20 60; do
  timeout -k 10 900 python -u bench.py --gpus 1 --steps $st --warmup 2 --ingest bus --verbose > $O/b_$st.tmp 2>> $O/bench.err \
    || { echo "bench rc=$?"; tail -40 $O/bench.err; exit 1; }
  python - "$st" <<'PY' >> $O/ab.jsonl
import json, sys
d = json.loads(open(f"gpurun_out/r05hh/b_{sys.argv[1]}.tmp").read().strip().splitlines()[-1])
e = d.get("engine", {})
print(json.dumps({"steps": int(sys.argv[1]), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "gpu_idle_s": e.get("gpu_idle_s"), "prefill_batches": e.get("prefill_batches")}))
PY
  tail -1 $O/ab.jsonl
done
