#!/bin/bash
# round 6, call I: the speed-of-light table at the qa engine's shapes (VERDICT r05 #7:
# keep PERF.md's SOL table current), the prompt length of the round-6 traffic (52 rows
# per message incl. the 9 queries)
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python -u scripts/sol_table.py --no-spec --decode-m 221184 --prefill-m 110592 --prefill-len 53 \
  --rounds 2 > $O/sol.json 2> $O/sol.err || { echo "sol rc=$?"; tail -20 $O/sol.err; exit 1; }
cat $O/sol.json
