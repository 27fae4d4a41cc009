# Round-3 session 2: sparse arg-max v2 + folded counters + int32 embedding (GPU suite, bench,
# kernel profile), then the parser in-flight depth A/B.
set -o pipefail
bash scripts/gpu_r03_sparse.sh && bash scripts/gpu_r03_conc.sh
