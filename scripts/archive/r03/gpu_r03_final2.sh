# Round-3 session 2: final check of the committed tree, then the gate/up kernel A/B.
set -o pipefail
bash scripts/gpu_r03_final.sh && bash scripts/gpu_r03_swiglu.sh
