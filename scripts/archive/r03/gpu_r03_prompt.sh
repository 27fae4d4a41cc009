# Round-3 session 2: two-token task tag as the shared prefix (P0 = 4: merged key stream in the
# st attention kernels).  Retrain the bundled small extractor for the new prefix and use it in
# place, GPU suite + smoke with it, bench A/B (default vs --no-native-prefill vs --no-attn-merge),
# kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 420 python -u scripts/quality_probe.py --model small --run '{"steps": 12000, "batch": 64, "lr": 0.002, "n_examples": 400000}' --save gpurun_out/extractor-small.safetensors --out gpurun_out/r03_quality_small_tag.jsonl > gpurun_out/r03_quality_small_tag.log 2>&1 || { tail -5 gpurun_out/r03_quality_small_tag.log; exit 1; }
cut -c1-400 gpurun_out/r03_quality_small_tag.jsonl
cp gpurun_out/extractor-small.safetensors smsgate_amd/models/assets/extractor-small.safetensors
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 700 python -u bench.py --verbose "$@" > gpurun_out/ab5_$n.json 2> gpurun_out/ab5_$n.err || { tail -5 gpurun_out/ab5_$n.err; exit 1; }
  cut -c1-160 gpurun_out/ab5_$n.json
}
run m1
run np --no-native-prefill
run nm --no-attn-merge
run m2
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_tag -o run -- python $R/bench.py --steps 10 --warmup 2 --eval-n 0 > $R/gpurun_out/prof_tag.log 2>&1) || { tail -5 gpurun_out/prof_tag.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_tag
find gpurun_out/prof_tag -name "*kernel_trace.csv" -delete
python scripts/stats_top.py gpurun_out/prof_tag/run_kernel_stats.csv > gpurun_out/prof_tag/top.txt
head -16 gpurun_out/prof_tag/top.txt
