# Round-3 session 2: 4-wave 128x192 / 256x96 residual tiles and the 4-wave 128x192 QKV+RoPE
# tile (64x96 wave tiles): GEMM GPU tests, then an interleaved tile sweep at the engine's rows
# (decode halves 4 608 / 9 216, prefill halves ~15 104 / 16 384).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -1 gpurun_out/pytest_gemm.log
timeout -k 10 500 python -u scripts/gemm_tune.py --rows 4608,9216,15104 --only down,o,qkv_rope --cfgs 1,3,21,22,23,26,28,29 --rounds 4 > gpurun_out/r03_tiles_tune.json 2> gpurun_out/r03_tiles_tune.err || { tail -5 gpurun_out/r03_tiles_tune.err; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/r03_tiles_tune.json'))
for k,v in d.items(): print(k, 'auto', v.get('auto'), v.get('auto_us'), 'best', v.get('best'), sorted(v['us'].items(), key=lambda x: x[1])[:5])
"
