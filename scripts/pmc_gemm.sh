set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
python -m smsgate_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/pmc -o p1 -- python $R/scripts/gemm_pmc.py > $R/gpurun_out/pmc/p1.log 2>&1; echo "p1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc -o p2 -- python $R/scripts/gemm_pmc.py > $R/gpurun_out/pmc/p2.log 2>&1; echo "p2 rc=$?"
ls -R $R/gpurun_out/pmc | head -30
