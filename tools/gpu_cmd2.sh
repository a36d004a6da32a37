# large-window W-MSA: stage timings + PMC passes (stage 2 of SwinV2-B 384) for the fwd / bwd
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lp2
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_steps.py > $O/steps.log 2>&1; rc=$?
grep -E "PASS|FAIL|loss|Error|assert" $O/steps.log | head -20; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp || exit 1
pass() {  # name cmd counters...
  local name=$1 cmd=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$name -o run --output-format csv -- $cmd > $O/$name.log 2>&1
}
for d in fwd bwd; do
  cmd="python3 $R/tools/bench_wmsa.py --b384 --iters 2 --stage ${STAGE:-2} --only $d"
  pass sq_$d "$cmd" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
  pass lds_$d "$cmd" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  pass tr_$d "$cmd" SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAVES SQ_INST_CYCLES_VMEM_RD GRBM_COUNT || exit 1
done
cd $R && python3 tools/pmc_report.py $O wmsa > $O/pmc_report.txt 2>&1; cat $O/pmc_report.txt
