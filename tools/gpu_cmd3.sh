# large-window W-MSA: kernel tests, SwinV2-B 384 stage timings, PMC passes at stage 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lp3
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wmsa.py -k "12 or 16 or 24" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 > $O/bench.txt 2>&1 || { cat $O/bench.txt; exit 1; }
cat $O/bench.txt
cd /tmp && export TMPDIR=/tmp || exit 1
pass() {  # name cmd counters...
  local name=$1 cmd=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$name -o run --output-format csv -- $cmd > $O/$name.log 2>&1
}
for d in fwd bwd; do
  cmd="python3 $R/tools/bench_wmsa.py --b384 --iters 2 --stage ${STAGE:-2} --only $d"
  pass sq_$d "$cmd" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
  pass lds_$d "$cmd" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE || exit 1
done
cd $R && python3 tools/pmc_report.py $O wmsa > $O/pmc_report.txt 2>&1; cat $O/pmc_report.txt
