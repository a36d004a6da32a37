# Large-window W-MSA (SwinV2-B 384 w24, BASELINE config 5): per-stage timings, component
# probe builds (abl/lprobe*.so: no CPB-gradient bins / no phase 2 / no loop B), and PMC passes
# (SQ issue / wait mix, LDS) for the stage-2 forward and backward.  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/large_prof
mkdir -p $O
cd $R
timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 > $O/base.txt 2>&1 || { cat $O/base.txt; exit 1; }
cat $O/base.txt
for v in ${PROBES:-}; do  # probe builds (abl/lprobe*.so) when PROBES names them
  echo "== $v" | tee $O/$v.txt
  HVK_LIB_PATH=$R/abl/$v.so timeout -k 10 200 python tools/bench_wmsa.py --b384 --iters 5 --stage 2 --only bwd >> $O/$v.txt 2>&1 || { cat $O/$v.txt; exit 1; }
  cat $O/$v.txt
done
cd /tmp && export TMPDIR=/tmp || exit 1
CMD_F="python3 $R/tools/bench_wmsa.py --b384 --iters 2 --stage 2 --only fwd"
CMD_B="python3 $R/tools/bench_wmsa.py --b384 --iters 2 --stage 2 --only bwd"
pass() {  # name cmd counters...
  local name=$1 cmd=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$name -o run --output-format csv -- $cmd > $O/$name.log 2>&1
}
for d in F B; do
  eval cmd=\$CMD_$d
  pass sq_$d "$cmd" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
  pass lds_$d "$cmd" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
done
for d in F B; do  # last: a counter this ROCm may not know only fails its own pass
  eval cmd=\$CMD_$d
  pass trans_$d "$cmd" SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAVES
done
cd $R && python3 tools/pmc_report.py $O > $O/pmc_report.txt 2>&1; cat $O/pmc_report.txt
