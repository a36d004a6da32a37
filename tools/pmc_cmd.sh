# PMC passes (separate rocprofv3 runs, counters + kernel trace only) over any python command:
#   bash tools/pmc_cmd.sh TAG "tools/bench_mlp.py 0" [passes: sq,mem,lds]
set -o pipefail
TAG=$1
ARGS=$2
PASSES=${3:-sq,mem,lds}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp || exit 1
run() {  # name counters...
  local name=$1; shift
  case ",$PASSES," in *",$name,"*) ;; *) return 0 ;; esac
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 $R/$ARGS > $OUT/$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
run mem SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE || exit 1
run lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run lds2 SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE || exit 1
