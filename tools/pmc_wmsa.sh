# PMC passes for the W-MSA kernels at the SwinV2-T stage-0 shape (separate rocprofv3 runs,
# counters only with the kernel trace, per MI355X_MICROARCH.md "rocprofv3 PMC slots").
#   bash tools/pmc_wmsa.sh [fwd|bwd] [tag] [passes: sq,fetch,write,lds]
# Environment is inherited by the profiled process.
set -o pipefail
ONLY=${1:-fwd}
TAG=${2:-$ONLY}
PASSES=${3:-sq,fetch,write,lds}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp || exit 1
CMD="python3 $R/tools/bench_wmsa.py --iters 3 --stage ${STAGE:-0} --only $ONLY $WMSA_ARGS"
run() {  # name counters...
  local name=$1; shift
  case ",$PASSES," in *",$name,"*) ;; *) return 0 ;; esac
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o run --output-format csv -- $CMD > $OUT/$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit 1
