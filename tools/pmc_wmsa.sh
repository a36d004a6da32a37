# PMC passes for the W-MSA kernels at the SwinV2-T stage-0 shape (separate rocprofv3 runs,
# counters only with the kernel trace, per MI355X_MICROARCH.md "rocprofv3 PMC slots").
#   bash tools/pmc_wmsa.sh [fwd|bwd]
set -o pipefail
ONLY=${1:-fwd}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$ONLY
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp || exit 1
CMD="python3 $R/tools/bench_wmsa.py --iters 3 --stage 0 --only $ONLY"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d $OUT/sq -o run --output-format csv -- $CMD > $OUT/sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- $CMD > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $OUT/lds -o run --output-format csv -- $CMD > $OUT/lds.log 2>&1 || exit 1
