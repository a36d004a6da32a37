# one PMC pass (MFMA busy cycles, busy-CU cycles, GRBM active) over a short default bench run
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mfma_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/p -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --no-roofline > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
cd $R && python3 tools/mfma_pmc.py $O/p $O/mfma_pmc.json
