# PMC passes over the tiled GEMM (stage-2 qkv shape) and the weight-gradient kernel (s2.qkv)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_cmd.sh tile "tools/bench_skinny.py 50176:384:1152" sq,lds || exit 1
bash tools/pmc_cmd.sh dw "tools/bench_dw.py s2.qkv" sq,lds || exit 1
