set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_gemm.py ${GEMM_ARGS:-} || exit 1
