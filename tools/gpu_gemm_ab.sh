# Tile-GEMM k-loop variant check: the GEMM GPU tests on abl/$NEW.so, then per-shape GEMM timings
# of abl/$BASE.so vs abl/$NEW.so (interleaved), then the bench line A/B (tools/gpu_ab_lib.sh).
#   BASE=base NEW=dmamid bash tools/gpu_gemm_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm_ab
mkdir -p $O
HVK_LIB_PATH=$PWD/abl/$NEW.so timeout -k 10 600 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_bench_routing.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in $BASE $NEW; do
    timeout -k 10 300 python tools/bench_gemm.py --lib abl/$v.so --only "${ONLY:-s2|s3}" > $O/${v}_$r.txt 2>&1 || { cat $O/${v}_$r.txt; exit 1; }
    echo "== $v rep $r"; cat $O/${v}_$r.txt
  done
done
AB_LIBS="$BASE $NEW" bash tools/gpu_ab_lib.sh
