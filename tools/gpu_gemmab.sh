# GEMM A/B: the linear/GEMM GPU tests on abl/$TESTLIB.so, then bench_gemm per variant (KLV)
set -o pipefail
cd $GRAFT_REPO_ROOT
if [ -n "$TESTLIB" ]; then
  HVK_LIB_PATH=$PWD/abl/$TESTLIB.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_swinb.py > gpurun_out/gemmab_tests.log 2>&1; rc=$?
  tail -2 gpurun_out/gemmab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for v in $KLV; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 300 python tools/bench_gemm.py ${GEMM_ARGS:-} || exit 1
done
