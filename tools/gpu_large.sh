# large-window W-MSA: GPU tests of the large kernels, then the SwinV2-B 384 stage microbench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py -k "${LARGE_K:-12 or 16 or 24}" > gpurun_out/large_tests.log 2>&1; rc=$?
tail -4 gpurun_out/large_tests.log
[ $rc -eq 0 ] || exit $rc
fi
for v in ${KLV:-}; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 3 ${BW_ARGS:-} || exit 1
done
