# W-MSA forward A/B of library variants (abl/<v>.so), interleaved, + the W-MSA tests on the new lib
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py > gpurun_out/fwdab_tests.log 2>&1; rc=$?
tail -2 gpurun_out/fwdab_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in ${KLV:-base new}; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 300 python tools/bench_wmsa.py --only fwd || exit 1
done; done
