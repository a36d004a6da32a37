# W-MSA forward head-group A/B (HVK_WMSA_FWD_HG), interleaved, after the W-MSA tests with HG=6
set -o pipefail
cd $GRAFT_REPO_ROOT
HVK_WMSA_FWD_HG=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py > gpurun_out/hg_tests.log 2>&1; rc=$?
tail -2 gpurun_out/hg_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for hg in 0 6; do
  echo "== HG $hg"
  HVK_WMSA_FWD_HG=$hg timeout -k 10 300 python tools/bench_wmsa.py --only fwd --kl 0 || exit 1
done; done
