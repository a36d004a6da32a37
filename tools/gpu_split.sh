set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py -k "12 or 16 or 24" > gpurun_out/split_tests.log 2>&1; rc=$?
tail -2 gpurun_out/split_tests.log; [ $rc -eq 0 ] || { grep -B3 Error gpurun_out/split_tests.log | head -20; exit $rc; }
for sp in 0 1; do
  echo "== split $sp"
  HVK_LARGE_SPLIT=$sp timeout -k 10 300 python tools/bench_wmsa.py --b384 --kl 1 --iters 3 --only bwd || exit 1
done
