# Large-window backward change check: the W-MSA and whole-step GPU tests (TESTS), then the config-5
# per-stage W-MSA timings of the tree's libhvk.so and of each abl/<name>.so in LIBS (interleaved,
# REPS rounds).  Each GPU step under its own limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${AB_OUT:-large_ab}
mkdir -p $O
if [ -n "${TESTS:-tests/test_gpu_wmsa.py tests/test_gpu_steps.py}" ]; then
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${TESTS:-tests/test_gpu_wmsa.py tests/test_gpu_steps.py} -m gpu -x -q -rs -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
cp -r gpurun_out/parity $O/ 2>/dev/null
fi
for r in $(seq 1 ${REPS:-1}); do
  echo "== tree (rep $r)"
  timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 ${STAGE_ARGS:-} > $O/tree_$r.txt 2>&1 || { cat $O/tree_$r.txt; exit 1; }
  cat $O/tree_$r.txt
  for v in ${LIBS:-}; do
    echo "== $v (rep $r)"
    timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 ${STAGE_ARGS:-} --lib abl/$v.so > $O/${v}_$r.txt 2>&1 || { cat $O/${v}_$r.txt; exit 1; }
    cat $O/${v}_$r.txt
  done
done
