# Checkpoint: all -m gpu tests, smoke, the default bench (with its per-shape GEMM binding-roof
# table and library_fallbacks), the dp2 rehearsal (two gloo ranks sharing GPU 0: the multi-rank
# flow of bench.py end to end, with its `comm` block), rocprof stats.  Each GPU step under its own
# limit; stops at the first failure.  TESTS narrows the test selection (default: all of tests/).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-check}
mkdir -p $O
timeout -k 10 ${TEST_LIMIT:-800} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp -r gpurun_out/parity $O/ 2>/dev/null
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'], d['mfma']['binding'], d['library_fallbacks'])"
if [ -z "$NO_DP2" ]; then
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --cpu-baseline 0 > $O/dp2.json 2> $O/dp2.err || { tail -30 $O/dp2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/dp2.json').read().strip().splitlines()[-1]); print(d['value'], d['comm'])"
fi
if [ -z "$NO_PROF" ]; then
  PROF_OUT=${CK_OUT:-check}/prof bash tools/gpu_prof.sh > /dev/null || exit 1
  head -25 $O/prof/summary.txt
fi
