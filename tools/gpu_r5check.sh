# Round-5 checkpoint: all -m gpu tests, smoke, the default bench (with its per-shape GEMM
# binding-roof table), the dp2 rehearsal (two gloo ranks sharing GPU 0: the multi-rank flow of
# bench.py end to end), rocprof kernel stats.  Each GPU step under its own limit; stops at the
# first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${CK_OUT:-r5check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'], d['mfma']['binding'])"
if [ -z "$NO_DP2" ]; then
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --cpu-baseline 0 > $O/dp2.json 2> $O/dp2.err || { tail -30 $O/dp2.err; exit 1; }
cat $O/dp2.json | head -c 1500; echo
fi
if [ -z "$NO_PROF" ]; then
  PROF_OUT=${CK_OUT:-r5check}/prof bash tools/gpu_prof.sh > /dev/null || exit 1
  head -25 $O/prof/summary.txt
fi
