# Round checkpoint: all -m gpu tests, smoke, default bench, SwinV2-B benches, rocprof kernel stats,
# W-MSA PMC traffic passes (each GPU step under its own time limit; stops at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${FINAL_OUT:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python bench.py --model swinv2_base_window7_224 --loss multitask --steps 10 --warmup 3 > $O/b224.json 2> $O/b224.err || { tail -20 $O/b224.err; exit 1; }
timeout -k 10 600 python bench.py --model swinv2_base_window24_384 --loss hxe --steps 5 --warmup 2 > $O/b384.json 2> $O/b384.err || { tail -20 $O/b384.err; exit 1; }
python3 -c "
import json
for f in ('b224', 'b384'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'])"
if [ -z "$NO_PROF" ]; then
  bash tools/gpu_prof.sh > /dev/null || exit 1
  head -30 gpurun_out/prof/summary.txt
  bash tools/gpu_traffic.sh > /dev/null || exit 1
  cat gpurun_out/traffic/bench_traffic.json
fi
if [ -z "$NO_PROF" ]; then
  bash tools/gpu_mfma_pmc.sh > /dev/null || exit 1
  cat gpurun_out/mfma_pmc/mfma_pmc.json | head -c 3000
fi
