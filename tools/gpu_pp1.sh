set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pp1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_pp.py --model t > $O/pp_t.txt 2>&1 || { tail -20 $O/pp_t.txt; exit 1; }
cat $O/pp_t.txt
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['mfma'])"
