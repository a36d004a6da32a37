# quick GPU check: the named test files, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q/tests.log 2>&1 || { tail -40 gpurun_out/q/tests.log; exit 1; }
tail -2 gpurun_out/q/tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { tail -20 gpurun_out/q/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/q/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_bwd']['frac'])"
