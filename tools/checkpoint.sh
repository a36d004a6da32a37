# Full GPU checkpoint: tests, smoke, default bench line, graph-mode bench line, rocprof kernel
# stats of the bench.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ckpt
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 600 python bench.py --graph 1 --cpu-baseline 0 > $O/bench_graph.json 2> $O/bench_graph.err || exit 1
cd /tmp && export TMPDIR=/tmp || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --no-roofline > $O/$c.log 2>&1 || exit 1
done
python3 $R/tools/traffic.py $O/FETCH_SIZE $O/WRITE_SIZE $O/bench_traffic.json
