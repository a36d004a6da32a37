# Full GPU checkpoint: tests, smoke, default bench line, rocprof kernel stats of the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ckpt
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/ckpt/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ckpt/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/ckpt/bench.json 2> gpurun_out/ckpt/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ckpt/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $R/gpurun_out/ckpt/bench_prof.json 2> $R/gpurun_out/ckpt/bench_prof.err || exit 1
