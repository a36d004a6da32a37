# Full GPU check: all -m gpu tests, the default bench line, and a rocprofv3 kernel-stats run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/tests.log 2>&1 || { tail -40 gpurun_out/full/tests.log; exit 1; }
tail -2 gpurun_out/full/tests.log
timeout -k 10 400 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { tail -20 gpurun_out/full/bench.err; exit 1; }
cat gpurun_out/full/bench.json
bash tools/gpu_prof.sh > /dev/null || exit 1
head -50 gpurun_out/prof/summary.txt
