set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wmsa.py -k "12 or 16 or 24" > gpurun_out/large_tests.log 2>&1; rc=$?
tail -5 gpurun_out/large_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_wmsa.py --b384 --iters 5 > gpurun_out/large_bench.txt 2>&1 || { cat gpurun_out/large_bench.txt; exit 1; }
cat gpurun_out/large_bench.txt
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_steps.py tests/test_gpu_model.py -k "steps or reference_api" > gpurun_out/t2.log 2>&1; rc=$?
grep -E "PASS|FAIL|loss|Error|assert" gpurun_out/t2.log | head -40; exit $rc
