# round-2 GPU check: changed test files first (fast feedback), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest ${FIRST:-tests/test_gpu_wmsa.py} -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r2/first.log 2>&1 || { grep -E "ERRS" gpurun_out/r2/first.log | tail -40; tail -40 gpurun_out/r2/first.log; exit 1; }
grep -E "ERRS" gpurun_out/r2/first.log | tail -40; tail -2 gpurun_out/r2/first.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2/tests.log 2>&1 || { tail -40 gpurun_out/r2/tests.log; exit 1; }
tail -2 gpurun_out/r2/tests.log
