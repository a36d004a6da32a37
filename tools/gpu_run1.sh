set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wmsa.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/wmsa.log 2>&1 || { tail -40 gpurun_out/r1/wmsa.log; exit 1; }
tail -2 gpurun_out/r1/wmsa.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1/tests.log 2>&1 || { tail -40 gpurun_out/r1/tests.log; exit 1; }
tail -2 gpurun_out/r1/tests.log
AB_LIBS="base new" bash tools/gpu_ab_lib.sh
