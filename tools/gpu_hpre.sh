# EPI-2 h prefetch: linear GPU tests, then A/B of library builds on the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hp/tests.log 2>&1 || { tail -30 gpurun_out/hp/tests.log; exit 1; }
tail -1 gpurun_out/hp/tests.log
bash tools/gpu_ab_lib.sh
