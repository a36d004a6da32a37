set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wmsa.py -m gpu -q -s --timeout 120 --timeout-method thread -k scale100 > gpurun_out/r1/diag.log 2>&1; grep -E "ERRS|passed|failed" gpurun_out/r1/diag.log
