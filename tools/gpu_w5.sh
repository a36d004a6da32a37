set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w5
timeout -k 10 300 python -u -m pytest tests/test_gpu_wmsa.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w5/tests.log 2>&1; rc=$?
grep -E "FAIL|Error|assert|passed|failed" gpurun_out/w5/tests.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/bench_wmsa.py --only bwd > gpurun_out/w5/bench_v2.txt 2>&1 || exit 1
true
cat gpurun_out/w5/bench_v2.txt | grep -v amdgpu
