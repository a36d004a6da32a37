# W-MSA backward check: GPU W-MSA tests, the stage microbench of the key-on-lane backward (and
# of the query-on-lane one with KL0=1), phase stamps with STAMPS=1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py ${KL_TESTS:-} > gpurun_out/kl_tests.log 2>&1; rc=$?
tail -4 gpurun_out/kl_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/bench_wmsa.py --only bwd --kl 1 || exit 1
if [ -n "$KL0" ]; then timeout -k 10 300 python tools/bench_wmsa.py --only bwd --kl 0 || exit 1; fi
if [ -n "$STAMPS" ]; then HVK_LIB_PATH=$PWD/abl/stamp.so timeout -k 10 300 python tools/bench_wmsa.py --only bwd --kl 1 --stamps --iters 5 --stage 0 || exit 1; fi
