set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w2
timeout -k 10 300 python -u -m pytest tests/test_gpu_wmsa.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w2/tests.log 2>&1 || { tail -30 gpurun_out/w2/tests.log; exit 1; }
tail -3 gpurun_out/w2/tests.log
timeout -k 10 120 python tools/bench_wmsa.py --only fwd > gpurun_out/w2/bench_v2.txt 2>&1 || exit 1
HVK_WMSA_FWD_V1=1 timeout -k 10 120 python tools/bench_wmsa.py --only fwd > gpurun_out/w2/bench_v1.txt 2>&1 || exit 1
cat gpurun_out/w2/bench_v2.txt gpurun_out/w2/bench_v1.txt
bash tools/pmc_wmsa.sh fwd ring sq,lds || exit 1
HVK_WMSA_FWD_V1=1 bash tools/pmc_wmsa.sh fwd v1 sq,lds || exit 1
