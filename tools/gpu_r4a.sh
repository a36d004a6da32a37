# Round-4 first call: the new persistent row-range GEMM's parity test and A/B microbench, the
# LayerNorm access-shape probe and the W-MSA forward memory probe (built here), then the quick
# checkpoint (all -m gpu tests, smoke, bench).  Each GPU step has its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -k "xr" -x -q --timeout 120 --timeout-method thread > gpurun_out/probe/xr_test.log 2>&1 || { tail -30 gpurun_out/probe/xr_test.log; exit 1; }
tail -1 gpurun_out/probe/xr_test.log
timeout -k 10 300 python -u tools/bench_xr.py > gpurun_out/probe/bench_xr.txt 2>&1 || { tail -30 gpurun_out/probe/bench_xr.txt; exit 1; }
cat gpurun_out/probe/bench_xr.txt
timeout -k 10 120 ./tools/probe/ln_probe > gpurun_out/probe/ln_probe.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/probe/wmsa_mem 3 > gpurun_out/probe/wmsa_mem_stage0.txt 2>&1 || exit 1
bash tools/gpu_check.sh || exit 1
