# Round 4: persistent row-range GEMM v2 (3-stage ring, one barrier per step): its parity tests,
# then the interleaved A/B microbench against the tile kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -k "xr" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c/xr_test.log 2>&1 || { tail -30 gpurun_out/r4c/xr_test.log; exit 1; }
tail -1 gpurun_out/r4c/xr_test.log
timeout -k 10 300 python -u tools/bench_xr.py > gpurun_out/r4c/bench_xr.txt 2>&1 || { tail -30 gpurun_out/r4c/bench_xr.txt; exit 1; }
cat gpurun_out/r4c/bench_xr.txt
