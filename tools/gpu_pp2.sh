# ping-pong GEMM: its GEMM tests, the per-shape A/B against the 128-row tile kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/pp2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_pp.py --model ${PP_MODEL:-t} > $O/pp.txt 2>&1 || { tail -20 $O/pp.txt; exit 1; }
grep -v amdgpu.ids $O/pp.txt
