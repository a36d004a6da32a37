# Round 4: weight-gradient partial-slab stores as 8 rows x 128 B (row-pair DPP swap, dwp) against
# 16 rows x 64 B (lpair2 = HEAD): weight-gradient tests on dwp, per-shape dW microbench, e2e A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4u
HVK_LIB_PATH=$PWD/abl/dwp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weight_grad.py tests/test_gpu_linear.py tests/test_gpu_model.py > gpurun_out/r4u/tests.txt 2>&1 || { tail -30 gpurun_out/r4u/tests.txt; exit 1; }
tail -1 gpurun_out/r4u/tests.txt
for v in lpair2 dwp lpair2 dwp; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --lib abl/$v.so > gpurun_out/r4u/gemm_$v.txt 2>&1 || { tail gpurun_out/r4u/gemm_$v.txt; exit 1; }
  echo "== $v"; grep -E "^total" gpurun_out/r4u/gemm_$v.txt
done
AB_LIBS="lpair2 dwp" timeout -k 10 900 bash tools/gpu_ab_lib.sh
