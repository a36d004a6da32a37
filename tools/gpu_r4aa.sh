# Round 4: weight-gradient slab reduce with 32 chunk phases per workgroup for the deep (>= 128
# chunk) slab stacks (red32) against 8 (redbase = HEAD): tests, dW microbench, e2e A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4aa
HVK_LIB_PATH=$PWD/abl/red32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weight_grad.py tests/test_gpu_linear.py > gpurun_out/r4aa/tests.txt 2>&1 || { tail -30 gpurun_out/r4aa/tests.txt; exit 1; }
tail -1 gpurun_out/r4aa/tests.txt
for v in redbase red32 redbase red32; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --only "s[01]|embed" --lib abl/$v.so > gpurun_out/r4aa/gemm_$v.txt 2>&1 || { tail gpurun_out/r4aa/gemm_$v.txt; exit 1; }
  echo "== $v"; grep -E "^(s[01]|embed)" gpurun_out/r4aa/gemm_$v.txt | awk '{print $1, $9}'
done
AB_LIBS="redbase red32" timeout -k 10 900 bash tools/gpu_ab_lib.sh
