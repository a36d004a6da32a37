# Round 4: weight-gradient partial slabs laid out fragment-major (1-KB contiguous stores, the
# reduce decodes (n, k)) against the row-major slabs: parity tests on the new build, per-shape
# microbench (bench_gemm's dw column), end-to-end A/B on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4r
HVK_LIB_PATH=$PWD/abl/dwfrag.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weight_grad.py tests/test_gpu_linear.py tests/test_gpu_model.py tests/test_gpu_steps.py > gpurun_out/r4r/tests.txt 2>&1 || { tail -30 gpurun_out/r4r/tests.txt; exit 1; }
tail -1 gpurun_out/r4r/tests.txt
for v in dwbase dwfrag dwbase dwfrag; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --lib abl/$v.so > gpurun_out/r4r/gemm_$v.txt 2>&1 || { tail gpurun_out/r4r/gemm_$v.txt; exit 1; }
  echo "== $v"; grep -E "^(s[0-3]|total)" gpurun_out/r4r/gemm_$v.txt
done
AB_LIBS="dwbase dwfrag" timeout -k 10 900 bash tools/gpu_ab_lib.sh
