# Round 4: whole-line row-pair stores in the stage-0 fused MLP kernels too (lpair2) vs the skinny
# kernels only (lpair) vs neither (lpbase): linear tests on lpair2, MLP microbench, end-to-end A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4t
HVK_LIB_PATH=$PWD/abl/lpair2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py tests/test_gpu_steps.py > gpurun_out/r4t/tests.txt 2>&1 || { tail -30 gpurun_out/r4t/tests.txt; exit 1; }
tail -1 gpurun_out/r4t/tests.txt
for v in lpbase lpair2 lpbase lpair2; do
  echo "== $v"; timeout -k 10 300 python3 tools/bench_mlp_fused.py --lib abl/$v.so 2>&1 | grep mlp_ || exit 1
done
AB_LIBS="lpbase lpair lpair2" timeout -k 10 1000 bash tools/gpu_ab_lib.sh
