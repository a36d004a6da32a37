# Round 4: tiled GEMM outputs staged through LDS and stored as whole row runs (gstg) against the
# fragment stores (gbase): GEMM parity tests on the staged build, per-shape microbench, end to end.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4o
HVK_LIB_PATH=$PWD/abl/gstg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py tests/test_gpu_qknorm.py tests/test_gpu_steps.py > gpurun_out/r4o/tests.txt 2>&1 || { tail -30 gpurun_out/r4o/tests.txt; exit 1; }
tail -2 gpurun_out/r4o/tests.txt
for v in gbase gstg gbase gstg; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --lib abl/$v.so > gpurun_out/r4o/gemm_$v.txt 2>&1 || { tail gpurun_out/r4o/gemm_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu gpurun_out/r4o/gemm_$v.txt | tail -40
done
AB_LIBS="gbase gstg" timeout -k 10 900 bash tools/gpu_ab_lib.sh
