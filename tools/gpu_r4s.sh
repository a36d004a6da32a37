# Round 4: skinny GEMM output slices stored in row pairs as whole 128-B lines (DPP row swap,
# lpair) against the plain 16 x 64-B fragment stores (lpbase): parity tests on the new build,
# per-shape microbench (SwinV2-T and SwinV2-B 224 shapes), end-to-end A/B on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4s
HVK_LIB_PATH=$PWD/abl/lpair.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py tests/test_gpu_qknorm.py tests/test_gpu_model.py tests/test_gpu_steps.py tests/test_gpu_swinb.py > gpurun_out/r4s/tests.txt 2>&1 || { tail -30 gpurun_out/r4s/tests.txt; exit 1; }
tail -1 gpurun_out/r4s/tests.txt
for v in lpbase lpair lpbase lpair; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --only "s[01]|embed" --lib abl/$v.so > gpurun_out/r4s/t_$v.txt 2>&1 || { tail gpurun_out/r4s/t_$v.txt; exit 1; }
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 10 --model b224 --only "s[01]|embed" --lib abl/$v.so > gpurun_out/r4s/b_$v.txt 2>&1 || { tail gpurun_out/r4s/b_$v.txt; exit 1; }
  echo "== $v"; grep -E "^(s[01]|embed)" gpurun_out/r4s/t_$v.txt; grep -E "^(s[01]|embed)" gpurun_out/r4s/b_$v.txt
done
AB_LIBS="lpbase lpair" timeout -k 10 900 bash tools/gpu_ab_lib.sh
