# Round 4: skinny GEMM / fused MLP operand slices loaded in row pairs as whole 128-B lines
# (DPP row swap at the consumer, lpl) against fragment-shaped 16 x 64-B loads (lpair2 = HEAD):
# parity tests on lpl, per-shape microbench (SwinV2-T / -B 224 stages 0-1, stage-0 MLP), e2e A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4v
HVK_LIB_PATH=$PWD/abl/lpl.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py tests/test_gpu_qknorm.py tests/test_gpu_model.py tests/test_gpu_steps.py tests/test_gpu_swinb.py > gpurun_out/r4v/tests.txt 2>&1 || { tail -30 gpurun_out/r4v/tests.txt; exit 1; }
tail -1 gpurun_out/r4v/tests.txt
for v in lpair2 lpl lpair2 lpl; do
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --only "s[01]|embed" --lib abl/$v.so > gpurun_out/r4v/t_$v.txt 2>&1 || { tail gpurun_out/r4v/t_$v.txt; exit 1; }
  timeout -k 10 300 python3 tools/bench_gemm.py --iters 10 --model b224 --only "s[01]|embed" --lib abl/$v.so > gpurun_out/r4v/b_$v.txt 2>&1 || { tail gpurun_out/r4v/b_$v.txt; exit 1; }
  echo "== $v"; timeout -k 10 300 python3 tools/bench_mlp_fused.py --lib abl/$v.so 2>&1 | grep mlp_ || exit 1
done
AB_LIBS="lpair2 lpl" timeout -k 10 900 bash tools/gpu_ab_lib.sh
