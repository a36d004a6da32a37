# skinny-GEMM branch-free accesses: GEMM / MLP / model parity tests, then interleaved end-to-end A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sk
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_linear.py tests/test_gpu_model.py tests/test_gpu_steps.py > gpurun_out/sk/tests.log 2>&1; rc=$?
tail -4 gpurun_out/sk/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_gemm.py --iters 10 --only "s0|s1" > gpurun_out/sk/gemm_new.txt 2>&1 || exit 1
HVK_LIB_PATH=$PWD/abl/base.so timeout -k 10 200 python tools/bench_gemm.py --iters 10 --only "s0|s1" > gpurun_out/sk/gemm_base.txt 2>&1 || exit 1
paste <(cut -c1-70 gpurun_out/sk/gemm_base.txt) <(cut -c60-100 gpurun_out/sk/gemm_new.txt) | head -14
AB_LIBS="base skinny" BENCH_ARGS="--no-roofline" bash tools/gpu_ab_lib.sh
