# Round 4: the ping-pong 256 x 256 / 128 x 384 GEMM with the LDS-staged epilogue (option gemm_pp
# 1 = wherever a ping-pong tile divides N) against the 128-row tiles, per stage 1-3 shape x2;
# parity test of the pp kernels first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4y
HVK_LIB_PATH=$PWD/abl/ppstg.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear.py -k "pingpong" > gpurun_out/r4y/tests.txt 2>&1 || { tail -30 gpurun_out/r4y/tests.txt; exit 1; }
tail -1 gpurun_out/r4y/tests.txt
for rep in 1 2; do
  for pp in 0 1; do
    timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --only "s[123]" --lib abl/ppstg.so --option gemm_pp=$pp > gpurun_out/r4y/pp${pp}_$rep.txt 2>&1 || { tail gpurun_out/r4y/pp${pp}_$rep.txt; exit 1; }
    echo "== gemm_pp=$pp rep $rep"; grep -E "^s[123]" gpurun_out/r4y/pp${pp}_$rep.txt
  done
done
