# Round 4: pair-backward P / dS image swizzle (4-bit, conflict-free under the §LDS bank model)
# and the LayerNorm forward's residual loaded with the branch output.  Parity tests on the new
# build, microbench A/B (normed W-MSA backward all stages; LayerNorm per stage) against the
# previous build, the stage-0 LDS counters, then the end-to-end A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wmsa.py tests/test_gpu_qknorm.py tests/test_gpu_model.py -k "wmsa or qk or norm or ln or layer" > gpurun_out/r4n/tests.txt 2>&1 || { tail -30 gpurun_out/r4n/tests.txt; exit 1; }
tail -2 gpurun_out/r4n/tests.txt
for v in bwdbase bwdswz bwdbase bwdswz; do
  timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --only bwd --normed --lib abl/$v.so > gpurun_out/r4n/mb_$v.txt 2>&1 || { tail gpurun_out/r4n/mb_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu gpurun_out/r4n/mb_$v.txt
done
for v in bwdswz lnx0 bwdswz lnx0; do
  timeout -k 10 300 python3 tools/bench_ln.py --iters 20 --lib abl/$v.so > gpurun_out/r4n/ln_$v.txt 2>&1 || { tail gpurun_out/r4n/ln_$v.txt; exit 1; }
  echo "== ln $v"; grep -v amdgpu gpurun_out/r4n/ln_$v.txt
done
WMSA_ARGS=--normed timeout -k 10 400 bash tools/pmc_wmsa.sh bwd bwd_swz lds || exit 1
AB_LIBS="bwdbase bwdswz lnx0" timeout -k 10 1000 bash tools/gpu_ab_lib.sh
