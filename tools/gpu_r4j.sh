# Round 4: slab chunk swizzle of the w <= 8 forward (abl/swz.so vs abl/noswz.so: parity tests
# on the swizzled build, W-MSA microbench, end-to-end A/B, LDS counters), and the pipelined head
# GEMMs against hipBLASLt.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wmsa.py tests/test_gpu_qknorm.py tests/test_gpu_head.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/bench_head.py > $O/head.txt 2>&1 || { tail $O/head.txt; exit 1; }
cat $O/head.txt
for r in 1 2; do
  for v in noswz swz; do
    timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --normed --only fwd --lib abl/$v.so > $O/wmsa_$v.txt 2>&1 || exit 1
    echo "== $v"; grep -v amdgpu $O/wmsa_$v.txt
  done
done
AB_LIBS="noswz swz" bash tools/gpu_ab_lib.sh
export WMSA_ARGS=--normed
STAGE=0 bash tools/pmc_wmsa.sh fwd fwd_s0_swz lds || exit 1
python3 tools/pmc_report.py gpurun_out/pmc_fwd_s0_swz/lds "wmsa" > gpurun_out/pmc_fwd_s0_swz/lds.txt 2>&1 && cat gpurun_out/pmc_fwd_s0_swz/lds.txt
