# Round 4: W-MSA counters after the q / k normalisation moved into the qkv GEMM epilogue (the
# model's path: tools/bench_wmsa.py --normed): forward stages 0 and 3, backward stage 0 (sq and lds
# passes, separate rocprofv3 runs), plus the per-stage microbench table of both forms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export WMSA_ARGS=--normed
STAGE=0 bash tools/pmc_wmsa.sh fwd fwd_s0 sq,lds || exit 1
STAGE=3 bash tools/pmc_wmsa.sh fwd fwd_s3 sq,lds || exit 1
STAGE=0 bash tools/pmc_wmsa.sh bwd bwd_s0 sq,lds || exit 1
for t in fwd_s0 fwd_s3 bwd_s0; do
  for p in sq lds; do
    python3 tools/pmc_report.py gpurun_out/pmc_$t/$p "wmsa" > gpurun_out/pmc_$t/$p.txt 2>&1 && cat gpurun_out/pmc_$t/$p.txt
  done
done
timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 > gpurun_out/wmsa_raw.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --normed > gpurun_out/wmsa_normed.txt 2>&1 || exit 1
cat gpurun_out/wmsa_raw.txt gpurun_out/wmsa_normed.txt
# timing probe: the w <= 8 backward without its CPB-gradient atomics (abl/probe_noatomic.so)
timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --normed --only bwd --lib abl/probe_noatomic.so > gpurun_out/wmsa_noatomic.txt 2>&1 || exit 1
cat gpurun_out/wmsa_noatomic.txt
# the CPB-gradient bins folded per workgroup (HVK_BWD_BIN 1, abl/binnew.so) vs NT^2*256 atomics (binold)
for r in 1 2; do
  for v in binold binnew; do
    timeout -k 10 300 python3 tools/bench_wmsa.py --iters 20 --normed --only bwd --lib abl/$v.so > gpurun_out/wmsa_$v.txt 2>&1 || exit 1
    echo "== $v"; cat gpurun_out/wmsa_$v.txt
  done
done
