# Round 4: PMC passes for the config-5 large-window W-MSA backward (wmsa_bwd_large_kernel<24>,
# SwinV2-B 384 w24 stage 0 shape) -- what binds it at 0.1 of every roof: instruction mix,
# waits, LDS bank conflicts -- plus the forward for comparison.  Separate rocprofv3 runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_cmd.sh b384bwd "tools/bench_wmsa.py --b384 --only bwd --iters 3 --stage 0" sq,lds,lds2 || exit 1
bash tools/pmc_cmd.sh b384fwd "tools/bench_wmsa.py --b384 --only fwd --iters 3 --stage 0" sq,lds || exit 1
for t in b384bwd b384fwd; do
  for p in sq lds lds2; do
    d=gpurun_out/pmc_$t/$p
    [ -d $d ] && python3 tools/pmc_report.py $d "wmsa" > gpurun_out/pmc_$t/$p.txt 2>&1 && cat gpurun_out/pmc_$t/$p.txt
  done
done
# the stage-2 qkv shapes of the weight-gradient kernel and the tiled forward GEMM
bash tools/pmc_cmd.sh dwqkv "tools/gemm_one.py dw 50176 1152 384" sq,lds,lds2 || exit 1
bash tools/pmc_cmd.sh fwdqkv "tools/gemm_one.py fwd 50176 1152 384" sq,lds,lds2 || exit 1
for t in dwqkv fwdqkv; do
  for p in sq lds lds2; do
    d=gpurun_out/pmc_$t/$p
    [ -d $d ] && python3 tools/pmc_report.py $d "dw_kernel|gemm_nt|gemm_xr" > gpurun_out/pmc_$t/$p.txt 2>&1 && cat gpurun_out/pmc_$t/$p.txt
  done
done
# bucket all-reduce enqueue points against the backward (one-rank RCCL, buckets forced, bs256)
timeout -k 10 300 python3 tools/ddp_trace.py --batch 256 > gpurun_out/r4d_ddp_enqueue.txt 2>&1 || { tail -20 gpurun_out/r4d_ddp_enqueue.txt; exit 1; }
cat gpurun_out/r4d_ddp_enqueue.txt
