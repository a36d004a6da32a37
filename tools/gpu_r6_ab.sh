# Round 6 measurements on one box: host enqueue time per step (tools/host_overhead.py), the qkv
# weight gradient on / off the side stream (interleaved A/B, 3 pairs), and the PMC passes of the
# stage-2 fc2 tile GEMM (gemm_nt<0,192> 50176 x 384 x 1536, tools/gemm_one.py) and its weight
# gradient.  Each GPU step under its own limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ab
mkdir -p $O
timeout -k 10 300 python tools/host_overhead.py > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 1; }
cat $O/host.txt
for rep in 1 2 3; do
  for arm in A B; do
    if [ $arm = A ]; then args="--host-opt wgrad_stream_qkv=0"; else args=""; fi
    timeout -k 10 300 python bench.py --cpu-baseline 0 --no-roofline $args > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    echo "$arm [$args] $(python3 -c "import json; d=json.load(open('$O/b.json')); print(d['value'], d['ms_per_step'], d['library_fallbacks'])")" | tee -a $O/ab_qkv.txt
  done
done
bash tools/pmc_cmd.sh gemm_fc2 "tools/gemm_one.py fwd 50176 384 1536 5" sq,mem,lds,lds2 || exit 1
bash tools/pmc_cmd.sh dw_fc2 "tools/gemm_one.py dw 50176 384 1536 5" sq,lds,lds2 || exit 1
for d in gemm_fc2 dw_fc2; do
  for p in sq mem lds lds2; do
    [ -d gpurun_out/pmc_$d/$p ] && python3 tools/pmc_report.py gpurun_out/pmc_$d/$p "gemm_nt|dw_kernel" > gpurun_out/pmc_$d/$p.txt 2>&1
  done
done
head -50 gpurun_out/pmc_gemm_fc2/*.txt
