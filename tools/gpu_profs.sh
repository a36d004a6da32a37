# checkpoint profiles: rocprof kernel stats, W-MSA traffic passes, MFMA-busy PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh > /dev/null || exit 1
head -30 gpurun_out/prof/summary.txt
bash tools/gpu_traffic.sh > /dev/null || exit 1
cat gpurun_out/traffic/bench_traffic.json
bash tools/gpu_mfma_pmc.sh > /dev/null || exit 1
head -c 1500 gpurun_out/mfma_pmc/mfma_pmc.json
