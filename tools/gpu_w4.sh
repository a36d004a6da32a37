set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w4
for HG in 3 4 2; do
  echo "== HG=$HG"; HVK_WMSA_FWD_HG=$HG timeout -k 10 120 python tools/bench_wmsa.py --only fwd || exit 1
done > gpurun_out/w4/hg.txt 2>&1
cat gpurun_out/w4/hg.txt | grep -v amdgpu.ids
bash tools/pmc_wmsa.sh fwd ring2 sq,lds || exit 1
STAGE=2 bash tools/pmc_wmsa.sh fwd ring2s2 sq || exit 1
