# W-MSA w7 backward: parity tests, A/B timing of the one-wave (HVK_WMSA_BWD_V1=1) and pair
# kernels, then SQ/LDS PMC passes of both at the stage-0 shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bwdab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py > gpurun_out/bwdab/tests.log 2>&1; rc=$?
tail -5 gpurun_out/bwdab/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  HVK_WMSA_BWD_V1=$v timeout -k 10 120 python tools/bench_wmsa.py --only bwd --iters 20 > gpurun_out/bwdab/b$v.txt 2>&1 || { cat gpurun_out/bwdab/b$v.txt; exit 1; }
  echo "V1=$v"; cat gpurun_out/bwdab/b$v.txt
done
if [ -z "$NO_PMC" ]; then
HVK_WMSA_BWD_V1=1 bash tools/pmc_wmsa.sh bwd bwd_v1 sq,lds || exit 1
HVK_WMSA_BWD_V1=0 bash tools/pmc_wmsa.sh bwd bwd_pair sq,lds || exit 1
fi
[ -f abl/stamps.so ] && HVK_LIB_PATH=$PWD/abl/stamps.so timeout -k 10 120 python tools/bwd_stamps.py --stage 0
