# ring (slab) W-MSA backward: parity tests, then A/B timing against the pair kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rb
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wmsa.py > gpurun_out/rb/tests.log 2>&1; rc=$?
tail -15 gpurun_out/rb/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  HVK_WMSA_BWD_RING=$v timeout -k 10 120 python tools/bench_wmsa.py --only bwd --iters 20 > gpurun_out/rb/b$v.txt 2>&1 || { cat gpurun_out/rb/b$v.txt; exit 1; }
  echo "RING=$v"; grep -v amdgpu.ids gpurun_out/rb/b$v.txt
done
[ -f abl/stamps.so ] && HVK_LIB_PATH=$PWD/abl/stamps.so timeout -k 10 120 python tools/bwd_stamps.py --stage 2 --ring
