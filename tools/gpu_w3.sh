set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w3
timeout -k 10 300 python -u -m pytest tests/test_gpu_wmsa.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w3/tests.log 2>&1 || { tail -30 gpurun_out/w3/tests.log; exit 1; }
tail -2 gpurun_out/w3/tests.log
for L in hierarchical-vision_amd/libhvk.so tools/probe/libhvk_ringmem.so tools/probe/libhvk_ringmath.so; do
  echo "== $L"; timeout -k 10 120 python tools/bench_wmsa.py --only fwd --lib $L || exit 1
done > gpurun_out/w3/ab.txt 2>&1
cat gpurun_out/w3/ab.txt
