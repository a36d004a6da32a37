# large-window backward phase-2 probes (abl/base|nobins|nolse.so): config-5 stage shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/largeprobe
for v in base nobins nolse; do
  echo "== $v"
  HVK_LIB_PATH=$PWD/abl/$v.so timeout -k 10 200 python tools/bench_wmsa.py --b384 --only bwd --iters 5 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/largeprobe/micro.txt
