set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sk
for v in 0 1 3; do
  HVK_LINEAR_VARIANT=$v timeout -k 10 120 python tools/bench_skinny.py 50176:384:1152 50176:384:384 50176:384:1536 || exit 1
done 2>&1 | grep -v amdgpu.ids > gpurun_out/sk/out.txt
cat gpurun_out/sk/out.txt
