set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sk; rm -f gpurun_out/sk/out.txt
for v in 0 1; do HVK_TILE_PIPE=$v timeout -k 10 200 python tools/bench_skinny.py 50176:384:1152 50176:384:384 50176:384:1536 50176:1536:384 50176:1152:384 12544:768:2304 12544:768:768 12544:768:3072 12544:3072:768 12544:1536:768 2>&1 | grep -v amdgpu.ids >> gpurun_out/sk/out.txt || exit 1; done
cat gpurun_out/sk/out.txt
