# per-workgroup timelines of the tiled GEMM (HVK_GEMM_PROBE=4 build) for the stage-2 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tl
for s in "50176 384 1152" "50176 384 1536 gelu" "50176 384 1536 gelu_bwd" "50176 1536 384"; do
  n=$(echo $s | tr ' ' _)
  timeout -k 10 120 python tools/gemm_timeline.py $s > gpurun_out/tl/$n.txt 2>&1 || { tail -5 gpurun_out/tl/$n.txt; exit 1; }
  head -6 gpurun_out/tl/$n.txt; grep "restart gap" gpurun_out/tl/$n.txt
done
