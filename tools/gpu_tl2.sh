# EPI1 / EPI2 tiled-GEMM timelines: full build vs GELU-free build (HVK_PROBE_NOGELU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tl2
for lib in libhvk_gemm4 libhvk_gemm4ng; do
  for s in "50176 384 1536 gelu" "50176 384 1536 gelu_bwd"; do
    n=${lib}_$(echo $s | tr ' ' _)
    HVK_TL_LIB=tools/probe/$lib.so timeout -k 10 120 python tools/gemm_timeline.py $s > gpurun_out/tl2/$n.txt 2>&1 || { tail -5 gpurun_out/tl2/$n.txt; exit 1; }
    echo "== $lib $s"; sed -n 2,6p gpurun_out/tl2/$n.txt
  done
done
