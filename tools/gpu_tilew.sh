# fused-GELU tiled GEMM shapes: default tile choice vs forced 128-column tiles (HVK_TILE_WIDE=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tw
for r in 1 2; do
  for w in ${TW_VALUES:--1 0}; do
    HVK_TILE_WIDE=$w timeout -k 10 200 python tools/bench_pp.py --model ${PP_MODEL:-t} --rounds 3 > gpurun_out/tw/w${w}_$r.txt 2>&1 || { tail -5 gpurun_out/tw/w${w}_$r.txt; exit 1; }
    echo "== HVK_TILE_WIDE=$w round $r"; grep -E "fc1 |fc2.dx|fc1\.dx|qkv |sum" gpurun_out/tw/w${w}_$r.txt
  done
done
