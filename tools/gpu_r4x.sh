# Round 4: tiled fc1 + GELU (EPI 1) and fc2-input-gradient-through-GELU' (EPI 2) kernels with the
# LDS-staged epilogue: 128- vs 192-column tiles per stage (option tile_wide), interleaved x2.
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for w in -1 0 1; do
    echo "== tile_wide=$w"; timeout -k 10 300 python3 tools/bench_mlp_tile.py tile_wide=$w 2>&1 | grep "M=" || exit 1
  done
done
