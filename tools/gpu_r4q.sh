# Round 4: with the LDS-staged epilogue, 128- vs 192-column tiles per stage 1-3 shape (option
# tile_wide -1 = the shape rule, 0 = 128 where 128 | N, 1 = 192 where 192 | N), interleaved x2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4q
for rep in 1 2; do
  for w in -1 0 1; do
    timeout -k 10 300 python3 tools/bench_gemm.py --iters 20 --only "s[123]" --option tile_wide=$w > gpurun_out/r4q/w${w}_$rep.txt 2>&1 || { tail gpurun_out/r4q/w${w}_$rep.txt; exit 1; }
    echo "== tile_wide=$w rep $rep"; grep -E "^s[123]" gpurun_out/r4q/w${w}_$rep.txt
  done
done
