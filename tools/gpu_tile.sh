# tiled GEMM variants: parity tests under each env setting in $VARS (a,b = two settings), then interleaved
# per-shape timings (tools/bench_gemm.py) -> gpurun_out/tile/g<i>_<round>.txt
set -o pipefail
mkdir -p gpurun_out/tile
VARS=${VARS:-"HVK_TILE_PIPE=1 HVK_TILE_PIPE=0"}
i=0
for v in $VARS; do
  env ${v//,/ } timeout -k 10 180 python -u -m pytest tests/test_gpu_linear.py -k tile -x -q --timeout 60 --timeout-method thread > gpurun_out/tile/t$i.log 2>&1 || { tail -30 gpurun_out/tile/t$i.log; exit 1; }
  i=$((i+1))
done
for r in 1 2; do
  i=0
  for v in $VARS; do
    env ${v//,/ } timeout -k 10 200 python tools/bench_gemm.py --iters 20 --only "${ONLY:-s1.merge|s2|s3}" > gpurun_out/tile/g${i}_$r.txt 2>&1 || exit 1
    i=$((i+1))
  done
done
