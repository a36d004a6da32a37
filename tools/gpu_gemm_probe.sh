# tiled GEMM probes: full kernel vs no-MFMA / no-store / no-DMA builds (make -C tools/probe libhvk_gemm{1,2,3}.so)
set -o pipefail
mkdir -p gpurun_out/gp
for r in 1 2; do
  for v in "" ${PROBES:-tools/probe/libhvk_gemm1.so tools/probe/libhvk_gemm2.so tools/probe/libhvk_gemm3.so}; do
    n=$(basename "${v:-full}" .so)
    timeout -k 10 200 python tools/bench_gemm.py --iters 20 --only "s2|s3" ${v:+--lib $v} > gpurun_out/gp/${n}_$r.txt 2>&1 || exit 1
  done
done
