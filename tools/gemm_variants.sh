# time the hvk_linear variants (HVK_LINEAR_VARIANT 0-3) on the shapes they cover
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3; do
  HVK_LINEAR_VARIANT=$v timeout -k 10 300 python tools/bench_gemm.py --only 's0|s1.qkv|s1.proj|s1.fc1|embed' > gpurun_out/gemm_v$v.log 2>&1 || exit 1
done
